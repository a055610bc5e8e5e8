#!/usr/bin/env bash
# bench.py (config 3, no CPU baseline / Solve leg) once per setting, each in its own process; prints LM it/s and the
# per-phase split.  A setting is environment assignments and/or bench.py options, e.g. "INSFM_X=1 --cluster-size 12";
# "-" = defaults.  usage: tools/bench_env.sh SETTING ...
cd "$(dirname "$0")/.."
for spec in "$@"; do
  [ "$spec" = "-" ] && spec=""
  envs=(); args=()
  for w in $spec; do
    if [[ "$w" == *=* && "$w" != --* ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-cpu --no-solve "${args[@]}" 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('[${spec:--}]', d['value'], 'it/s', d['ms_per_step'], 'ms', 'phases', d['phase_ms_per_step'], 'iters', sum(d['pcg_iters']), 'rmse', d['final_rmse_px'])" || exit 1
done
