#!/usr/bin/env bash
# Same-box A/B of bench.py arguments: alternates `bench.py --no-cpu --no-solve <args>` over the given argument
# strings, `rounds` times.   usage: tools/ab_args.sh rounds "args A" "args B" ...
set -e
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for a in "$@"; do
    timeout -k 10 150 python -u bench.py --no-cpu --no-solve $a 2>>gpurun_out/ab_args.err | python3 -c "
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print('[$a]', d['value'], d['ms_per_step'], d['phase_ms_per_step'].get('cg_iterations'), sum(d['pcg_iters']), d['final_rmse_px'], flush=True)"
  done
done
