#!/usr/bin/env bash
# Same-box A/B of an environment setting on the default bench: alternates `bench.py --no-cpu --no-solve` without and
# with the given INSFM_DIAG value, `rounds` times, printing value / ms_per_step / CG phase per run.
#   usage: tools/ab_env.sh rounds diag_value
set -e
cd "$(dirname "$0")/.."
rounds=$1; diagv=$2
one() {
  timeout -k 10 150 python -u bench.py --no-cpu --no-solve 2>/dev/null | python3 -c "
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print('$1', d['value'], d['ms_per_step'], d['phase_ms_per_step']['cg_iterations'], flush=True)"
}
for r in $(seq "$rounds"); do
  INSFM_DIAG= one default
  INSFM_DIAG=$diagv one "$diagv"
done
