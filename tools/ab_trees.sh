#!/usr/bin/env bash
# Same-box A/B of two source trees' default bench (e.g. the previous round's tree copied to abtree/old, built there):
# alternates `bench.py --no-cpu --no-solve` of this tree and of each given tree, `rounds` times.
#   usage: tools/ab_trees.sh rounds dir...
set -e
cd "$(dirname "$0")/.."
rounds=$1; shift
one() {
  timeout -k 10 150 python -u "$1/bench.py" --no-cpu --no-solve 2>/dev/null | python3 -c "
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print('$1', d['value'], d['ms_per_step'], d['phase_ms_per_step'].get('cg_iterations'), d['pcg_iters'], flush=True)"
}
for r in $(seq "$rounds"); do
  one .
  for v in "$@"; do one "$v"; done
done
