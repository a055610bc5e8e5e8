#!/usr/bin/env bash
# A/B of the side-chain schedule (INSFM_SIDE_SCHED 0 / 1) and E-build grid: benches, then a kernel trace.
# usage: tools/ab_side.sh "ENV=.. ENV2=.." ...   (each spec one bench run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
n=0
for spec in "$@"; do
  n=$((n + 1))
  env $spec timeout -k 10 100 python bench.py --no-cpu --no-solve > gpurun_out/ab_$n.log 2>&1 || exit 1
  echo "[$spec] $(grep -o '"value": [0-9.]*' gpurun_out/ab_$n.log | head -1) $(grep -o 'phase_ms_per_step[^}]*' gpurun_out/ab_$n.log)"
done
