#!/usr/bin/env bash
# Round-3 profile session: kernel stats of the default bench and the FETCH_SIZE / WRITE_SIZE passes behind
# profiles/pmc_traffic.json (tools/pmc_traffic.py).  Each step under its own time limit via tools/gpu_session.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
exec tools/gpu_session.sh \
  "stats|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --no-cpu --no-solve" \
  "pmc_fetch|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "pmc_write|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve"
