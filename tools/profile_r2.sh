#!/usr/bin/env bash
# Round-2 profile session: kernel stats of the default bench, FETCH/WRITE and SQ (MFMA / VALU) PMC passes, the widened
# benches.  Each step under its own time limit via tools/gpu_session.sh; outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
exec tools/gpu_session.sh \
  "stats|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --no-cpu --no-solve" \
  "pmc_fetch|120|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "pmc_write|120|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "pmc_sq|120|cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "bench_gp|240|python3 bench.py --path gp" \
  "bench_tracks|240|python3 bench.py --path tracks" \
  "bench_passes|240|python3 bench.py --path passes" \
  "bench_mapper|400|python3 bench.py --path mapper"
