#!/usr/bin/env bash
# Round-5 GPU session (each step under its own time limit via tools/gpu_session.sh; stops at a fault-class exit).
#   usage: tools/profile_r5.sh step [step ...]   (steps: cgp dist gpu bench bench_hold trace trace_hold pmc_fetch
#          pmc_write solve smoke)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
declare -A S
S[cgp]="cgp|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cgp.py"
S[dist]="dist|800|python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py"
S[gpu]="gpu|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
S[smoke]="smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'"
S[bench]="bench|240|python -u bench.py --no-cpu > $R/gpurun_out/bench.json"
S[benchcpu]="benchcpu|300|python -u bench.py --steps 20 --warmup 5 > $R/gpurun_out/bench_full.json"
S[bench_hold]="bench_hold|200|INSFM_DIAG=chain_hold python -u bench.py --no-cpu --no-solve > $R/gpurun_out/bench_hold.json"
S[trace]="trace|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o run -- python3 $R/bench.py --no-cpu --no-solve"
S[trace_hold]="trace_hold|240|cd /tmp && INSFM_DIAG=chain_hold rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_hold -o run -- python3 $R/bench.py --no-cpu --no-solve"
S[pmc_fetch]="pmc_fetch|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve"
S[pmc_write]="pmc_write|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve"
S[solve]="solve|200|python -u tools/solve_probe.py --modes alive,solve,warm --reps 2"
args=()
for k in "$@"; do args+=("${S[$k]}"); done
exec tools/gpu_session.sh "${args[@]}"
