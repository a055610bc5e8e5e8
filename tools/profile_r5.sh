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
S[stamps]="stamps|200|INSFM_DIAG=stamps python -u tools/stamp_probe.py > $R/gpurun_out/stamps.log"
S[ab_old]="ab_old|600|tools/ab_trees.sh 3 abtree/old"
S[cgtrace]="cgtrace|300|INSFM_DIAG=cgp_trace python -u bench.py --no-cpu --no-solve --steps 6 > $R/gpurun_out/cgtrace_new.json 2> $R/gpurun_out/cgtrace_new.err; INSFM_DIAG=cgp_trace python -u abtree/old/bench.py --no-cpu --no-solve --steps 6 > $R/gpurun_out/cgtrace_old.json 2> $R/gpurun_out/cgtrace_old.err"
S[gj]="gj|200|for m in 567 639 747; do tools/bench_dense_p5 \$m 30; tools/bench_dense_p6 \$m 30; done"
S[ab_k]="ab_k|600|tools/ab_args.sh 2 --cluster-size=14 --cluster-size=12 --cluster-size=10 --cluster-size=16"
S[sp]="sp|300|python -u -m pytest tests/test_gpu_parity.py -q -k test_solve_parity --timeout 120 --timeout-method thread > $R/gpurun_out/sp_default.log 2>&1; INSFM_DIAG=no_cgp python -u -m pytest tests/test_gpu_parity.py -q -k test_solve_parity --timeout 120 --timeout-method thread > $R/gpurun_out/sp_nocgp.log 2>&1; INSFM_DIAG=cgp_trace python -u -m pytest tests/test_gpu_parity.py -q -k \"test_solve_parity and 1-32-True-2\" -s --timeout 120 --timeout-method thread > $R/gpurun_out/sp_trace.log 2>&1; true"
S[ab_prio]="ab_prio|400|tools/ab_env.sh 3 side_hi; tools/ab_env.sh 2 side_normal"
S[ab_late]="ab_late|500|tools/ab_env.sh 3 late_chain"
S[trace_late]="trace_late|240|cd /tmp && INSFM_DIAG=late_chain rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_late -o run -- python3 $R/bench.py --no-cpu --no-solve"
S[tl]="tl|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k \"lagged or two_level or coarse or config3 or solve_parity\""
S[gloo2]="gloo2|400|INSFM_DIST_BACKEND=gloo python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $R/gpurun_out/gloo2.json"
S[pmc_cgp_f]="pmc_cgp_f|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_fetch -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_fetch.json"
S[pmc_cgp_w]="pmc_cgp_w|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_write -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_write.json"
S[par]="par|600|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py"
S[ab_rd]="ab_rd|500|tools/ab_env.sh 3 schur_y"
S[rdq]="rdq|300|INSFM_DIAG=create python -u bench.py --no-cpu --no-solve > $R/gpurun_out/rdq.json 2> $R/gpurun_out/rdq.err; grep -h 'Schur build' $R/gpurun_out/rdq.err; python3 -c \"import json; d=json.loads([l for l in open('$R/gpurun_out/rdq.json') if l.startswith('{')][-1]); print(d['value'], d['kernel_us'], d['phase_ms_per_step'])\""
S[ab_cu]="ab_cu|600|tools/ab_env.sh 2 side_cu16 && tools/ab_env.sh 2 side_cu32 && tools/ab_env.sh 2 side_cu64"
S[ab_fork]="ab_fork|500|tools/ab_env.sh 4 lin_fork_early"
S[benchdef]="benchdef|400|python -u bench.py > $R/gpurun_out/bench_default.json"
S[adef]="adef|400|for i in 1 2; do timeout -k 10 150 python -u bench.py --no-cpu --no-solve --precond 2 > $R/gpurun_out/adef_\$i.json 2> $R/gpurun_out/adef_\$i.err || exit 1; timeout -k 10 150 python -u bench.py --no-cpu --no-solve > $R/gpurun_out/ad_\$i.json 2>> $R/gpurun_out/adef_\$i.err || exit 1; done; for f in adef_1 ad_1 adef_2 ad_2; do python3 -c \"import json; d=json.loads([l for l in open('$R/gpurun_out/\$f.json') if l.startswith('{')][-1]); print('\$f', d['value'], d['ms_per_step'], d['phase_ms_per_step']['cg_iterations'], d['pcg_iters'], sum(d['pcg_iters']), d['final_rmse_px'], d['kernel_us'])\"; done"
S[solve]="solve|200|python -u tools/solve_probe.py --modes alive,solve,warm --reps 2"
args=()
for k in "$@"; do args+=("${S[$k]}"); done
exec tools/gpu_session.sh "${args[@]}"
