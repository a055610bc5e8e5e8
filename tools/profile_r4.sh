#!/usr/bin/env bash
# Round-4 profile session (each step under its own time limit via tools/gpu_session.sh):
#   stats       rocprofv3 kernel trace + stats of the default bench (k_tl_cgp, k_schur on Y records, the side chain)
#   pmc_fetch / pmc_write   FETCH_SIZE / WRITE_SIZE passes behind profiles/pmc_traffic.json (tools/pmc_traffic.py)
#   pmc_schur   the SQ counter sets of k_schur (tools/pmc_schur.sh: SQ_INSTS_LDS, LDS bank conflicts, MFMA busy)
#   schur_det   k_schur timed in the order-fixed deterministic form against the default (tools/schur_probe.py)
#   gj          the pivot-block inversion variants of the Gauss-Jordan chain (tools/bench_dense_p4 / _p5)
#   create      the host phases of insfm_ba_create and TorchBA.Solve (tools/create_probe.py, INSFM_DIAG=create)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
exec tools/gpu_session.sh \
  "stats|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --no-cpu --no-solve" \
  "pmc_fetch|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "pmc_write|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
  "pmc_schur|300|tools/pmc_schur.sh" \
  "schur_det|200|python3 tools/schur_probe.py && DET=1 python3 tools/schur_probe.py" \
  "gj|200|for m in 567 639 747; do tools/bench_dense_p4 \$m 30; tools/bench_dense_p5 \$m 30; done" \
  "create|300|INSFM_DIAG=create python3 tools/create_probe.py --reps 3"
