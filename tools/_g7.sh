cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v5; mkdir -p $O
INSFM_DIAG=cgp_trace timeout -k 10 200 python -u bench.py --no-cpu --no-solve --steps 6 > $O/cgtrace.json 2> $O/cgtrace.err || exit 1
INSFM_DIAG=cgp_trace timeout -k 10 200 python -u bench.py --no-cpu --no-solve --steps 6 --deterministic > $O/cgtrace_det.json 2> $O/cgtrace_det.err || exit 1
