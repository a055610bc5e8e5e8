cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v6; mkdir -p $O
INSFM_DIAG=cgp_trace timeout -k 10 200 python -u bench.py --no-cpu --no-solve --steps 6 > $O/cgtrace.json 2> $O/cgtrace.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cgp.py -m gpu -q -x --timeout 600 --timeout-method thread > $O/pytest_parity_cgp.log 2>&1; echo "rc=$?" >> $O/pytest_parity_cgp.log
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu --no-solve > $O/bench_$i.json 2> $O/bench_$i.err || exit 1; done
