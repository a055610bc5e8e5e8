cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v8; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cgp.py tests/test_gpu_dist.py tests/test_gpu_gp.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_det.log 2>&1; echo "rc=$?" >> $O/pytest_det.log
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu --no-solve --deterministic > $O/bench_det_$i.json 2> $O/bench_det_$i.err || exit 1; done
timeout -k 10 200 python -u bench.py --no-cpu --no-solve > $O/bench_nocpu.json 2> $O/bench_nocpu.err || exit 1
