cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_nocpu.json 2> $O/bench_nocpu.err || exit 1
timeout -k 10 200 python -u bench.py --deterministic --no-cpu --no-solve > $O/bench_det.json 2> $O/bench_det.err || exit 1
