cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests/test_gpu_cgp.py tests/test_gpu_parity.py -m gpu -v --maxfail=8 --timeout 600 --timeout-method thread -k "cgp or reject or adef2 or product_default or deterministic" > gpurun_out/r6/pytest_gpu_b.log 2>&1
echo "rc=$?" >> gpurun_out/r6/pytest_gpu_b.log
