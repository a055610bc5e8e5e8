cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 600 --timeout-method thread > gpurun_out/r6/pytest_gpu_a.log 2>&1
echo "rc=$?" >> gpurun_out/r6/pytest_gpu_a.log
