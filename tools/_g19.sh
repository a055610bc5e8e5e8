cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "deterministic" -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_det.log 2>&1; echo "rc=$?" >> $O/pytest_det.log
