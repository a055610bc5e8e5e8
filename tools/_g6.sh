cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v4; mkdir -p $O
timeout -k 10 600 bash tools/ab_libs.sh 3 fb0 > $O/factor_basis_ab.log 2>&1 || exit 1
INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_fb1.log 2>&1 || exit 1
INSFM_LIB=tools/lib_fb0.so INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_fb0.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cgp.py -m gpu -q -x --timeout 600 --timeout-method thread > $O/pytest_parity_cgp.log 2>&1; echo "rc=$?" >> $O/pytest_parity_cgp.log
