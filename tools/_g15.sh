cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v12; mkdir -p $O
INSFM_DIAG=cgp_trace timeout -k 10 200 python -u bench.py --no-cpu --no-solve --steps 6 > $O/cgtrace_glds.json 2> $O/cgtrace_glds.txt || exit 1
INSFM_LIB=tools/lib_g0.so INSFM_DIAG=cgp_trace timeout -k 10 200 python -u bench.py --no-cpu --no-solve --steps 6 > $O/cgtrace_reg.json 2> $O/cgtrace_reg.txt || exit 1
timeout -k 10 700 bash tools/ab_libs.sh 3 g0 > $O/glds_ab.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cgp.py tests/test_gpu_dist.py tests/test_gpu_smoke.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "rc=$?" >> $O/pytest.log
