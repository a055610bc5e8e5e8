cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v14; mkdir -p $O
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh 4 fact_event > $O/fact_ab.txt 2>&1 || exit 1
INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cgp.py tests/test_gpu_dist.py tests/test_gpu_smoke.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "rc=$?" >> $O/pytest.log
