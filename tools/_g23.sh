cd $GRAFT_REPO_ROOT
R=$PWD
tools/gpu_session.sh \
 "gpu|1000|python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread" \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchcpu|400|python -u bench.py > $R/gpurun_out/bench_default2.json"
