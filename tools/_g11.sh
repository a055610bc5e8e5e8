cd $GRAFT_REPO_ROOT
R=$PWD
tools/gpu_session.sh \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "smoketest|300|python -u -m pytest tests/test_gpu_smoke.py tests/test_gpu_passes.py tests/test_gpu_mapper.py -m gpu -v --timeout 200 --timeout-method thread" \
 "pmc_fetch|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
 "pmc_write|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
 "pmc_cgp_f|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_fetch -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_fetch.json" \
 "pmc_cgp_w|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_write -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_write.json"
