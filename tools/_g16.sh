cd $GRAFT_REPO_ROOT
R=$PWD
tools/gpu_session.sh \
 "gpu|1000|python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread" \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchcpu|400|python -u bench.py > $R/gpurun_out/bench_default.json" \
 "benchdet|200|python -u bench.py --deterministic --no-cpu --no-solve > $R/gpurun_out/bench_det.json" \
 "trace|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o run -- python3 $R/bench.py --no-cpu --no-solve" \
 "pmc_fetch|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
 "pmc_write|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-solve" \
 "pmc_cgp_f|150|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_fetch -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_fetch.json" \
 "pmc_cgp_w|150|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_cgp_write -o run -- python3 $R/tools/cgp_pmc_probe.py > $R/gpurun_out/cgp_probe_write.json"
