cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v20; mkdir -p $O
timeout -k 10 200 python -u bench.py --no-cpu --no-solve > $O/bench_lds.json 2> $O/bench_lds.err || exit 1
