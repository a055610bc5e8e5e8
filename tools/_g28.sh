cd $GRAFT_REPO_ROOT
R=$PWD
O=gpurun_out/r6_v21; mkdir -p $O
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_det -o run -- python3 $R/bench.py --deterministic --no-cpu --no-solve > $R/$O/bench_det_traced.json 2> $R/$O/bench_det_traced.err || exit 1
