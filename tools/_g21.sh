cd $GRAFT_REPO_ROOT
R=$PWD
O=gpurun_out/r6_v17; mkdir -p $O
timeout -k 10 300 python -u bench.py --path gp --no-cpu > $O/bench_gp.json 2> $O/bench_gp.err || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_gp -o run -- python3 $R/bench.py --path gp --no-cpu > /dev/null 2>&1 || exit 1
