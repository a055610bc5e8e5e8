cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v9; mkdir -p $O
timeout -k 10 300 python -u tools/wb_probe.py > $O/wb_probe.txt 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_$i.json 2> $O/bench_$i.err || exit 1; done
