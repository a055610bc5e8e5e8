cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v2; mkdir -p $O
timeout -k 10 600 bash tools/ab_libs.sh 2 p1 p2 p3 > $O/schur_probes.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_nocpu.json 2> $O/bench_nocpu.err || exit 1
