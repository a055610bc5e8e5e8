cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v20; mkdir -p $O
timeout -k 10 120 ./tools/lds_bench > $O/lds_bench.txt 2>&1 || exit 1
