cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v16; mkdir -p $O
timeout -k 10 900 bash tools/ab_libs.sh 3 p6 p4 p8 > $O/pipe_ab.txt 2>&1 || exit 1
