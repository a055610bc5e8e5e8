cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v13; mkdir -p $O
timeout -k 10 900 bash tools/ab_libs.sh 3 x2 x4 x8 > $O/xcd_ab.txt 2>&1 || exit 1
