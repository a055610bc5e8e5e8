cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v10; mkdir -p $O
timeout -k 10 700 bash tools/ab_libs.sh 3 snt nt0 > $O/snt_ab.txt 2>&1 || exit 1
INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_nt.txt 2>&1 || exit 1
