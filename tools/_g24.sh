cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v18; mkdir -p $O
timeout -k 10 900 bash tools/ab_libs.sh 4 b512 > $O/final_ab.txt 2>&1 || exit 1
INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_default.txt 2>&1 || exit 1
INSFM_LIB=tools/lib_b512.so INSFM_DIAG=stamps timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_b512.txt 2>&1 || exit 1
