cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v22; mkdir -p $O
for r in 1 2; do
  DET=1 timeout -k 10 150 python -u tools/schur_probe.py >> $O/det_lds.txt 2>&1 || exit 1
  for v in l48 l56 l60; do
    DET=1 INSFM_LIB=tools/lib_$v.so timeout -k 10 150 python -u tools/schur_probe.py >> $O/det_lds.txt 2>&1 || exit 1
  done
done
