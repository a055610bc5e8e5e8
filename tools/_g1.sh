set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
timeout -k 10 200 python -u tools/xchg_diag.py --overlap --out gpurun_out/r6/xchg_ov.json > gpurun_out/r6/xchg_ov.log 2>&1
timeout -k 10 120 python -u tools/xchg_diag.py --overlap --order plain,xchg --out gpurun_out/r6/xchg_ov_rev.json > gpurun_out/r6/xchg_ov_rev.log 2>&1
INSFM_DIAG=own_streams timeout -k 10 120 python -u tools/xchg_diag.py --overlap --out gpurun_out/r6/xchg_ov_own.json > gpurun_out/r6/xchg_ov_own.log 2>&1
timeout -k 10 120 python -u tools/xchg_diag.py --order xchg,plain --out gpurun_out/r6/xchg_seq_x1.json > gpurun_out/r6/xchg_seq_x1.log 2>&1
