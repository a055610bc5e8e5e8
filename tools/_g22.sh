cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v17; mkdir -p $O
for r in 1 2 3; do
  for v in default gnt; do
    if [ $v = default ]; then L=""; else L=tools/lib_$v.so; fi
    INSFM_LIB=$L timeout -k 10 200 python -u bench.py --path gp --no-cpu 2>/dev/null | python3 -c "
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print('$v', d['value'], d['ms_per_step'], d.get('kernel_us'), flush=True)" >> $O/gp_nt_ab.txt || exit 1
  done
done
