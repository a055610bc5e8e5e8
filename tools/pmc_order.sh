#!/usr/bin/env bash
# L2 hit rate and L1->L2 read latency of k_schur under the observation / work orders (tools/order_probe.sh),
# one rocprofv3 --pmc pass per counter set and order.  usage: tools/pmc_order.sh 0:0 1:1 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/pmc_order
mkdir -p $out
for spec in "$@"; do
  o="${spec%%:*}"; x="${spec#*:}"
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
    i=$((i+1))
    d=$out/o${o}x${x}_p$i
    INSFM_SCHUR_ORDER=$o INSFM_SCHUR_XCD=$x timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $d -o run -- \
      python3 tools/schur_probe.py > $d.log 2>&1 || { echo "order $spec pass $i failed"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*counter_collection.csv" | head -1)
    echo "== order=$o xcd=$x pass $i"
    python3 tools/pmc_summary.py "$f" $d.json k_schur | grep -B1 mean_per_dispatch | grep -v dispatches
  done
done
