"""Per-kernel averages of rocprofv3 --pmc counters (counter_collection.csv) -> JSON.
usage: pmc_summary.py counter_collection.csv out.json [kernel substrings...]"""
import csv
import json
import sys
from collections import defaultdict


def main(path, out, names):
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        for k in names:
            if k in r["Kernel_Name"]:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {k: {c: {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)} for c, v in cs.items()}
           for k, cs in agg.items()}
    json.dump({"source": path, "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["k_gj_step", "k_gj_pinv0", "k_schur", "k_tl_pspmv", "k_tl_pc"])
