"""Summarize a rocprofv3 --pmc counter_collection.csv per kernel: wave-cycle split and instruction counts."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    agg[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = d.get("SQ_WAVE_CYCLES")
    if not wc:
        continue
    parts = [f"{k:28s} wave {wc:9.3g}"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in d:
            parts.append(f"{c[3:].lower()} {d[c] / wc:.2f}")
    for c in sorted(d):
        if c not in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            parts.append(f"{c[3:].lower()} {d[c]:.3g}")
    print("  ".join(parts))
