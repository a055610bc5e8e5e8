"""Timeline of one LM step from a rocprofv3 kernel_trace.csv: kernel, start offset, duration, gap to the previous
kernel on the same queue (us).  usage: step_timeline.py trace.csv [step index]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("insfm::", "")
    return re.split(r"\(", n, maxsplit=1)[0]


idx = [i for i, r in enumerate(rows) if "k_lin_points" in r["Kernel_Name"]]
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev = {}
agg = {}
for r in rows[i0:i1]:
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
    gap = (s - prev[q]) / 1000 if q in prev else 0.0
    prev[q] = e
    n = short(r["Kernel_Name"])[:30]
    agg[n] = agg.get(n, 0.0) + (e - s) / 1000
    print(f"{(s - t0) / 1000:8.1f} {n:30s} {(e - s) / 1000:8.2f} gap {gap:7.2f} q{q}")
print("step span us", (int(rows[i1]["Start_Timestamp"]) - t0) / 1000)
for n, v in sorted(agg.items(), key=lambda x: -x[1])[:12]:
    print(f"  {n:30s} {v:8.1f}")

# every step of the trace: the main queue's (k_lin_points') busy fraction and the union of all queues' kernels
qm = rows[idx[0]]["Queue_Id"]
fr, un = [], []
for a, b in zip(idx[:-1], idx[1:]):
    s0, s1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b] if r["Queue_Id"] == qm)
    iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), s1)) for r in rows[a:b])
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    fr.append(busy / (s1 - s0))
    un.append(tot / (s1 - s0))
if fr:
    fr_s, un_s = sorted(fr), sorted(un)
    print(f"steps {len(fr)}: main queue busy median {fr_s[len(fr) // 2]:.3f} (min {fr_s[0]:.3f}, max {fr_s[-1]:.3f}); "
          f"any queue busy median {un_s[len(un) // 2]:.3f}")
