"""Build profiles/pmc_traffic.json from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

hbm_bytes per launch = (corr * FETCH_SIZE + WRITE_SIZE) * 1024, where corr = 2 for kernels whose reads are 16-B/lane
streaming loads (gfx950 FETCH_SIZE counts half of those, MI355X_MICROARCH.md HBM section) and 1 otherwise.
Launches that exit early (CG iterations after convergence) are excluded by a minimum-duration filter.
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"k_schur": 1.0, "k_tl_pspmv": 2.0, "k_cg_iter": 2.0, "k_tl_cgp": 1.0, "k_lin_points": 1.0}


def load(path, counter):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k in KERNELS:
            if k + "<" in name or k + "(" in name:
                out[k].append((float(r["Counter_Value"]), dur))
    return out


def main(fetch_csv, write_csv, out_json, config, source, cgp=None):
    """cgp: (fetch csv, write csv, probe json) of tools/cgp_pmc_probe.py -- k_tl_cgp's entry from its last `reps`
    launches (the re-run of one solve at a known iteration count) instead of the bench pass's mixed solves."""
    f, w = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    res = {}
    if cgp is not None:
        pr = json.loads([ln for ln in open(cgp[2]) if ln.startswith("{")][-1])
        cf = load(cgp[0], "FETCH_SIZE")["k_tl_cgp"][-pr["reps"]:]
        cw = load(cgp[1], "WRITE_SIZE")["k_tl_cgp"][-pr["reps"]:]
        fk, wk = sum(v for v, _ in cf) / len(cf), sum(v for v, _ in cw) / len(cw)
        res["k_tl_cgp"] = {"FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk, "fetch_correction": 1.0,
                           "hbm_bytes_per_launch": int((fk + wk) * 1024), "samples": len(cf),
                           "iterations": pr["iterations"],
                           "note": "tools/cgp_pmc_probe.py: the last solve of 10 LM steps re-run by "
                                   "insfm_ba_debug_time_cgp, the launch bench.py's roofline entry times"}
    for k, corr in KERNELS.items():
        if k in res or not f.get(k) or not w.get(k):
            continue
        dmax = max(d for _, d in f[k])
        fv = [v for v, d in f[k] if d > 0.3 * dmax]
        wv = [v for v, d in w[k] if d > 0.3 * max(dd for _, dd in w[k])]
        fk, wk = sum(fv) / len(fv), sum(wv) / len(wv)
        res[k] = {"FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk, "fetch_correction": corr,
                  "hbm_bytes_per_launch": int((corr * fk + wk) * 1024), "samples": len(fv)}
    json.dump({"config": config, "source": source, "kernels": res}, open(out_json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    # usage: pmc_traffic.py fetch.csv write.csv out.json config [cgp_fetch.csv cgp_write.csv cgp_probe.json]
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]),
         "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over 'python bench.py --steps 2 --warmup 0 "
         "--no-cpu'; hbm_bytes = (corr*FETCH_SIZE + WRITE_SIZE) * 1024 (corr = 2 for 16-B/lane streaming reads: gfx950 "
         "FETCH_SIZE counts half of those, MI355X_MICROARCH.md HBM section); early-exit CG launches excluded",
         cgp=tuple(sys.argv[5:8]) if len(sys.argv) >= 8 else None)
