#!/usr/bin/env python3
"""Tracer-free main-queue timeline of config-3 LM steps: INSFM_DIAG=stamps makes the main-queue
kernels of a step -- k_lin_points, k_schur, k_cg_factor, k_tl_basis, k_tl_cgp, k_cg_finish, k_backsub_rc, k_cost,
k_final, k_publish -- record device-clock (100 MHz) entry / exit stamps (engine.STAMP_KERNELS); this prints, per step
and as medians, the step span (k_lin_points entry to the next one), each kernel's duration, the main queue's busy
time (the sum of the stamped kernels: the kernels a lagged trial runs on the main queue are all stamped) and the
gaps between consecutive kernels.  Steps with more than one trial (a rejected trial relaunches k_schur .. k_publish,
and the stamps keep the last launch) are left out of the medians.  The stamped run's wall time per step is printed
beside (each stamped kernel's workgroups add one atomic; bench.py gives the unstamped rate).

    INSFM_DIAG=stamps python tools/stamp_probe.py [--steps 20] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from instantsfm_amd.engine import STAMP_KERNELS, BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    if "stamps" not in os.environ.get("INSFM_DIAG", ""):
        raise SystemExit("run with INSFM_DIAG=stamps")
    prob = make_config(a.config)
    dev = torch.device("cuda:0")
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
    c0, p0 = torch.from_numpy(prob.cams_init).to(dev), torch.from_numpy(prob.points_init).to(dev)
    cams, pts = c0.clone(), p0.clone()
    for _ in range(a.warmup):
        eng.step(cams, pts)
    eng.reset()
    cams.copy_(c0)
    pts.copy_(p0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters, trials = [], []
    for _ in range(a.steps):
        stt = eng.step(cams, pts)[1]
        iters.append(stt["pcg_iters"])
        trials.append(stt["trials"])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    st = eng.debug_stamps()[-a.steps:].astype(np.float64) / 100.0  # microseconds
    names = list(STAMP_KERNELS)
    order = ["k_lin_points", "k_schur", "k_cg_factor", "k_tl_basis", "k_tl_cgp", "k_cg_finish", "k_backsub_rc",
             "k_cost", "k_final", "k_publish"]
    ix = [names.index(n) for n in order]
    rows = []
    for k in range(len(st) - 1):
        s, n = st[k], st[k + 1]
        t0, t1 = s[ix[0], 0], n[ix[0], 0]
        r = {"span": t1 - t0, "trials": trials[k], "pcg": iters[k]}
        busy, prev_end = 0.0, None
        for name, i in zip(order, ix):
            b, e = s[i]
            if not (t0 <= b < t1):  # not launched in this step
                r[name] = float("nan")
                continue
            r[name] = e - b
            busy += e - b
            if prev_end is not None:
                r["gap>" + name] = b - prev_end
            prev_end = e
        r["gap>next"] = t1 - prev_end
        r["busy"] = busy
        r["busy_frac"] = busy / r["span"]
        rows.append(r)
        print(f"step {k:2d}: " + " ".join(f"{q} {v:.1f}" if isinstance(v, float) else f"{q} {v}" for q, v in r.items()),
              flush=True)
    keep = [r for r in rows if r["trials"] == 1]
    keys = [q for q in rows[0] if q not in ("trials", "pcg")]
    med = {q: float(np.nanmedian([r.get(q, np.nan) for r in keep])) for q in keys}
    gaps = {q: round(v, 2) for q, v in med.items() if q.startswith("gap>")}
    print(json.dumps({"wall_ms_per_step_stamped_run": round(wall, 4),
                      "steps_used": len(keep), "median_us": {q: round(v, 2) for q, v in med.items()},
                      "main_queue_busy_frac_median": round(med["busy_frac"], 4),
                      "gaps_us_median": gaps, "gaps_us_sum_of_medians": round(sum(gaps.values()), 2)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
