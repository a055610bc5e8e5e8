#!/usr/bin/env python3
"""Tracer-free main-queue timeline of config-3 LM steps: INSFM_DIAG=stamps makes k_lin_points,
k_schur, k_tl_cgp, k_cg_finish and k_publish record device-clock (100 MHz) entry / exit stamps; this prints, per step
and as medians, the step span and the regions between the stamped kernels:

  lin        k_lin_points                          boundary   k_publish exit -> next k_lin_points entry
  lin>schur  k_lin_points exit -> k_schur entry     schur      k_schur
  pre-CG     k_schur exit -> k_tl_cgp entry (k_cg_factor, [k_cg_scale], k_tl_basis, dispatch)
  cgp        k_tl_cgp                              post-CG    k_tl_cgp exit -> k_cg_finish entry
  tail       k_cg_finish entry -> k_publish exit (back-substitution, cost, k_final, k_publish)

The gaps are measured without a tracer; the kernels inside pre-CG and tail are not stamped (their busy time is the
sum of their standalone durations).  The unstamped rate of the same run is printed beside.

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

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
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
    iters = []
    for _ in range(a.steps):
        iters.append(eng.step(cams, pts)[1]["pcg_iters"])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    st = eng.debug_stamps()[-a.steps:].astype(np.float64) / 100.0  # microseconds
    LIN, SCH, CGP, FIN, PUB = range(5)
    rows = []
    for k in range(len(st) - 1):
        s, n = st[k], st[k + 1]
        r = {"span": n[LIN, 0] - s[LIN, 0], "lin": s[LIN, 1] - s[LIN, 0], "lin>schur": s[SCH, 0] - s[LIN, 1],
             "schur": s[SCH, 1] - s[SCH, 0], "pre-CG": s[CGP, 0] - s[SCH, 1], "cgp": s[CGP, 1] - s[CGP, 0],
             "post-CG": s[FIN, 0] - s[CGP, 1], "tail": s[PUB, 1] - s[FIN, 0], "boundary": n[LIN, 0] - s[PUB, 1],
             "pcg": iters[k]}
        rows.append(r)
        print(f"step {k:2d}: " + " ".join(f"{q} {v:.1f}" if q != "pcg" else f"pcg {v}" for q, v in r.items()),
              flush=True)
    med = {q: float(np.median([r[q] for r in rows])) for q in rows[0] if q != "pcg"}
    stamped = sum(med[q] for q in ("lin", "schur", "cgp"))
    print(json.dumps({"wall_ms_per_step_stamped_run": round(wall, 4), "median_us": {q: round(v, 2) for q, v in med.items()},
                      "stamped_kernels_busy_frac": round(stamped / med["span"], 4),
                      "gaps_us": {q: round(med[q], 2) for q in ("lin>schur", "post-CG", "boundary")}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
