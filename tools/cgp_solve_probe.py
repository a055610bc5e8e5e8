#!/usr/bin/env python3
"""One debug_solve of test_gpu_parity's small scene (30 cameras, 800 points, seed 5), printing the PCG iterations
(or the error) and a hash of dc: run it with and without INSFM_DIAG=no_cgp to chase a CG breakdown of one path
(INSFM_DIAG=cgp_trace adds k_tl_cgp's per-iteration gamma / delta / rho).
    usage: tools/cgp_solve_probe.py [--det] [--cluster 6] [--model 2]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--det", action="store_true")
    ap.add_argument("--cluster", type=int, default=6)
    ap.add_argument("--model", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    prob = make_problem(30, 800, seed=5, model=a.model)
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                         device=dev, deterministic=a.det, precond=1, cluster_size=a.cluster)
    eng.debug_linearize(torch.from_numpy(prob.cams_init.copy()).to(dev), torch.from_numpy(prob.points_init.copy()).to(dev))
    f = 1.0 + 1e-4
    try:
        it_g = eng.debug_solve(f)
    except Exception as e:  # noqa: BLE001
        it_g = f"error: {e}"
    C, D = prob.n_cams, eng.D
    out = dict(diag=os.environ.get("INSFM_DIAG", ""), det=a.det, cluster=a.cluster, iters=it_g)
    if isinstance(it_g, int):
        dc = eng.debug_get(7, (C, D))
        out["dc_norm"] = float(np.linalg.norm(dc))
    print(out, flush=True)


if __name__ == "__main__":
    main()
