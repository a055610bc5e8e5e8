"""Time k_schur (and the whole LM step) of config 3 for the library named by INSFM_LIB (tools/schur_variants.sh)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prob = make_config(int(os.environ.get("CFG", "3")))
if os.environ.get("REORDER"):
    # points sorted by their lowest camera (W records of the tracks a band of camera rows touches become contiguous)
    import numpy as np
    P = prob.n_points
    mincam = np.full(P, 1 << 30)
    np.minimum.at(mincam, prob.pt_idx, prob.cam_idx)
    perm = np.argsort(mincam, kind="stable")            # new point k = old point perm[k]
    inv = np.empty(P, np.int64)
    inv[perm] = np.arange(P)
    newpt = inv[prob.pt_idx]
    order = np.argsort(newpt, kind="stable")
    prob.uv, prob.cam_idx, prob.pt_idx = prob.uv[order], prob.cam_idx[order], newpt[order].astype(np.int32)
    prob.points_init = prob.points_init[perm].copy()
dev = torch.device("cuda:0")
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                     deterministic=bool(os.environ.get("DET")))  # DET=1: the order-fixed one-wave-per-row k_schur
cams = torch.from_numpy(prob.cams_init).to(dev)
pts = torch.from_numpy(prob.points_init).to(dev)
for _ in range(2):
    eng.step(cams, pts)
torch.cuda.synchronize()
t0 = time.perf_counter()
losses = [eng.step(cams, pts)[0] for _ in range(8)]
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 8
us = eng.debug_time_kernel(1, 20)
ul = eng.debug_time_kernel(5, 20)
print(f"{os.path.basename(os.environ.get('INSFM_LIB', 'default'))}{' det' if os.environ.get('DET') else ''}: k_schur {us:.1f} us, "
      f"k_lin_points {ul:.1f} us, step {dt*1e3:.3f} ms, loss {losses[-1]:.10e}", flush=True)
