"""Timing probe for the CG iteration kernel (run under rocprofv3 --kernel-trace --stats with INSFM_CG_PROBE set).
One linearization + one damped solve of config 3 with a fixed iteration cap."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prob = make_config(int(os.environ.get("CFG", "3")))
dev = torch.device("cuda:0")
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                     pcg_max_iter=int(os.environ.get("ITERS", "100")))
cams = torch.from_numpy(prob.cams_init).to(dev)
pts = torch.from_numpy(prob.points_init).to(dev)
eng.debug_linearize(cams, pts)
for _ in range(2):
    try:
        print("iters", eng.debug_solve(1.0001))
    except Exception as e:  # probe modes produce garbage numerics
        print("solve:", e)
torch.cuda.synchronize()
