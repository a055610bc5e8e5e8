"""A few linearize + solve calls on config 3 (counter collection target for rocprofv3 --pmc)."""
import sys

import torch

sys.path.insert(0, '.')
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

DEV = torch.device('cuda:0')
prob = make_config(3)
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=DEV)
c, p = torch.from_numpy(prob.cams_init).to(DEV), torch.from_numpy(prob.points_init).to(DEV)
eng.debug_linearize(c, p)
for _ in range(3):
    eng.debug_solve(1 + 1e-4)
torch.cuda.synchronize()
print("done")
