"""Phase timestamps of k_tl_pc (library built with -DPC_TRACE, see tools/schur_variants.sh): wall clock ticks (100 MHz)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prob = make_config(3)
dev = torch.device("cuda:0")
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
cams = torch.from_numpy(prob.cams_init).to(dev)
pts = torch.from_numpy(prob.points_init).to(dev)
for _ in range(3):
    eng.step(cams, pts)
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
from instantsfm_amd import _capi  # noqa: E402
buf = np.zeros(4096)
n = _capi.load().insfm_ba_debug_get(eng._h, 22, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
ts = buf[:6]
print("k_tl_pc phase deltas (us):", [round((ts[k + 1] - ts[k]) / 100.0, 2) for k in range(5)])
