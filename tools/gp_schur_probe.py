"""Time k_schur_gp (insfm_ba_debug_time_kernel 1) on the GP bench scene; INSFM_CG_PROBE selects a timing probe
(0 exact, 1 non-atomic LDS adds, 2 no accumulation)."""
import os
import sys

import numpy as np
import torch
from instantsfm_amd import _capi
from instantsfm_amd.engine import GlobalPositioner

if len(sys.argv) > 1:  # alternative build of the library (experiments)
    _capi.load(os.path.abspath(sys.argv[1]))
from instantsfm_amd.synth import make_gp_problem

p = make_gp_problem(1000, 200000, track_len=10, seed=0, init="random")
eng = GlobalPositioner(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, device="cuda:0")
d = [torch.from_numpy(a).cuda() for a in (p.cams_init, p.points_init, p.scales_init)]
for _ in range(3):
    eng.step(*d)
print(sys.argv[1:], "k_schur_gp us", eng.debug_time_kernel(1, 20))
