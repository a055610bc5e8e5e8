#!/usr/bin/env python3
"""Config-3 LM steps with INSFM_DIAG=trace2 (set it in the environment): the library prints, per step, the host
timestamps (us since the step began) of its API calls to stderr.  usage: INSFM_DIAG=trace2 python tools/host_trace.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prob = make_config(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
dev = torch.device("cuda:0")
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
cams = torch.from_numpy(prob.cams_init.copy()).to(dev)
pts = torch.from_numpy(prob.points_init.copy()).to(dev)
for k in range(10):
    t0 = time.perf_counter()
    eng.step(cams, pts)
    print(f"python step {k}: {1e6 * (time.perf_counter() - t0):.0f} us", file=sys.stderr, flush=True)
