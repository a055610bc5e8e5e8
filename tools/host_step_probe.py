"""Host-side cost of one BundleAdjuster.step call outside the C library (config 3): the Python wrapper pieces timed
in isolation, and the wall time per step of the timed loop.  Diagnostics for the inter-step host gap."""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from instantsfm_amd import _capi  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prob = make_config(3)
dev = torch.device("cuda:0")
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
cams0 = torch.from_numpy(prob.cams_init).to(dev)
pts0 = torch.from_numpy(prob.points_init).to(dev)
cams, pts = cams0.clone(), pts0.clone()
N = 2000


def tm(f):
    t0 = time.perf_counter()
    for _ in range(N):
        f()
    return (time.perf_counter() - t0) / N * 1e6


st = _capi.Stats()
print(f"Stats()            {tm(lambda: _capi.Stats()):6.2f} us")
print(f"_capi.load()       {tm(_capi.load):6.2f} us")
print(f"_ptr x2            {tm(lambda: (eng._ptr(cams, (eng.n_cams, eng.D + 1)), eng._ptr(pts, (eng.n_points, 3)))):6.2f} us")


def ctx():
    with eng._on_stream():
        pass


print(f"_on_stream enter/exit {tm(ctx):6.2f} us")
print(f"as_dict            {tm(st.as_dict):6.2f} us")
L = _capi.load()
print(f"ctypes nnzb call   {tm(lambda: L.insfm_ba_nnzb(eng._h)):6.2f} us")
for _ in range(2):
    eng.step(cams, pts)
for rep in range(3):
    eng.reset()
    cams.copy_(cams0)
    pts.copy_(pts0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        eng.step(cams, pts)
        ts.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    print("step wall ms:", " ".join(f"{t:.3f}" for t in ts), f"sum {sum(ts):.3f}")
