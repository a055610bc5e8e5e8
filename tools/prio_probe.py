"""LM it/s of config 3 (bench.py's timed loop: 2 warm-up steps, reset, 10 timed steps) with the library stream created
at a given torch stream priority.  usage: PRIO=-1|0|default python tools/prio_probe.py"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402

prio = os.environ.get("PRIO", "default")
dev = torch.device("cuda:0")
prob = make_config(3)
ctx = torch.cuda.stream(torch.cuda.Stream(dev, priority=int(prio))) if prio != "default" else None
if ctx:
    ctx.__enter__()
eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
cams0 = torch.from_numpy(prob.cams_init).to(dev)
pts0 = torch.from_numpy(prob.points_init).to(dev)
cams, pts = cams0.clone(), pts0.clone()
for _ in range(2):
    eng.step(cams, pts)
eng.reset()
cams.copy_(cams0)
pts.copy_(pts0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    eng.step(cams, pts)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 10
print(f"prio={prio}: {1.0 / dt:.1f} LM it/s ({dt * 1e3:.3f} ms/step), range {torch.cuda.Stream.priority_range()}",
      flush=True)
