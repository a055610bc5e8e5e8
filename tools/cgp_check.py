#!/usr/bin/env python3
"""The persistent register-resident CG (k_tl_cgp) against the launch-per-iteration two-level CG (INSFM_DIAG=no_cgp,
read once per process): run this twice, once with each setting, and compare the JSON lines.  Per scene: LM losses and
PCG iterations of a few non-deterministic steps, the CG launches per step (k_tl_cgp: one per trial), wall-clock LM
steps per second.  Used by tests/test_gpu_cgp.py; `--steps` / `--scenes` for timing runs."""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config, make_problem  # noqa: E402


def scene(name):
    """(problem, engine options) of a named scene; "fine": 300 cameras in clusters of 4, so the coarse dimension
    (75 clusters x 9 = 675) exceeds two entries per thread of a k_tl_cgp workgroup."""
    if name == "small":
        return make_problem(40, 1500, seed=3), {}
    if name == "fine":
        return make_problem(300, 12000, seed=8), dict(cluster_size=4)
    if name == "config2":
        return make_config(2), {}
    if name == "config3":
        return make_config(3), {}
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="small,fine,config2")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--det", action="store_true", help="deterministic mode (the fixed-order k_tl_cgp variant)")
    ap.add_argument("--repeat", type=int, default=1, help="run each scene this many times (bitwise reproducibility)")
    ap.add_argument("--precond", type=int, default=1,
                    help="1: the additive form both CG paths run (default); 2: A-DEF2 (k_tl_cgp only)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = dict(env=os.environ.get("INSFM_DIAG", ""), scenes={})
    for name in [n for n in a.scenes.split(",") for _ in range(a.repeat)]:
        prob, opts = scene(name)
        if a.det:
            opts = dict(opts, deterministic=True)
        eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                             device=dev, precond=a.precond, **opts)
        cg = torch.from_numpy(prob.cams_init.copy()).to(dev)
        pg = torch.from_numpy(prob.points_init.copy()).to(dev)
        eng.step(cg, pg)  # warm-up (first-touch allocations, code objects)
        losses, iters, launches, trials, failed = [], [], [], [], []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loss, st = eng.step(cg, pg)
            if st["failed"]:
                print(f"{name}: solver failed: {eng.last_error()}", file=sys.stderr, flush=True)
            losses.append(float(loss))
            iters.append(int(st["pcg_iters"]))
            failed.append(int(st["failed"]))
            launches.append(int(st["cg_launches"]))
            trials.append(int(st["trials"]))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        _, nc = eng.clusters()
        key = name if name not in out["scenes"] else f"{name}#{sum(k.split('#')[0] == name for k in out['scenes'])}"
        out["scenes"][key] = dict(params_sha=hashlib.sha256(cg.cpu().numpy().tobytes() + pg.cpu().numpy().tobytes()).hexdigest(),
                                   losses_hex=[float(x).hex() for x in losses],losses=losses, iters=iters, launches=launches, trials=trials, failed=failed, nc=nc,
                                   steps_per_s=a.steps / dt, D=eng.D, path=eng.cg_info()[0])
        eng.close()
        print(json.dumps(dict(scene=key, **out["scenes"][key])), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
