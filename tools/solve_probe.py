#!/usr/bin/env python3
"""Where does a TorchBA.Solve's LM-step time go, against the bench's timed loop?

Per-step wall times (each insfm_ba_step blocks for the trial's loss) of:
  solve      TorchBA.Solve on fresh copies of the config-3 scene (a fresh engine per Solve, like global_mapper.py:115)
  fresh      a fresh BundleAdjuster on the same packed problem, steps right after create
  fresh_sync the same with a device synchronization after create (create's queued device work drained first)
  idle50     fresh_sync, then 50 ms of host sleep before the first step (GPU idle -> clock state)
  busy       fresh_sync, then ~30 ms of GPU work (torch matmuls) right before the first step
  warm       the last engine again after insfm_ba_reset (the bench's timed loop: warmup steps, reset, steps)

    python tools/solve_probe.py [--config 3] [--steps 9] [--reps 2]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from instantsfm_amd.config.colmap import BUNDLE_ADJUSTER_OPTIONS  # noqa: E402
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.processors import bundle_adjustment as BA  # noqa: E402
from instantsfm_amd.synth import make_config, to_scene  # noqa: E402


def fmt(ms, stats):
    return (" ".join(f"{m:.2f}" for m in ms) + f" | sum {sum(ms):.2f} ms, mean {np.mean(ms):.3f} | pcg "
            + ",".join(str(s["pcg_iters"]) for s in stats) + " | cg_launches "
            + ",".join(str(s["cg_launches"]) for s in stats) + " | trials " + ",".join(str(s["trials"]) for s in stats))


def run_steps(eng, cams, pts, n):
    ms, st = [], []
    for _ in range(n):
        t = time.perf_counter()
        _, s = eng.step(cams, pts)
        ms.append(1e3 * (time.perf_counter() - t))
        st.append(s)
    return ms, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--modes", default="solve,fresh,fresh_sync,idle50,busy,warm")
    a = ap.parse_args()
    modes = a.modes.split(",")
    prob = make_config(a.config)
    dev = torch.device("cuda:0")
    x = torch.randn(2048, 2048, device=dev)
    torch.cuda.synchronize()
    keep = None
    if "alive" in modes:  # the bench's situation: another config-3 engine (its own streams) alive during the Solves
        keep = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                              device=dev)
        kc, kp = torch.from_numpy(prob.cams_init).to(dev), torch.from_numpy(prob.points_init).to(dev)
        for _ in range(3):
            keep.step(kc, kp)
        torch.cuda.synchronize()
    if "solve" in modes or "alive" in modes:
        for r in range(a.reps + 1):
            cams, ims, tracks = to_scene(prob)
            ba = BA.TorchBA(device=str(dev))
            ba.Solve(cams, ims, tracks, BUNDLE_ADJUSTER_OPTIONS, progress=False)
            t = ba.timings
            print(f"{'alive' if keep is not None else 'solve'} rep {r}: pack {1e3 * t['pack_s']:.1f} create {1e3 * t['create_s']:.1f} steps "
                  f"{1e3 * t['steps_s']:.1f} update {1e3 * t['update_s']:.1f} ms | steps: " + fmt(t["step_ms"], t["step_stats"]),
                  flush=True)
    if keep is not None:
        keep.close()
    cams_s, ims_s, tracks_s = to_scene(prob)
    pk = BA.pack(cams_s, ims_s, tracks_s, BUNDLE_ADJUSTER_OPTIONS)
    cam32, pt32 = pk.indices32()
    eng = None
    for mode in [m for m in modes if m not in ("solve", "warm", "alive")]:
        for r in range(a.reps):
            if eng is not None:
                eng.close()
            t0 = time.perf_counter()
            eng = BundleAdjuster(pk.model.value, pk.points_2d, cam32, pt32, pk.camera_pps, pk.camera_params.shape[0],
                                 pk.points_3d.shape[0], device=dev)
            cams = torch.from_numpy(pk.camera_params).to(dev)
            pts = torch.from_numpy(pk.points_3d).to(dev)
            t1 = time.perf_counter()
            sync_ms = 0.0
            if mode != "fresh":
                torch.cuda.synchronize()
                sync_ms = 1e3 * (time.perf_counter() - t1)
            if mode == "idle50":
                time.sleep(0.05)
            elif mode == "busy":
                tb = time.perf_counter()
                while time.perf_counter() - tb < 0.03:
                    for _ in range(8):
                        x = (x @ x) * 1e-3
                    torch.cuda.synchronize()
            ms, st = run_steps(eng, cams, pts, a.steps)
            print(f"{mode} rep {r}: create+H2D {1e3 * (t1 - t0):.1f} ms, drain after create {sync_ms:.2f} ms | steps: "
                  + fmt(ms, st), flush=True)
    if "warm" in modes and eng is not None:
        for r in range(a.reps):
            eng.reset()
            cams = torch.from_numpy(pk.camera_params).to(dev)
            pts = torch.from_numpy(pk.points_3d).to(dev)
            torch.cuda.synchronize()
            ms, st = run_steps(eng, cams, pts, a.steps)
            print(f"warm rep {r}: steps: " + fmt(ms, st), flush=True)
    if eng is not None:
        eng.close()


if __name__ == "__main__":
    main()
