#!/usr/bin/env python3
"""Host-side cost of one TorchBA.Solve on the config-3 scene, phase by phase: pack(), engine creation
(insfm_ba_create's host phases via INSFM_DIAG=create, printed to stderr), the LM steps and the write-back.

    INSFM_DIAG=create python tools/create_probe.py [--config 3] [--reps 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    prob = make_config(a.config)
    cameras, images, tracks = to_scene(prob)
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    for r in range(a.reps):
        t0 = time.perf_counter()
        ph = {}
        pk = BA.pack(cameras, images, tracks, BUNDLE_ADJUSTER_OPTIONS, phases=ph)
        t1 = time.perf_counter()
        cam32, pt32 = pk.indices32()
        eng = BundleAdjuster(pk.model.value, pk.points_2d, cam32, pt32, pk.camera_pps,
                             pk.camera_params.shape[0], pk.points_3d.shape[0], device=dev)
        t2 = time.perf_counter()
        cams = torch.from_numpy(pk.camera_params).to(dev)
        pts = torch.from_numpy(pk.points_3d).to(dev)
        t3 = time.perf_counter()
        eng.step(cams, pts)
        t4 = time.perf_counter()
        BA.update(cameras, images, tracks, pk, cams, pts)
        t5 = time.perf_counter()
        eng.close()
        t6 = time.perf_counter()
        print(f"rep {r}: pack {1e3 * (t1 - t0):.1f} ms, create {1e3 * (t2 - t1):.1f}, params H2D {1e3 * (t3 - t2):.1f}, "
              f"1 step {1e3 * (t4 - t3):.1f}, update {1e3 * (t5 - t4):.1f}, close {1e3 * (t6 - t5):.1f}; pack phases "
              + ", ".join(f"{k} {1e3 * v:.1f}" for k, v in ph.items()), flush=True)


if __name__ == "__main__":
    main()
