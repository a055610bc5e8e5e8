#!/usr/bin/env python3
"""Host-side write-back probe (no GPU): TorchBA.Solve's pack() and update() on a config-3 scene with numpy parameters,
four Solves in one process as bench.py's solve_end_to_end runs them, with update()'s phase split; and _pose_matrices
alone.  python tools/wb_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from instantsfm_amd.config.colmap import BUNDLE_ADJUSTER_OPTIONS  # noqa: E402
from instantsfm_amd.processors.bundle_adjustment import _pose_matrices, pack, update  # noqa: E402
from instantsfm_amd.synth import make_config, to_scene  # noqa: E402

prob = make_config(3)
rows = np.ascontiguousarray(prob.cams_init[:, :7])
for k in range(3):
    t = time.perf_counter()
    _pose_matrices(rows)
    print(f"_pose_matrices alone #{k}: {1e3 * (time.perf_counter() - t):.3f} ms", flush=True)
for rep in range(4):
    cams, ims, tracks = to_scene(prob)
    ph = {}
    t0 = time.perf_counter()
    pk = pack(cams, ims, tracks, BUNDLE_ADJUSTER_OPTIONS, phases=ph)
    t1 = time.perf_counter()
    wb = {}
    update(cams, ims, tracks, pk, pk.camera_params.copy(), pk.points_3d.copy(), phases=wb)
    t2 = time.perf_counter()
    print(f"solve {rep}: pack {1e3 * (t1 - t0):.1f} ms, update {1e3 * (t2 - t1):.1f} ms: " +
          ", ".join(f"{k} {1e3 * v:.2f}" for k, v in wb.items()), flush=True)
    del cams, ims, tracks, pk
