#!/usr/bin/env python3
"""Device vs host derivation of the Schur block pattern and the co-visibility graph in insfm_ba_create
(INSFM_DIAG=pattern_host selects the host pass; read once per process).  For a few scenes -- config 2, a scene with
duplicated observations (two observations of one track on one camera), one with a camera that sees nothing and the
24-camera scene of the multi-rank tests (one coarse cluster) --
prints one JSON line with the block count, the two-level cluster labels and the bits of three deterministic LM steps.
Run twice by tests/test_gpu_parity.py::test_device_block_pattern_matches_host_pass and compared."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config, make_problem  # noqa: E402


def scenes():
    yield "config2", make_config(2)
    prob = make_problem(40, 1500, seed=9)
    rng = np.random.default_rng(9)
    dup = rng.random(prob.n_obs) < 0.05  # duplicate 5 % of the observations (same camera, same track)
    idx = np.sort(np.concatenate([np.arange(prob.n_obs), np.flatnonzero(dup)]), kind="stable")
    prob.uv = np.ascontiguousarray(prob.uv[idx] + rng.normal(0, 0.3, (idx.size, 2)) * np.isin(idx, np.flatnonzero(dup))[:, None])
    prob.cam_idx = np.ascontiguousarray(prob.cam_idx[idx])
    prob.pt_idx = np.ascontiguousarray(prob.pt_idx[idx])
    yield "duplicates", prob
    prob = make_problem(30, 800, seed=4)
    keep = prob.cam_idx != 7  # camera 7 sees nothing
    prob.uv, prob.cam_idx, prob.pt_idx = (np.ascontiguousarray(a[keep]) for a in (prob.uv, prob.cam_idx, prob.pt_idx))
    yield "empty_camera", prob
    # the multi-rank tests' 24-camera scene (tools/dist_check.py --small): one coarse cluster at the default target
    yield "dist_small", make_problem(24, 900, seed=9)


def main():
    dev = torch.device("cuda:0")
    out = dict(env=os.environ.get("INSFM_DIAG", ""), scenes={})
    for name, prob in scenes():
        eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                             device=dev, deterministic=True)
        lab, nc = eng.clusters()
        cg = torch.from_numpy(prob.cams_init.copy()).to(dev)
        pg = torch.from_numpy(prob.points_init.copy()).to(dev)
        losses = [eng.step(cg, pg)[0] for _ in range(3)]
        hsh = hashlib.sha256(cg.cpu().numpy().tobytes() + pg.cpu().numpy().tobytes()).hexdigest()
        out["scenes"][name] = dict(n_obs=int(prob.uv.shape[0]), nnzb=eng.nnzb(), nc=nc, labels=lab.tolist(),
                                   losses=[float(x).hex() for x in losses], params=hsh)
        eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
