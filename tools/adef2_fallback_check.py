#!/usr/bin/env python3
"""A-DEF2 breakdown fallback, run by tests/test_gpu_parity.py::test_adef2_breakdown_falls_back_to_additive
under INSFM_DIAG=adef2_breakdown (read once per process: the first A-DEF2 k_tl_cgp launch of the process reports a
breakdown at iteration 2).  Steps config 2 three times on a handle whose first solve breaks down, then three times on
a fresh handle (no fault left), and prints one JSON line: per step loss / PCG iterations / failed flag of both and
the fallback count of each handle (insfm_ba_cg_fallbacks)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402


def run(prob, dev, steps=3):
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                         precond=2)
    cg = torch.from_numpy(prob.cams_init.copy()).to(dev)
    pg = torch.from_numpy(prob.points_init.copy()).to(dev)
    out = [eng.step(cg, pg) for _ in range(steps)]
    path = eng.cg_info()[0]
    fb = eng.adef2_fallbacks()
    eng.close()
    return out, path, fb


def main():
    dev = torch.device("cuda:0")
    prob = make_config(2)
    a, path, fa = run(prob, dev)
    b, _, fb = run(prob, dev)
    print(json.dumps(dict(cg_path=path, fallbacks=[fa, fb], losses=[x[0] for x in a], losses_ref=[x[0] for x in b],
                          iters=[int(x[1]["pcg_iters"]) for x in a], iters_ref=[int(x[1]["pcg_iters"]) for x in b],
                          failed=[int(x[1]["failed"]) for x in a], failed_ref=[int(x[1]["failed"]) for x in b])),
          flush=True)


if __name__ == "__main__":
    main()
