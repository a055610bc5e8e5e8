#!/usr/bin/env python3
"""Parity of an opt-in CG path switched by an environment variable read once per process (argv[1], default
INSFM_PC_CLUSTER: the cluster reduction of the CG's row partials; INSFM_CG_STREAM: the CG on its own stream):
config-2 LM steps on the GPU vs the oracle, same PCG iterations and trials, parameters to 1e-9.  Prints one JSON line.
Run by tests/test_gpu_parity.py (test_pc_cluster_reduction_parity, test_cg_stream_parity) in a subprocess with the
variable set."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    prob = make_config(2)
    dev = torch.device("cuda:0")
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev)
    ora = O.OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points)
    cg, pg = torch.from_numpy(prob.cams_init.copy()).to(dev), torch.from_numpy(prob.points_init.copy()).to(dev)
    co, po = prob.cams_init.copy(), prob.points_init.copy()
    var = sys.argv[1] if len(sys.argv) > 1 else "INSFM_PC_CLUSTER"
    out = dict(env=os.environ.get(var), steps=[])
    for _ in range(3):
        lg, st = eng.step(cg, pg)
        lo = ora.step(co, po)
        so = ora.stats()
        rc = float(np.abs(cg.cpu().numpy() - co).max() / np.abs(co).max())
        rp = float(np.abs(pg.cpu().numpy() - po).max() / np.abs(po).max())
        out["steps"].append(dict(pcg=[st["pcg_iters"], so["pcg_iters"]], trials=[st["trials"], so["trials"]],
                                 loss_rel=abs(lg - lo) / lo, cams_rel=rc, points_rel=rp))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
