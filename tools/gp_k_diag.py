"""GP step parity diagnostic across cluster sizes (prints GPU vs oracle stats per step)."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from instantsfm_amd.engine import GlobalPositioner
from instantsfm_amd.synth import make_gp_problem
from oracle import oracle as O
DEV = torch.device("cuda:0")
for K in (32, 16, 12, 8):
    p = make_gp_problem(30, 1000, seed=1, init="perturbed", depth_frac=0.0)
    eng = GlobalPositioner(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, device=DEV, precond=1,
                           cluster_size=K)
    ora = O.OracleGP(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, precond=1, cluster_size=K)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(DEV)  # noqa: E731
    cg, pg, sg = d(p.cams_init), d(p.points_init), d(p.scales_init)
    co, po, so = p.cams_init.copy(), p.points_init.copy(), p.scales_init.copy()
    print("K", K, "clusters gpu", eng.clusters()[1], "oracle", ora.clusters()[1])
    for s in range(4):
        lg, st = eng.step(cg, pg, sg)
        lo = ora.step(co, po, so)
        sto = ora.stats()
        print(" step", s, "gpu", st["pcg_iters"], st["trials"], st["coarse_used"], f"{lg:.12e}", "ora", sto["pcg_iters"],
              sto["trials"], sto["coarse_used"], f"{lo:.12e}")
    eng.close()
