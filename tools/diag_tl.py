import numpy as np, torch, sys
sys.path.insert(0, '.')
from instantsfm_amd.engine import BundleAdjuster
from instantsfm_amd.synth import make_problem
from oracle import oracle as O
DEV = torch.device('cuda:0')
for model in (2, 4, 6):
    for det in (True, False):
        for K in (32, 6):
            prob = make_problem(30, 800, seed=5, model=model)
            eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=DEV, deterministic=det, cluster_size=K)
            eng.debug_linearize(torch.from_numpy(prob.cams_init).to(DEV), torch.from_numpy(prob.points_init).to(DEV))
            try:
                it = eng.debug_solve(1 + 1e-4)
            except Exception as e:
                it = str(e)[:40]
            ora = O.OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, precond=1, cluster_size=K)
            ora.linearize(prob.cams_init, prob.points_init)
            print(model, det, K, 'gpu', it, 'oracle', ora.solve(1 + 1e-4), eng.clusters()[1], ora.clusters()[1], flush=True)
            eng.close()
