"""Repeat the two-level first solve on small scenes (both Schur modes) and report any PCG failure with its status."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_problem  # noqa: E402

DEV = torch.device('cuda:0')
if len(sys.argv) > 2 and sys.argv[2] == "stream":
    _st = torch.cuda.Stream(DEV)
    torch.cuda.set_stream(_st)
    print("using non-default torch stream", _st.cuda_stream)
fails = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    for model in (2, 4, 6):
        for det in (True, False):
            prob = make_problem(30, 800, seed=5, model=model)
            eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                                 device=DEV, deterministic=det, cluster_size=6)
            eng.debug_linearize(torch.from_numpy(prob.cams_init).to(DEV), torch.from_numpy(prob.points_init).to(DEV))
            res = []
            for k in range(3):
                try:
                    res.append(eng.debug_solve(1 + 1e-4))
                except Exception as e:  # noqa: BLE001
                    res.append(str(e))
                    fails += 1
            if any(isinstance(r, str) for r in res) or rep == 0:
                print(rep, model, det, res, flush=True)
            if isinstance(res[-1], str):
                C, D = prob.n_cams, eng.D
                m = eng.debug_get(11, (-1,)).size if False else None
                u = eng.debug_get(9, (C, D)); w = eng.debug_get(10, (C, D)); r = eng.debug_get(15, (C, D))
                gd = eng.debug_get(14, (2, C))
                nc = eng.clusters()[1]
                mm = nc * (D + 1)
                E0 = eng.debug_get(12, (mm, mm)); E1 = eng.debug_get(13, (mm, mm))
                def st(a):
                    return "nan=%d max=%.3e" % (np.isnan(a).sum(), np.nanmax(np.abs(a)))
                nB = (mm + 31) // 32
                for sl in (0, 1):
                    Lf_ = eng.debug_get(16 + sl, (mm, mm)); Dv_ = eng.debug_get(18 + sl, (nB * 32 * 32,)); Li_ = eng.debug_get(20 + sl, (mm, mm))
                    if np.isnan(Li_).any():
                        rr_, cc_ = np.nonzero(np.isnan(Li_))
                        print("   NaN rows", sorted(set(rr_.tolist()))[:10], "cols", sorted(set(cc_.tolist()))[:40], "m", mm, flush=True)
                        L_ = np.tril(Lf_)
                        Lref = np.linalg.inv(L_)
                        ok_ = ~np.isnan(Li_)
                        print("   Linv err (non-NaN)", np.max(np.abs(Li_[ok_] - Lref[ok_])) / np.max(np.abs(Lref)),
                              "Dinv finite", np.isfinite(Dv_).all(), flush=True)
                        for R in range(nB):
                            r0 = 32 * R; nb_ = min(32, mm - r0)
                            Dref = np.linalg.inv(L_[r0:r0 + nb_, r0:r0 + nb_])
                            Dg = Dv_[R * 1024:(R + 1) * 1024].reshape(32, 32)
                            print("     Dinv block", R, "err", np.max(np.abs(Dg[:nb_, :nb_] - Dref)) / np.max(np.abs(Dref)),
                                  "pad max", np.max(np.abs(Dg[nb_:, :])) if nb_ < 32 else 0.0,
                                  "pad-col max", np.max(np.abs(Dg[:nb_, nb_:])) if nb_ < 32 else 0.0, flush=True)
                    print("   slot", sl, "L(lower) nan=%d" % np.isnan(np.tril(Lf_)).sum(), "Dinv nan=%d" % np.isnan(Dv_).sum(),
                          "Linv nan=%d" % np.isnan(Li_).sum(), "Linv upper nonzero=%d" % (np.triu(Li_, 1) != 0).sum(), flush=True)
                print("   u", st(u), "w", st(w), "r", st(r), "gd", st(gd), "sum w.u %.3e" % gd[1].sum(),
                      "E0", st(E0), "E1", st(E1), "sym0 %.2e sym1 %.2e" % (np.max(np.abs(E0 - E0.T)), np.max(np.abs(E1 - E1.T))),
                      flush=True)
            eng.close()
print("failures", fails)
