"""Global positioning (TorchGP) on the HIP path vs the C oracle (oracle/ba_oracle.c ora_gp_*).  Needs an MI355X.

Tolerances as for bundle adjustment: linear-solve outputs 1e-8 relative at equal PCG iteration count,
parameters after an LM step 1e-9, loss 1e-10.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from instantsfm_amd.engine import GlobalPositioner  # noqa: E402
from instantsfm_amd.synth import make_gp_problem  # noqa: E402
from oracle import oracle as O  # noqa: E402

DEV = torch.device("cuda:0")


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(DEV)


def engines(p, **kw):
    eng = GlobalPositioner(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, device=DEV, **kw)
    okw = {k: v for k, v in kw.items() if k in ("precond", "cluster_size")}
    ora = O.OracleGP(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, **okw)
    return eng, ora


@pytest.mark.parametrize("depth_frac", [0.0, 0.3])
@pytest.mark.parametrize("precond,cluster", [(0, 32), (1, 32), (1, 6)])
@pytest.mark.parametrize("f", [1.001, 1.5])
def test_gp_solve_parity(depth_frac, precond, cluster, f):
    p = make_gp_problem(40, 1500, seed=2, depth_frac=depth_frac, init="perturbed", init_sigma=0.5)
    eng, ora = engines(p, precond=precond, cluster_size=cluster)
    eng.debug_linearize(dev(p.cams_init), dev(p.points_init), dev(p.scales_init))
    ora.linearize(p.cams_init, p.points_init, p.scales_init)
    it_g = eng.debug_solve(f)
    it_o = ora.solve(f)
    assert it_g == it_o
    C, P = p.n_cams, p.n_points
    assert rel(eng.debug_get(1, (P, 6)), ora.get(O.V)) < 1e-12
    assert rel(eng.debug_get(2, (P, 3)), ora.get(O.GP)) < 1e-12
    assert rel(eng.debug_get(6, (C, 3)), ora.get(O.B)) < 1e-10
    assert rel(eng.debug_get(7, (C, 3)), ora.get(O.DC)) < 1e-8
    assert rel(eng.debug_get(8, (P, 3)), ora.get(O.DP)) < 1e-8
    ds_g, ds_o = eng.debug_ds(), ora.ds()
    assert rel(ds_g, ds_o) < 1e-8
    assert np.all(ds_g[p.sfree == 0] == 0.0)


def test_gp_cost_parity():
    p = make_gp_problem(20, 600, seed=4, depth_frac=0.2, init="random")
    eng, ora = engines(p)
    lg, rg = eng.cost(dev(p.cams_init), dev(p.points_init), dev(p.scales_init))
    lo, ro = ora.cost(p.cams_init, p.points_init, p.scales_init)
    assert abs(lg - lo) / lo < 1e-12 and abs(rg - ro) / ro < 1e-12


@pytest.mark.parametrize("init,depth_frac,precond", [("perturbed", 0.0, 1), ("random", 0.0, 1), ("random", 0.3, 0)])
def test_gp_step_parity(init, depth_frac, precond):
    p = make_gp_problem(30, 1000, seed=1, init=init, depth_frac=depth_frac)
    eng, ora = engines(p, precond=precond)
    cg, pg, sg = dev(p.cams_init), dev(p.points_init), dev(p.scales_init)
    co, po, so = p.cams_init.copy(), p.points_init.copy(), p.scales_init.copy()
    for s in range(6):
        lg, st = eng.step(cg, pg, sg)
        lo = ora.step(co, po, so)
        sto = ora.stats()
        assert st["pcg_iters"] == sto["pcg_iters"] and st["trials"] == sto["trials"], (s, st, sto)
        assert abs(lg - lo) / lo < 1e-10, (s, lg, lo)
        assert rel(cg.cpu().numpy(), co) < 1e-9
        assert rel(pg.cpu().numpy(), po) < 1e-9
        assert rel(sg.cpu().numpy(), so) < 1e-9
    fixed = p.sfree == 0
    assert np.array_equal(sg.cpu().numpy()[fixed], p.scales_init[fixed])


def test_gp_converges_like_oracle():
    p = make_gp_problem(40, 2000, seed=9, init="random")
    eng, _ = engines(p)
    cg, pg, sg = dev(p.cams_init), dev(p.points_init), dev(p.scales_init)
    hist = []
    for _ in range(100):
        hist.append(eng.step(cg, pg, sg)[0])
        if len(hist) >= 8:
            a, b = np.mean(hist[-4:]), np.mean(hist[-8:-4])
            if abs((b - a) / b) < 5e-4:
                break
    _, _, _, hist_o = O.gp_solve_to_convergence(p)
    assert len(hist) == len(hist_o)
    assert abs(hist[-1] - hist_o[-1]) / hist_o[-1] < 1e-6
    # translation + scale gauge: positions match ground truth after a similarity fit
    A = np.vstack([cg.cpu().numpy(), pg.cpu().numpy()])
    B = np.vstack([p.cams_gt, p.points_gt])
    Ac, Bc = A - A.mean(0), B - B.mean(0)
    k = (Ac * Bc).sum() / (Ac * Ac).sum()
    assert np.median(np.linalg.norm(k * Ac - Bc, axis=1)) < 0.1


def test_torchgp_optimize_end_to_end():
    """The TorchGP processor on a reference-class scene: filters, packing, LM loop, write-back, ConvertResults."""
    from scipy.spatial.transform import Rotation
    from instantsfm_amd.processors.global_positioning import TorchGP
    from instantsfm_amd.scene.defs import Camera, CameraModelId, Image, Track
    p = make_gp_problem(24, 800, seed=5, init="random", outlier_frac=0.0)
    rng = np.random.default_rng(0)
    C = p.n_cams
    order = np.argsort(p.cam_idx, kind="stable")
    counts = np.bincount(p.cam_idx, minlength=C)
    starts = np.concatenate([[0], np.cumsum(counts)])
    feat = np.empty(p.n_obs, np.int64)
    feat[order] = np.arange(p.n_obs) - np.repeat(starts[:-1], counts)
    cams, imgs = [], []
    for c in range(C):
        R = Rotation.from_rotvec(rng.normal(0, 0.3, 3)).as_matrix()
        w2c = np.eye(4)
        w2c[:3, :3] = R
        cams.append(Camera(id=c, model_id=CameraModelId.SIMPLE_RADIAL, params=[1000.0, 500.0, 400.0, 0.0],
                           has_prior_focal_length=bool(p.fcam[c] == 1.0)))
        imgs.append(Image(id=c, cam_id=c, is_registered=True, world2cam=w2c,
                          features_undist=p.trans[order[starts[c]:starts[c + 1]]] @ R.T))
    ptr = np.concatenate([[0], np.cumsum(np.bincount(p.pt_idx, minlength=p.n_points))])
    pairs = np.stack([p.cam_idx.astype(np.int64), feat], 1)
    tracks = {q: Track(id=q, xyz=np.zeros(3), observations=pairs[ptr[q]:ptr[q + 1]]) for q in range(p.n_points)}
    gp = TorchGP(device="cuda:0")
    np.random.seed(1)
    gp.InitializeRandomPositions(cams, imgs, tracks)
    opts = dict(min_num_view_per_track=3, thres_loss_function=1e-1, max_num_iterations=100, function_tolerance=5e-4)
    gp.Optimize(cams, imgs, tracks, None, opts, progress=False)
    assert gp.loss_history[-1] < 1e-3 * gp.loss_history[0]
    centers = np.stack([-im.world2cam[:3, :3].T @ im.world2cam[:3, 3] for im in imgs])   # undo ConvertResults
    A = np.vstack([centers, np.stack([tracks[q].xyz for q in range(p.n_points)])])
    B = np.vstack([p.cams_gt, p.points_gt])
    Ac, Bc = A - A.mean(0), B - B.mean(0)
    k = (Ac * Bc).sum() / (Ac * Ac).sum()
    assert np.median(np.linalg.norm(k * Ac - Bc, axis=1)) < 0.1
