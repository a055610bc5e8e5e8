"""Global-positioning oracle (TorchGP.Optimize, global_positioning.py:45-206) against an independent dense numpy
restatement of the same damped Gauss-Newton system: unknowns [camera positions, points, free scales], residual
r_o = f_o (t_o - s_o (X_p - c_i)) (utils/cost_function.py:23-29), Huber kernel with Triggs weighting."""
import numpy as np
import pytest

from oracle import oracle as O
from instantsfm_amd.synth import make_gp_problem


def dense_gp_step(p, cams, pts, scales, f, delta=0.1, cmin=1e-6, cmax=1e32):
    """Dense damped normal equations of one LM solve; returns (dc, dX, ds)."""
    C, P, N = p.n_cams, p.n_points, p.n_obs
    free = np.flatnonzero(p.sfree)
    sidx = -np.ones(N, np.int64)
    sidx[free] = np.arange(free.size)
    n = 3 * C + 3 * P + free.size
    J = np.zeros((3 * N, n))
    r = np.zeros(3 * N)
    fo = p.fcam[p.cam_idx]
    for o in range(N):
        c, q = p.cam_idx[o], p.pt_idx[o]
        e = pts[q] - cams[c]
        ro = fo[o] * (p.trans[o] - scales[o] * e)
        nr = np.linalg.norm(ro)
        sw = np.sqrt(1.0 if nr < delta else delta / nr)
        rows = slice(3 * o, 3 * o + 3)
        r[rows] = sw * ro
        J[rows, 3 * c:3 * c + 3] = sw * fo[o] * scales[o] * np.eye(3)
        J[rows, 3 * C + 3 * q:3 * C + 3 * q + 3] = -sw * fo[o] * scales[o] * np.eye(3)
        if sidx[o] >= 0:
            J[rows, 3 * C + 3 * P + sidx[o]] = -sw * fo[o] * e
    H = J.T @ J
    H[np.diag_indices(n)] = np.clip(np.diag(H), cmin, cmax) * f
    x = np.linalg.solve(H, -J.T @ r)
    ds = np.zeros(N)
    ds[free] = x[3 * C + 3 * P:]
    return x[:3 * C].reshape(C, 3), x[3 * C:3 * C + 3 * P].reshape(P, 3), ds


@pytest.mark.parametrize("depth_frac", [0.0, 0.3, 1.0])
@pytest.mark.parametrize("precond", [0, 1])
@pytest.mark.parametrize("f", [1.5, 1.001])
def test_gp_solve_matches_dense(depth_frac, precond, f):
    p = make_gp_problem(12, 60, track_len=5, seed=3, depth_frac=depth_frac, init="perturbed", init_sigma=0.3)
    gp = O.OracleGP(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points, pcg_tol=1e-13,
                    precond=precond, cluster_size=4)
    gp.linearize(p.cams_init, p.points_init, p.scales_init)
    it = gp.solve(f)
    assert it > 0
    dc_ref, dX_ref, ds_ref = dense_gp_step(p, p.cams_init, p.points_init, p.scales_init, f)
    dc = gp.get(O.DC)
    dX = gp.get(O.DP)
    ds = gp.ds()
    scale = max(np.abs(dc_ref).max(), np.abs(dX_ref).max())
    rtol = 1e-7 if f > 1.1 else 1e-5
    np.testing.assert_allclose(dc.reshape(-1, 3), dc_ref, atol=rtol * scale)
    np.testing.assert_allclose(dX.reshape(-1, 3), dX_ref, atol=rtol * scale)
    np.testing.assert_allclose(ds, ds_ref, atol=rtol * max(np.abs(ds_ref).max(), 1e-12))
    assert np.all(ds[p.sfree == 0] == 0.0)


def test_gp_cost_is_huber_of_pairwise_residual():
    p = make_gp_problem(10, 40, track_len=4, seed=5, init="perturbed")
    gp = O.OracleGP(p.trans, p.cam_idx, p.pt_idx, p.fcam, p.sfree, p.n_cams, p.n_points)
    e = p.points_init[p.pt_idx] - p.cams_init[p.cam_idx]
    res = p.fcam[p.cam_idx][:, None] * (p.trans - p.scales_init[:, None] * e)
    s = (res ** 2).sum(1)
    d = 0.1
    ref = np.where(np.sqrt(s) < d, s, 2 * d * np.sqrt(s) - d * d).sum()
    loss, rmse = gp.cost(p.cams_init, p.points_init, p.scales_init)
    assert loss == pytest.approx(ref, rel=1e-12)
    assert rmse == pytest.approx(np.sqrt(s.mean()), rel=1e-12)


@pytest.mark.parametrize("init", ["random", "perturbed"])
def test_gp_converges_to_ground_truth_up_to_similarity(init):
    p = make_gp_problem(30, 800, seed=1, init=init, outlier_frac=0.0)
    cams, pts, scales, hist = O.gp_solve_to_convergence(p, max_iters=100)
    assert hist[-1] < 1e-2 * hist[0]
    # gauge: global translation + scale (rotation is fixed by the world-frame rays)
    A = np.vstack([cams, pts])
    B = np.vstack([p.cams_gt, p.points_gt])
    Ac, Bc = A - A.mean(0), B - B.mean(0)
    k = (Ac * Bc).sum() / (Ac * Ac).sum()
    err = np.linalg.norm(k * Ac - Bc, axis=1)
    assert np.median(err) < 0.1
    assert np.median(err[:p.n_cams]) < 0.1


def test_gp_fixed_scales_stay_fixed():
    p = make_gp_problem(16, 200, track_len=6, seed=2, depth_frac=0.5, init="perturbed")
    cams, pts, scales, hist = O.gp_solve_to_convergence(p, max_iters=20)
    fixed = p.sfree == 0
    assert fixed.any() and (~fixed).any()
    np.testing.assert_array_equal(scales[fixed], p.scales_init[fixed])
    assert np.abs(scales[~fixed] - 1.0).max() > 1e-3


def test_gp_cost_matches_reference_pairwise_cost(golden_dir):
    """The oracle's residual is the reference's pairwise_cost (golden vectors from the reference itself)."""
    import os
    g = np.load(os.path.join(golden_dir, "gp_cost_golden.npz"))
    ref = g["out"]
    C, P = g["cams"].shape[0], g["pts"].shape[0]
    fcam = np.where(g["calibrated"], 1.0, 0.5)
    for delta in (0.1, 1e6):  # Huber active / inactive (then loss = sum ||r||^2)
        gp = O.OracleGP(g["trans"], g["cam_idx"], g["pt_idx"], fcam, np.ones(len(ref), np.int32), C, P, huber_delta=delta)
        loss, rmse = gp.cost(g["cams"], g["pts"], g["scales"])
        s = (ref ** 2).sum(1)
        exp = np.where(np.sqrt(s) < delta, s, 2 * delta * np.sqrt(s) - delta * delta).sum()
        assert loss == pytest.approx(exp, rel=1e-13)
        assert rmse == pytest.approx(np.sqrt(s.mean()), rel=1e-13)
