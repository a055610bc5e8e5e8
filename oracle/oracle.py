"""ORACLE / TEST INFRASTRUCTURE ONLY -- ctypes wrapper of oracle/ba_oracle.c.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libba_oracle.so")
# "fma": the same source built with fused multiply-adds contracted wherever the compiler likes (-ffp-contract=fast),
# i.e. the same algorithm with different last-bit rounding -- the reference point for how far rounding alone moves a
# result (tests/test_oracle.py::test_pcg_rounding_sensitivity_lives_in_the_near_null_space)
_VARIANTS = {"": _LIB_PATH, "fma": os.path.join(_HERE, "build", "libba_oracle_fma.so")}
_lib = None
_libs = {}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)

# buffer ids for ora_get
W, V, GP, U, GC, S, B, DC, DP = range(9)


def build(quiet=True):
    subprocess.run(["make", "-C", _HERE], check=True, capture_output=quiet)


def lib(variant=""):
    global _lib
    if variant:
        if variant not in _libs:
            path = _VARIANTS[variant]
            if not os.path.exists(path):
                build()
            _libs[variant] = _bind(ctypes.CDLL(path))
        return _libs[variant]
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = _bind(ctypes.CDLL(_LIB_PATH))
    return _lib


def _bind(L):
    if True:
        L.ora_create.restype = ctypes.c_void_p
        L.ora_create.argtypes = [ctypes.c_int] * 4 + [_dp, _ip, _ip, _dp, _dp, _ip]
        L.ora_destroy.argtypes = [ctypes.c_void_p]
        L.ora_step.argtypes = [ctypes.c_void_p, _dp, _dp, _dp]
        L.ora_cost.restype = ctypes.c_double
        L.ora_cost.argtypes = [ctypes.c_void_p, _dp, _dp, _dp]
        L.ora_linearize.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.ora_solve.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.ora_build_reduced.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.ora_get.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp]
        L.ora_nnzb.argtypes = [ctypes.c_void_p]
        L.ora_pattern.argtypes = [ctypes.c_void_p, _ip, _ip]
        L.ora_stats.argtypes = [ctypes.c_void_p, _dp]
        L.ora_eval.argtypes = [ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.ora_retract_pose.argtypes = [_dp, _dp, _dp]
        L.ora_n_intr.argtypes = [ctypes.c_int]
        L.ora_clusters.argtypes = [ctypes.c_void_p, _ip]
        L.ora_gp_create.restype = ctypes.c_void_p
        L.ora_gp_create.argtypes = [ctypes.c_int] * 3 + [_dp, _ip, _ip, _dp, _ip, _dp, _ip]
        L.ora_gp_step.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.ora_gp_cost.restype = ctypes.c_double
        L.ora_gp_cost.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.ora_gp_linearize.argtypes = [ctypes.c_void_p, _dp, _dp, _dp]
        L.ora_gp_solve.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.ora_gp_get_ds.argtypes = [ctypes.c_void_p, _dp]
        L.ora_spd_inverse.argtypes = [ctypes.c_int, _dp, _dp]
        L.ora_spd_inverse.restype = ctypes.c_int
    return L


def _d(a):
    return a.ctypes.data_as(_dp)


def _i(a):
    return a.ctypes.data_as(_ip)


def n_intr(model):
    return lib().ora_n_intr(model)


def evaluate(model, X, cam, pp, uv=None, want_jac=True):
    """Residual (or projection when uv is None) and analytic Jacobians for n observations."""
    X = np.ascontiguousarray(X, np.float64)
    cam = np.ascontiguousarray(cam, np.float64)
    pp = np.ascontiguousarray(pp, np.float64)
    n = X.shape[0]
    D = 6 + n_intr(model)
    r = np.zeros((n, 2))
    Jc = np.zeros((n, 2, D)) if want_jac else None
    Jp = np.zeros((n, 2, 3)) if want_jac else None
    u = np.ascontiguousarray(uv, np.float64) if uv is not None else None
    lib().ora_eval(model, n, _d(X), _d(cam), _d(pp), _d(u) if u is not None else None, _d(r),
                   _d(Jc) if want_jac else None, _d(Jp) if want_jac else None)
    return r, Jc, Jp


def spd_inverse(E):
    """The two-level preconditioner's coarse inverse as the oracle forms it (equilibrated blocked Gauss-Jordan).
    Returns (E^-1, positive definite?)."""
    E = np.ascontiguousarray(E, np.float64)
    X = np.zeros_like(E)
    ok = lib().ora_spd_inverse(E.shape[0], _d(E), _d(X))
    return X, bool(ok)


def retract_pose(x7, d6):
    x7 = np.ascontiguousarray(x7, np.float64)
    d6 = np.ascontiguousarray(d6, np.float64)
    out = np.zeros(7)
    lib().ora_retract_pose(_d(x7), _d(d6), _d(out))
    return out


DEFAULTS = dict(huber_delta=1.0, tr_radius=1e4, tr_max=1e10, tr_min=1e-6, tr_up=2.0, tr_down=0.5 ** 4,
                tr_factor=0.25, tr_high=0.5, tr_low=1e-3, clamp_min=1e-6, clamp_max=1e32, pcg_tol=1e-5,
                max_rejects=30, pcg_max_iter=500, optimize_poses=1, threads=0, precond=1, cluster_size=24,
                order_seed=0, order_mode=0)


class OracleBA:
    """CPU LM-BA restatement on a packed problem (track-major obs, pypose camera rows)."""

    def __init__(self, model, uv, cam_idx, pt_idx, pp, n_cams, n_points, variant="", **opts):
        o = dict(DEFAULTS, **opts)
        self.L = lib(variant)
        self.model = int(model)
        self.C, self.P = int(n_cams), int(n_points)
        self.uv = np.ascontiguousarray(uv, np.float64)
        self.cam = np.ascontiguousarray(cam_idx, np.int32)
        self.pt = np.ascontiguousarray(pt_idx, np.int32)
        self.pp = np.ascontiguousarray(pp, np.float64)
        self.N = self.uv.shape[0]
        self.D = 6 + n_intr(self.model)
        dopt = np.array([o['huber_delta'], o['tr_radius'], o['tr_max'], o['tr_min'], o['tr_up'], o['tr_down'],
                         o['tr_factor'], o['tr_high'], o['tr_low'], o['clamp_min'], o['clamp_max'], o['pcg_tol']])
        iopt = np.array([o['max_rejects'], o['pcg_max_iter'], o['optimize_poses'], o['threads'], o['precond'],
                         o['cluster_size'], o['order_seed'], o['order_mode']], np.int32)
        self.h = self.L.ora_create(self.model, self.C, self.P, self.N, _d(self.uv), _i(self.cam), _i(self.pt),
                                  _d(self.pp), _d(dopt), _i(iopt))
        if not self.h:
            raise ValueError("ora_create failed (bad sizes/model or obs not track-major)")

    def __del__(self):
        if getattr(self, "h", None):
            try:
                self.L.ora_destroy(self.h)
            except TypeError:  # interpreter shutdown: the module globals are already gone
                pass
            self.h = None

    def step(self, cams, pts):
        """One LM step; cams [C,stride] / pts [P,3] float64 arrays are updated in place."""
        assert cams.flags.c_contiguous and pts.flags.c_contiguous
        loss = ctypes.c_double()
        self.L.ora_step(self.h, _d(cams), _d(pts), ctypes.byref(loss))
        return loss.value

    def stats(self):
        s = np.zeros(9)
        self.L.ora_stats(self.h, _d(s))
        return dict(trials=int(s[0]), pcg_iters=int(s[1]), pcg_total=int(s[2]), damp_factor=s[3],
                    damping=s[4], failed=int(s[5]), rejects=int(s[6]), coarse_used=int(s[7]), adef2_fallbacks=int(s[8]))

    def cost(self, cams, pts):
        sq = ctypes.c_double()
        loss = self.L.ora_cost(self.h, _d(np.ascontiguousarray(cams)), _d(np.ascontiguousarray(pts)), ctypes.byref(sq))
        return loss, float(np.sqrt(sq.value / self.N))

    def linearize(self, cams, pts):
        self.L.ora_linearize(self.h, _d(np.ascontiguousarray(cams)), _d(np.ascontiguousarray(pts)))

    def solve(self, f):
        return self.L.ora_solve(self.h, float(f))

    def build_reduced(self, f):
        """Unscaled reduced camera system for damping factor f: (S upper blocks, b)."""
        if self.L.ora_build_reduced(self.h, float(f)) != 0:
            raise RuntimeError("non-PD point block")
        return self.get(S), self.get(B)

    def clusters(self):
        """Camera cluster labels of the two-level preconditioner's coarse space and the cluster count."""
        lab = np.zeros(self.C, np.int32)
        nc = self.L.ora_clusters(self.h, _i(lab))
        return lab, nc

    def nnzb(self):
        return self.L.ora_nnzb(self.h)

    def pattern(self):
        rp = np.zeros(self.C + 1, np.int32)
        col = np.zeros(self.nnzb(), np.int32)
        self.L.ora_pattern(self.h, _i(rp), _i(col))
        return rp, col

    def get(self, which):
        shapes = {W: (self.N, self.D, 3), V: (self.P, 6), GP: (self.P, 3), U: (self.C, self.D, self.D),
                  GC: (self.C, self.D), S: (self.nnzb(), self.D, self.D), B: (self.C, self.D),
                  DC: (self.C, self.D), DP: (self.P, 3)}
        out = np.zeros(shapes[which])
        self.L.ora_get(self.h, which, _d(out))
        return out


def solve_to_convergence(problem, max_iters=200, ftol=5e-4, window=4, **opts):
    """TorchBA.Solve's loop (bundle_adjustment.py:128-150) driven by the oracle step."""
    ba = OracleBA(problem.model, problem.uv, problem.cam_idx, problem.pt_idx, problem.pp,
                  problem.n_cams, problem.n_points, **opts)
    cams = problem.cams_init.copy()
    pts = problem.points_init.copy()
    hist = []
    for _ in range(max_iters):
        hist.append(ba.step(cams, pts))
        if len(hist) >= 2 * window:
            recent = np.mean(hist[-window:])
            prev = np.mean(hist[-2 * window:-window])
            if abs((prev - recent) / prev) < ftol:
                break
            if hist[-1] == hist[-2]:
                break
    loss, rmse = ba.cost(cams, pts)
    return cams, pts, hist, rmse


# TorchGP LM options (global_positioning.py:157-160): TrustRegion(radius=1e3, max=1e8, up=2.0, down=0.5**4), PCG(1e-5),
# Huber(thres_loss_function), reject=30; pypose defaults for the rest.
# TorchGP.Optimize (global_positioning.py:158-161): TrustRegion(radius=1e3, max=1e8), PCG(tol=1e-5), reject=30;
# Huber threshold GLOBAL_POSITIONER_OPTIONS['thres_loss_function'] = 0.1 (config/colmap.py:41-46)
GP_DEFAULTS = dict(DEFAULTS, huber_delta=0.1, tr_radius=1e3, tr_max=1e8)


class OracleGP:
    """CPU restatement of TorchGP's LM (oracle/ba_oracle.c ora_gp_*) on a packed global-positioning problem:
    rays t [N,3] (world frame), camera index / point index per observation (track-major), per-camera factor
    (1.0 calibrated, 0.5 otherwise), per-observation scale-free flag."""

    def __init__(self, trans, cam_idx, pt_idx, fcam, sfree, n_cams, n_points, variant="", **opts):
        o = dict(GP_DEFAULTS, **opts)
        self.L = lib(variant)
        self.C, self.P = int(n_cams), int(n_points)
        self.t = np.ascontiguousarray(trans, np.float64)
        self.cam = np.ascontiguousarray(cam_idx, np.int32)
        self.pt = np.ascontiguousarray(pt_idx, np.int32)
        self.fcam = np.ascontiguousarray(fcam, np.float64)
        self.sfree = np.ascontiguousarray(sfree, np.int32)
        self.N = self.t.shape[0]
        self.D = 3
        dopt = np.array([o['huber_delta'], o['tr_radius'], o['tr_max'], o['tr_min'], o['tr_up'], o['tr_down'],
                         o['tr_factor'], o['tr_high'], o['tr_low'], o['clamp_min'], o['clamp_max'], o['pcg_tol']])
        iopt = np.array([o['max_rejects'], o['pcg_max_iter'], 1, o['threads'], o['precond'], o['cluster_size'], 0, 0],
                        np.int32)
        self.h = self.L.ora_gp_create(self.C, self.P, self.N, _d(self.t), _i(self.cam), _i(self.pt), _d(self.fcam),
                                     _i(self.sfree), _d(dopt), _i(iopt))
        if not self.h:
            raise ValueError("ora_gp_create failed")

    __del__ = OracleBA.__del__
    stats = OracleBA.stats
    clusters = OracleBA.clusters
    nnzb = OracleBA.nnzb
    get = OracleBA.get

    def step(self, cams, pts, scales):
        assert cams.flags.c_contiguous and pts.flags.c_contiguous and scales.flags.c_contiguous
        loss = ctypes.c_double()
        self.L.ora_gp_step(self.h, _d(cams), _d(pts), _d(scales), ctypes.byref(loss))
        return loss.value

    def cost(self, cams, pts, scales):
        sq = ctypes.c_double()
        loss = self.L.ora_gp_cost(self.h, _d(np.ascontiguousarray(cams)), _d(np.ascontiguousarray(pts)),
                                 _d(np.ascontiguousarray(scales)), ctypes.byref(sq))
        return loss, float(np.sqrt(sq.value / self.N))

    def linearize(self, cams, pts, scales):
        self.L.ora_gp_linearize(self.h, _d(np.ascontiguousarray(cams)), _d(np.ascontiguousarray(pts)),
                               _d(np.ascontiguousarray(scales)))

    def solve(self, f):
        return self.L.ora_gp_solve(self.h, float(f))

    def ds(self):
        out = np.zeros(self.N)
        self.L.ora_gp_get_ds(self.h, _d(out))
        return out


def gp_solve_to_convergence(problem, max_iters=100, ftol=5e-4, window=4, **opts):
    """TorchGP.Optimize's loop (global_positioning.py:176-186): window 4, |improvement| < function_tolerance."""
    gp = OracleGP(problem.trans, problem.cam_idx, problem.pt_idx, problem.fcam, problem.sfree, problem.n_cams,
                  problem.n_points, **opts)
    cams, pts, scales = problem.cams_init.copy(), problem.points_init.copy(), problem.scales_init.copy()
    hist = []
    for _ in range(max_iters):
        hist.append(gp.step(cams, pts, scales))
        if len(hist) >= 2 * window:
            recent, prev = np.mean(hist[-window:]), np.mean(hist[-2 * window:-window])
            if abs((prev - recent) / prev) < ftol:
                break
    return cams, pts, scales, hist


def dense_reduced(ora, f):
    """The damped reduced camera system (S = U' - W V^-1 W^T, both triangles, and b) of `ora`'s current linearization
    for damping factor f, as a dense (C*D)^2 matrix: the yardstick for comparing two PCG solutions (small C only)."""
    S, b = ora.build_reduced(f)
    rp, col = ora.pattern()
    C, D = ora.C, ora.D
    Sf = np.zeros((C * D, C * D))
    for i in range(C):
        for e in range(rp[i], rp[i + 1]):
            j = col[e]
            Sf[i * D:(i + 1) * D, j * D:(j + 1) * D] = S[e]
            if j != i:
                Sf[j * D:(j + 1) * D, i * D:(i + 1) * D] = S[e].T
    return Sf, b.ravel().copy()


def solve_differences(S, b, x, x_ref):
    """How far apart two solutions of S x = b are, three ways:
      max    max|x - x_ref| / max|x_ref|                  (dominated by the near-null space of S)
      energy ||x - x_ref||_S / ||x_ref||_S                 (the norm CG minimizes the error in)
      resid  ||S (x - x_ref)|| / ||b||                     (on the scale of the PCG's relative-residual tolerance)"""
    x, x_ref = np.ravel(x), np.ravel(x_ref)
    d = x - x_ref
    return dict(max=float(np.abs(d).max() / np.abs(x_ref).max()),
                energy=float(np.sqrt(max(d @ S @ d, 0.0) / max(x_ref @ S @ x_ref, 1e-300))),
                resid=float(np.linalg.norm(S @ d) / np.linalg.norm(b)))
