"""ctypes binding of the C ABI in include/insfm_ba.h, insfm_gp.h and insfm_passes.h (libinsfm_ba.so, built in-tree for
gfx950).

There is no CPU fallback: if the HIP library is missing or no GPU is visible, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libinsfm_ba.so")

INSFM_BA_OK = 0
INSFM_BA_EINVAL = -22
INSFM_BA_ENOMEM = -12
INSFM_BA_EHIP = -100
INSFM_BA_ECOMM = -101
INSFM_BA_ESOLVER = -102

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64)
ALLREDUCE_ASYNC_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int64,
                                      ctypes.c_void_p)


class Desc(ctypes.Structure):
    _fields_ = [
        ("n_cams", ctypes.c_int32), ("n_points", ctypes.c_int32), ("n_obs", ctypes.c_int32),
        ("cam_model", ctypes.c_int32), ("optimize_poses", ctypes.c_int32), ("deterministic", ctypes.c_int32),
        ("huber_delta", ctypes.c_double),
        ("tr_radius", ctypes.c_double), ("tr_max", ctypes.c_double), ("tr_min", ctypes.c_double),
        ("tr_up", ctypes.c_double), ("tr_down", ctypes.c_double), ("tr_factor", ctypes.c_double),
        ("tr_high", ctypes.c_double), ("tr_low", ctypes.c_double),
        ("clamp_min", ctypes.c_double), ("clamp_max", ctypes.c_double),
        ("max_rejects", ctypes.c_int32), ("pcg_max_iter", ctypes.c_int32),
        ("pcg_tol", ctypes.c_double),
        ("world_size", ctypes.c_int32), ("rank", ctypes.c_int32),
        ("shard_point_begin", ctypes.c_int32), ("shard_point_end", ctypes.c_int32),
        ("allreduce", ALLREDUCE_FN), ("allreduce_ctx", ctypes.c_void_p),
        ("precond", ctypes.c_int32), ("cluster_size", ctypes.c_int32), ("schur_variant", ctypes.c_int32),
        ("allreduce_async", ALLREDUCE_ASYNC_FN), ("exchange_chunks", ctypes.c_int32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("loss", ctypes.c_double), ("loss_before", ctypes.c_double), ("damping", ctypes.c_double),
        ("trials", ctypes.c_int32), ("rejects", ctypes.c_int32), ("pcg_iters_last", ctypes.c_int32),
        ("pcg_iters_total", ctypes.c_int32), ("solver_failed", ctypes.c_int32), ("cg_launches", ctypes.c_int32),
        ("time_ms", ctypes.c_double * 8), ("coarse_used", ctypes.c_int32),
    ]

    def as_dict(self):
        return dict(loss=self.loss, loss_before=self.loss_before, damping=self.damping, trials=self.trials,
                    rejects=self.rejects, pcg_iters=self.pcg_iters_last, pcg_total=self.pcg_iters_total,
                    failed=self.solver_failed, cg_launches=self.cg_launches, time_ms=list(self.time_ms),
                    coarse_used=self.coarse_used)


# exported symbols (every one declared in include/*.h)
SYMBOLS = ("insfm_build_info", "insfm_ba_default_desc", "insfm_ba_create", "insfm_ba_step", "insfm_ba_cost", "insfm_ba_reset",
           "insfm_ba_destroy", "insfm_ba_last_error", "insfm_ba_debug_linearize", "insfm_ba_debug_solve",
           "insfm_ba_debug_get", "insfm_ba_nnzb", "insfm_ba_exchange_count", "insfm_ba_set_exchange",
           "insfm_ba_debug_time_kernel", "insfm_ba_set_timing", "insfm_ba_debug_clusters", "insfm_ba_debug_spd_inverse",
           "insfm_ba_release_cache", "insfm_ba_set_ranks_per_device", "insfm_ba_cg_info", "insfm_ba_set_persistent_cg", "insfm_ba_cg_fallbacks", "insfm_ba_cg_window", "insfm_ba_cg_attach", "insfm_ba_cg_partition",
           "insfm_ba_debug_time_xchg", "insfm_ba_debug_time_cgp", "insfm_ba_debug_stamps",
           "insfm_gp_default_desc", "insfm_gp_create", "insfm_gp_step", "insfm_gp_cost", "insfm_gp_debug_linearize",
           "insfm_gp_debug_get_ds",
           "insfm_undistort", "insfm_filter_reproj_normalized", "insfm_filter_angle", "insfm_filter_tri_angle",
           "insfm_filter_reproj_pixel", "insfm_reproj_candidates",
           "insfm_tracks_establish")

_lib = None


class BAError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"insfm_ba error {code}: {msg}")
        self.code = code


def build_info(L=None):
    """The provenance string the library was built with ("src=<hash> arch=... flags=...")."""
    L = L or load()
    L.insfm_build_info.argtypes = []
    L.insfm_build_info.restype = ctypes.c_char_p
    return L.insfm_build_info().decode()


def _check_provenance(L, path):
    """The in-tree library must have been built from the sources in this tree (instantsfm_amd/build.py hashes them):
    a stale or foreign binary fails loudly instead of running unverified code."""
    from . import build as _b
    if not all(os.path.exists(p) for p in _b.SRCS + _b.HEADERS):
        return  # (an installed copy without sources: nothing to compare against)
    info = build_info(L)
    want = _b.source_hash()
    if f"src={want} " not in info + " ":
        raise RuntimeError(f"{path} was built from other sources ({info}; this tree hashes to src={want}): "
                           "rebuild it (python -c 'import __graft_entry__ as g; g.build()')")


def load(path=None):
    """Load the HIP library (no GPU needed to load it).  Raises if it was not built.  ``INSFM_LIB`` names another
    build of the same library (A/B timing of kernel variants on one box; its provenance is not checked)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("INSFM_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(path)
    if not os.environ.get("INSFM_LIB"):
        _check_provenance(L, path)
    vp, dp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
    L.insfm_ba_default_desc.argtypes = [ctypes.POINTER(Desc)]
    L.insfm_ba_default_desc.restype = None
    L.insfm_ba_create.argtypes = [ctypes.POINTER(Desc), dp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                  dp, vp, ctypes.POINTER(vp)]
    L.insfm_ba_create.restype = ctypes.c_int
    L.insfm_ba_step.argtypes = [vp, vp, vp, ctypes.POINTER(Stats)]
    L.insfm_ba_step.restype = ctypes.c_int
    L.insfm_ba_cost.argtypes = [vp, vp, vp, dp, dp]
    L.insfm_ba_cost.restype = ctypes.c_int
    L.insfm_ba_reset.argtypes = [vp]
    L.insfm_ba_reset.restype = ctypes.c_int
    L.insfm_ba_destroy.argtypes = [vp]
    L.insfm_ba_destroy.restype = None
    L.insfm_ba_last_error.argtypes = [vp]
    L.insfm_ba_last_error.restype = ctypes.c_char_p
    L.insfm_ba_debug_linearize.argtypes = [vp, vp, vp]
    L.insfm_ba_debug_linearize.restype = ctypes.c_int
    L.insfm_ba_debug_solve.argtypes = [vp, ctypes.c_double]
    L.insfm_ba_debug_solve.restype = ctypes.c_int
    L.insfm_ba_debug_get.argtypes = [vp, ctypes.c_int32, dp]
    L.insfm_ba_debug_get.restype = ctypes.c_int64
    L.insfm_ba_nnzb.argtypes = [vp]
    L.insfm_ba_nnzb.restype = ctypes.c_int64
    L.insfm_ba_exchange_count.argtypes = [vp]
    L.insfm_ba_exchange_count.restype = ctypes.c_int64
    L.insfm_ba_set_exchange.argtypes = [vp, vp, ctypes.c_int64]
    L.insfm_ba_set_exchange.restype = ctypes.c_int
    L.insfm_ba_debug_time_kernel.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, dp]
    L.insfm_ba_debug_time_kernel.restype = ctypes.c_int
    L.insfm_ba_debug_stamps.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
    L.insfm_ba_debug_stamps.restype = ctypes.c_int32
    L.insfm_ba_debug_time_cgp.argtypes = [vp, ctypes.c_int32, dp]
    L.insfm_ba_debug_time_cgp.restype = ctypes.c_int
    L.insfm_ba_set_timing.argtypes = [vp, ctypes.c_int32]
    L.insfm_ba_set_timing.restype = ctypes.c_int
    L.insfm_ba_debug_clusters.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
    L.insfm_ba_debug_clusters.restype = ctypes.c_int32
    L.insfm_ba_debug_spd_inverse.argtypes = [ctypes.c_int32, vp, vp, vp, ctypes.c_int32, dp]
    L.insfm_ba_debug_spd_inverse.restype = ctypes.c_int
    L.insfm_ba_release_cache.argtypes = []
    L.insfm_ba_release_cache.restype = ctypes.c_int64
    L.insfm_ba_set_ranks_per_device.argtypes = [vp, ctypes.c_int32]
    L.insfm_ba_set_ranks_per_device.restype = ctypes.c_int
    L.insfm_ba_cg_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
    L.insfm_ba_cg_info.restype = ctypes.c_int
    L.insfm_ba_set_persistent_cg.argtypes = [vp, ctypes.c_int32]
    L.insfm_ba_set_persistent_cg.restype = ctypes.c_int
    L.insfm_ba_cg_fallbacks.argtypes = [vp]
    L.insfm_ba_cg_fallbacks.restype = ctypes.c_int32
    L.insfm_ba_cg_window.argtypes = [vp, ctypes.c_char_p]
    L.insfm_ba_cg_window.restype = ctypes.c_int
    L.insfm_ba_cg_attach.argtypes = [vp, ctypes.c_char_p]
    L.insfm_ba_cg_attach.restype = ctypes.c_int
    L.insfm_ba_cg_partition.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
    L.insfm_ba_cg_partition.restype = ctypes.c_int
    L.insfm_ba_debug_time_xchg.argtypes = [vp, ctypes.c_int32, dp]
    L.insfm_ba_debug_time_xchg.restype = ctypes.c_int
    ip = ctypes.POINTER(ctypes.c_int32)
    L.insfm_gp_default_desc.argtypes = [ctypes.POINTER(Desc)]
    L.insfm_gp_default_desc.restype = None
    L.insfm_gp_create.argtypes = [ctypes.POINTER(Desc), dp, ip, ip, dp, ip, vp, ctypes.POINTER(vp)]
    L.insfm_gp_create.restype = ctypes.c_int
    L.insfm_gp_step.argtypes = [vp, vp, vp, vp, ctypes.POINTER(Stats)]
    L.insfm_gp_step.restype = ctypes.c_int
    L.insfm_gp_cost.argtypes = [vp, vp, vp, vp, dp, dp]
    L.insfm_gp_cost.restype = ctypes.c_int
    L.insfm_gp_debug_linearize.argtypes = [vp, vp, vp, vp]
    L.insfm_gp_debug_linearize.restype = ctypes.c_int
    L.insfm_gp_debug_get_ds.argtypes = [vp, dp]
    L.insfm_gp_debug_get_ds.restype = ctypes.c_int64
    i64, f64, i32 = ctypes.c_int64, ctypes.c_double, ctypes.c_int32
    L.insfm_undistort.argtypes = [i64, vp, i32, vp, vp, vp, vp, vp]
    L.insfm_filter_reproj_normalized.argtypes = [i64, vp, vp, vp, vp, vp, vp, f64, vp, vp, vp]
    L.insfm_filter_angle.argtypes = [i64, vp, vp, vp, vp, vp, vp, f64, vp, vp]
    L.insfm_filter_tri_angle.argtypes = [i64, vp, vp, vp, vp, f64, vp, vp]
    L.insfm_filter_reproj_pixel.argtypes = [i64, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp, f64, vp, vp, vp]
    L.insfm_reproj_candidates.argtypes = [i64, i32, vp, vp, vp, vp, i32, vp, vp, vp, f64, vp, vp, vp]
    L.insfm_tracks_establish.argtypes = [i64, vp, vp, i32, i64, vp, vp, f64, vp, vp, vp, vp, vp,
                                         ctypes.POINTER(ctypes.c_int64), vp]
    for fn in ("insfm_tracks_establish", "insfm_undistort", "insfm_filter_reproj_normalized", "insfm_filter_angle", "insfm_filter_tri_angle",
               "insfm_filter_reproj_pixel", "insfm_reproj_candidates",
           "insfm_tracks_establish"):
        getattr(L, fn).restype = ctypes.c_int
    _lib = L
    return L


def default_desc():
    d = Desc()
    load().insfm_ba_default_desc(ctypes.byref(d))
    return d


def gp_default_desc():
    d = Desc()
    load().insfm_gp_default_desc(ctypes.byref(d))
    return d


def release_device_cache():
    """Free the device buffers destroyed handles parked for reuse (insfm_ba_release_cache); returns the bytes freed.
    Those buffers are invisible to PyTorch's caching allocator: call this before large torch allocations."""
    return int(load().insfm_ba_release_cache())


def check(h, rc):
    if rc < 0:
        msg = load().insfm_ba_last_error(h).decode() if h else ""
        raise BAError(rc, msg)
    return rc
