"""LM engine bound to one packed BA problem -- the replacement for
``bae.optim.LM(model, strategy=TrustRegion(...), solver=PCG(tol=1e-5), kernel=Huber(thres), reject=30)``
(instantsfm/processors/bundle_adjustment.py:115-119) and its ``step(input)`` (:132).

All arithmetic runs in the HIP library (libinsfm_ba.so) through the C ABI of include/insfm_ba.h; torch ROCm tensors
only hold device memory and provide the stream / torch.distributed plumbing.  There is no CPU path.
"""
import ctypes
import time

import numpy as np
import torch

from . import _capi

# TrustRegion / LM / PCG options TorchBA passes (bundle_adjustment.py:116-119) + pypose defaults it relies on.  The
# preconditioner is the product's (TorchBA.Solve, bench.py): precond 2, the A-DEF2 coarse correction wherever the
# persistent CG runs (k_tl_cgp, D = 8: single rank, deterministic mode and every rank of a multi-rank run), the additive
# form of precond 1 elsewhere (effective_precond).
LM_DEFAULTS = dict(tr_radius=1e4, tr_max=1e10, tr_min=1e-6, tr_up=2.0, tr_down=0.5 ** 4, tr_factor=0.25,
                   tr_high=0.5, tr_low=1e-3, clamp_min=1e-6, clamp_max=1e32, max_rejects=30, pcg_tol=1e-5,
                   pcg_max_iter=500, precond=2, cluster_size=24, exchange_chunks=4)


# insfm_ba_debug_stamps' kernel order (ba_common.h StampKind)
STAMP_KERNELS = ("k_lin_points", "k_schur", "k_tl_cgp", "k_cg_finish", "k_publish", "k_cg_factor", "k_tl_basis",
                 "k_backsub_rc", "k_cost", "k_final")
CG_PATHS = {0: "launch-per-iteration two-level CG", 1: "k_tl_cgp (persistent, atomic cluster sums)",
            2: "k_tl_cgp (persistent, fixed-order)", 3: "row-partitioned CG",
            4: "k_tl_cgp (persistent, atomic cluster sums, A-DEF2 coarse correction: precond 2)",
            5: "k_tl_cgp (persistent, fixed-order, A-DEF2 coarse correction: precond 2)"}
# the persistent-CG paths (k_tl_cgp) and the fixed-order ones a replicated multi-rank CG may keep
CGP_PATHS = (1, 2, 4, 5)
CGP_DET_PATHS = (2, 5)


def effective_precond(requested, path):
    """The preconditioner a handle runs: A-DEF2 (2) only on the persistent CG's A-DEF2 paths (4, 5); a request for 2
    runs the additive form (1) on the launch path; 0 and 1 as requested."""
    if path in (4, 5):
        return 2
    return min(int(requested), 1)


def device_key(device):
    """(host name, PCI domain / bus / device) of ``device``: ranks with equal keys share one GPU."""
    import socket
    p = torch.cuda.get_device_properties(device)
    return (socket.gethostname(), int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))


def ranks_per_device(device, group=None):
    """The most ranks of ``group`` that run on one GPU (host name + PCI address of each rank's device, all-gathered)."""
    import torch.distributed as dist
    ids = [None] * dist.get_world_size(group)
    dist.all_gather_object(ids, device_key(device), group=group)
    return max(ids.count(x) for x in ids)


def cg_path_decision(allv):
    """The pure part of agree_cg_path on the all-gathered (device key, path, grid, slots) of every rank: (ranks on the
    most shared GPU, keep k_tl_cgp).  The same list on every rank gives the same answer on every rank."""
    keys = [a[0] for a in allv]
    rpd = max(keys.count(k) for k in keys)
    paths = {a[1] for a in allv}
    keep = len(paths) == 1 and paths <= set(CGP_DET_PATHS) and all(keys.count(a[0]) * a[2] <= a[3] for a in allv)
    return rpd, keep


def agree_cg_path(handle, device, group=None):
    """Collective: the CG every rank of a replicated multi-rank handle runs.  The ranks must all take the same path
    (the persistent k_tl_cgp and the launch path sum S~ m in different orders, so mixed paths would give dc that differ
    in rounding and replicated cameras that drift apart silently).  Every rank all-gathers its device key and
    insfm_ba_cg_info (its own eligibility: grid, slots, INSFM_DIAG, the host-mapped progress word ...); k_tl_cgp stays
    only if every rank runs the same fixed-order form (additive or A-DEF2) and every GPU holds the grids of all ranks
    placed on it at once.
    Returns (ranks on the most shared GPU, the agreed path code)."""
    import torch.distributed as dist
    L = _capi.load()
    info = (ctypes.c_int32 * 4)()
    _capi.check(handle, L.insfm_ba_cg_info(handle, info))
    me = (device_key(device), int(info[0]), int(info[1]), int(info[2]))
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, me, group=group)
    rpd, keep = cg_path_decision(allv)
    if not keep and int(info[0]) in CGP_PATHS:
        _capi.check(handle, L.insfm_ba_set_persistent_cg(handle, 0))
    _capi.check(handle, L.insfm_ba_cg_info(handle, info))
    return rpd, int(info[0])


def make_allreduce_callback(get_buffer, group=None, errors=None, counter=None):
    """The C ABI's allreduce callback (insfm_ba_allreduce_fn) over torch.distributed.

    The library only ever passes sub-ranges of the exchange tensor returned by ``get_buffer()``; the slice is summed
    in place across ranks.  RCCL ("nccl") reduces the device tensor directly on the current stream (the library's
    stream); gloo reduces a host copy (pinned), which also lets several ranks share one GPU in tests.
    """
    import torch.distributed as dist

    def _allreduce(ctx, ptr, count):
        t0 = time.perf_counter()
        try:
            if counter is not None:
                counter[0] += 1
            buf = get_buffer()
            addr = ctypes.cast(ptr, ctypes.c_void_p).value
            off = (addr - buf.data_ptr()) // buf.element_size()
            if off < 0 or off + count > buf.numel():
                raise ValueError("allreduce range outside the exchange buffer")
            view = buf[off:off + count]
            if view.is_cuda and dist.get_backend(group) == "gloo":
                host = view.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
                view.copy_(host)
            else:
                dist.all_reduce(view, op=dist.ReduceOp.SUM, group=group)
            return 0
        except Exception as e:  # surfaced to the caller as INSFM_BA_ECOMM
            if errors is not None:
                errors.append(e)
            return -1
        finally:
            if counter is not None and len(counter) > 1:
                counter[1] += time.perf_counter() - t0  # host seconds inside the callback (gloo: the whole reduce)
    return _allreduce


def make_allreduce_async_callback(get_buffer, group=None, errors=None, counter=None):
    """The C ABI's asynchronous exchange callback (insfm_ba_allreduce_async_fn): sum the slice in place across ranks,
    enqueued on the library's exchange stream ``stream`` without waiting for it.  RCCL ("nccl"): the all_reduce is
    issued with that stream current (the process group's stream waits for it, and it waits for the collective);
    gloo: the stream is synchronized and the slice reduced through host memory, then copied back on that stream."""
    import torch.distributed as dist

    def _allreduce_async(ctx, ptr, count, stream):
        try:
            if counter is not None:
                counter[0] += 1
            buf = get_buffer()
            addr = ctypes.cast(ptr, ctypes.c_void_p).value
            off = (addr - buf.data_ptr()) // buf.element_size()
            if off < 0 or off + count > buf.numel():
                raise ValueError("allreduce range outside the exchange buffer")
            view = buf[off:off + count]
            xs = torch.cuda.ExternalStream(stream, device=buf.device)
            if dist.get_backend(group) == "gloo":
                xs.synchronize()
                host = view.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
                with torch.cuda.stream(xs):
                    view.copy_(host)
            else:
                with torch.cuda.stream(xs):
                    dist.all_reduce(view, op=dist.ReduceOp.SUM, group=group)
            return 0
        except Exception as e:  # surfaced to the caller as INSFM_BA_ECOMM
            if errors is not None:
                errors.append(e)
            return -1
    return _allreduce_async


def _require_gpu(device):
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError(f"insfm_ba runs on an MI355X (ROCm 'cuda' device); got device={device!r}. There is no CPU path.")
    if not torch.cuda.is_available():
        raise RuntimeError("insfm_ba: no ROCm GPU visible (torch.cuda.is_available() is False); there is no CPU fallback")
    return dev


class _LibraryStream:
    """Context: library stream current; ordered after the caller's stream on entry, caller's after it on exit."""

    def __init__(self, lib_stream):
        self.lib = lib_stream
        self.ctx = None
        self.caller = None

    def __enter__(self):
        self.caller = torch.cuda.current_stream(self.lib.device)
        self.ctx = None
        if self.caller != self.lib:  # (the common case -- the library stream is already current -- costs one query)
            self.lib.wait_stream(self.caller)
            self.ctx = torch.cuda.stream(self.lib)
            self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            self.caller.wait_stream(self.lib)
        return False


class BundleAdjuster:
    """One LM problem on one GPU (or one track shard of it)."""

    def __init__(self, model, uv, cam_idx, pt_idx, pp, n_cams, n_points, device="cuda:0", optimize_poses=True,
                 huber_delta=1.0, deterministic=False, world_size=1, rank=0, shard=None, process_group=None,
                 force_exchange=False, **lm):
        self.device = _require_gpu(device)
        L = _capi.load()
        opts = dict(LM_DEFAULTS, **lm)
        uv = np.ascontiguousarray(uv, dtype=np.float64).reshape(-1, 2)
        cam_idx = np.ascontiguousarray(cam_idx, dtype=np.int32).reshape(-1)
        pt_idx = np.ascontiguousarray(pt_idx, dtype=np.int32).reshape(-1)
        pp = np.ascontiguousarray(pp, dtype=np.float64).reshape(-1, 2)
        d = _capi.default_desc()
        d.n_cams, d.n_points, d.n_obs = int(n_cams), int(n_points), int(uv.shape[0])
        d.cam_model = int(model)
        d.optimize_poses = int(bool(optimize_poses))
        d.deterministic = int(bool(deterministic))
        d.huber_delta = float(huber_delta)
        for k, v in opts.items():
            setattr(d, k, type(getattr(d, k))(v))
        d.world_size, d.rank = int(world_size), int(rank)
        d.shard_point_begin, d.shard_point_end = (0, -1) if shard is None else (int(shard[0]), int(shard[1]))
        self._xbuf = None
        self._cb = None
        self._errors = []
        self.exchange_calls = [0, 0.0]  # exchange callbacks made, host seconds spent in the synchronous one
        exchange = world_size > 1 or force_exchange
        if exchange:
            self._cb = _capi.ALLREDUCE_FN(make_allreduce_callback(lambda: self._xbuf, process_group, self._errors,
                                                                  self.exchange_calls))
            d.allreduce = self._cb
            if d.exchange_chunks > 1:
                # the reduced camera system is summed in row chunks behind the Schur build (exchange stream)
                self._cb_async = _capi.ALLREDUCE_ASYNC_FN(make_allreduce_async_callback(
                    lambda: self._xbuf, process_group, self._errors, self.exchange_calls))
                d.allreduce_async = self._cb_async
        self._stream = torch.cuda.current_stream(self.device)
        stream = self._stream.cuda_stream
        h = ctypes.c_void_p()
        rc = L.insfm_ba_create(ctypes.byref(d), uv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                               cam_idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                               pt_idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                               pp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.c_void_p(stream), ctypes.byref(h))
        if rc != 0:
            msg = L.insfm_ba_last_error(h).decode() if h.value else ""
            if h.value:
                L.insfm_ba_destroy(h)
            raise _capi.BAError(rc, msg)
        self._h = h
        self.desc = d
        self.n_cams, self.n_points, self.n_obs = d.n_cams, d.n_points, d.n_obs
        self.D = 6 + {0: 1, 1: 2, 2: 2, 3: 3, 4: 6, 5: 6, 6: 10, 8: 2, 9: 3}[int(model)]
        if exchange:
            n = L.insfm_ba_exchange_count(h)
            self._xbuf = torch.zeros(int(n), dtype=torch.float64, device=self.device)
            _capi.check(h, L.insfm_ba_set_exchange(h, ctypes.c_void_p(self._xbuf.data_ptr()), n))
        self.cg_path = self.cg_info()[0]
        if world_size > 1:
            self.ranks_per_device, self.cg_path = agree_cg_path(h, self.device, process_group)

    # ------------------------------------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _capi.load().insfm_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def partition_cg(self, process_group=None):
        """Switch a multi-rank two-level handle to the row-partitioned CG (insfm_ba_cg_window / _attach, DESIGN.md
        section 5): every rank exports its exchange window, the IPC handles are all-gathered over ``process_group``
        (any backend: the handles are host bytes), and every rank maps its peers' windows.  Collective; call before
        the first step.  Returns this rank's [begin, end) cluster-ordered camera rows."""
        import torch.distributed as dist
        L = _capi.load()
        hbuf = ctypes.create_string_buffer(64)
        _capi.check(self._h, L.insfm_ba_cg_window(self._h, hbuf))
        world = dist.get_world_size(process_group)
        handles = [None] * world
        dist.all_gather_object(handles, bytes(hbuf.raw), group=process_group)
        _capi.check(self._h, L.insfm_ba_cg_attach(self._h, b"".join(handles)))
        rows = (ctypes.c_int32 * 2)()
        _capi.check(self._h, L.insfm_ba_cg_partition(self._h, rows))
        return int(rows[0]), int(rows[1])

    def debug_time_exchange(self, reps=200):
        """Collective: microseconds per flag exchange of the partitioned CG (insfm_ba_debug_time_xchg)."""
        us = ctypes.c_double()
        _capi.check(self._h, _capi.load().insfm_ba_debug_time_xchg(self._h, int(reps), ctypes.byref(us)))
        return us.value

    def last_error(self):
        """The handle's last error message (e.g. why a step reported ``failed``)."""
        return _capi.load().insfm_ba_last_error(self._h).decode() if getattr(self, "_h", None) is not None else ""

    def _ptr(self, t, shape):
        if not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
            raise ValueError("parameters must be contiguous float64 tensors on the GPU")
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {shape}, got {tuple(t.shape)}")
        return ctypes.c_void_p(t.data_ptr())

    def _on_stream(self):
        """The library launches on the stream captured at create.  Callers may be inside another torch stream context:
        order the library stream after the caller's current stream, and make the library stream current while the
        library runs, so the all-reduce callback (RCCL on the current stream, or gloo's device->host copy) is ordered
        with the library's kernels.  The caller's stream is ordered after the library's on exit."""
        return _LibraryStream(self._stream)

    def step(self, cam_params, points):
        """One LM step; updates ``cam_params`` [C, 7+ni] and ``points`` [P, 3] in place.  Returns (loss, stats)."""
        st = _capi.Stats()
        L = _capi.load()
        with self._on_stream():
            rc = L.insfm_ba_step(self._h, self._ptr(cam_params, (self.n_cams, self.D + 1)),
                                 self._ptr(points, (self.n_points, 3)), ctypes.byref(st))
        _capi.check(self._h, rc)
        return st.loss, st.as_dict()

    def cost(self, cam_params, points):
        loss, rmse = ctypes.c_double(), ctypes.c_double()
        L = _capi.load()
        with self._on_stream():
            rc = L.insfm_ba_cost(self._h, self._ptr(cam_params, (self.n_cams, self.D + 1)),
                                 self._ptr(points, (self.n_points, 3)), ctypes.byref(loss), ctypes.byref(rmse))
        _capi.check(self._h, rc)
        return loss.value, rmse.value

    def set_timing(self, on):
        """Per-phase hipEvent timing in the step stats (off by default)."""
        _capi.check(self._h, _capi.load().insfm_ba_set_timing(self._h, int(bool(on))))

    def reset(self):
        _capi.check(self._h, _capi.load().insfm_ba_reset(self._h))

    # ---- parity introspection -----------------------------------------------------------------------------------
    def debug_linearize(self, cam_params, points):
        L = _capi.load()
        _capi.check(self._h, L.insfm_ba_debug_linearize(self._h, self._ptr(cam_params, (self.n_cams, self.D + 1)),
                                                        self._ptr(points, (self.n_points, 3))))

    def debug_solve(self, f):
        return _capi.check(self._h, _capi.load().insfm_ba_debug_solve(self._h, float(f)))

    def debug_time_kernel(self, which, reps=50):
        """Average device time (us) of `reps` back-to-back launches: 0 k_cg_iter, 1 k_schur, 2 one two-level CG
        iteration (k_tl_pc + k_tl_pspmv), 3 k_tl_pspmv, 4 the two-level setup (basis, E build, E^-1), 5 k_lin_points,
        6 the coarse inverse alone (k_gj_pinv0 + the k_gj_step chain), 7 the E build alone (include/insfm_ba.h)."""
        us = ctypes.c_double()
        _capi.check(self._h, _capi.load().insfm_ba_debug_time_kernel(self._h, int(which), int(reps), ctypes.byref(us)))
        return us.value

    def debug_stamps(self, max_steps=1024):
        """INSFM_DIAG=stamps: int64 [steps, 10, 2] device-clock (100 MHz) entry / exit of k_lin_points, k_schur,
        k_tl_cgp, k_cg_finish, k_publish, k_cg_factor, k_tl_basis, k_backsub_rc, k_cost, k_final per LM step
        (insfm_ba_debug_stamps; STAMP_KERNELS names them); an empty array when off."""
        out = np.zeros((max_steps, len(STAMP_KERNELS), 2), dtype=np.int64)
        n = _capi.load().insfm_ba_debug_stamps(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), max_steps)
        _capi.check(self._h, n)
        return out[:n]

    def cg_info(self):
        """(path code, k_tl_cgp grid, workgroup slots, register blocks per row) -- insfm_ba_cg_info; CG_PATHS names
        the codes."""
        info = (ctypes.c_int32 * 4)()
        _capi.check(self._h, _capi.load().insfm_ba_cg_info(self._h, info))
        return tuple(int(x) for x in info)

    def debug_time_cgp(self, reps=10):
        """The persistent CG (k_tl_cgp) of the last solve re-run `reps` times: (us per k_tl_cgp launch, reserved (always
        0: the setup launch it once timed now runs inside k_tl_cgp), PCG iterations per solve); None when this handle
        does not run k_tl_cgp (insfm_ba_debug_time_cgp)."""
        out = (ctypes.c_double * 3)()
        rc = _capi.load().insfm_ba_debug_time_cgp(self._h, int(reps), out)
        if rc == _capi.INSFM_BA_EINVAL:
            return None
        _capi.check(self._h, rc)
        return float(out[0]), float(out[1]), float(out[2])

    def adef2_fallbacks(self):
        """A-DEF2 solves of this handle that broke down and were repeated additively (insfm_ba_cg_fallbacks)."""
        return int(_capi.check(self._h, _capi.load().insfm_ba_cg_fallbacks(self._h)))

    def nnzb(self):
        return int(_capi.load().insfm_ba_nnzb(self._h))

    def coarse_dim(self):
        """Dimension m of the two-level preconditioner's coarse matrix E (clusters x (D + 1)); 0 when it is off."""
        return self.clusters()[1] * (self.D + 1)

    def clusters(self):
        """Camera cluster labels of the two-level preconditioner and the cluster count (0 when it is off)."""
        lab = np.zeros(self.n_cams, dtype=np.int32)
        nc = _capi.load().insfm_ba_debug_clusters(self._h, lab.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        _capi.check(self._h, nc)
        return lab, int(nc)

    def debug_get(self, which, shape):
        out = np.zeros(shape, dtype=np.float64)
        n = _capi.load().insfm_ba_debug_get(self._h, int(which), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        _capi.check(self._h, n)
        assert n == out.size, (n, out.shape)
        return out


# TorchGP.Optimize's LM (global_positioning.py:158-161): TrustRegion(radius=1e3, max=1e8, up=2, down=1/16), PCG(1e-5),
# Huber(GLOBAL_POSITIONER_OPTIONS['thres_loss_function'] = 0.1), reject=30.
# (the additive two-level form: global positioning has D = 3 and runs the launch-per-iteration CG)
GP_DEFAULTS = dict(LM_DEFAULTS, tr_radius=1e3, tr_max=1e8, precond=1)


class GlobalPositioner(BundleAdjuster):
    """One global-positioning LM problem (include/insfm_gp.h): camera positions [C,3], points [P,3] and one scale per
    observation [N] -- the replacement for the LM TorchGP builds around PairwiseNonBatched (global_positioning.py:51-71,
    :155-161).  ``scale_free`` [N] (or None = all free) marks the observations whose scale is optimized; the others
    (valid depth) keep theirs (scales.optimize_indices, :57-59)."""

    def __init__(self, trans, cam_idx, pt_idx, cam_factor, scale_free, n_cams, n_points, device="cuda:0",
                 huber_delta=0.1, deterministic=False, world_size=1, rank=0, shard=None, process_group=None, **lm):
        self.device = _require_gpu(device)
        L = _capi.load()
        opts = dict(GP_DEFAULTS, **lm)
        trans = np.ascontiguousarray(trans, dtype=np.float64).reshape(-1, 3)
        cam_idx = np.ascontiguousarray(cam_idx, dtype=np.int32).reshape(-1)
        pt_idx = np.ascontiguousarray(pt_idx, dtype=np.int32).reshape(-1)
        cam_factor = np.ascontiguousarray(cam_factor, dtype=np.float64).reshape(-1)
        sf = None if scale_free is None else np.ascontiguousarray(scale_free, dtype=np.int32).reshape(-1)
        d = _capi.gp_default_desc()
        d.n_cams, d.n_points, d.n_obs = int(n_cams), int(n_points), int(trans.shape[0])
        d.deterministic = int(bool(deterministic))
        d.huber_delta = float(huber_delta)
        for k, v in opts.items():
            setattr(d, k, type(getattr(d, k))(v))
        d.world_size, d.rank = int(world_size), int(rank)
        d.shard_point_begin, d.shard_point_end = (0, -1) if shard is None else (int(shard[0]), int(shard[1]))
        self._xbuf = None
        self._cb = None
        self._errors = []
        self.exchange_calls = [0]
        if world_size > 1:
            self._cb = _capi.ALLREDUCE_FN(make_allreduce_callback(lambda: self._xbuf, process_group, self._errors,
                                                                  self.exchange_calls))
            d.allreduce = self._cb
        self._stream = torch.cuda.current_stream(self.device)
        stream = self._stream.cuda_stream
        h = ctypes.c_void_p()
        dp, ip = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
        rc = L.insfm_gp_create(ctypes.byref(d), trans.ctypes.data_as(dp), cam_idx.ctypes.data_as(ip),
                               pt_idx.ctypes.data_as(ip), cam_factor.ctypes.data_as(dp),
                               None if sf is None else sf.ctypes.data_as(ip), ctypes.c_void_p(stream), ctypes.byref(h))
        if rc != 0:
            msg = L.insfm_ba_last_error(h).decode() if h.value else ""
            if h.value:
                L.insfm_ba_destroy(h)
            raise _capi.BAError(rc, msg)
        self._h = h
        self.desc = d
        self.n_cams, self.n_points, self.n_obs = d.n_cams, d.n_points, d.n_obs
        self.D = 3
        if world_size > 1:
            n = L.insfm_ba_exchange_count(h)
            self._xbuf = torch.zeros(int(n), dtype=torch.float64, device=self.device)
            _capi.check(h, L.insfm_ba_set_exchange(h, ctypes.c_void_p(self._xbuf.data_ptr()), n))

    def _args(self, positions, points, scales):
        return (self._ptr(positions, (self.n_cams, 3)), self._ptr(points, (self.n_points, 3)),
                self._ptr(scales, (self.n_obs,)))

    def step(self, positions, points, scales):
        """One LM step; updates ``positions`` [C,3], ``points`` [P,3], ``scales`` [N] in place.  Returns (loss, stats)."""
        st = _capi.Stats()
        with self._on_stream():
            rc = _capi.load().insfm_gp_step(self._h, *self._args(positions, points, scales), ctypes.byref(st))
        _capi.check(self._h, rc)
        return st.loss, st.as_dict()

    def cost(self, positions, points, scales):
        loss, rmse = ctypes.c_double(), ctypes.c_double()
        with self._on_stream():
            rc = _capi.load().insfm_gp_cost(self._h, *self._args(positions, points, scales), ctypes.byref(loss),
                                            ctypes.byref(rmse))
        _capi.check(self._h, rc)
        return loss.value, rmse.value

    def debug_linearize(self, positions, points, scales):
        _capi.check(self._h, _capi.load().insfm_gp_debug_linearize(self._h, *self._args(positions, points, scales)))

    def debug_ds(self):
        out = np.zeros(self.n_obs, dtype=np.float64)
        _capi.check(self._h, _capi.load().insfm_gp_debug_get_ds(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return out
