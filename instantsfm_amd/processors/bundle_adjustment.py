"""TorchBA -- drop-in for ``instantsfm/processors/bundle_adjustment.py`` (reference :1-154).

Same constructor and ``Solve(cameras, images, tracks, BUNDLE_ADJUSTER_OPTIONS)`` signature, same filters, ordering,
stop rule and in-place write-back; the LM engine underneath is the MI355X HIP library (``engine.BundleAdjuster``)
instead of bae/pypose.  Packing (reference :66-113, a Python double loop over tracks x observations) is vectorized.
"""
import time

import numpy as np
import torch

from ..engine import BundleAdjuster, effective_precond
from ..scene.defs import CameraModelId, IMPLEMENTED_MODELS, get_camera_model_info


def _load_packx():
    """The native packing extension (csrc/packx.c, built by instantsfm_amd.build next to libinsfm_ba.so).  Missing: a
    warning, and the bit-identical numpy path packs instead.  Built from other sources than this tree's packx.c: an
    error, as for the main library (_capi._check_provenance)."""
    import importlib.util
    import os
    import sysconfig
    import warnings
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib",
                        "_packx" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    if not os.path.exists(path):
        warnings.warn(f"{path} not built: TorchBA packs with the (slower, bit-identical) numpy path", RuntimeWarning)
        return None
    spec = importlib.util.spec_from_file_location("_packx", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from .. import build as _b
    if os.path.exists(_b.PACKX_SRC) and getattr(mod, "SRC_HASH", None) != _b.packx_hash():
        raise RuntimeError(f"{path} was built from other sources (SRC_HASH {getattr(mod, 'SRC_HASH', None)}, this tree's "
                           f"packx.c hashes to {_b.packx_hash()}): rebuild it (python -c 'import __graft_entry__ as g; "
                           "g.build()')")
    return mod


_PACKX = []


def packx():
    """The native packing extension, loaded (and its provenance checked) on first use: the package must stay
    importable while build() rebuilds a stale extension."""
    if not _PACKX:
        _PACKX.append(_load_packx())
    return _PACKX[0]


def _quat_xyzw_from_matrix(R):
    """pp.mat2SE3 rotation part: rotation matrix (or a batch) -> quaternion [x, y, z, w] (sign: w >= 0)."""
    from scipy.spatial.transform import Rotation
    q = Rotation.from_matrix(np.asarray(R, dtype=np.float64)).as_quat()
    return np.where(q[..., 3:4] < 0, -q, q)


def _pose_matrices(cam_rows):
    """pp.SE3(rows[:, :7]).matrix(): the 4x4 of the action p -> p + 2w(q x p) + 2 q x (q x p) + t, i.e. the rotation
    I + 2w[q]x + 2[q]x^2 written out entry by entry ([q]x^2 = q q^T - |q|^2 I) into one preallocated array (the
    stacked 3x3 temporaries and their matmul were most of the write-back's pose time)."""
    c = np.ascontiguousarray(cam_rows[:, :7], dtype=np.float64).T
    qx, qy, qz, w = c[3], c[4], c[5], c[6]
    n = cam_rows.shape[0]
    M = np.empty((n, 4, 4))
    xx, yy, zz = qx * qx, qy * qy, qz * qz
    xy, xz, yz = qx * qy, qx * qz, qy * qz
    wx, wy, wz = w * qx, w * qy, w * qz
    M[:, 0, 0] = 1.0 - 2.0 * (yy + zz)
    M[:, 0, 1] = 2.0 * (xy - wz)
    M[:, 0, 2] = 2.0 * (xz + wy)
    M[:, 1, 0] = 2.0 * (xy + wz)
    M[:, 1, 1] = 1.0 - 2.0 * (xx + zz)
    M[:, 1, 2] = 2.0 * (yz - wx)
    M[:, 2, 0] = 2.0 * (xz - wy)
    M[:, 2, 1] = 2.0 * (yz + wx)
    M[:, 2, 2] = 1.0 - 2.0 * (xx + yy)
    M[:, :3, 3] = c[:3].T
    M[:, 3, :3] = 0.0
    M[:, 3, 3] = 1.0
    return M


def _as_torch_like_params(params):
    """``torch.tensor(cameras[id].params)`` (reference :71-72): a Python list of floats becomes float32 in torch
    (default dtype) before it is concatenated with the float64 pose; a numpy array keeps its dtype."""
    if isinstance(params, np.ndarray):
        return params.astype(np.float64)
    if torch.is_tensor(params):
        return params.detach().cpu().numpy().astype(np.float64)
    vals = list(params)
    # torch infers the default dtype (float32) for plain Python scalars when at least one is a float; numpy
    # scalars keep their own dtype (np.float64 -> float64) and promote the result.
    plain = all(type(x) in (float, int, bool) for x in vals)
    arr = np.asarray(vals, dtype=np.float64)
    if plain and any(type(x) is float for x in vals):
        return arr.astype(np.float32).astype(np.float64)
    return arr


def _rotated_z(points, pt, pose, cam):
    """z of bae's rotate_quat(points[pt], pose[cam]) = p + 2(w (q x p) + q x (q x p)) + t, the same products and
    sums as the vector form (numpy's cross), computed only for the z row; the per-observation operands are gathered
    column by column from contiguous per-point / per-camera columns."""
    P = np.ascontiguousarray(points.T)
    Q = np.ascontiguousarray(pose[:, :7].T)
    px, py, pz = P[0][pt], P[1][pt], P[2][pt]
    qx, qy, qz, w = Q[3][cam], Q[4][cam], Q[5][cam], Q[6][cam]
    uvx = qy * pz - qz * py
    uvy = qz * px - qx * pz
    uvz = qx * py - qy * px
    return pz + 2.0 * (w * uvz + (qx * uvy - qy * uvx)) + Q[2][cam]


def _compact(ids, n):
    """np.unique(ids, return_inverse=True) for ids in [0, n): bincount instead of a sort."""
    present = np.bincount(ids, minlength=n) > 0
    uniq = np.flatnonzero(present)
    remap = np.cumsum(present) - 1
    return uniq, remap[ids]


class PackedProblem:
    """What TorchBA.Solve hands the LM (reference :98-126): compacted, track-major arrays + bookkeeping."""

    def __init__(self, model, points_2d, camera_indices, point_indices, camera_pps, camera_params, points_3d,
                 unique_cameras, unique_points, track_keys, remaining_indices, pp_indices, track_vals=None,
                 indices_i32=None):
        self.model = model
        self.points_2d = points_2d
        self.camera_indices = camera_indices
        self.point_indices = point_indices
        self.camera_pps = camera_pps
        self.camera_params = camera_params
        self.points_3d = points_3d
        self.unique_cameras = unique_cameras
        self.unique_points = unique_points
        self.track_keys = track_keys
        self.remaining_indices = remaining_indices
        self.pp_indices = pp_indices
        self.track_vals = track_vals  # the Track objects in track_keys order (update() writes xyz through it)
        # int32 copies of (camera_indices, point_indices) for insfm_ba_create (native pack), else made on demand
        self.indices_i32 = indices_i32

    def indices32(self):
        if self.indices_i32 is None:
            self.indices_i32 = (self.camera_indices.astype(np.int32), self.point_indices.astype(np.int32))
        return self.indices_i32


def pack(cameras, images, tracks, options, native=True, phases=None):
    """Vectorized restatement of bundle_adjustment.py:66-113.  With the native extension (csrc/packx.c) the per-Track
    reads and the per-observation filtering run in C on all host cores; ``native=False`` (or Track attributes that are
    not plain ndarrays) takes the numpy path, which gives the same arrays (tests/test_packing.py checks both).
    ``phases``: a dict that receives the wall seconds of the native path's parts (keys, collect, images, features,
    finish, outputs)."""
    tp = [time.perf_counter()]

    def mark(name):
        if phases is not None:
            tp.append(time.perf_counter())
            phases[name] = tp[-1] - tp[-2]
    model = cameras[0].model_id  # :45 "assume all cameras are under the same model"
    info = get_camera_model_info(model)
    if model.value not in IMPLEMENTED_MODELS:
        raise NotImplementedError("Unsupported camera model")
    min_len = options['min_num_view_per_track']
    track_keys = list(tracks.keys())
    track_vals = list(tracks.values())
    mark("keys")
    got = packx().collect(track_vals, int(min_len)) if (native and packx() is not None) else None
    mark("collect")
    if got is not None:
        lengths = np.frombuffer(got[0], np.int64)
        obs_valid = np.frombuffer(got[1], np.int64).reshape(-1, 2)
        xyz = None
        points_3d = np.frombuffer(got[2], np.float64).reshape(-1, 3)
    else:
        obs_all = [t.observations for t in track_vals]
        lengths = np.fromiter(map(len, obs_all), dtype=np.int64, count=len(obs_all))
        xyz = [t.xyz for t in track_vals]                                                     # :82-83
    is_valid = lengths >= min_len                                                             # :66-68
    registered = np.array([img.is_registered for img in images], dtype=bool)                  # :70
    # :71-73, one batched matrix -> quaternion conversion; unregistered images get the identity row
    se3 = np.tile(np.array([0, 0, 0, 0, 0, 0, 1.0]), (len(images), 1))
    reg = np.flatnonzero(registered)
    if reg.size:
        w2c = np.array([np.asarray(images[i].world2cam, dtype=np.float64) for i in reg.tolist()]).reshape(-1, 4, 4)
        se3[reg, :3] = w2c[:, :3, 3]
        se3[reg, 3:] = _quat_xyzw_from_matrix(w2c[:, :3, :3])
    intr = {}
    for img in images:
        if img.cam_id not in intr:
            intr[img.cam_id] = _as_torch_like_params(cameras[img.cam_id].params)
    camera_params = np.concatenate([se3, np.array([intr[img.cam_id] for img in images])], axis=1).astype(np.float64)
    pp_indices = np.asarray(info['pp']) + 7                                                   # :75-80
    remaining = np.array([i for i in range(camera_params.shape[1]) if i not in pp_indices])
    camera_pps = camera_params[:, pp_indices]
    camera_params = camera_params[:, remaining]
    mark("images")
    feats = [np.asarray(im.features).reshape(-1, 2) for im in images]
    foff = np.concatenate([[0], np.cumsum([f.shape[0] for f in feats])]).astype(np.int64)
    feat_all = np.ascontiguousarray(np.concatenate(feats), dtype=np.float64) if feats else np.zeros((0, 2))
    if got is not None:
        # :85-113 in C: registered filter, feature gather, cheirality z > 0.1, torch.unique compaction
        cp = np.ascontiguousarray(camera_params)
        mark("features")
        r = packx().finish(obs_valid, lengths, int(min_len), registered.astype(np.uint8), feat_all, foff,
                          np.ascontiguousarray(points_3d), cp, cp.shape[1])
        mark("finish")
        points_2d = np.frombuffer(r[0], np.float64).reshape(-1, 2)
        cam_inv, pt_inv = np.frombuffer(r[1], np.int64), np.frombuffer(r[2], np.int64)
        unique_cameras, unique_points = np.frombuffer(r[3], np.int64), np.frombuffer(r[4], np.int64)
        out = PackedProblem(model, points_2d, cam_inv, pt_inv, np.ascontiguousarray(camera_pps[unique_cameras]),
                            np.ascontiguousarray(camera_params[unique_cameras]),
                            np.ascontiguousarray(points_3d[unique_points]), unique_cameras, unique_points,
                            track_keys, remaining, pp_indices, track_vals,
                            (np.frombuffer(r[5], np.int32), np.frombuffer(r[6], np.int32)))
        mark("outputs")
        return out
    try:
        points_3d = np.concatenate(xyz).astype(np.float64, copy=False).reshape(-1, 3)
        if points_3d.shape[0] != len(xyz):
            raise ValueError
    except ValueError:
        points_3d = np.stack([np.asarray(x, dtype=np.float64).reshape(3) for x in xyz])

    valid_ids = np.flatnonzero(is_valid)                                                      # :85-96
    if valid_ids.size:
        sel = [obs_all[t] for t in valid_ids.tolist()]
        try:
            obs = np.concatenate(sel)
            if obs.ndim != 2 or obs.shape[1] != 2:
                raise ValueError
        except ValueError:
            obs = np.concatenate([np.asarray(o).reshape(-1, 2) for o in sel])
        obs = obs.astype(np.int64, copy=False)
        tid = np.repeat(valid_ids, lengths[valid_ids])
    else:
        obs = np.zeros((0, 2), np.int64)
        tid = np.zeros(0, np.int64)
    img_id, feat_id = obs[:, 0], obs[:, 1]
    keep = registered[img_id]
    if not keep.all():
        img_id, feat_id, tid = img_id[keep], feat_id[keep], tid[keep]
    # one 16-byte gather per observation (a row of feat_all viewed as one complex128)
    points_2d = feat_all.view(np.complex128).reshape(-1)[foff[img_id] + feat_id].view(np.float64).reshape(-1, 2)

    z = _rotated_z(points_3d, tid, camera_params, img_id)                                    # :102-107
    ok = z > 0.1
    if not ok.all():
        points_2d, img_id, tid = points_2d[ok], img_id[ok], tid[ok]
    unique_cameras, cam_inv = _compact(img_id, len(images))                                   # :108-113
    unique_points, pt_inv = _compact(tid, len(track_vals))
    return PackedProblem(model, np.ascontiguousarray(points_2d), cam_inv.astype(np.int64), pt_inv.astype(np.int64),
                         np.ascontiguousarray(camera_pps[unique_cameras]),
                         np.ascontiguousarray(camera_params[unique_cameras]),
                         np.ascontiguousarray(points_3d[unique_points]), unique_cameras, unique_points, track_keys,
                         remaining, pp_indices, track_vals)


def update(cameras, images, tracks, packed, camera_params, points_3d, phases=None):
    """bundle_adjustment.py:18-36: write the optimized parameters back into the scene objects.  ``phases`` (a dict)
    gets the wall-time split: d2h (the device-to-host copies), xyz (every track's ``xyz`` set to its row), poses (the
    pose matrices, ``world2cam`` per image, ``set_params`` per camera)."""
    t0 = time.perf_counter()
    cp = camera_params.detach().cpu().numpy() if torch.is_tensor(camera_params) else np.asarray(camera_params)
    pts = points_3d.detach().cpu().numpy() if torch.is_tensor(points_3d) else np.asarray(points_3d)
    t1 = time.perf_counter()
    full = np.zeros((cp.shape[0], cp.shape[1] + 2))
    full[:, packed.remaining_indices] = cp
    full[:, packed.pp_indices] = packed.camera_pps
    keys = packed.track_keys
    if packx() is not None and pts.dtype == np.float64 and pts.flags.c_contiguous and pts.ndim == 2:
        packx().assign_xyz(list(tracks.values()) if packed.track_vals is None else packed.track_vals,
                          np.ascontiguousarray(packed.unique_points, np.int64), pts)
    else:
        for orig, xyz in zip(packed.unique_points.tolist(), pts):
            tracks[keys[orig]].xyz = xyz
    t2 = time.perf_counter()
    mats = _pose_matrices(full[:, :7])
    t3 = time.perf_counter()
    last = {}
    for i, image_id in enumerate(packed.unique_cameras.tolist()):
        image = images[image_id]
        image.world2cam = mats[i]
        last[image.cam_id] = i            # :33-36 set_params per image: the last image of a camera wins
    t4 = time.perf_counter()
    for cam_id, i in last.items():
        cameras[cam_id].set_params(full[i, 7:])
    if phases is not None:
        t5 = time.perf_counter()
        phases.update(d2h=t1 - t0, xyz=t2 - t1, poses=t5 - t2, poses_mats=t3 - t2, poses_images=t4 - t3,
                      poses_set_params=t5 - t4)


class TorchBA:
    """bundle_adjustment.py:38-154 with the HIP engine underneath."""

    def __init__(self, visualizer=None, device="cuda:0"):
        self.device = device
        self.visualizer = visualizer
        self.loss_history = []
        self.last_stats = None
        self.timings = {}

    def Solve(self, cameras, images, tracks, BUNDLE_ADJUSTER_OPTIONS, progress=True):
        """bundle_adjustment.py:44-154.  ``self.timings`` gets the wall-time split of the call (pack, create,
        steps, write-back) and the step count."""
        opts = BUNDLE_ADJUSTER_OPTIONS
        t0 = time.perf_counter()
        phases = {}
        packed = pack(cameras, images, tracks, opts, phases=phases)
        t1 = time.perf_counter()
        self.timings = dict(pack_s=t1 - t0, pack_phases=phases, create_s=0.0, steps_s=0.0, update_s=0.0, total_s=t1 - t0, steps=0,
                            n_cams=int(packed.camera_params.shape[0]), n_points=int(packed.points_3d.shape[0]),
                            n_obs=int(packed.points_2d.shape[0]))
        if packed.points_2d.shape[0] == 0:
            return
        # the engine wants track-major observations: point_indices from np.unique are already nondecreasing because
        # observations were gathered track by track (reference :88-96), so no reordering is needed.
        cam32, pt32 = packed.indices32()
        eng = BundleAdjuster(packed.model.value, packed.points_2d, cam32, pt32,
                             packed.camera_pps, packed.camera_params.shape[0], packed.points_3d.shape[0],
                             device=self.device, optimize_poses=opts['optimize_poses'],
                             huber_delta=opts['thres_loss_function'], deterministic=opts.get('deterministic', False),
                             precond=opts.get('precond', 2),
                             **{k: opts[k] for k in ('pcg_max_iter', 'pcg_tol') if k in opts})
        # the preconditioner the engine runs: A-DEF2 (precond 2) where the persistent CG runs (D = 8), else the
        # additive two-level form (insfm_ba_cg_info path codes, engine.CG_PATHS / effective_precond)
        self.cg_path = eng.cg_info()[0]
        self.precond_effective = effective_precond(opts.get('precond', 2), self.cg_path)
        dev = torch.device(self.device)
        cams_t = torch.from_numpy(packed.camera_params).to(dev).contiguous()
        pts_t = torch.from_numpy(packed.points_3d).to(dev).contiguous()
        t2 = time.perf_counter()
        window_size = 4                                                                       # :128-150
        loss_history = []
        step_ms, step_stats = [], []
        it = range(opts['max_num_iterations'])
        bar = None
        if progress:
            try:
                import tqdm
                bar = tqdm.trange(opts['max_num_iterations'])
                it = bar
            except ImportError:
                pass
        for _ in it:
            ts = time.perf_counter()
            loss, stats = eng.step(cams_t, pts_t)
            step_ms.append(1e3 * (time.perf_counter() - ts))
            step_stats.append(stats)
            self.last_stats = stats
            loss_history.append(loss)
            if len(loss_history) >= 2 * window_size:
                avg_recent = np.mean(loss_history[-window_size:])
                avg_previous = np.mean(loss_history[-2 * window_size:-window_size])
                improvement = (avg_previous - avg_recent) / avg_previous
                if abs(improvement) < opts['function_tolerance']:
                    break
                if loss_history[-1] == loss_history[-2]:
                    break
            if bar is not None:
                bar.set_postfix({"loss": loss})
            if self.visualizer:
                update(cameras, images, tracks, packed, cams_t, pts_t)
                self.visualizer.add_step(cameras, images, tracks, "bundle_adjustment")
        if bar is not None:
            bar.close()
        self.loss_history = loss_history
        t3 = time.perf_counter()
        self.final_loss, self.final_rmse = eng.cost(cams_t, pts_t)
        t3a = time.perf_counter()
        wb = {}
        update(cameras, images, tracks, packed, cams_t, pts_t, phases=wb)
        t3b = time.perf_counter()
        eng.close()
        t4 = time.perf_counter()
        self.timings.update(create_s=t2 - t1, steps_s=t3 - t2, update_s=t4 - t3, total_s=t4 - t0,
                            update_phases=dict(cost=t3a - t3, write_back=t3b - t3a, close=t4 - t3b,
                                               **{"write_back_" + k: v for k, v in wb.items()}),
                            steps=len(loss_history), final_rmse=self.final_rmse, step_ms=step_ms,
                            step_stats=step_stats)
