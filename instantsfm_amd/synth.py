"""Seeded synthetic BA scenes.

* C cameras on a ring of radius 30 around the origin (height jitter +-2), looking at the origin.
* SIMPLE_RADIAL by default: f=1000, image 2000x1500, pp=(1000,750), GT k=-0.02.
* P points uniform in a ball of radius 8; every track has L=10 observations whose cameras are L
  distinct indices from the window {h-30..h+30} mod C around a uniform home camera h
  (the whole ring when C <= 61).
* observations = GT projection + N(0, 0.5^2) px; 1% outliers get +-U(5,20) px per coordinate.
* initial values: rotation (+) N(0, 0.002^2) rad, translation + N(0, 0.05^2), points + N(0, 0.05^2),
  focal * (1 + N(0, 0.005^2)), distortion = 0.
* observations are stored track-major (the order ``TorchBA.Solve`` packs them in,
  bundle_adjustment.py:85-100); camera rows are pypose ``[t, q_xyzw, intrinsics-without-pp]``.
"""
from dataclasses import dataclass

import numpy as np

from .scene.defs import Camera, CameraModelId, Image, Track, num_intrinsics

# Ground-truth intrinsics (without the principal point) per model id.
_GT_INTR = {
    0: [1000.0],
    1: [1000.0, 1010.0],
    2: [1000.0, -0.02],
    3: [1000.0, -0.02, 0.004],
    4: [1000.0, 1010.0, -0.02, 0.004, 1e-4, -2e-4],
    5: [1000.0, 1010.0, -0.01, 0.002, -3e-4, 0.0],
    6: [1000.0, 1010.0, -0.02, 0.004, 1e-4, -2e-4, 1e-3, 0.01, -0.002, 3e-4],
    8: [1000.0, -0.01],
    9: [1000.0, -0.01, 0.002],
}
_FOCAL_COUNT = {0: 1, 1: 2, 2: 1, 3: 1, 4: 2, 5: 2, 6: 2, 8: 1, 9: 1}


@dataclass
class BAProblem:
    model: int
    cams_gt: np.ndarray      # [C, 7+ni] f64
    cams_init: np.ndarray    # [C, 7+ni] f64
    pp: np.ndarray           # [C, 2] f64
    points_gt: np.ndarray    # [P, 3] f64
    points_init: np.ndarray  # [P, 3] f64
    uv: np.ndarray           # [N, 2] f64, track-major
    cam_idx: np.ndarray      # [N] int32
    pt_idx: np.ndarray       # [N] int32, nondecreasing

    @property
    def n_cams(self):
        return self.cams_init.shape[0]

    @property
    def n_points(self):
        return self.points_init.shape[0]

    @property
    def n_obs(self):
        return self.uv.shape[0]


def _quat_mul(a, b):
    """Hamilton product of xyzw quaternions (broadcasting)."""
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz], axis=-1)


def _quat_from_rotvec(v):
    th = np.linalg.norm(v, axis=-1, keepdims=True)
    half = 0.5 * th
    s = np.where(th > 1e-12, np.sin(half) / np.maximum(th, 1e-300), 0.5 - th * th / 48.0)
    return np.concatenate([v * s, np.cos(half)], axis=-1)


def _quat_from_matrix(R):
    """Rotation matrix -> xyzw quaternion with w >= 0 (batched)."""
    from scipy.spatial.transform import Rotation
    q = Rotation.from_matrix(R).as_quat()
    return np.where(q[..., 3:4] < 0, -q, q)


def quat_to_matrix(q):
    x, y, z, w = np.moveaxis(q, -1, 0)
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def _project(model, X, cams, pp):
    R = quat_to_matrix(cams[:, 3:7])
    pc = np.einsum('nij,nj->ni', R, X) + cams[:, :3]
    uv = pc[:, :2] / pc[:, 2:3]
    intr = cams[:, 7:]
    nf = _FOCAL_COUNT[model]
    ff = intr[:, :nf] if nf == 2 else np.repeat(intr[:, :1], 2, axis=1)
    k = intr[:, nf:]
    r2 = np.sum(uv * uv, axis=1, keepdims=True)
    if model in (0, 1):
        d = uv
    elif model == 2:
        d = uv * (1 + k[:, 0:1] * r2)
    elif model == 3:
        d = uv * (1 + k[:, 0:1] * r2 + k[:, 1:2] * r2 ** 2)
    elif model in (4, 6):
        k1, k2, p = k[:, 0:1], k[:, 1:2], k[:, 2:4]
        if model == 4:
            radial = k1 * r2 + k2 * r2 ** 2
        else:
            k3, k4, k5, k6 = k[:, 4:5], k[:, 5:6], k[:, 6:7], k[:, 7:8]
            radial = (1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3) / (1 + k4 * r2 + k5 * r2 ** 2 + k6 * r2 ** 3) - 1
        uvp = uv[:, 0:1] * uv[:, 1:2]
        d = uv + uv * radial + 2 * p * uvp + p[:, ::-1] * (r2 + 2 * uv ** 2)
    elif model in (5, 8, 9):
        r = np.sqrt(r2)
        g = np.arctan(r) / r
        if model == 5:
            d = uv * g * (1 + k[:, 0:1] * r2 + k[:, 1:2] * r2 ** 2 + k[:, 2:3] * r2 ** 3)
        elif model == 8:
            d = uv * g * (1 + k[:, 0:1] * r2)
        else:
            d = uv * g * (1 + k[:, 0:1] * r2 + k[:, 1:2] * r2 ** 2)
    else:
        raise NotImplementedError
    return d * ff + pp, pc


def make_problem(n_cams, n_points, track_len=10, seed=0, model=2, noise_px=0.5, outlier_frac=0.01,
                 window=30, rot_sigma=0.002, trans_sigma=0.05, point_sigma=0.05, focal_sigma=0.005):
    """Build a seeded BAProblem; see module docstring for the recipe."""
    if model not in _GT_INTR:
        raise NotImplementedError(f"camera model {model}")
    rng = np.random.default_rng(seed)
    C, P, L = int(n_cams), int(n_points), int(track_len)
    if L > C:
        raise ValueError("track_len exceeds number of cameras")
    ni = num_intrinsics(model)

    ang = 2 * np.pi * np.arange(C) / C
    centers = np.stack([30 * np.cos(ang), 30 * np.sin(ang), rng.uniform(-2, 2, C)], axis=1)
    zax = -centers / np.linalg.norm(centers, axis=1, keepdims=True)
    up = np.array([0.0, 0.0, 1.0])
    xax = np.cross(zax, up)
    xax /= np.linalg.norm(xax, axis=1, keepdims=True)
    yax = np.cross(zax, xax)
    Rw2c = np.stack([xax, yax, zax], axis=1)
    t = -np.einsum('cij,cj->ci', Rw2c, centers)
    q = _quat_from_matrix(Rw2c)
    intr = np.tile(np.asarray(_GT_INTR[model], dtype=np.float64), (C, 1))
    cams_gt = np.concatenate([t, q, intr], axis=1)
    pp = np.tile(np.array([1000.0, 750.0]), (C, 1))

    d = rng.normal(size=(P, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    points_gt = d * (8.0 * rng.uniform(0, 1, (P, 1)) ** (1.0 / 3.0))

    if C <= 2 * window + 1:
        keys = rng.uniform(size=(P, C))
        cams_of = np.argsort(keys, axis=1)[:, :L]
    else:
        home = rng.integers(0, C, P)
        keys = rng.uniform(size=(P, 2 * window + 1))
        offs = np.argsort(keys, axis=1)[:, :L] - window
        cams_of = (home[:, None] + offs) % C
    cams_of = np.sort(cams_of, axis=1)
    cam_idx = cams_of.reshape(-1).astype(np.int32)
    pt_idx = np.repeat(np.arange(P, dtype=np.int32), L)

    uv, _ = _project(model, points_gt[pt_idx], cams_gt[cam_idx], pp[cam_idx])
    uv = uv + rng.normal(0, noise_px, uv.shape)
    n_out = int(round(outlier_frac * uv.shape[0]))
    if n_out:
        which = rng.choice(uv.shape[0], n_out, replace=False)
        uv[which] += rng.choice([-1.0, 1.0], (n_out, 2)) * rng.uniform(5, 20, (n_out, 2))

    dq = _quat_from_rotvec(rng.normal(0, rot_sigma, (C, 3)))
    q0 = _quat_mul(dq, q)
    t0 = t + rng.normal(0, trans_sigma, (C, 3))
    intr0 = np.zeros_like(intr)
    nf = _FOCAL_COUNT[model]
    intr0[:, :nf] = intr[:, :nf] * (1 + rng.normal(0, focal_sigma, (C, 1)))
    cams_init = np.concatenate([t0, q0, intr0], axis=1)
    points_init = points_gt + rng.normal(0, point_sigma, (P, 3))
    assert cams_init.shape[1] == 7 + ni
    return BAProblem(model, cams_gt, cams_init, pp, points_gt, points_init,
                     np.ascontiguousarray(uv), cam_idx, pt_idx)


# reference configs (BASELINE.json "configs")
CONFIGS = {
    1: dict(n_cams=20, n_points=2000),
    2: dict(n_cams=200, n_points=50000),
    3: dict(n_cams=1000, n_points=200000),
}


def make_config(cfg, seed=0, **kw):
    return make_problem(seed=seed, **CONFIGS[cfg], **kw)


def full_params(model, cam_row, pp):
    """Re-insert the pp columns into an intrinsics vector (inverse of bundle_adjustment.py:75-80)."""
    from .scene.defs import get_camera_model_info
    info = get_camera_model_info(CameraModelId(model))
    out = np.zeros(info['num_params'])
    rest = [i for i in range(info['num_params']) if i not in info['pp']]
    out[rest] = cam_row
    out[info['pp']] = pp
    return out


def to_scene(problem: BAProblem, use_init=True, image_features_dtype=np.float64):
    """Scene objects (cameras list, images list, tracks dict) for ``TorchBA.Solve``.

    One camera per image; image i observes its features in track order.
    """
    cams = problem.cams_init if use_init else problem.cams_gt
    pts = problem.points_init if use_init else problem.points_gt
    C = problem.n_cams
    model = CameraModelId(problem.model)
    cameras, images = [], []
    order = np.argsort(problem.cam_idx, kind='stable')
    counts = np.bincount(problem.cam_idx, minlength=C)
    starts = np.concatenate([[0], np.cumsum(counts)])
    feat_id = np.empty(problem.n_obs, dtype=np.int64)
    feat_id[order] = np.arange(problem.n_obs) - np.repeat(starts[:-1], counts)
    for c in range(C):
        cameras.append(Camera(id=c, model_id=model, width=2000, height=1500,
                              params=full_params(problem.model, cams[c, 7:], problem.pp[c])))
        R = quat_to_matrix(cams[c, 3:7])
        w2c = np.eye(4)
        w2c[:3, :3] = R
        w2c[:3, 3] = cams[c, :3]
        feats = problem.uv[order[starts[c]:starts[c + 1]]].astype(image_features_dtype)
        images.append(Image(id=c, cam_id=c, is_registered=True, world2cam=w2c, features=feats))
    tracks = {}
    L_ptr = np.concatenate([[0], np.cumsum(np.bincount(problem.pt_idx, minlength=problem.n_points))])
    obs_pairs = np.stack([problem.cam_idx.astype(np.int64), feat_id], axis=1)
    for p in range(problem.n_points):
        tracks[p] = Track(id=p, xyz=pts[p].copy(), observations=obs_pairs[L_ptr[p]:L_ptr[p + 1]].copy(),
                          is_initialized=True)
    return cameras, images, tracks


# ------------------------------------------------------------------------------------------------------------
# global positioning scenes (TorchGP.Optimize, global_positioning.py:45-206)
# ------------------------------------------------------------------------------------------------------------
@dataclass
class GPProblem:
    trans: np.ndarray        # [N, 3] world-frame ray of each observation (R_img^T features_undist, unit norm)
    cam_idx: np.ndarray      # [N] int32
    pt_idx: np.ndarray       # [N] int32, nondecreasing
    fcam: np.ndarray         # [C] 1.0 calibrated camera (has_prior_focal_length), 0.5 otherwise
    sfree: np.ndarray        # [N] int32: 1 scale optimized, 0 fixed (valid depth)
    cams_gt: np.ndarray      # [C, 3] camera positions
    points_gt: np.ndarray    # [P, 3]
    cams_init: np.ndarray
    points_init: np.ndarray
    scales_init: np.ndarray  # [N] (1 where free, 1/depth where fixed, as TorchGP builds them)

    @property
    def n_cams(self):
        return self.cams_init.shape[0]

    @property
    def n_points(self):
        return self.points_init.shape[0]

    @property
    def n_obs(self):
        return self.trans.shape[0]


def make_gp_problem(n_cams, n_points, track_len=10, seed=0, window=30, ray_sigma=0.002, outlier_frac=0.01,
                    calibrated_frac=0.8, depth_frac=0.0, init="random", scene_scale=100.0, init_sigma=0.5):
    """Seeded global-positioning scene on the same ring geometry as make_problem: rays from camera centres to points
    (angular noise ray_sigma, outlier_frac of rays off by 0.05-0.2 rad), a calibrated_frac of cameras with factor 1
    (else 0.5), a depth_frac of observations with a fixed scale 1/depth.  init="random" follows
    TorchGP.InitializeRandomPositions (uniform in +-scene_scale, global_positioning.py:22-39); "perturbed" starts
    from ground truth + N(0, init_sigma)."""
    rng = np.random.default_rng(seed)
    C, P, L = int(n_cams), int(n_points), int(track_len)
    ang = 2 * np.pi * np.arange(C) / C
    centers = np.stack([30 * np.cos(ang), 30 * np.sin(ang), rng.uniform(-2, 2, C)], axis=1)
    d = rng.normal(size=(P, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    points = d * (8.0 * rng.uniform(0, 1, (P, 1)) ** (1.0 / 3.0))
    if C <= 2 * window + 1:
        cams_of = np.argsort(rng.uniform(size=(P, C)), axis=1)[:, :L]
    else:
        home = rng.integers(0, C, P)
        offs = np.argsort(rng.uniform(size=(P, 2 * window + 1)), axis=1)[:, :L] - window
        cams_of = (home[:, None] + offs) % C
    cams_of = np.sort(cams_of, axis=1)
    cam_idx = cams_of.reshape(-1).astype(np.int32)
    pt_idx = np.repeat(np.arange(P, dtype=np.int32), L)
    v = points[pt_idx] - centers[cam_idx]
    depth = np.linalg.norm(v, axis=1)
    rays = v / depth[:, None]
    n = rays.shape[0]
    sig = np.full(n, ray_sigma)
    n_out = int(round(outlier_frac * n))
    if n_out:
        sig[rng.choice(n, n_out, replace=False)] = rng.uniform(0.05, 0.2, n_out)
    rays = rays + rng.normal(size=rays.shape) * sig[:, None]
    rays /= np.linalg.norm(rays, axis=1, keepdims=True)
    fcam = np.where(rng.uniform(size=C) < calibrated_frac, 1.0, 0.5)
    has_depth = rng.uniform(size=n) < depth_frac
    sfree = (~has_depth).astype(np.int32)
    scales_init = np.where(has_depth, 1.0 / depth, 1.0)
    if init == "random":
        cams_init = scene_scale * rng.uniform(-1, 1, (C, 3))
        points_init = scene_scale * rng.uniform(-1, 1, (P, 3))
    else:
        cams_init = centers + rng.normal(0, init_sigma, (C, 3))
        points_init = points + rng.normal(0, init_sigma, (P, 3))
    return GPProblem(np.ascontiguousarray(rays), cam_idx, pt_idx, fcam, sfree, centers, points,
                     np.ascontiguousarray(cams_init), np.ascontiguousarray(points_init), np.ascontiguousarray(scales_init))


# ------------------------------------------------------------------------------------------------------------
# retriangulation scenes (RetriangulateTracks, track_retriangulation.py:215-259)
# ------------------------------------------------------------------------------------------------------------
def make_retri_scene(model=2, n_cams=20, n_points=600, seed=0, point_sigma=0.01, drop_frac=0.25, wrong_frac=0.03,
                     far_frac=0.02, missing_frac=0.05, features_dtype=np.float32):
    """(cameras, images, tracks, tracks_orig) for complete_tracks / RetriangulateTracks.

    Ground-truth poses; float32 features (the database's keypoint type).  ``tracks_orig`` holds every track's full
    observation list (as TrackEngine.EstablishFullTracks returns: id -> int array [k, 2]) plus a few wrong
    observations (another track's feature in a random image); ``tracks`` keeps a random subset of each track's
    observations (the completion re-adds the rest), perturbed points, some points moved far away (no candidate
    passes), and lacks a few ids of ``tracks_orig`` altogether.  Track ids are non-contiguous."""
    prob = make_problem(n_cams, n_points, seed=seed, model=model)
    cameras, images, tracks0 = to_scene(prob, use_init=False, image_features_dtype=features_dtype)
    rng = np.random.default_rng(seed + 1000)
    nfeat = np.array([len(im.features) for im in images])
    tracks, tracks_orig = {}, {}
    for p, t in tracks0.items():
        tid = 7 * p + 3
        full = t.observations.astype(np.int64)
        if rng.uniform() < wrong_frac:
            img = int(rng.integers(0, n_cams))
            full = np.concatenate([full, [[img, int(rng.integers(0, nfeat[img]))]]])
        tracks_orig[tid] = full
        if rng.uniform() < missing_frac:
            continue
        keep = rng.uniform(size=t.observations.shape[0]) >= drop_frac
        keep[:2] = True
        xyz = t.xyz + rng.normal(0, point_sigma, 3)
        if rng.uniform() < far_frac:
            xyz = xyz + rng.normal(0, 3.0, 3)
        tracks[tid] = Track(id=tid, xyz=xyz, observations=t.observations[keep].copy(), is_initialized=True)
    return cameras, images, tracks, tracks_orig


# ------------------------------------------------------------------------------------------------------------
# COLMAP database scenes (ReadColmapDatabase + TrackEngine)
# ------------------------------------------------------------------------------------------------------------
def write_match_database(path, n_images=24, n_points=1500, track_len=6, window=5, seed=0, distractors=40,
                         wrong_frac=0.03, dup_frac=0.03, bad_index_frac=0.002, kp_cols=6, feature_name="superpoint",
                         min_common=12):
    """Write a seeded COLMAP database.db (utils/database.py schema) of a ring of images looking at a point cloud.

    Images get DB ids 1..n with one gap and share cameras (one per 3 images, SIMPLE_RADIAL, a third with a focal
    prior); keypoints are the float32 projections of the points each image sees plus random distractors, shuffled
    (``kp_cols`` columns like SIFT's affine shape; one image has no keypoints row).  Every image pair with at least
    ``min_common`` common points gets a matches row (random order, ``wrong_frac`` random wrong matches, ``dup_frac``
    near-duplicate features -- a second keypoint within 2 px matched to the same partner -- and a few out-of-range
    indices) and a two_view_geometries row whose config is mostly valid (2, 3, 4) and sometimes invalid (0, 1, 7, 8);
    one pair has NULL match data, one has matches but no geometry, some are stored with the larger image id first.
    Returns the number of match rows written."""
    from .utils.database import COLMAPDatabase
    rng = np.random.default_rng(seed)
    prob = make_problem(n_images, n_points, track_len=track_len, seed=seed, window=window)
    C, P = prob.n_cams, prob.n_points
    db = COLMAPDatabase.connect(path)
    db.create_tables()
    cam_ids = []
    for c in range(0, C, 3):
        f = float(prob.cams_gt[c, 7])
        cam_ids.append(db.add_camera(2, 2000, 1500, [f, 1000.0, 750.0, float(prob.cams_gt[c, 8])],
                                     prior_focal_length=(c // 3) % 3 == 0))
    img_ids = [i + 1 + (1 if i >= n_images // 2 else 0) for i in range(C)]  # one gap in the ids
    for i in range(C):
        db.add_image(f"img_{i:04d}.jpg", cam_ids[i // 3], image_id=img_ids[i])
    # features: projections (float32) + distractors, shuffled; near-duplicates of some observations
    feat_of = {}
    feats_per_img = []
    no_kp = C // 3
    for c in range(C):
        sel = np.flatnonzero(prob.cam_idx == c)
        pts = prob.pt_idx[sel]
        xy = prob.uv[sel]
        dup = rng.uniform(size=sel.size) < dup_frac
        extra = rng.uniform([0, 0], [2000, 1500], (distractors, 2))
        near = xy[dup] + rng.uniform(-1.4, 1.4, (int(dup.sum()), 2))
        allxy = np.concatenate([xy, near, extra])
        order = rng.permutation(allxy.shape[0])
        inv = np.empty_like(order)
        inv[order] = np.arange(order.size)
        for k, p in enumerate(pts):
            feat_of[(c, int(p))] = [int(inv[k])]
        for j, k in enumerate(np.flatnonzero(dup)):
            feat_of[(c, int(pts[k]))].append(int(inv[sel.size + j]))
        kp = np.zeros((allxy.shape[0], kp_cols), np.float32)
        kp[:, :2] = allxy[order]
        if kp_cols > 2:
            kp[:, 2:] = rng.normal(size=(allxy.shape[0], kp_cols - 2))
        feats_per_img.append(kp.shape[0])
        if c != no_kp:
            db.add_keypoints(img_ids[c], kp)
    seen = [set(prob.pt_idx[prob.cam_idx == c].tolist()) for c in range(C)]
    n_rows = 0
    pairs = [(i, j) for i in range(C) for j in range(i + 1, C) if len(seen[i] & seen[j]) >= min_common]
    null_pair = pairs[len(pairs) // 2]
    nogeo_pair = pairs[len(pairs) // 3]
    for i, j in pairs:
        common = sorted(seen[i] & seen[j])
        m = []
        for p in common:
            fi, fj = feat_of[(i, p)], feat_of[(j, p)]
            m.append((fi[0], fj[0]))
            if len(fi) > 1:
                m.append((fi[1], fj[0]))
            if len(fj) > 1:
                m.append((fi[0], fj[1]))
        n_wrong = int(np.ceil(wrong_frac * len(m))) if rng.uniform() < 0.7 else 0
        for _ in range(n_wrong):
            m.append((int(rng.integers(0, feats_per_img[i])), int(rng.integers(0, feats_per_img[j]))))
        m = np.array(m, dtype=np.int64)[rng.permutation(len(m))]
        if rng.uniform() < 0.2:
            k = max(1, int(bad_index_frac * len(m)))
            rows = rng.choice(len(m), k, replace=False)
            m[rows, rng.integers(0, 2)] = feats_per_img[i] + feats_per_img[j] + 5
        a, b = (img_ids[i], img_ids[j]) if rng.uniform() < 0.8 else (img_ids[j], img_ids[i])
        mm = m if a == img_ids[i] else m[:, ::-1]
        if (i, j) == null_pair:
            db.add_null_matches(a, b)
        else:
            db.add_matches(a, b, mm)
        n_rows += 1
        if (i, j) == nogeo_pair:
            continue
        u = rng.uniform()
        config = 2 if u < 0.7 else 3 if u < 0.8 else 4 if u < 0.85 else int(rng.choice([0, 1, 7, 8]))
        F = rng.normal(size=(3, 3))
        db.add_two_view_geometry(a, b, mm, F=F, E=rng.normal(size=(3, 3)), H=rng.normal(size=(3, 3)), config=config)
    if feature_name:
        db.add_feature_name(feature_name)
    db.commit()
    db.close()
    return n_rows


def assign_inliers(view_graph, seed=0, frac=0.9):
    """Seeded inlier subsets (the relative-pose stage's output, image_pair_inliers.py) for every pair, in order."""
    for pair_id, pair in view_graph.image_pairs.items():
        rng = np.random.default_rng([seed, pair_id % (2 ** 63)])
        n = len(pair.matches)
        pair.inliers = np.flatnonzero(rng.uniform(size=n) < frac)


def make_match_graph(n_images=500, n_points=600_000, track_len=8, window=12, reach=2, distractors=2000,
                     wrong_frac=0.01, seed=0):
    """Config-5-sized matches without a database: (view_graph, images) for TrackEngine.

    n_images images on a ring; each point is seen by ``track_len`` distinct images of a ``window`` of consecutive ones;
    every image holds its observations plus ``distractors`` random keypoints (float32, shuffled).  Each image pair
    gets the matches of the points both see whose observations are at most ``reach`` apart in the track (sequential
    matching), plus ``wrong_frac`` random wrong matches, in random order; pairs are in pair-id order, all matches are
    inliers.  Vectorized: builds ~8M matches in seconds."""
    from .scene.defs import ImagePair, Image, Ids2PairId, ViewGraph
    rng = np.random.default_rng(seed)
    C, P, L = int(n_images), int(n_points), int(track_len)
    home = rng.integers(0, C, P)
    offs = np.sort(np.argsort(rng.uniform(size=(P, window)), axis=1)[:, :L], axis=1)
    img = (home[:, None] + offs) % C                               # [P, L]
    n_obs_img = np.bincount(img.reshape(-1), minlength=C)
    nfeat = n_obs_img + distractors
    # feature index of each observation: a random slot of its image
    feat = np.empty(P * L, np.int64)
    flat_img = img.reshape(-1)
    order = np.lexsort((rng.uniform(size=P * L), flat_img))
    start = np.concatenate([[0], np.cumsum(n_obs_img)])
    rank_in_img = np.arange(P * L) - start[flat_img[order]]
    slots = [rng.permutation(nfeat[c]) for c in range(C)]
    slot_cat = np.concatenate(slots)
    slot_off = np.concatenate([[0], np.cumsum(nfeat)])
    feat[order] = slot_cat[slot_off[flat_img[order]] + rank_in_img]
    feat = feat.reshape(P, L)
    a_img, a_feat, b_img, b_feat = [], [], [], []
    for d in range(1, reach + 1):
        a_img.append(img[:, :-d].reshape(-1)); a_feat.append(feat[:, :-d].reshape(-1))
        b_img.append(img[:, d:].reshape(-1)); b_feat.append(feat[:, d:].reshape(-1))
    ai, af, bi, bf = (np.concatenate(x) for x in (a_img, a_feat, b_img, b_feat))
    n_wrong = int(wrong_frac * ai.size)
    wi = rng.integers(0, C, n_wrong)
    wj = (wi + rng.integers(1, window, n_wrong)) % C
    ai = np.concatenate([ai, wi]); bi = np.concatenate([bi, wj])
    af = np.concatenate([af, (rng.uniform(size=n_wrong) * nfeat[wi]).astype(np.int64)])
    bf = np.concatenate([bf, (rng.uniform(size=n_wrong) * nfeat[wj]).astype(np.int64)])
    swap = ai > bi
    ai[swap], bi[swap] = bi[swap], ai[swap].copy()
    af[swap], bf[swap] = bf[swap], af[swap].copy()
    key = ai * C + bi
    order = np.lexsort((rng.uniform(size=key.size), key))
    key, af, bf = key[order], af[order], bf[order]
    ukey, first = np.unique(key, return_index=True)
    bounds = np.concatenate([first, [key.size]])
    vg = ViewGraph()
    for k, (s, e) in enumerate(zip(bounds[:-1], bounds[1:])):
        i, j = divmod(int(ukey[k]), C)
        p = ImagePair(image_id1=i, image_id2=j)
        p.matches = np.stack([af[s:e], bf[s:e]], 1).astype(np.uint32)
        p.inliers = np.arange(e - s)
        vg.image_pairs[Ids2PairId(i, j)] = p
    images = [Image(id=c, cam_id=0, features=rng.uniform([0, 0], [2000, 1500], (nfeat[c], 2)).astype(np.float32))
              for c in range(C)]
    return vg, images


# ------------------------------------------------------------------------------------------------------------
# Config-5 mapper scenes: a COLMAP database.db with geometrically consistent tracks (global_mapper.py:80-146)
# ------------------------------------------------------------------------------------------------------------
@dataclass
class MapperScene:
    """What write_mapper_database wrote, plus the ground truth the stand-in for rotation averaging draws from."""
    path: str
    n_images: int
    n_points: int
    n_matches: int
    n_pairs: int
    rot_gt: np.ndarray       # [C, 3, 3] world-to-camera rotations, DB image order (= reader's list order)
    centers_gt: np.ndarray   # [C, 3]
    points_gt: np.ndarray    # [P, 3]


def write_mapper_database(path, n_images=500, n_points=100_000, track_len=8, window=12, reach=3, seed=0,
                          images_per_camera=50, distractors=200, wrong_frac=0.01, min_matches=15,
                          focal_sigma=0.01):
    """Write a seeded COLMAP database.db (utils/database.py schema) for the mapper's BA half (config 5).

    Geometry is make_problem's ring (SIMPLE_RADIAL, GT f = 1000, k = -0.02, 0.5 px noise, 1 % outliers): each point
    is seen by ``track_len`` distinct images of a window of 2*window+1 consecutive ones.  Keypoints are those
    observations (float32, COLMAP's type) plus ``distractors`` random ones per image, shuffled.  Matches are the
    sequential-matching subset of every track (observations at most ``reach`` apart in camera order) plus
    ``wrong_frac`` random wrong matches; a pair with fewer than ``min_matches`` matches is not stored.  Each stored
    pair gets a matches row and a two_view_geometries row holding the same matches (config CALIBRATED, a few
    UNCALIBRATED).  Cameras are shared by ``images_per_camera`` images; their stored focal is the GT one times
    1 + N(0, focal_sigma^2) and their distortion 0 (BA recovers both).  Vectorized: a 500-image database in seconds."""
    from .utils.database import COLMAPDatabase
    rng = np.random.default_rng([seed, 5])
    prob = make_problem(n_images, n_points, track_len=track_len, seed=seed, window=window)
    C, P, L = prob.n_cams, prob.n_points, int(track_len)
    cam_idx = prob.cam_idx.astype(np.int64)
    n_obs = cam_idx.size
    n_obs_img = np.bincount(cam_idx, minlength=C)
    nfeat = n_obs_img + distractors
    # feature slot of every observation: a random permutation of its image's keypoints
    order = np.argsort(cam_idx, kind="stable")
    start = np.concatenate([[0], np.cumsum(n_obs_img)])
    rank = np.empty(n_obs, np.int64)
    rank[order] = np.arange(n_obs) - start[cam_idx[order]]
    slot_off = np.concatenate([[0], np.cumsum(nfeat)])
    slots = np.concatenate([rng.permutation(int(n)) for n in nfeat])
    feat = slots[slot_off[cam_idx] + rank]
    kps = []
    for c in range(C):
        kp = np.empty((int(nfeat[c]), 2), np.float32)
        kp[:] = rng.uniform([0, 0], [2000, 1500], (int(nfeat[c]), 2))
        sel = order[start[c]:start[c + 1]]
        kp[feat[sel]] = prob.uv[sel]
        kps.append(kp)
    # sequential matches inside each track
    img = cam_idx.reshape(P, L)
    ft = feat.reshape(P, L)
    ai, af, bi, bf = [], [], [], []
    for d in range(1, min(reach, L - 1) + 1):
        ai.append(img[:, :-d].ravel()); af.append(ft[:, :-d].ravel())
        bi.append(img[:, d:].ravel()); bf.append(ft[:, d:].ravel())
    ai, af, bi, bf = (np.concatenate(x) for x in (ai, af, bi, bf))
    n_wrong = int(wrong_frac * ai.size)
    w = rng.integers(0, ai.size, n_wrong)                # wrong partner feature on an existing pair
    ai = np.concatenate([ai, ai[w]]); bi = np.concatenate([bi, bi[w]]); af = np.concatenate([af, af[w]])
    bf = np.concatenate([bf, (rng.uniform(size=n_wrong) * nfeat[bi[ai.size - n_wrong:]]).astype(np.int64)])
    swap = ai > bi
    ai[swap], bi[swap] = bi[swap], ai[swap].copy()
    af[swap], bf[swap] = bf[swap], af[swap].copy()
    key = ai * C + bi
    o = np.lexsort((rng.uniform(size=key.size), key))
    key, af, bf = key[o], af[o], bf[o]
    ukey, first, cnt = np.unique(key, return_index=True, return_counts=True)

    db = COLMAPDatabase.connect(path)
    db.create_tables()
    n_cam_rows = (C + images_per_camera - 1) // images_per_camera
    f0 = 1000.0 * (1 + rng.normal(0, focal_sigma, n_cam_rows))
    cam_ids = [db.add_camera(2, 2000, 1500, [f0[k], 1000.0, 750.0, 0.0], prior_focal_length=(k % 2 == 0))
               for k in range(n_cam_rows)]
    for c in range(C):
        db.add_image(f"img_{c:04d}.jpg", cam_ids[c // images_per_camera], image_id=c + 1)
        db.add_keypoints(c + 1, kps[c])
    n_pairs = n_matches = 0
    for k in range(ukey.size):
        if cnt[k] < min_matches:
            continue
        i, j = divmod(int(ukey[k]), C)
        m = np.stack([af[first[k]:first[k] + cnt[k]], bf[first[k]:first[k] + cnt[k]]], 1)
        db.add_matches(i + 1, j + 1, m)
        db.add_two_view_geometry(i + 1, j + 1, m, config=2 if rng.uniform() < 0.95 else 3)
        n_pairs += 1
        n_matches += int(cnt[k])
    db.add_feature_name("colmap")
    db.commit()
    db.close()
    Rgt = quat_to_matrix(prob.cams_gt[:, 3:7])
    centers = -np.einsum('cji,cj->ci', Rgt, prob.cams_gt[:, :3])
    return MapperScene(path, C, P, n_matches, n_pairs, Rgt, centers, prob.points_gt)


def stand_in_rotation_averaging(view_graph, images, scene: MapperScene, rot_sigma_deg=0.1, seed=0):
    """What the mapper's stages before track establishment leave behind (global_mapper.py:22-78, out of scope here):
    every pair's inlier set (relpose estimation, image_pair_inliers.py) = the geometrically verified matches the
    database's two_view_geometries rows hold, and every image registered with a world-to-camera rotation = ground
    truth composed with a N(0, rot_sigma_deg^2) rotation (rotation averaging's output)."""
    rng = np.random.default_rng([seed, 7])
    for pair in view_graph.image_pairs.values():
        pair.inliers = np.arange(len(pair.matches))
    C = len(images)
    dq = _quat_from_rotvec(rng.normal(0, np.deg2rad(rot_sigma_deg), (C, 3)))
    R = np.einsum('cij,cjk->cik', quat_to_matrix(dq), scene.rot_gt)
    for i, im in enumerate(images):
        im.world2cam = np.eye(4)
        im.world2cam[:3, :3] = R[i]
        im.is_registered = True
