"""CPU restatement of the between-round caller passes -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, as the checker; the product path
(instantsfm_amd/processors/{image_undistortion,track_filter}.py) runs the HIP kernels of csrc/passes.hip.

* ``img2cam`` / ``undistort_images`` -- image_undistortion.py:3-10 + Camera.img2cam (scene/defs.py:315-369).  Eight of
  the eleven models call ``cv2.undistortPoints`` (opencv-python==4.10.0.84, pyproject.toml:18), which is absent from
  this image.  Its published algorithm (calib3d/src/undistort.dispatch.cpp, cvUndistortPointsInternal, default
  criteria TermCriteria(COUNT, 5, 0.01): five fixed-point iterations, no tilt, R = I, P = none, output in the input's
  float type) is restated in ``cv_undistort_points``.  PARITY: SIMPLE_PINHOLE / PINHOLE are pinned by golden vectors
  from the reference; the cv2 models are pinned only through the reference's own forward model (``cam2img``, golden
  vectors of it: undistort(cam2img(x)) == x where five iterations converge) -- "parity unpinned" against cv2 itself.
* ``filter_reproj_normalized`` -- track_filter.py:26-66 (FilterTracksByReprojectionNormalized), including its
  counter, which tests the slice of the *next* track (``count`` is advanced before the test).  Pinned by golden
  vectors from the reference.
* ``filter_angle`` -- track_filter.py:5-24 (FilterTracksByAngle).  Pinned by golden vectors.
"""
import numpy as np

EPSILON = 1e-10

# cv2 distortion-coefficient vector (k1,k2,p1,p2,k3,k4,k5,k6,s1,s2,s3,s4) built by Camera.img2cam, per model, from the
# reference's parameter vector (Camera.set_params, defs.py:176-237): index into params, or None for 0.
_CV = {
    2: (3, None, None, None),                                   # SIMPLE_RADIAL  [k, 0, 0, 0]
    3: (3, 4, None, None),                                      # RADIAL
    4: (4, 5, 6, 7),                                            # OPENCV [k1, k2, p1, p2]
    5: (4, 5, None, None, 6),                                   # OPENCV_FISHEYE [k1, k2, 0, 0, k3] (k4 ignored)
    6: (4, 5, 6, 7, 8, 9, 10, 11),                              # FULL_OPENCV
    8: (3, None, None, None),                                   # SIMPLE_RADIAL_FISHEYE
    9: (3, 4, None, None),                                      # RADIAL_FISHEYE
    10: (4, 5, 6, 7, 8, None, None, None, 10, 11, None, None),  # THIN_PRISM_FISHEYE
}
_FISHEYE = (5, 8, 9, 10)


def focal_pp(model, params):
    """(fx, fy, cx, cy) as Camera.set_params stores them."""
    p = params
    if model in (0, 2, 3, 8, 9):
        return p[0], p[0], p[1], p[2]
    return p[0], p[1], p[2], p[3]


def cv_coeffs(model, params):
    k = np.zeros(14)
    for j, src in enumerate(_CV[model]):
        if src is not None:
            k[j] = params[src]
    return k


def cv_undistort_points(xy, fx, fy, cx, cy, k, iters=5):
    """cvUndistortPointsInternal (OpenCV 4.10) for R = I, P = none, no tilt, criteria COUNT 5: double arithmetic,
    result cast back to the input dtype."""
    src = np.asarray(xy)
    u = src[:, 0].astype(np.float64)
    v = src[:, 1].astype(np.float64)
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (u - cx) * ifx
    y = (v - cy) * ify
    x0, y0 = x.copy(), y.copy()
    done = np.zeros(x.shape, bool)
    for _ in range(iters):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        neg = (icdist < 0) & ~done   # regression_14583: fall back to the undistorted-by-K point and stop
        x = np.where(neg, (u - cx) * ifx, x)
        y = np.where(neg, (v - cy) * ify, y)
        done |= neg
        deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
        deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
        x = np.where(done, x, (x0 - deltaX) * icdist)
        y = np.where(done, y, (y0 - deltaY) * icdist)
    return np.stack([x, y], 1).astype(src.dtype)


def normal_from_fisheye(uv):
    """Camera.normal_from_fisheye (defs.py:252-255), in the array's own dtype."""
    theta = np.linalg.norm(uv, axis=-1, keepdims=True)
    theta_cos_theta = theta * np.cos(theta)
    # the reference divides unguarded: uv = 0 gives 0/0 = NaN there too (the kernel matches it)
    with np.errstate(invalid="ignore", divide="ignore"):
        return uv * np.sin(theta) / theta_cos_theta


def img2cam(model, params, xy):
    """Camera.img2cam (defs.py:315-369) for the implemented models (FOV restated as written: r2 of raw pixels)."""
    params = np.asarray(params, dtype=np.float64)
    fx, fy, cx, cy = focal_pp(model, params)
    if model == 0:
        return (xy - np.array([cx, cy])) / float(np.mean([fx, fy]))
    if model == 1:
        return (xy - np.array([cx, cy])) / np.array([fx, fy])
    if model == 7:
        omega = float(params[4])  # a Python float in the reference (Camera.params is a list): float32 inputs stay float32
        r2 = np.expand_dims(np.sum(xy ** 2, axis=-1), axis=-1)
        omega2 = omega ** 2
        eps = 1e-4
        if omega2 < eps:
            factor = (omega2 * r2) / 3 - omega2 / 12 + 1
        else:
            m = r2 < eps
            factor = np.zeros_like(r2)
            factor[m] = (omega * (omega2 * r2[m] + 3)) / (6 * np.tan(omega / 2))
            radius = np.sqrt(r2[~m])
            factor[~m] = np.tan(radius * omega) / (radius * 2 * np.tan(omega / 2))
        return (xy - np.array([cx, cy])) / np.array([fx, fy]) * factor
    uv = cv_undistort_points(xy, fx, fy, cx, cy, cv_coeffs(model, params))
    if model in _FISHEYE:
        uv = normal_from_fisheye(uv)
    return uv


def undistort_rays(model, params, xy):
    """undistort_process (image_undistortion.py:3-6): unit rays [n, 3] (float64)."""
    fu = img2cam(model, params, xy)
    fu = np.hstack([fu, np.ones((fu.shape[0], 1))])
    return fu / np.linalg.norm(fu, axis=1, keepdims=True)


def gather_obs(tracks, images):
    """Observations of all tracks in dict order: image ids, feature ids, track rows, and per-track counts."""
    obs = [np.asarray(t.observations, dtype=np.int64).reshape(-1, 2) for t in tracks.values()]
    counts = np.array([o.shape[0] for o in obs], dtype=np.int64)
    allobs = np.concatenate(obs) if obs else np.zeros((0, 2), np.int64)
    return allobs[:, 0], allobs[:, 1], np.repeat(np.arange(len(obs)), counts), counts


def filter_reproj_normalized(images, tracks, max_reprojection_error):
    """FilterTracksByReprojectionNormalized (track_filter.py:26-66) on plain arrays: returns (valid mask over the
    concatenated observations, per-track counts, counter)."""
    img, feat, trow, counts = gather_obs(tracks, images)
    w2c = np.array([im.world2cam for im in images])[img]
    xyz = np.hstack([np.array([t.xyz for t in tracks.values()]), np.ones((len(tracks), 1))])[trow]
    fu = np.array([images[i].features_undist[f] for i, f in zip(img.tolist(), feat.tolist())]).reshape(-1, 3)
    fu_r = fu[:, :2] / (fu[:, 2:] + EPSILON)
    pc = np.einsum('ijk,ik->ij', w2c, xyz)[:, :3]
    valid = pc[:, 2] > EPSILON
    pr = pc[:, :2] / (pc[:, 2:] + EPSILON)
    err = np.linalg.norm(pr - fu_r, axis=1)
    valid = valid & (err < max_reprojection_error)
    return valid, counts, quirk_counter(valid, counts), err


def quirk_counter(valid, counts):
    """The reference's counter: after advancing ``count`` past track j it tests valid[count : count + len_j]."""
    starts = np.concatenate([[0], np.cumsum(counts)])
    inv = np.concatenate([[0], np.cumsum(~valid)])
    n = valid.shape[0]
    a = starts[1:]
    b = np.minimum(a + counts, n)
    return int(np.sum(inv[b] - inv[np.minimum(a, n)] > 0))


def filter_angle(images, tracks, max_angle_error):
    """FilterTracksByAngle (track_filter.py:5-24): valid mask, per-track counts, number of tracks changed."""
    thres = np.cos(np.deg2rad(max_angle_error))
    img, feat, trow, counts = gather_obs(tracks, images)
    valid = np.zeros(img.shape[0], bool)
    xyz = [t.xyz for t in tracks.values()]
    for x in range(img.shape[0]):
        image = images[img[x]]
        pt = image.world2cam[:3, :3] @ xyz[trow[x]] + image.world2cam[:3, 3]
        if pt[2] < EPSILON:
            continue
        pt = pt / np.linalg.norm(pt)
        valid[x] = np.dot(pt, image.features_undist[feat[x]]) > thres
    starts = np.concatenate([[0], np.cumsum(counts)])
    changed = int(sum(1 for j in range(len(counts)) if not valid[starts[j]:starts[j + 1]].all()))
    return valid, counts, changed


def filter_tri_angle(images, tracks, min_angle):
    """FilterTracksTriangulationAngle (track_filter.py:116-137): keys of the tracks it deletes."""
    thres = np.cos(np.deg2rad(min_angle))
    centers = np.array([im.center() for im in images])
    out = []
    for key, track in tracks.items():
        ids = np.unique(np.asarray(track.observations).reshape(-1, 2)[:, 0])
        v = track.xyz - centers[ids]
        pts = v / (np.linalg.norm(v, axis=1, keepdims=True) + EPSILON)
        if np.all(pts @ pts.T > thres):
            out.append(key)
    return out


# ---------------------------------------------------------------------------------------------------------------------
# Retriangulation passes: Camera.cam2img, FilterTracksByReprojection, complete_tracks.

def cam2img(model, params, uvw):
    """Camera.cam2img (scene/defs.py:371-412) with Camera.Distortion (defs.py:257-313) and fisheye_from_normal
    (defs.py:246-250), numpy float64, the reference's operation order.  Pinned by camera_models_golden.npz."""
    params = np.asarray(params, dtype=np.float64)
    fx, fy, cx, cy = focal_pp(model, params)
    pp = np.array([cx, cy])
    ff = np.array([fx, fy])
    f = np.mean(ff)
    uv = uvw[..., :2] / (np.expand_dims(uvw[..., 2], axis=-1) + 1e-10)

    def fisheye_from_normal(uv):
        r = np.linalg.norm(uv, axis=-1, keepdims=True)
        r = np.clip(r, 1e-8, None)
        return uv * np.arctan(r) / r

    def r2_of(uv):
        return np.sum(uv ** 2, axis=-1, keepdims=True)

    def tangential(uv, p, r2):
        uv_ = np.expand_dims(uv[..., 0] * uv[..., 1], axis=-1)
        return 2 * p * uv_, p[::-1] * (r2 + 2 * uv ** 2)

    if model == 0:
        return uv * f + pp
    if model == 1:
        return uv * ff + pp
    if model in (2, 8):
        if model == 8:
            uv = fisheye_from_normal(uv)
        r2 = r2_of(uv)
        uv += uv * params[3] * r2
        return uv * f + pp
    if model in (3, 9):
        if model == 9:
            uv = fisheye_from_normal(uv)
        r2 = r2_of(uv)
        uv += uv * params[3] * r2 + uv * params[4] * r2 ** 2
        return uv * f + pp
    if model == 4:
        r2 = r2_of(uv)
        p = params[6:8]
        a, b = tangential(uv, p, r2)
        d = uv * (params[4] * r2 + params[5] * r2 ** 2) + a
        d += b
        uv += d
        return uv * ff + pp
    if model == 5:
        uv = fisheye_from_normal(uv)
        r2 = r2_of(uv)
        uv += uv * (params[4] * r2 + params[5] * r2 ** 2 + params[6] * r2 ** 3)
        return uv * ff + pp
    if model == 6:
        r2 = r2_of(uv)
        k = params[[4, 5, 8, 9, 10, 11]]
        radial = (1 + k[0] * r2 + k[1] * r2 ** 2 + k[2] * r2 ** 3) / (1 + k[3] * r2 + k[4] * r2 ** 2 + k[5] * r2 ** 3) - 1
        a, b = tangential(uv, params[6:8], r2)
        d = uv * radial + a
        d += b
        uv += d
        return uv * ff + pp
    if model == 7:
        omega = params[4]
        r2 = r2_of(uv)
        omega2 = omega ** 2
        eps = 1e-4
        if omega2 < eps:
            factor = (omega2 * r2) / 3 - omega2 / 12 + 1
        else:
            factor = np.zeros_like(r2)
            m = r2 < eps
            th = np.tan(omega / 2)
            factor[m] = (-2 * th * (4 * r2[m] * th ** 2 - 3)) / (3 * omega)
            radius = np.sqrt(r2[~m])
            factor[~m] = np.arctan(radius * 2 * np.tan(omega / 2)) / (radius * omega)
        return uv * factor * f + pp
    if model == 10:
        uv = fisheye_from_normal(uv)
        r2 = r2_of(uv)
        k = params[[4, 5, 8, 9]]
        a, b = tangential(uv, params[6:8], r2)
        d = uv * (k[0] * r2 + k[1] * r2 ** 2 + k[2] * r2 ** 3) + a
        d += b
        d += params[10:12] * r2
        uv += d
        return uv * ff + pp
    raise NotImplementedError


def filter_reproj_pixel(cameras, images, tracks, max_reprojection_error):
    """FilterTracksByReprojection (track_filter.py:68-113): valid mask over the concatenated observations, per-track
    counts, the reference's counter (same next-track-slice quirk as the normalized filter) and the errors."""
    img, feat, trow, counts = gather_obs(tracks, images)
    w2c = np.array([im.world2cam for im in images])[img]
    cam_of = np.array([im.cam_id for im in images])[img]
    xyz = np.hstack([np.array([t.xyz for t in tracks.values()]), np.ones((len(tracks), 1))])[trow]
    feats = np.array([images[i].features[f] for i, f in zip(img.tolist(), feat.tolist())]).reshape(-1, 2)
    pc = np.einsum('ijk,ik->ij', w2c, xyz)[:, :3]
    valid = pc[:, 2] > EPSILON
    pr = np.zeros((len(feats), 2))
    for i, cam in enumerate(cameras):
        m = cam_of == i
        pr[m] = cam2img(cam.model_id.value, cam.params, pc[m])
    err = np.linalg.norm(pr - feats, axis=1)
    valid = valid & (err < max_reprojection_error)
    return valid, counts, quirk_counter(valid, counts), err


def complete_candidates(cameras, images, tracks, tracks_orig, max_reproj_error):
    """complete_tracks' candidate test (track_retriangulation.py:43-92): for every observation of every track of
    ``tracks_orig`` whose id is in ``tracks``, reproject the current track point through ``reproject_funcs`` with the
    image's pose (scipy quaternion of world2cam) and camera; keep z > 1e-7 and ||err|| <= threshold.
    Returns (obs_info [n,2], track row [n], passing mask [n], errors [n])."""
    from scipy.spatial.transform import Rotation
    from . import projection_ref as PR
    model = cameras[0].model_id.value
    if model in (7, 10):
        raise NotImplementedError
    id2idx = {k: i for i, k in enumerate(tracks.keys())}
    obs, rows = [], []
    for k, o in tracks_orig.items():
        if k in id2idx:
            o = np.asarray(o).reshape(-1, 2)
            obs.append(o)
            rows.append(np.full(o.shape[0], id2idx[k]))
    obs = np.concatenate(obs).astype(np.int64)
    rows = np.concatenate(rows)
    uv = np.array([images[i].features[f] for i, f in obs.tolist()], dtype=np.float64)
    pp_idx = {0: [1, 2], 1: [2, 3], 2: [1, 2], 3: [1, 2], 8: [1, 2], 9: [1, 2]}.get(model, [2, 3])
    cams = []
    for im in images:
        prm = np.asarray(cameras[im.cam_id].params, dtype=np.float64)
        cams.append(np.concatenate([im.world2cam[:3, 3], Rotation.from_matrix(im.world2cam[:3, :3]).as_quat(), prm]))
    cams = np.array(cams)
    keep = [j for j in range(cams.shape[1]) if j - 7 not in pp_idx]
    rowcam = cams[obs[:, 0]]
    X = np.array([np.asarray(t.xyz, dtype=np.float64) for t in tracks.values()])[rows]
    z = PR.rotate_quat(X, rowcam[:, :7])[:, 2]
    err = np.linalg.norm(PR.reproject(model, X, rowcam[:, keep], rowcam[:, [7 + j for j in pp_idx]]) - uv, axis=-1)
    return obs, rows, (err <= max_reproj_error) & (z > 1e-7), err
