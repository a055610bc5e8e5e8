"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path (instantsfm_amd/).

numpy float64 restatement of the reference's per-observation reprojection functions,
``instantsfm/utils/cost_function.py:32-208``, plus the SE3 point action ``rotate_quat`` that
the reference imports from the un-vendored ``bae.utils.ba`` (pypose layout ``[t(3), q_xyzw(4)]``,
p_c = R(q) p + t).  Camera rows are the reference's BA rows: ``[t, q, intrinsics-without-pp]``
(bundle_adjustment.py:70-80).

Pinned by ``tests/golden/projection_golden.npz`` (generated from the reference itself by
``tools/gen_golden.py``).
"""
import numpy as np

# Number of optimized intrinsics per model id after the principal point is removed.
N_INTR = {0: 1, 1: 2, 2: 2, 3: 3, 4: 6, 5: 6, 6: 10, 8: 2, 9: 3}


def rotate_quat(points, pose):
    """bae.utils.ba.rotate_quat (un-vendored; call sites cost_function.py:34, bundle_adjustment.py:102).

    v' = v + 2 w (q_v x v) + 2 q_v x (q_v x v) + t  with q = (x, y, z, w).
    """
    t = pose[..., 0:3]
    qv = pose[..., 3:6]
    w = pose[..., 6:7]
    uv = np.cross(qv, points)
    uuv = np.cross(qv, uv)
    return points + 2.0 * (w * uv + uuv) + t


def _normalize(points, cam):
    pc = rotate_quat(points, cam[..., :7])
    return pc[..., :2] / pc[..., 2:3]


def reproject(model, points, cam, pp):
    """Dispatch like ``reproject_funcs[model]`` (cost_function.py:206-208)."""
    uv = _normalize(points, cam)
    if model == 0:  # SIMPLE_PINHOLE :32-38
        f = cam[..., -1:]
        return uv * f + pp
    if model == 1:  # PINHOLE :40-46
        return uv * cam[..., -2:] + pp
    if model == 2:  # SIMPLE_RADIAL :48-56
        f, k = cam[..., -2:-1], cam[..., -1:]
        r2 = np.sum(uv ** 2, axis=-1, keepdims=True)
        return uv * (1 + k * r2) * f + pp
    if model == 3:  # RADIAL :58-67
        f, k1, k2 = cam[..., -3:-2], cam[..., -2:-1], cam[..., -1:]
        r2 = np.sum(uv ** 2, axis=-1, keepdims=True)
        return uv * (1 + k1 * r2 + k2 * r2 ** 2) * f + pp
    if model in (4, 6):  # OPENCV :69-85, FULL_OPENCV :104-123
        if model == 4:
            ff, k1, k2, p = cam[..., -6:-4], cam[..., -4:-3], cam[..., -3:-2], cam[..., -2:]
        else:
            ff, k1, k2, p = cam[..., -10:-8], cam[..., -8:-7], cam[..., -7:-6], cam[..., -6:-4]
            k3, k4, k5, k6 = cam[..., -4:-3], cam[..., -3:-2], cam[..., -2:-1], cam[..., -1:]
        r2 = np.sum(uv ** 2, axis=-1, keepdims=True)
        uvp = uv[..., 0:1] * uv[..., 1:2]
        if model == 4:
            radial = k1 * r2 + k2 * r2 ** 2
        else:
            radial = (1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3) / (1 + k4 * r2 + k5 * r2 ** 2 + k6 * r2 ** 3) - 1
        d = uv * radial + 2 * p * uvp
        d = d + p[..., ::-1] * (r2 + 2 * uv ** 2)
        return (uv + d) * ff + pp
    if model in (5, 8, 9):  # OPENCV_FISHEYE :87-102, SIMPLE_RADIAL_FISHEYE :130-140, RADIAL_FISHEYE :142-153
        r2 = np.sum(uv ** 2, axis=-1, keepdims=True)
        r = np.sqrt(r2)
        uvt = uv * np.arctan(r) / r
        if model == 5:
            ff, k1, k2, k3 = cam[..., -6:-4], cam[..., -4:-3], cam[..., -3:-2], cam[..., -2:-1]
            return uvt * (1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3) * ff + pp
        if model == 8:
            f, k = cam[..., -2:-1], cam[..., -1:]
            return uvt * (1 + k * r2) * f + pp
        f, k1, k2 = cam[..., -3:-2], cam[..., -2:-1], cam[..., -1:]
        return uvt * (1 + k1 * r2 + k2 * r2 ** 2) * f + pp
    raise NotImplementedError  # FOV (7) and THIN_PRISM_FISHEYE (10) raise in the reference too


def huber(s, delta):
    """pypose.optim.kernel.Huber on squared norms s (un-vendored; bundle_adjustment.py:118)."""
    rs = np.sqrt(s)
    return np.where(rs < delta, s, 2.0 * delta * rs - delta * delta)
