"""UndistortImages -- drop-in for ``instantsfm/processors/image_undistortion.py`` (reference :1-10).

Every image's ``features`` go through its camera's ``img2cam`` (scene/defs.py:315-369) and are normalized to unit
rays in ``image.features_undist`` -- on the GPU (``insfm_undistort``, csrc/passes.hip), all images in one launch per
feature dtype.  Features stored as float32 (the database's type) are undistorted like cv2 does for float32 input
(double arithmetic, float32 result).
"""
import numpy as np

from .. import passes
from ..scene.defs import CameraModelId


def _camera_table(cameras, images):
    """Rows for the cameras the images use: model id and the reference's params vector."""
    cam_ids = sorted({int(im.cam_id) for im in images})
    row = {c: i for i, c in enumerate(cam_ids)}
    models, params = [], []
    for c in cam_ids:
        cam = cameras[c]
        mid = cam.model_id.value if isinstance(cam.model_id, CameraModelId) else int(cam.model_id)
        if mid < 0 or mid > 10:
            raise NotImplementedError  # Camera.img2cam raises for unknown models
        models.append(mid)
        params.append(np.asarray(cam.params, dtype=np.float64).reshape(-1))
    return row, np.array(models, np.int32), params


def UndistortImages(cameras, images, device="cuda:0"):
    """image_undistortion.py:8-10: ``image.features_undist`` = normalized [img2cam(features), 1] for every image."""
    if not len(images):
        return
    row, models, params = _camera_table(cameras, images)
    feats = [np.asarray(im.features) for im in images]
    feats = [f.reshape(-1, 2) if f.size else np.zeros((0, 2)) for f in feats]
    groups = {}
    for i, f in enumerate(feats):
        groups.setdefault(f.dtype == np.float32, []).append(i)
    for f32, idx in groups.items():
        xy = np.concatenate([feats[i] for i in idx]).astype(np.float32 if f32 else np.float64, copy=False)
        counts = [feats[i].shape[0] for i in idx]
        fc = np.repeat(np.array([row[int(images[i].cam_id)] for i in idx], np.int32), counts)
        rays = passes.undistort(xy, fc, models, params, device)
        off = np.concatenate([[0], np.cumsum(counts)])
        for j, i in enumerate(idx):
            images[i].features_undist = rays[off[j]:off[j + 1]]
