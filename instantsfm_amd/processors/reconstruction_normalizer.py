"""NormalizeReconstruction -- drop-in for ``instantsfm/processors/reconstruction_normalizer.py`` (reference :1-47).

Host-side scene bookkeeping (C camera centres, a percentile box, one similarity applied to every pose and track),
vectorized numpy with the reference's arithmetic; the per-observation depth ratios of the depth branch are gathered
as arrays instead of a Python double loop.
"""
import numpy as np


def NormalizeReconstruction(images, tracks, depths=None, fixed_scale=False, extent=10., p0=0.1, p1=0.9):
    coords = np.array([image.center() for image in images])
    coords_sorted = np.sort(coords, axis=0)
    P0 = int(p0 * (coords.shape[0] - 1)) if coords.shape[0] > 3 else 0
    P1 = int(p1 * (coords.shape[0] - 1)) if coords.shape[0] > 3 else coords.shape[0] - 1
    bbox_min = coords_sorted[P0]
    bbox_max = coords_sorted[P1]
    mean_coord = np.mean(coords_sorted[P0:P1 + 1], axis=0)

    if depths is not None:
        # depth-based normalization (:14-30): log(depth_gt) - log(||xyz - C||) over observations with depth_gt > 0
        obs = [np.asarray(t.observations).reshape(-1, 2).astype(np.int64) for t in tracks.values()]
        xyz = [np.asarray(t.xyz, dtype=np.float64) for t in tracks.values()]
        counts = np.array([o.shape[0] for o in obs], dtype=np.int64)
        allobs = np.concatenate(obs) if obs else np.zeros((0, 2), np.int64)
        # depths keep the depth map's dtype: np.log(np.array(depth_gt_list)) is a float32 log for float32 maps
        dep_img = [np.asarray(im.depths).reshape(-1) for im in images]
        dep_off = np.concatenate([[0], np.cumsum([d.shape[0] for d in dep_img])]).astype(np.int64)
        dep_all = np.concatenate(dep_img) if dep_img else np.zeros(0)
        dep = dep_all[dep_off[allobs[:, 0]] + allobs[:, 1]] if allobs.shape[0] else dep_all[:0]
        m = dep > 0
        if m.any():
            P = np.repeat(np.array(xyz).reshape(-1, 3), counts, axis=0)[m]
            C = coords[allobs[m, 0]]
            pred = np.linalg.norm(P - C, axis=1)
            log_scales = np.log(dep[m]) - np.log(pred)
            scale = np.exp(np.median(log_scales))
        else:
            scale = 1.0
    else:
        scale = 1.
        if not fixed_scale:
            old_extent = np.linalg.norm(bbox_max - bbox_min)
            if old_extent >= 1e-6:
                scale = extent / old_extent

    coords = (coords - mean_coord) * scale
    for idx, image in enumerate(images):
        image.world2cam[:3, 3] = -image.world2cam[:3, :3] @ coords[idx]
    for track in tracks.values():
        track.xyz = (track.xyz - mean_coord) * scale
