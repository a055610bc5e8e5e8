"""Rebuild the retriangulation golden scenes (tools/gen_golden.py gen_retri) as scene objects."""
import os

import numpy as np

from instantsfm_amd.scene.defs import Camera, CameraModelId, Image, Track

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ("retri_simple_radial", "retri_opencv", "retri_radial_fisheye")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def scene(g):
    cameras = [Camera(id=i, model_id=CameraModelId(int(m)), params=np.asarray(p, dtype=np.float64))
               for i, (m, p) in enumerate(zip(g["cam_model"], g["cam_params"]))]
    fp = g["feat_ptr"]
    images = [Image(id=i, cam_id=int(c), is_registered=True, world2cam=g["w2c"][i].copy(),
                    features=g["feats"][fp[i]:fp[i + 1]].copy()) for i, c in enumerate(g["img_cam"])]
    tp = g["track_ptr"]
    tracks = {int(k): Track(id=int(k), xyz=g["track_xyz"][j].copy(), observations=g["track_obs"][tp[j]:tp[j + 1]].copy())
              for j, k in enumerate(g["track_keys"])}
    op = g["orig_ptr"]
    tracks_orig = {int(k): g["orig_obs"][op[j]:op[j + 1]].copy() for j, k in enumerate(g["orig_keys"])}
    return cameras, images, tracks, tracks_orig


def flat(tracks):
    keys = np.array(list(tracks.keys()))
    ptr = np.concatenate([[0], np.cumsum([len(t.observations) for t in tracks.values()])])
    obs = np.concatenate([np.asarray(t.observations).reshape(-1, 2) for t in tracks.values()]).astype(np.int64)
    return keys, ptr, obs


def apply_completion(tracks, obs, rows, passing):
    """complete_tracks' update (track_retriangulation.py:91-106) from a passing mask over the candidates."""
    keys = list(tracks.keys())
    obs = obs[passing].astype(np.int32)
    rows = rows[passing]
    bounds = np.concatenate([[0], np.flatnonzero(np.diff(rows)) + 1, [rows.shape[0]]])
    n = 0
    for i in range(len(bounds) - 1):
        a, b = bounds[i], bounds[i + 1]
        t = tracks[keys[rows[a]]]
        n += abs((b - a) - t.observations.shape[0])
        t.observations = obs[a:b]
    return n
