"""Track filters -- drop-in for ``instantsfm/processors/track_filter.py`` (reference :1-137, all four filters): the per-observation
and per-track geometry on the GPU (csrc/passes.hip), the scene bookkeeping (gathering, per-track compaction, the
counters and messages the reference prints) on the host, vectorized.

Same signatures, same in-place effects on ``tracks`` and the same return values, including
FilterTracksByReprojectionNormalized's counter, which the reference computes on the slice of the *next* track
(track_filter.py:59-63: ``count`` is advanced before the test).
"""
import numpy as np

from .. import passes
from .bundle_adjustment import packx

EPSILON = 1e-10


def collect_tracks(tracks, with_obs=True):
    """(per-track counts int64, observations [X,2] int64 in dict order, xyz [T,3] float64) read in one C loop by the
    native pack extension (csrc/packx.c ``collect``), or None when it is missing or a Track's attributes are not the
    plain (n, 2) integer / (3,) float arrays it takes.  ``with_obs=False`` skips copying the observations."""
    if packx() is None or not tracks:
        return None
    got = packx().collect(list(tracks.values()), 0 if with_obs else (1 << 62))
    if got is None:
        return None
    return (np.frombuffer(got[0], np.int64), np.frombuffer(got[1], np.int64).reshape(-1, 2),
            np.frombuffer(got[2], np.float64).reshape(-1, 3))


def _gather_obs(tracks):
    """All observations of all tracks in dict order: (the per-track arrays or None, [X,2] int64, per-track counts,
    track row of each observation, -, the tracks' xyz or None).  Natively when collect_tracks takes the tracks, else
    one concatenation over the tracks' own arrays; tracks whose observations are not (n, 2) arrays (lists, empty 1-D
    arrays) go through the per-track reshape."""
    if not tracks:
        raise ValueError("need at least one array to concatenate")  # what the reference's np.concatenate raises
    got = collect_tracks(tracks)
    if got is not None:
        counts, allobs, xyz = got
        trow = np.repeat(np.arange(counts.size, dtype=np.int64), counts)
        return None, allobs, counts, trow, None, xyz
    raw = [t.observations for t in tracks.values()]
    try:
        if not all(isinstance(o, np.ndarray) and o.ndim == 2 for o in raw):
            raise ValueError
        counts = np.fromiter((o.shape[0] for o in raw), dtype=np.int64, count=len(raw))
        allobs = np.concatenate(raw).astype(np.int64, copy=False).reshape(-1, 2)
        obs = raw
    except ValueError:
        obs = [np.asarray(o).reshape(-1, 2).astype(np.int64, copy=False) for o in raw]
        counts = np.array([o.shape[0] for o in obs], dtype=np.int64)
        allobs = np.concatenate(obs)
    trow = np.repeat(np.arange(len(obs), dtype=np.int64), counts)
    return obs, allobs, counts, trow, None, None


def _apply_mask(tracks, valid, counts):
    """track.observations = track.observations[mask] for every track (track_filter.py:62-63 / :107-110); a track whose
    observations all pass keeps its array (the same values the reference's copy holds)."""
    starts = np.concatenate([[0], np.cumsum(counts)])
    bad = np.concatenate([[0], np.cumsum(~valid)])
    touched = np.flatnonzero(bad[starts[1:]] - bad[starts[:-1]] > 0)
    if touched.size == 0:
        return
    vals = list(tracks.values())
    for j in touched.tolist():
        track = vals[j]
        track.observations = track.observations[valid[starts[j]:starts[j + 1]]]


def _gather(images, tracks):
    """Observations of all tracks in dict order -> (obs [X,2], per-track counts, track rows, global feature row of each
    observation into the concatenated features_undist, the rays themselves, the tracks' xyz or None)."""
    obs, allobs, counts, trow, _, xyz = _gather_obs(tracks)
    fu = [np.asarray(im.features_undist, dtype=np.float64).reshape(-1, 3) if len(im.features_undist) else np.zeros((0, 3))
          for im in images]
    foff = np.concatenate([[0], np.cumsum([f.shape[0] for f in fu])]).astype(np.int64)
    rays = np.concatenate(fu) if fu else np.zeros((0, 3))
    ray_row = foff[allobs[:, 0]] + allobs[:, 1]
    return obs, allobs, counts, trow, ray_row, rays, xyz


def _world2cams(images):
    return np.array([np.asarray(im.world2cam, dtype=np.float64) for im in images]).reshape(-1, 16)


def _xyz(tracks, xyz=None):
    if xyz is not None:  # (already read by collect_tracks: the same float64 values)
        return xyz
    return np.array([t.xyz for t in tracks.values()], dtype=np.float64).reshape(-1, 3)


def quirk_counter(valid, counts):
    """track_filter.py:57-63: after ``count += len_j`` the test reads valid[count : count + len_j]."""
    starts = np.concatenate([[0], np.cumsum(counts)])
    inv = np.concatenate([[0], np.cumsum(~valid)])
    n = valid.shape[0]
    a = np.minimum(starts[1:], n)
    b = np.minimum(starts[1:] + counts, n)
    return int(np.sum(inv[b] - inv[a] > 0))


def FilterTracksByReprojectionNormalized(cameras, images, tracks, max_reprojection_error, device="cuda:0"):
    """track_filter.py:26-66."""
    obs, allobs, counts, trow, ray_row, rays, xyz = _gather(images, tracks)
    valid = passes.filter_reproj_normalized(allobs[:, 0], trow, ray_row, _world2cams(images), _xyz(tracks, xyz), rays,
                                            max_reprojection_error, device)
    _apply_mask(tracks, valid, counts)
    counter = quirk_counter(valid, counts)
    print(f'Filtered {counter} / {len(tracks)} tracks by reprojection error')
    return counter


def _features(images):
    """Concatenated raw features of all images [F,2] and each image's first row.  float32 when every image's
    features are float32 (the database's keypoint type), else float64 (the reference's ``np.array(features)`` then
    promotes against the float64 projection either way, so the values are exact)."""
    fs = [np.asarray(im.features).reshape(-1, 2) for im in images]
    f32 = all(f.dtype == np.float32 for f in fs if f.size)
    fs = [f.astype(np.float32 if f32 else np.float64, copy=False) for f in fs]
    off = np.concatenate([[0], np.cumsum([f.shape[0] for f in fs])]).astype(np.int64)
    return (np.concatenate(fs) if fs else np.zeros((0, 2))), off


def FilterTracksByReprojection(cameras, images, tracks, max_reprojection_error, device="cuda:0"):
    """track_filter.py:68-113: pixel reprojection error through each image's Camera.cam2img."""
    obs, allobs, counts, trow, _, xyz = _gather_obs(tracks)
    feats, foff = _features(images)
    img_cam = np.array([im.cam_id for im in images], dtype=np.int32)
    valid = passes.filter_reproj_pixel(allobs[:, 0], trow, foff[allobs[:, 0]] + allobs[:, 1], feats, img_cam,
                                       [cam.model_id.value for cam in cameras], [cam.params for cam in cameras],
                                       _world2cams(images), _xyz(tracks, xyz), max_reprojection_error, device)
    _apply_mask(tracks, valid, counts)
    counter = quirk_counter(valid, counts)
    print(f'Filtered {counter} / {len(tracks)} tracks by reprojection error')
    return counter


def FilterTracksByAngle(cameras, images, tracks, max_angle_error, device="cuda:0"):
    """track_filter.py:5-24."""
    thres = np.cos(np.deg2rad(max_angle_error))
    obs, allobs, counts, trow, ray_row, rays, xyz = _gather(images, tracks)
    valid = passes.filter_angle(allobs[:, 0], trow, ray_row, _world2cams(images), _xyz(tracks, xyz), rays, thres,
                                device)
    starts = np.concatenate([[0], np.cumsum(counts)])
    bad = np.concatenate([[0], np.cumsum(~valid)])
    touched = np.flatnonzero(bad[starts[1:]] - bad[starts[:-1]] > 0)  # the tracks with a failing observation
    counter = int(touched.size)
    vals = list(tracks.values()) if counter else []
    for j in touched.tolist():
        track = vals[j]
        track.observations = track.observations[np.flatnonzero(valid[starts[j]:starts[j + 1]])]
    print(f'Filtered {counter} / {len(tracks)} tracks by angle error')
    return tracks


def FilterTracksTriangulationAngle(cameras, images, tracks, min_angle, device="cuda:0"):
    """track_filter.py:116-137: drop tracks whose viewing directions are all within ``min_angle`` of each other."""
    thres = np.cos(np.deg2rad(min_angle))
    centers = np.array([np.asarray(im.center(), dtype=np.float64) for im in images]).reshape(-1, 3)
    keys = list(tracks.keys())
    got = collect_tracks(tracks)
    if got is not None:
        counts, allobs, xyz = got
        img = allobs[:, 0].astype(np.int32)
    else:
        obs = [np.asarray(tracks[k].observations).reshape(-1, 2) for k in keys]
        counts = np.array([o.shape[0] for o in obs], dtype=np.int64)
        img = np.concatenate([o[:, 0] for o in obs]).astype(np.int32) if obs else np.zeros(0, np.int32)
        xyz = None
    ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    remove = passes.filter_tri_angle(ptr, img, centers, _xyz(tracks, xyz), thres, device) if keys else np.zeros(0, bool)
    counter = 0
    for k, r in zip(keys, remove.tolist()):
        if r:
            del tracks[k]
            counter += 1
    print(f'Filtered {counter} / {counter + len(tracks)} tracks by too small triangulation angle')
    return counter
