"""TrackEngine -- drop-in for ``instantsfm/processors/track_establishment.py`` (reference :1-106).

``EstablishFullTracks`` (:14-21) = ``BlindConcatenation`` (:23-37) + ``TrackCollection`` (:39-86).  The reference
walks every inlier match twice in Python (a dict-based union-find, then per-track dicts, a per-track consistency loop
and a per-track ``np.unique``); here the matches are flattened once on the host and the whole computation runs in
csrc/tracks.hip (``insfm_tracks_establish``): lock-free union-find, then an exact replay of the reference's
order-dependent ``UnionFind.Union`` per component (the root -- the track id -- depends on the union order), first
appearance order, reference counts, the inconsistency test and the per-image deduplication.  The host turns the
per-track rows back into the reference's ``{track_id: int64 [k, 2] (image_id, feature_id)}`` dict, in the same order.

Global feature ids follow the reference, ``(image_id << 32) | feature_id`` (the reference pins numpy 1.26, where
``int | np.uint32`` promotes to int64).  ``FindTracksForProblem`` (:88-106) is the reference's filter, vectorized.
"""
import ctypes
import time

import numpy as np
import torch

from .. import _capi
from ..engine import _require_gpu
from ..scene.defs import Track, ViewGraph


def flatten_matches(view_graph: ViewGraph, images):
    """The inlier matches of every valid pair in the reference's iteration order (track_establishment.py:24-29) as
    global feature numbers, plus the per-image feature offsets and the concatenated feature coordinates."""
    nfeat = np.array([len(im.features) for im in images], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(nfeat)]).astype(np.int64)
    a_parts, b_parts = [], []
    for pair in view_graph.image_pairs.values():
        if not pair.is_valid:
            continue
        inl = np.asarray(pair.inliers, dtype=np.int64).reshape(-1)
        if inl.size == 0:
            continue
        m = np.asarray(pair.matches)[inl].astype(np.int64, copy=False)
        i1, i2 = int(pair.image_id1), int(pair.image_id2)
        if m.size and (m[:, 0].max() >= nfeat[i1] or m[:, 1].max() >= nfeat[i2] or m.min() < 0):
            # the reference indexes images[image_id].features[feature_id] (:64)
            raise IndexError(f"match of pair ({i1}, {i2}) refers to a feature outside its image")
        a_parts.append(off[i1] + m[:, 0])
        b_parts.append(off[i2] + m[:, 1])
    ea = np.concatenate(a_parts) if a_parts else np.zeros(0, np.int64)
    eb = np.concatenate(b_parts) if b_parts else np.zeros(0, np.int64)
    feats = [np.asarray(im.features).reshape(-1, 2) for im in images]
    f32 = all(f.dtype == np.float32 for f in feats if f.size)
    xy = np.concatenate([f.astype(np.float32 if f32 else np.float64, copy=False) for f in feats]) if feats else np.zeros((0, 2))
    return ea, eb, off, xy


def establish(ea, eb, off, xy, thres_inconsistency, device="cuda:0"):
    """Run insfm_tracks_establish.  Returns (track ids int64 [T], bad flags [T], distinct observations per track [T],
    row image [R], row feature [R], row track [R]) with tracks in first-appearance order."""
    dev = _require_gpu(device)
    L = _capi.load()
    ne = int(ea.shape[0])
    nn = int(off[-1])
    if ne == 0:
        z = np.zeros(0, np.int64)
        return z, z.astype(bool), z, z, z, z
    if nn >= 2 ** 31 - 1 or 2 * ne >= 2 ** 31 - 1:
        raise ValueError("too many features / matches for 32-bit node numbering")
    node_img = np.repeat(np.arange(len(off) - 1, dtype=np.int32), np.diff(off))
    f32 = xy.dtype == np.float32

    def d(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)

    t_img, t_xy = d(node_img, np.int32), d(xy, np.float32 if f32 else np.float64)
    t_a, t_b = d(ea, np.int32), d(eb, np.int32)
    root = torch.empty(ne, dtype=torch.int32, device=dev)
    bad = torch.empty(ne, dtype=torch.uint8, device=dev)
    nodes = torch.empty(ne, dtype=torch.int32, device=dev)
    rnode = torch.empty(2 * ne, dtype=torch.int32, device=dev)
    rtrack = torch.empty(2 * ne, dtype=torch.int32, device=dev)
    counts = (ctypes.c_int64 * 2)()
    with torch.cuda.device(dev):
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = L.insfm_tracks_establish(nn, p(t_img), p(t_xy), int(f32), ne, p(t_a), p(t_b), float(thres_inconsistency),
                                  p(root), p(bad), p(nodes), p(rnode), p(rtrack), counts, stream)
    if rc != 0:
        raise _capi.BAError(rc, "insfm_tracks_establish")
    T, R = int(counts[0]), int(counts[1])
    root = root[:T].cpu().numpy().astype(np.int64)
    rnode = rnode[:R].cpu().numpy().astype(np.int64)
    rimg = node_img[root].astype(np.int64)
    track_ids = (rimg << 32) | (root - off[rimg])
    row_img = node_img[rnode].astype(np.int64)
    return (track_ids, bad[:T].cpu().numpy().astype(bool), nodes[:T].cpu().numpy().astype(np.int64), row_img,
            rnode - off[row_img], rtrack[:R].cpu().numpy().astype(np.int64))


class TrackEngine:
    """track_establishment.py:7-106."""

    def __init__(self, view_graph: ViewGraph, images, device="cuda:0"):
        self.view_graph = view_graph
        self.images = images
        self.device = device

    def EstablishFullTracks(self, TRACK_ESTABLISHMENT_OPTIONS):
        start_time = time.time()
        ea, eb, off, xy = flatten_matches(self.view_graph, self.images)
        print(f"Blind concatenation took {time.time() - start_time} seconds")
        tracks = self._collect(ea, eb, off, xy, TRACK_ESTABLISHMENT_OPTIONS)
        print(f"Track collection took {time.time() - start_time} seconds")
        return tracks

    def _collect(self, ea, eb, off, xy, options):
        ids, bad, nodes, row_img, row_feat, row_track = establish(ea, eb, off, xy, options['thres_inconsistency'],
                                                                  self.device)
        keep_row = ~bad[row_track]
        rows = np.stack([row_img[keep_row], row_feat[keep_row]], axis=1)
        per_track = np.bincount(row_track, minlength=len(ids))
        discarded = int(bad.sum()) + int((nodes - per_track)[~bad].sum())
        kept = np.flatnonzero(~bad)
        bounds = np.cumsum(per_track[kept])[:-1]
        tracks = dict(zip(ids[kept].tolist(), np.split(rows, bounds) if kept.size else []))
        print(f"Discarded {discarded} features due to deduplication")
        return tracks

    def FindTracksForProblem(self, tracks_full, TRACK_ESTABLISHMENT_OPTIONS):
        """track_establishment.py:88-106: keep tracks with min..max views, observations of registered images only."""
        registered = np.array([bool(im.is_registered) for im in self.images] + [False])
        lo = TRACK_ESTABLISHMENT_OPTIONS['min_num_view_per_track']
        hi = TRACK_ESTABLISHMENT_OPTIONS['max_num_view_per_track']
        # every image registered and every image index in range: the mask keeps every row, a plain copy is the same
        all_reg = bool(registered[:-1].all())
        if all_reg and tracks_full:
            img = np.concatenate([o[:, 0] for o in tracks_full.values()])
            all_reg = img.size == 0 or (int(img.min()) >= 0 and int(img.max()) < len(self.images))
        tracks = {}
        for track_id, track_obs in tracks_full.items():
            if track_obs.shape[0] < lo or track_obs.shape[0] > hi:
                continue
            t = Track(id=track_id)
            t.observations = track_obs.copy() if all_reg else track_obs[registered[track_obs[:, 0]]]
            tracks[track_id] = t
        return tracks
