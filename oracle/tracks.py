"""CPU restatement of track establishment -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench.py's cpu_baseline leg use this module, as the checker; the product path
(instantsfm_amd/processors/track_establishment.py) runs csrc/tracks.hip.

Restates processors/track_establishment.py:7-86 and utils/union_find.py:2-23 loop for loop (a dict-based union-find
with path compression, Union(larger, smaller) in view-graph order, per-track first-appearance dicts with reference
counts, the inconsistency test, the np.unique deduplication).  The only deliberate difference: global ids are built
with Python ints, which is what the reference's pinned numpy 1.26 computes for ``(image_id << 32) | np.uint32``
(under numpy 2 that expression overflows).  Pinned by tests/golden/tracks_*.npz, captured from the reference itself.
"""
from collections import defaultdict

import numpy as np


class UnionFind:
    """utils/union_find.py:2-23 (iterative Find with full path compression, same roots)."""

    def __init__(self):
        self.parent = {}

    def Find(self, x):
        parent = self.parent
        if x not in parent:
            parent[x] = x
            return x
        root = x
        while parent[root] != root:
            root = parent[root]
        while parent[x] != root:
            parent[x], x = root, parent[x]
        return root

    def Union(self, x, y):
        rx, ry = self.Find(x), self.Find(y)
        if rx != ry:
            self.parent[rx] = ry


def _edges(view_graph):
    for pair in view_graph.image_pairs.values():
        if not pair.is_valid:
            continue
        m = np.asarray(pair.matches)
        for idx in np.asarray(pair.inliers, dtype=np.int64).reshape(-1).tolist():
            p1, p2 = int(m[idx, 0]), int(m[idx, 1])
            yield pair.image_id1, p1, pair.image_id2, p2


def establish_full_tracks(view_graph, images, thres_inconsistency):
    """TrackEngine.EstablishFullTracks: returns ({track_id: int64 [k, 2]}, discarded counter)."""
    uf = UnionFind()
    for i1, p1, i2, p2 in _edges(view_graph):
        g1, g2 = (i1 << 32) | p1, (i2 << 32) | p2
        if g2 < g1:
            uf.Union(g1, g2)
        else:
            uf.Union(g2, g1)
    track_map = {}
    for i1, p1, i2, p2 in _edges(view_graph):
        tid = uf.Find((i1 << 32) | p1)
        if tid not in track_map:
            track_map[tid] = defaultdict(int)
        track_map[tid][(i1, p1)] += 1
        track_map[tid][(i2, p2)] += 1
    tracks = {tid: np.concatenate([np.array(list(c.keys()), dtype=np.int64),
                                   -np.array(list(c.values()), dtype=np.int64)[:, None]], axis=-1)
              for tid, c in track_map.items()}
    discarded = 0
    for tid in list(tracks.keys()):
        seen = {}
        bad = False
        for image_id, feature_id, _ in tracks[tid]:
            f = images[image_id].features[feature_id]
            if image_id not in seen:
                seen[image_id] = f.reshape(1, 2)
            else:
                if np.any(np.linalg.norm(seen[image_id] - f, axis=1) > thres_inconsistency):
                    bad = True
                    break
                seen[image_id] = np.vstack([seen[image_id], f.reshape(1, 2)])
        if bad:
            del tracks[tid]
            discarded += 1
            continue
        corr = tracks[tid]
        prio, first = np.unique(corr[:, [0, 2]], axis=0, return_index=True)
        _, per_image = np.unique(prio[:, 0], return_index=True)
        discarded += len(corr) - len(per_image)
        tracks[tid] = corr[first[per_image], :2]
    return tracks, discarded


def find_tracks_for_problem(tracks_full, images, options):
    """TrackEngine.FindTracksForProblem (:88-106): {track_id: observations of registered images}."""
    registered = [i for i, im in enumerate(images) if im.is_registered]
    out = {}
    for tid, obs in tracks_full.items():
        if obs.shape[0] < options['min_num_view_per_track'] or obs.shape[0] > options['max_num_view_per_track']:
            continue
        out[tid] = obs[np.isin(obs[:, 0], registered)]
    return out
