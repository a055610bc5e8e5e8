/*
 * insfm_tracks.h -- C ABI of track establishment, same library as insfm_ba.h.
 *
 * Replaces the Python core of TrackEngine.EstablishFullTracks (processors/track_establishment.py:14-86):
 *   - BlindConcatenation (:23-37): union-find over every inlier match of every valid image pair, in view-graph
 *     order, with UnionFind.Union(larger global id, smaller global id) (utils/union_find.py:16-20) -- the root, and so
 *     the track id, depends on that order; it is reproduced exactly;
 *   - TrackCollection (:39-86): per track, the distinct (image, feature) observations in order of first appearance
 *     with their reference counts, the inconsistency check (two features of one image farther apart than
 *     thres_inconsistency discard the track) and the per-image deduplication (keep the most-referenced feature,
 *     the earliest on ties; rows sorted by image id).
 *
 * Features are numbered globally: node = first_feature[image] + feature_index, so node order is the reference's
 * global-id order ((image << 32) | feature).  Edges are the inlier matches flattened in the reference's iteration
 * order: edge k joins node edge_a[k] = (pair.image_id1, point1) and edge_b[k] = (pair.image_id2, point2).
 *
 * All array arguments are DEVICE pointers except `counts` (host).  The call enqueues the work on `stream`, then
 * waits for it (the output sizes are data-dependent).  Returns 0 or INSFM_BA_EINVAL / INSFM_BA_ENOMEM / INSFM_BA_EHIP.
 */
#ifndef INSFM_TRACKS_H
#define INSFM_TRACKS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Inputs: node_img [n_nodes] image of each node; node_xy [n_nodes, 2] feature coordinates (float32 when xy_f32 != 0,
 * the database's keypoint type, else float64 -- the distance test runs in that type like numpy); edge_a / edge_b
 * [n_edges] (n_nodes and 2 * n_edges below 2^31).
 * Outputs (capacity n_edges for the per-track arrays, 2 * n_edges for the per-row arrays), tracks in order of first
 * appearance, rows grouped by track and sorted by image id:
 *   track_root [T]  node whose global id is the track id;
 *   track_bad  [T]  1 = discarded by the inconsistency check;
 *   track_nodes[T]  distinct observations before deduplication;
 *   row_node   [R]  the observation kept for one (track, image);
 *   row_track  [R]  its track;
 *   counts[0] = T, counts[1] = R. */
int insfm_tracks_establish(int64_t n_nodes, const int32_t* node_img, const void* node_xy, int32_t xy_f32,
                           int64_t n_edges, const int32_t* edge_a, const int32_t* edge_b, double thres_inconsistency,
                           int32_t* track_root, uint8_t* track_bad, int32_t* track_nodes, int32_t* row_node,
                           int32_t* row_track, int64_t* counts, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* INSFM_TRACKS_H */
