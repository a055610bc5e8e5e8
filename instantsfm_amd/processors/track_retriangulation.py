"""RetriangulateTracks -- drop-in for ``instantsfm/processors/track_retriangulation.py`` (reference :1-259).

The last stage of the global mapper (global_mapper.py:154-156): complete the tracks from the full tracks of the
track engine, then up to ``ba_global_max_refinements`` rounds of points-only bundle adjustment (TorchBA with
``optimize_poses=False``: block-diagonal 3x3 systems on the same HIP engine), completion and filtering.

* ``complete_tracks`` (:18-108): the candidate reprojection (every observation of every full track whose id is still
  in ``tracks``, through ``reproject_funcs`` with the image's scipy quaternion) runs on the GPU
  (``insfm_reproj_candidates``, the BA kernels' projection); the per-track replacement of ``observations`` and the
  ``num_completed`` count are the reference's, vectorized.
* ``filter_points`` (:200-204): FilterTracksByReprojection + FilterTracksTriangulationAngle (processors/track_filter).
* ``merge_tracks`` (:110-198) calls faiss, which the reference never imports, and its caller has it commented out
  (:210-212); it is not part of the path and raises here.
"""
import numpy as np
from scipy.spatial.transform import Rotation as R

from .. import passes
from ..scene.defs import CameraModelId, get_camera_model_info
from .bundle_adjustment import TorchBA, _as_torch_like_params
from .track_filter import FilterTracksByReprojection, FilterTracksTriangulationAngle, _features

EPSILON = 1e-7


def _image_rows(cameras, images, pp_idx):
    """The reference's per-image rows (:65-79): [t, scipy as_quat(world2cam), camera params] with the principal point
    columns split off."""
    w2c = np.array([np.asarray(im.world2cam, dtype=np.float64) for im in images]).reshape(-1, 4, 4)
    quat = R.from_matrix(w2c[:, :3, :3]).as_quat().reshape(-1, 4) if len(images) else np.zeros((0, 4))
    prm = np.array([_as_torch_like_params(cameras[im.cam_id].params) for im in images], dtype=np.float64)
    rows = np.concatenate([w2c[:, :3, 3], quat, prm], axis=1)
    pcols = [7 + i for i in pp_idx]
    keep = [j for j in range(rows.shape[1]) if j not in pcols]
    return np.ascontiguousarray(rows[:, keep]), np.ascontiguousarray(rows[:, pcols])


def complete_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, device="cuda:0"):
    """track_retriangulation.py:18-108.  Returns the number of observations changed across all tracks."""
    reproj_threshold = TRIANGULATOR_OPTIONS['complete_max_reproj_error']
    camera_model = cameras[0].model_id  # the reference assumes one model for all cameras
    info = get_camera_model_info(camera_model)
    if camera_model in (CameraModelId.FOV, CameraModelId.THIN_PRISM_FISHEYE, CameraModelId.INVALID):
        raise NotImplementedError("Unsupported camera model")  # reproject_fov / _thin_prism raise (cost_function.py)

    keys = list(tracks.keys())
    track_id2idx = {track_id: idx for idx, track_id in enumerate(keys)}
    cand, cidx = [], []
    for track_id, track_obs in tracks_orig.items():
        idx = track_id2idx.get(track_id)
        if idx is None:
            continue
        cand.append(track_obs if isinstance(track_obs, np.ndarray) and track_obs.ndim == 2
                    else np.asarray(track_obs).reshape(-1, 2))
        cidx.append(idx)
    ccount = np.fromiter((c.shape[0] for c in cand), dtype=np.int64, count=len(cand))
    if not cand or int(ccount.sum()) == 0:
        # the reference indexes obs_info_tensor[:, 0] of an empty 1-D tensor
        raise IndexError("too many indices for tensor of dimension 1")
    obs_info = np.concatenate(cand).astype(np.int32).reshape(-1, 2)  # torch.tensor(..., dtype=torch.int32) (:61)
    point_rows = np.repeat(np.asarray(cidx, dtype=np.int32), ccount)

    feats, foff = _features(images)
    image_rows, image_pps = _image_rows(cameras, images, info['pp'])
    xyz = np.array([np.asarray(t.xyz, dtype=np.float64) for t in tracks.values()]).reshape(-1, 3)
    passing = passes.reproj_candidates(camera_model.value, obs_info[:, 0], point_rows,
                                       foff[obs_info[:, 0]] + obs_info[:, 1], feats, image_rows, image_pps, xyz,
                                       reproj_threshold, device)

    obs_info = obs_info[passing]
    point_rows = point_rows[passing]
    if point_rows.shape[0] == 0:
        # the reference reads point_indices_tensor[0] of an empty tensor (:102)
        raise IndexError("index 0 is out of bounds for dimension 0 with size 0")
    split = np.flatnonzero(np.diff(point_rows)) + 1
    bounds = np.concatenate([[0], split, [point_rows.shape[0]]]).tolist()
    firsts = point_rows[np.asarray(bounds[:-1], dtype=np.int64)].tolist()
    vals = list(tracks.values())
    num_completed = 0
    for a, b, r in zip(bounds[:-1], bounds[1:], firsts):
        track = vals[r]
        num_completed += abs((b - a) - track.observations.shape[0])
        track.observations = obs_info[a:b]
    return num_completed


def merge_tracks(cameras, images, tracks, TRIANGULATOR_OPTIONS):
    """track_retriangulation.py:110-198 -- not on the path, and not callable in the reference either: its k-NN search
    is `faiss.IndexFlatL2` (:136), but the module never imports faiss (:1-14), so a call raises NameError there before
    any track is touched; its only caller has the call commented out (:210-212, "current version of merge does not
    have a good result and is not used in the pipeline").  This raises at the same point, with the reason."""
    raise NotImplementedError("merge_tracks: the reference's version cannot run (faiss is used at "
                              "track_retriangulation.py:136 but never imported) and its only call is commented out "
                              "(:210-212)")


def filter_points(cameras, images, tracks, TRIANGULATOR_OPTIONS, device="cuda:0"):
    """track_retriangulation.py:200-204."""
    num_filtered = 0
    num_filtered += FilterTracksByReprojection(cameras, images, tracks, TRIANGULATOR_OPTIONS['filter_max_reproj_error'],
                                               device=device)
    num_filtered += FilterTracksTriangulationAngle(cameras, images, tracks, TRIANGULATOR_OPTIONS['filter_min_tri_angle'],
                                                   device=device)
    return num_filtered


def complete_and_merge_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, device="cuda:0"):
    """track_retriangulation.py:206-213 (merging is disabled in the reference)."""
    num_completed_observations = complete_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, device)
    print('Number of completed observations:', num_completed_observations)
    num_merged_observations = 0
    return num_completed_observations + num_merged_observations


def RetriangulateTracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, BUNDLE_ADJUSTER_OPTIONS,
                        device="cuda:0"):
    """track_retriangulation.py:215-259: complete, then points-only BA / complete / filter rounds until the changed
    fraction drops below ``ba_global_max_refinement_change``."""
    image_registered = [image.is_registered for image in images]

    complete_and_merge_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, device)

    for i in range(TRIANGULATOR_OPTIONS['ba_global_max_refinements']):
        print(f'Running bundle adjustment iteration {i+1} / {TRIANGULATOR_OPTIONS["ba_global_max_refinements"]}')
        ba_engine = TorchBA(device=device)
        LOCAL_BUNDLE_ADJUSTER_OPTIONS = BUNDLE_ADJUSTER_OPTIONS.copy()
        LOCAL_BUNDLE_ADJUSTER_OPTIONS['optimize_poses'] = False
        ba_engine.Solve(cameras, images, tracks, LOCAL_BUNDLE_ADJUSTER_OPTIONS)
        num_changed_observations = 0
        num_changed_observations += abs(complete_and_merge_tracks(cameras, images, tracks, tracks_orig,
                                                                  TRIANGULATOR_OPTIONS, device))
        num_changed_observations += filter_points(cameras, images, tracks, TRIANGULATOR_OPTIONS, device)
        changed_percentage = num_changed_observations / len(tracks)
        if changed_percentage < TRIANGULATOR_OPTIONS['ba_global_max_refinement_change']:
            break

    for i, image in enumerate(images):
        image.is_registered = image_registered[i]
