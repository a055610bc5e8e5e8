"""CPU restatement of the mapper's BA half (global_mapper.py:80-146) on oracle stages -- TEST INFRASTRUCTURE ONLY.

Only tests/ use this module, as the checker of ``instantsfm_amd.controllers.global_mapper.SolveGlobalMapper``.  Every
stage the product runs on the GPU runs here on its CPU restatement:

* track establishment (:85-89)       -> oracle/tracks.py (the reference's union-find restated loop for loop)
* UndistortImages (:98, :117, ...)   -> oracle/passes.py ``undistort_rays`` per image
* TorchGP.Optimize's LM (:100-104)   -> oracle/ba_oracle.c ``ora_gp_*`` (OracleGP), TorchGP's stop rule
* TorchBA.Solve's LM (:114-116, :138) -> oracle/ba_oracle.c (OracleBA), TorchBA's stop rule (:128-150)
* the track filters (:105, :118, :123-124, :144-145) -> oracle/passes.py
* RetriangulateTracks (:133)         -> oracle/passes.py ``complete_candidates`` / ``filter_reproj_pixel`` /
  ``filter_tri_angle`` + points-only OracleBA (track_retriangulation.py:215-259)

Host-side scene bookkeeping that has no device part is shared with the product, because it is pinned bit-exactly by
fixtures captured from the reference itself: ``pack`` / ``update`` of TorchBA (packing_*.npz), ``pack_gp``
(gp_packing_*.npz) and ``NormalizeReconstruction`` (passes_golden.npz).  ``trace`` records (stage, tracks,
observations, loss or RMSE) after every stage so a test can compare the two pipelines stage by stage.
"""
import numpy as np

from . import oracle as O
from . import passes as OP
from . import tracks as OT


def _n_obs(tracks):
    return int(sum(np.asarray(t.observations).reshape(-1, 2).shape[0] for t in tracks.values()))


def undistort_images(cameras, images):
    """image_undistortion.py:3-10."""
    for im in images:
        cam = cameras[im.cam_id]
        f = np.asarray(im.features).reshape(-1, 2)
        im.features_undist = OP.undistort_rays(cam.model_id.value, np.asarray(cam.params, np.float64), f) \
            if f.shape[0] else np.zeros((0, 3))


def _apply_mask(tracks, valid):
    counts = [np.asarray(t.observations).reshape(-1, 2).shape[0] for t in tracks.values()]
    starts = np.concatenate([[0], np.cumsum(counts)])
    for j, t in enumerate(tracks.values()):
        t.observations = t.observations[valid[starts[j]:starts[j + 1]]]


def filter_angle(images, tracks, max_angle_error):
    valid, counts, _ = OP.filter_angle(images, tracks, max_angle_error)
    starts = np.concatenate([[0], np.cumsum(counts)])
    for j, t in enumerate(tracks.values()):
        v = valid[starts[j]:starts[j + 1]]
        if not v.all():
            t.observations = t.observations[np.flatnonzero(v)]


def filter_reproj_normalized(images, tracks, thr):
    valid, _, _, _ = OP.filter_reproj_normalized(images, tracks, thr)
    _apply_mask(tracks, valid)


def filter_reproj_pixel(cameras, images, tracks, thr):
    valid, _, counter, _ = OP.filter_reproj_pixel(cameras, images, tracks, thr)
    _apply_mask(tracks, valid)
    return counter


def filter_tri_angle(images, tracks, min_angle):
    drop = OP.filter_tri_angle(images, tracks, min_angle)
    for k in drop:
        del tracks[k]
    return len(drop)


def gp_optimize(cameras, images, tracks, options):
    """TorchGP.Optimize (global_positioning.py:45-206) with the oracle LM."""
    from types import SimpleNamespace
    from instantsfm_amd.processors.global_positioning import pack_gp
    pk = pack_gp(cameras, images, tracks, None, options)
    prob = SimpleNamespace(trans=pk.translations, cam_idx=pk.camera_indices, pt_idx=pk.point_indices,
                           fcam=np.where(pk.is_calibrated, 1.0, 0.5), sfree=pk.scale_free,
                           n_cams=pk.camera_translations.shape[0], n_points=pk.points_3d.shape[0],
                           cams_init=pk.camera_translations.copy(), points_init=pk.points_3d.copy(),
                           scales_init=pk.scales.copy())
    cams, pts, _, hist = O.gp_solve_to_convergence(prob, max_iters=options['max_num_iterations'],
                                                   ftol=options['function_tolerance'],
                                                   huber_delta=options['thres_loss_function'])
    for t, xyz in zip(pk.track_list, pts):
        t.xyz = xyz
    for idx, image_id in enumerate(pk.image_idx2id.tolist()):
        images[image_id].world2cam[:3, 3] = cams[idx]
    for image in images:                                                        # ConvertResults (:41-43)
        image.world2cam[:3, 3] = -(image.world2cam[:3, :3] @ image.world2cam[:3, 3])
    return hist


def ba_solve(cameras, images, tracks, options):
    """TorchBA.Solve (bundle_adjustment.py:44-154) with the oracle LM.  Returns (loss history, final RMSE)."""
    from types import SimpleNamespace
    from instantsfm_amd.processors.bundle_adjustment import pack, update
    pk = pack(cameras, images, tracks, options)
    if pk.points_2d.shape[0] == 0:
        return [], None
    prob = SimpleNamespace(model=pk.model.value, uv=pk.points_2d, cam_idx=pk.camera_indices,
                           pt_idx=pk.point_indices, pp=pk.camera_pps, n_cams=pk.camera_params.shape[0],
                           n_points=pk.points_3d.shape[0], cams_init=np.ascontiguousarray(pk.camera_params),
                           points_init=np.ascontiguousarray(pk.points_3d))
    cams, pts, hist, rmse = O.solve_to_convergence(prob, max_iters=options['max_num_iterations'],
                                                   ftol=options['function_tolerance'],
                                                   huber_delta=options['thres_loss_function'],
                                                   optimize_poses=int(bool(options['optimize_poses'])),
                                                   precond=options.get('precond', 2))  # (TorchBA's default)
    update(cameras, images, tracks, pk, cams, pts)
    return hist, rmse


def complete_tracks(cameras, images, tracks, tracks_orig, options):
    """track_retriangulation.py:18-108."""
    obs, rows, passing, _ = OP.complete_candidates(cameras, images, tracks, tracks_orig,
                                                   options['complete_max_reproj_error'])
    obs, rows = obs[passing].astype(np.int32), rows[passing]
    keys = list(tracks.keys())
    bounds = np.concatenate([[0], np.flatnonzero(np.diff(rows)) + 1, [rows.shape[0]]])
    n = 0
    for i in range(len(bounds) - 1):
        a, b = int(bounds[i]), int(bounds[i + 1])
        t = tracks[keys[int(rows[a])]]
        n += abs((b - a) - t.observations.shape[0])
        t.observations = obs[a:b]
    return n


def retriangulate(cameras, images, tracks, tracks_orig, tri_opts, ba_opts):
    """track_retriangulation.py:215-259."""
    registered = [im.is_registered for im in images]
    complete_tracks(cameras, images, tracks, tracks_orig, tri_opts)
    for i in range(tri_opts['ba_global_max_refinements']):
        local = dict(ba_opts, optimize_poses=False)
        ba_solve(cameras, images, tracks, local)
        changed = abs(complete_tracks(cameras, images, tracks, tracks_orig, tri_opts))
        changed += filter_reproj_pixel(cameras, images, tracks, tri_opts['filter_max_reproj_error'])
        changed += filter_tri_angle(images, tracks, tri_opts['filter_min_tri_angle'])
        if changed / len(tracks) < tri_opts['ba_global_max_refinement_change']:
            break
    for im, r in zip(images, registered):
        im.is_registered = r


def solve_global_mapper(view_graph, cameras, images, config, trace=None):
    """global_mapper.py:80-146 on the oracle stages; the caller seeds numpy's global RNG like for the product run
    (InitializeRandomPositions draws from it)."""
    from instantsfm_amd.processors.reconstruction_normalizer import NormalizeReconstruction
    from instantsfm_amd.scene.defs import Track
    trace = trace if trace is not None else []
    te = config.TRACK_ESTABLISHMENT_OPTIONS
    full, _ = OT.establish_full_tracks(view_graph, images, te['thres_inconsistency'])
    obs = OT.find_tracks_for_problem(full, images, te)
    tracks = {tid: Track(id=tid, observations=o) for tid, o in obs.items()}
    trace.append(('tracks', len(tracks), _n_obs(tracks), None))

    thr = config.INLIER_THRESHOLD_OPTIONS
    undistort_images(cameras, images)
    scene_scale = 100                                                           # InitializeRandomPositions (:23-39)
    for image in images:
        image.world2cam[:3, 3] = scene_scale * np.random.uniform(-1, 1, 3)
    for track in tracks.values():
        track.xyz = scene_scale * np.random.uniform(-1, 1, 3)
        track.is_initialized = True
    hist = gp_optimize(cameras, images, tracks, config.GLOBAL_POSITIONER_OPTIONS)
    trace.append(('gp', len(tracks), _n_obs(tracks), hist[-1]))
    filter_angle(images, tracks, thr['max_angle_error'])
    NormalizeReconstruction(images, tracks, None)
    trace.append(('gp_filtered', len(tracks), _n_obs(tracks), None))

    for it in range(3):
        _, rmse = ba_solve(cameras, images, tracks, config.BUNDLE_ADJUSTER_OPTIONS)
        trace.append((f'ba{it}', len(tracks), _n_obs(tracks), rmse))
        undistort_images(cameras, images)
        filter_reproj_normalized(images, tracks, thr['max_reprojection_error'] * max(1, 3 - it))
    undistort_images(cameras, images)
    filter_reproj_normalized(images, tracks, thr['max_reprojection_error'])
    filter_tri_angle(images, tracks, thr['min_triangulation_angle'])
    NormalizeReconstruction(images, tracks, None)
    trace.append(('ba_filtered', len(tracks), _n_obs(tracks), None))

    if not config.OPTIONS['skip_retriangulation']:
        retriangulate(cameras, images, tracks, full, config.TRIANGULATOR_OPTIONS, config.BUNDLE_ADJUSTER_OPTIONS)
        _, rmse = ba_solve(cameras, images, tracks, config.BUNDLE_ADJUSTER_OPTIONS)
        trace.append(('ba_final', len(tracks), _n_obs(tracks), rmse))
        undistort_images(cameras, images)
        filter_reproj_normalized(images, tracks, thr['max_reprojection_error'])
        filter_tri_angle(images, tracks, thr['min_triangulation_angle'])
        trace.append(('retri_filtered', len(tracks), _n_obs(tracks), None))
    return cameras, images, tracks
