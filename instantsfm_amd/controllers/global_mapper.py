"""SolveGlobalMapper -- drop-in for ``instantsfm/controllers/global_mapper.py`` (reference :21-156), the half of it
this build replaces: track establishment (:80-91), global positioning (:93-107), the bundle-adjustment block (:109-126)
and retriangulation (:128-146), every stage on the MI355X processors of this package.

The stages before track establishment (preprocessing, view-graph calibration, relative pose estimation, rotation
averaging: :22-78) and pruning (:148-154) are outside the hot-path scope.  Their ``skip_*``
switches must be set; their outputs -- each valid pair's ``inliers`` and each image's ``is_registered`` flag and
world-to-camera rotation -- are the caller's (``synth.stand_in_rotation_averaging`` supplies them for synthetic
databases).  With a switch left off the mapper raises NotImplementedError instead of silently skipping the stage.

``timings`` (optional dict) receives the wall time of every stage and, per TorchGP / TorchBA call, its
pack / create / steps / write-back split (``TorchGP.timings`` / ``TorchBA.timings``); ``timings['trace']`` lists
(stage, tracks, observations, final LM loss or RMSE) after every stage -- what the tests' CPU restatement of the
pipeline records too, so the two can be compared stage by stage.
"""
import time

from ..processors.bundle_adjustment import TorchBA
from ..processors.global_positioning import TorchGP
from ..processors.image_undistortion import UndistortImages
from ..processors.reconstruction_normalizer import NormalizeReconstruction
from ..processors.track_establishment import TrackEngine
from ..processors.track_filter import (FilterTracksByAngle, FilterTracksByReprojectionNormalized,
                                       FilterTracksTriangulationAngle, collect_tracks)
from ..processors.track_retriangulation import RetriangulateTracks
from .config import OUT_OF_SCOPE_STAGES


def _n_obs(tracks):
    got = collect_tracks(tracks, with_obs=False)  # (the per-track lengths in one C loop when the tracks allow it)
    if got is not None:
        return int(got[0].sum())
    return int(sum(len(t.observations) for t in tracks.values()))


def _banner(msg):
    print('-------------------------------------')
    print(msg)
    print('-------------------------------------')


def SolveGlobalMapper(view_graph, cameras, images, config, depths=None, visualizer=None, device="cuda:0",
                      timings=None, progress=False):
    """global_mapper.py:21-156 from track establishment on.  Returns (cameras, images, tracks) like the reference."""
    for key in OUT_OF_SCOPE_STAGES:
        if not config.OPTIONS[key]:
            raise NotImplementedError(f"{key}=False: that stage (global_mapper.py:22-78 / :148-154) is outside this "
                                      "build's scope; set the switch and supply its outputs (pair inliers, "
                                      "registered images with rotations)")
    T = timings if timings is not None else {}
    T.setdefault('ba', [])
    trace = T.setdefault('trace', [])
    tracks = tracks_orig = None

    if not config.OPTIONS['skip_track_establishment']:                                          # :80-91
        _banner('Running track establishment ...')
        start_time = time.time()
        track_engine = TrackEngine(view_graph, images, device=device)
        tracks_orig = track_engine.EstablishFullTracks(config.TRACK_ESTABLISHMENT_OPTIONS)
        print('Initialized', len(tracks_orig), 'tracks')
        tracks = track_engine.FindTracksForProblem(tracks_orig, config.TRACK_ESTABLISHMENT_OPTIONS)
        print('Before filtering:', len(tracks_orig), ', after filtering:', len(tracks))
        T['track_establishment_s'] = time.time() - start_time
        T['tracks_full'], T['tracks_problem'] = len(tracks_orig), len(tracks)
        trace.append(('tracks', len(tracks), _n_obs(tracks), None))
        print('Track establishment took: ', T['track_establishment_s'])
    if tracks is None:
        # the reference reads the local ``tracks`` below; it is unbound when track establishment is skipped
        raise UnboundLocalError("tracks: track establishment was skipped")

    if not config.OPTIONS['skip_global_positioning']:                                           # :93-107
        _banner('Running global positioning ...')
        start_time = time.time()
        UndistortImages(cameras, images, device=device)
        gp_engine = TorchGP(visualizer=visualizer, device=device)
        gp_engine.InitializeRandomPositions(cameras, images, tracks, depths)
        gp_engine.Optimize(cameras, images, tracks, depths, config.GLOBAL_POSITIONER_OPTIONS, progress=progress)
        trace.append(('gp', len(tracks), _n_obs(tracks),
                      gp_engine.loss_history[-1] if gp_engine.loss_history else None))
        tracks = FilterTracksByAngle(cameras, images, tracks, config.INLIER_THRESHOLD_OPTIONS['max_angle_error'],
                                     device=device)
        NormalizeReconstruction(images, tracks, depths)
        trace.append(('gp_filtered', len(tracks), _n_obs(tracks), None))
        T['global_positioning_s'] = time.time() - start_time
        T['gp'] = dict(gp_engine.timings, final_loss=getattr(gp_engine, 'final_loss', None))
        print('Global positioning took: ', T['global_positioning_s'])

    if not config.OPTIONS['skip_bundle_adjustment']:                                            # :109-126
        _banner('Running bundle adjustment ...')
        start_time = time.time()
        for iter in range(3):  # the reference hardcodes 3 (num_iteration_bundle_adjustment is unused)
            ba_engine = TorchBA(visualizer=visualizer, device=device)
            ba_engine.Solve(cameras, images, tracks, config.BUNDLE_ADJUSTER_OPTIONS, progress=progress)
            T['ba'].append(dict(ba_engine.timings, stage=f'ba{iter}'))
            trace.append((f'ba{iter}', len(tracks), _n_obs(tracks), getattr(ba_engine, 'final_rmse', None)))
            UndistortImages(cameras, images, device=device)
            FilterTracksByReprojectionNormalized(cameras, images, tracks,
                                                 config.INLIER_THRESHOLD_OPTIONS['max_reprojection_error']
                                                 * max(1, 3 - iter), device=device)
        print(f'{len([image for image in images if image.is_registered])} images are registered after BA.')
        print('Filtering tracks')
        UndistortImages(cameras, images, device=device)
        FilterTracksByReprojectionNormalized(cameras, images, tracks,
                                             config.INLIER_THRESHOLD_OPTIONS['max_reprojection_error'], device=device)
        FilterTracksTriangulationAngle(cameras, images, tracks,
                                       config.INLIER_THRESHOLD_OPTIONS['min_triangulation_angle'], device=device)
        NormalizeReconstruction(images, tracks, depths)
        trace.append(('ba_filtered', len(tracks), _n_obs(tracks), None))
        T['bundle_adjustment_s'] = time.time() - start_time
        print('Bundle adjustment took: ', T['bundle_adjustment_s'])

    if not config.OPTIONS['skip_retriangulation']:                                              # :128-146
        _banner('Running retriangulation ...')
        start_time = time.time()
        RetriangulateTracks(cameras, images, tracks, tracks_orig, config.TRIANGULATOR_OPTIONS,
                            config.BUNDLE_ADJUSTER_OPTIONS, device=device)
        _banner('Running bundle adjustment ...')
        ba_engine = TorchBA(device=device)
        ba_engine.Solve(cameras, images, tracks, config.BUNDLE_ADJUSTER_OPTIONS, progress=progress)
        T['ba'].append(dict(ba_engine.timings, stage='ba_final'))
        trace.append(('ba_final', len(tracks), _n_obs(tracks), getattr(ba_engine, 'final_rmse', None)))
        UndistortImages(cameras, images, device=device)
        print('Filtering tracks')
        FilterTracksByReprojectionNormalized(cameras, images, tracks,
                                             config.INLIER_THRESHOLD_OPTIONS['max_reprojection_error'], device=device)
        FilterTracksTriangulationAngle(cameras, images, tracks,
                                       config.INLIER_THRESHOLD_OPTIONS['min_triangulation_angle'], device=device)
        trace.append(('retri_filtered', len(tracks), _n_obs(tracks), None))
        T['retriangulation_s'] = time.time() - start_time
        print('Retriangulation took: ', T['retriangulation_s'])

    return cameras, images, tracks
