"""Options of ``instantsfm/config/colmap.py`` for the passes this build replaces (same keys and values):
BUNDLE_ADJUSTER_OPTIONS (:47-54, TorchBA.Solve), GLOBAL_POSITIONER_OPTIONS (:41-46, TorchGP.Optimize),
TRACK_ESTABLISHMENT_OPTIONS (:36-40, TrackEngine) and TRIANGULATOR_OPTIONS (:55-63, RetriangulateTracks)."""

TRACK_ESTABLISHMENT_OPTIONS = {
    'thres_inconsistency': 10.,
    'min_num_view_per_track': 3,
    'max_num_view_per_track': 200,
}

GLOBAL_POSITIONER_OPTIONS = {
    'min_num_view_per_track': 3,
    'thres_loss_function': 1e-1,
    'max_num_iterations': 100,
    'function_tolerance': 5e-4,
}

BUNDLE_ADJUSTER_OPTIONS = {
    'optimize_poses': True,
    'optimize_points': True,          # present but unused in the reference
    'min_num_view_per_track': 2,
    'thres_loss_function': 1.,
    'max_num_iterations': 200,
    'function_tolerance': 5e-4,
}

TRIANGULATOR_OPTIONS = {
    'min_num_view_per_track': 2,
    'complete_max_reproj_error': 3.0,
    'merge_max_reproj_error': 3.0,
    'filter_max_reproj_error': 3.0,
    'filter_min_tri_angle': 1.5,
    'ba_global_max_refinements': 5,
    'ba_global_max_refinement_change': 0.0005,
}

CONFIG = {'TRACK_ESTABLISHMENT_OPTIONS': TRACK_ESTABLISHMENT_OPTIONS,
          'GLOBAL_POSITIONER_OPTIONS': GLOBAL_POSITIONER_OPTIONS,
          'BUNDLE_ADJUSTER_OPTIONS': BUNDLE_ADJUSTER_OPTIONS,
          'TRIANGULATOR_OPTIONS': TRIANGULATOR_OPTIONS}
