"""Options of ``instantsfm/config/colmap.py`` (same keys and values): BUNDLE_ADJUSTER_OPTIONS (:47-54,
TorchBA.Solve), GLOBAL_POSITIONER_OPTIONS (:41-46, TorchGP.Optimize), TRACK_ESTABLISHMENT_OPTIONS (:36-40,
TrackEngine), TRIANGULATOR_OPTIONS (:55-63, RetriangulateTracks) and INLIER_THRESHOLD_OPTIONS (:11-21, the mapper's
track filters).  The option tables of the out-of-scope stages (view-graph calibration, rotation averaging, feature
handling) are kept so ``controllers.config.Config`` exposes the reference's attributes."""

VIEW_GRAPH_CALIBRATOR_OPTIONS = {
    'thres_lower_ratio': 0.1,
    'thres_higher_ratio': 10,
    'thres_two_view_error': 2.,
    'thres_loss_function': 1e-2,
    'max_num_iterations': 100,
    'function_tolerance': 5e-4,
}

INLIER_THRESHOLD_OPTIONS = {
    'max_angle_error': 1.,
    'max_reprojection_error': 1e-2,
    'min_triangulation_angle': 1.,
    'max_epipolar_error_E': 1.,
    'max_epipolar_error_F': 4.,
    'max_epipolar_error_H': 4.,
    'min_inlier_num': 30,
    'min_inlier_ratio': 0.25,
    'max_rotation_error': 10.,
}

ROTATION_ESTIMATOR_OPTIONS = {
    'max_num_l1_iterations': 10,
    'l1_step_convergence_threshold': 0.001,
    'max_num_irls_iterations': 100,
    'irls_step_convergence_threshold': 0.001,
    'irls_loss_parameter_sigma': 5.0,
}

L1_SOLVER_OPTIONS = {
    'max_num_iterations': 1000,
    'rho': 1.0,
    'alpha': 1.0,
    'absolute_tolerance': 1e-4,
    'relative_tolerance': 1e-2,
}

FEATURE_HANDLER_OPTIONS = {
    'min_num_matches': 30,
}

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

CONFIG = {'VIEW_GRAPH_CALIBRATOR_OPTIONS': VIEW_GRAPH_CALIBRATOR_OPTIONS,
          'INLIER_THRESHOLD_OPTIONS': INLIER_THRESHOLD_OPTIONS,
          'ROTATION_ESTIMATOR_OPTIONS': ROTATION_ESTIMATOR_OPTIONS,
          'L1_SOLVER_OPTIONS': L1_SOLVER_OPTIONS,
          'TRACK_ESTABLISHMENT_OPTIONS': TRACK_ESTABLISHMENT_OPTIONS,
          'GLOBAL_POSITIONER_OPTIONS': GLOBAL_POSITIONER_OPTIONS,
          'BUNDLE_ADJUSTER_OPTIONS': BUNDLE_ADJUSTER_OPTIONS,
          'TRIANGULATOR_OPTIONS': TRIANGULATOR_OPTIONS,
          'FEATURE_HANDLER_OPTIONS': FEATURE_HANDLER_OPTIONS}
