"""BA options of ``instantsfm/config/colmap.py:47-54`` (the dict passed to ``TorchBA.Solve``)."""

BUNDLE_ADJUSTER_OPTIONS = {
    'optimize_poses': True,
    'optimize_points': True,          # present but unused in the reference
    'min_num_view_per_track': 2,
    'thres_loss_function': 1.,
    'max_num_iterations': 200,
    'function_tolerance': 5e-4,
}

CONFIG = {'BUNDLE_ADJUSTER_OPTIONS': BUNDLE_ADJUSTER_OPTIONS}
