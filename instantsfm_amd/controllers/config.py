"""Config -- drop-in for ``instantsfm/controllers/config.py`` (reference :1-51).

Same ``GENERAL_OPTIONS`` keys and defaults and the same ``Config(feature_name, manual_config_name=None)`` attributes.
The stages this build does not replace (preprocessing, view-graph calibration, relative pose estimation, rotation
averaging, pruning: SURVEY.md section 7) keep their ``skip_*`` switches; ``SolveGlobalMapper`` requires them to be set
(``Config.for_ba_half`` sets them) and raises NotImplementedError otherwise.
"""
import copy
import importlib

# general options that do not vary with feature_name (config.py:3-19)
GENERAL_OPTIONS = {
    'skip_preprocessing': False,
    'skip_view_graph_calibration': False,
    'skip_relative_pose_estimation': False,
    'skip_rotation_averaging': False,
    'skip_track_establishment': False,
    'skip_global_positioning': False,
    'skip_bundle_adjustment': False,
    'num_iteration_bundle_adjustment': 3,
    'skip_retriangulation': True,
    'num_iteration_retriangulation': 1,
    'skip_pruning': True,
    'uniform_camera': True,
}

# the stages before track establishment and after retriangulation (global_mapper.py:22-78, :148-154)
OUT_OF_SCOPE_STAGES = ('skip_preprocessing', 'skip_view_graph_calibration', 'skip_relative_pose_estimation',
                       'skip_rotation_averaging', 'skip_pruning')


class Config:
    """config.py:21-51: option tables of ``instantsfm_amd.config.<name>`` (``colmap`` for every COLMAP database)."""

    def __init__(self, feature_name, manual_config_name=None):
        self.feature_name = feature_name
        config_module_names = {'colmap': 'instantsfm_amd.config.colmap'}
        if manual_config_name is not None:
            config_module_name = 'instantsfm_amd.config.' + manual_config_name
        elif feature_name in config_module_names:
            config_module_name = config_module_names[feature_name]
        else:
            raise ValueError('Invalid feature_name')
        CONFIG = getattr(importlib.import_module(config_module_name), 'CONFIG')
        # copies, so that one run's option changes do not leak into the next Config (the reference shares the dicts)
        self.OPTIONS = copy.deepcopy(GENERAL_OPTIONS)
        self.VIEW_GRAPH_CALIBRATOR_OPTIONS = copy.deepcopy(CONFIG['VIEW_GRAPH_CALIBRATOR_OPTIONS'])
        self.INLIER_THRESHOLD_OPTIONS = copy.deepcopy(CONFIG['INLIER_THRESHOLD_OPTIONS'])
        self.ROTATION_ESTIMATOR_OPTIONS = copy.deepcopy(CONFIG['ROTATION_ESTIMATOR_OPTIONS'])
        self.L1_SOLVER_OPTIONS = copy.deepcopy(CONFIG['L1_SOLVER_OPTIONS'])
        self.TRACK_ESTABLISHMENT_OPTIONS = copy.deepcopy(CONFIG['TRACK_ESTABLISHMENT_OPTIONS'])
        self.GLOBAL_POSITIONER_OPTIONS = copy.deepcopy(CONFIG['GLOBAL_POSITIONER_OPTIONS'])
        self.BUNDLE_ADJUSTER_OPTIONS = copy.deepcopy(CONFIG['BUNDLE_ADJUSTER_OPTIONS'])
        self.TRIANGULATOR_OPTIONS = copy.deepcopy(CONFIG['TRIANGULATOR_OPTIONS'])
        self.FEATURE_HANDLER_OPTIONS = copy.deepcopy(CONFIG['FEATURE_HANDLER_OPTIONS'])

    @classmethod
    def for_ba_half(cls, feature_name='colmap', retriangulation=True, manual_config_name=None):
        """The configuration the mapper runs with here: the out-of-scope stages skipped (their outputs -- pair
        inliers, registered images with rotations -- are supplied by the caller), track establishment, global
        positioning and bundle adjustment on, retriangulation on unless ``retriangulation`` is False."""
        cfg = cls(feature_name, manual_config_name)
        for k in OUT_OF_SCOPE_STAGES:
            cfg.OPTIONS[k] = True
        cfg.OPTIONS['skip_retriangulation'] = not retriangulation
        return cfg
