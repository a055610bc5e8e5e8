"""Scene data contract kept at the BA boundary.

Restates the subset of ``instantsfm/scene/defs.py`` that ``TorchBA.Solve`` reads and writes:

* ``Image``               -- defs.py:8-39   (``world2cam`` 4x4, ``features`` [F,2], ``cam_id``, ``is_registered``)
* ``CameraModelId``       -- defs.py:101-113
* ``get_camera_model_info`` -- defs.py:115-140 (focal / pp / k index maps)
* ``Camera``              -- defs.py:142-237 (``model_id``, ``params``, ``set_params``)
* ``Track``               -- defs.py:414-423 (``xyz``, ``observations`` [k,2] = (image_id, feature_id))
* ``ConfigurationType``, ``ImagePair``, pair-id helpers, ``ViewGraph`` (pairs only) -- defs.py:41-97, 425-430: what
  the COLMAP database reader produces and the track engine consumes

The reference module imports cv2 for undistortion helpers that are off the BA path; this
restatement has no cv2 dependency.
"""
from enum import Enum
from typing import List, Optional

import numpy as np


class Image:
    """defs.py:8-39."""

    def __init__(self, id: int = -1, cam_id: int = -1, filename: str = "", is_registered: bool = False,
                 cluster_id: int = -1, world2cam: Optional[np.ndarray] = None,
                 features: Optional[np.ndarray] = None, depths=None, features_undist=None,
                 point3d_ids=None, num_points3d: int = 0):
        self.id = id
        self.cam_id = cam_id
        self.filename = filename
        self.is_registered = is_registered
        self.cluster_id = cluster_id
        self.world2cam = world2cam if world2cam is not None else np.eye(4)
        self.features = features if features is not None else []
        self.depths = depths if depths is not None else []
        self.features_undist = features_undist if features_undist is not None else []
        self.point3d_ids = point3d_ids if point3d_ids is not None else []
        self.num_points3d = num_points3d

    def center(self):
        return self.world2cam[:3, :3].T @ -self.world2cam[:3, 3]


class ConfigurationType(Enum):
    """defs.py:41-50 (COLMAP's TwoViewGeometry::ConfigurationType values)."""
    UNDEFINED = 0
    DEGENERATE = 1
    CALIBRATED = 2
    UNCALIBRATED = 3
    PLANAR = 4
    PANORAMIC = 5
    PLANAR_OR_PANORAMIC = 6
    WATERMARK = 7
    MULTIPLE = 8


class ImagePair:
    """defs.py:52-86 (the fields; relative-pose helpers are off the path)."""

    def __init__(self, image_id1: int = -1, image_id2: int = -1, is_valid: bool = True, weight: float = 0.0,
                 E=None, F=None, H=None, rotation=None, translation=None, inliers=None,
                 config: ConfigurationType = ConfigurationType.UNDEFINED):
        self.image_id1 = image_id1
        self.image_id2 = image_id2
        self.is_valid = is_valid
        self.weight = weight
        self.E = E if E is not None else np.eye(3)
        self.F = F if F is not None else np.eye(3)
        self.H = H if H is not None else np.eye(3)
        self.rotation = rotation if rotation is not None else np.array([1, 0, 0, 0])
        self.translation = translation if translation is not None else np.zeros(3)
        self.inliers = inliers if inliers is not None else []
        self.config = config


C_MAX_INT = 2 ** 31 - 1  # defs.py:88


def PairId2Ids(pair_id):
    """defs.py:89-90."""
    return (pair_id % C_MAX_INT, pair_id // C_MAX_INT)


def PairId2IdsInversed(pair_id):
    """defs.py:92-93 (COLMAP's pair_id = id1 * (2^31 - 1) + id2)."""
    return (pair_id // C_MAX_INT, pair_id % C_MAX_INT)


def Ids2PairId(id1, id2):
    """defs.py:95-96."""
    return (id1 * C_MAX_INT + id2 if id1 < id2 else id2 * C_MAX_INT + id1)


class ViewGraph:
    """defs.py:425-430 plus establish_adjacency_list (:431-441)."""

    def __init__(self):
        self.image_pairs = {}  # pair_id -> ImagePair
        self.num_images = 0
        self.num_pairs = 0

    def establish_adjacency_list(self):
        self.adjacency_list = {}
        for pair in self.image_pairs.values():
            if not pair.is_valid:
                continue
            self.adjacency_list.setdefault(pair.image_id1, set()).add(pair.image_id2)
            self.adjacency_list.setdefault(pair.image_id2, set()).add(pair.image_id1)


class CameraModelId(Enum):
    """defs.py:101-113 (same integer values: they index ``reproject_funcs``)."""
    INVALID = -1
    SIMPLE_PINHOLE = 0
    PINHOLE = 1
    SIMPLE_RADIAL = 2
    RADIAL = 3
    OPENCV = 4
    OPENCV_FISHEYE = 5
    FULL_OPENCV = 6
    FOV = 7
    SIMPLE_RADIAL_FISHEYE = 8
    RADIAL_FISHEYE = 9
    THIN_PRISM_FISHEYE = 10


_MODEL_INFO = {
    # defs.py:115-140, verbatim index maps
    CameraModelId.SIMPLE_PINHOLE: dict(name='SIMPLE_PINHOLE', num_params=3, focal=[0], pp=[1, 2], k=[], p=[], omega=[], sx=[], optimize=[0]),
    CameraModelId.PINHOLE: dict(name='PINHOLE', num_params=4, focal=[0, 1], pp=[2, 3], k=[], p=[], omega=[], sx=[], optimize=[0, 1]),
    CameraModelId.SIMPLE_RADIAL: dict(name='SIMPLE_RADIAL', num_params=4, focal=[0], pp=[1, 2], k=[3], p=[], omega=[], sx=[], optimize=[0, 3]),
    CameraModelId.RADIAL: dict(name='RADIAL', num_params=5, focal=[0], pp=[1, 2], k=[3, 4], p=[], omega=[], sx=[], optimize=[0, 3, 4]),
    CameraModelId.OPENCV: dict(name='OPENCV', num_params=8, focal=[0, 1], pp=[2, 3], k=[4, 5], p=[6, 7], omega=[], sx=[], optimize=[0, 1, 4, 5, 6, 7]),
    CameraModelId.OPENCV_FISHEYE: dict(name='OPENCV_FISHEYE', num_params=8, focal=[0, 1], pp=[2, 3], k=[4, 5, 6, 7], omega=[], sx=[], optimize=[0, 1, 4, 5, 6, 7]),
    CameraModelId.FULL_OPENCV: dict(name='FULL_OPENCV', num_params=12, focal=[0, 1], pp=[2, 3], k=[4, 5, 8, 9, 10, 11], p=[6, 7], omega=[], sx=[], optimize=[0, 1, 4, 5, 6, 7, 8, 9, 10, 11]),
    CameraModelId.FOV: dict(name='FOV', num_params=5, focal=[0, 1], pp=[2, 3], k=[], p=[], omega=[4], sx=[], optimize=[0, 1, 4]),
    CameraModelId.SIMPLE_RADIAL_FISHEYE: dict(name='SIMPLE_RADIAL_FISHEYE', num_params=4, focal=[0], pp=[1, 2], k=[3], p=[], omega=[], sx=[], optimize=[0, 3]),
    CameraModelId.RADIAL_FISHEYE: dict(name='RADIAL_FISHEYE', num_params=5, focal=[0], pp=[1, 2], k=[3, 4], p=[], omega=[], sx=[], optimize=[0, 3, 4]),
    CameraModelId.THIN_PRISM_FISHEYE: dict(name='THIN_PRISM_FISHEYE', num_params=12, focal=[0, 1], pp=[2, 3], k=[4, 5, 8, 9], p=[6, 7], omega=[], sx=[10, 11], optimize=[0, 1, 4, 5, 6, 7, 8, 9, 10, 11]),
}

# Models whose projection the reference implements (cost_function.py:32-177); FOV (:125-128) and
# THIN_PRISM_FISHEYE (:179-182) raise NotImplementedError there.
IMPLEMENTED_MODELS = (0, 1, 2, 3, 4, 5, 6, 8, 9)


def get_camera_model_info(model_id):
    """defs.py:115-140. Raises NotImplementedError for INVALID like the reference."""
    if model_id not in _MODEL_INFO:
        raise NotImplementedError
    info = _MODEL_INFO[model_id]
    return {k: (list(v) if isinstance(v, list) else v) for k, v in info.items()}


def num_intrinsics(model_id) -> int:
    """Optimized intrinsics per camera after the pp columns are dropped (bundle_adjustment.py:75-80)."""
    info = get_camera_model_info(CameraModelId(model_id) if not isinstance(model_id, CameraModelId) else model_id)
    return info['num_params'] - len(info['pp'])


class Camera:
    """defs.py:142-237 (parameter bookkeeping only)."""

    def __init__(self, id: int = -1, model_id: CameraModelId = CameraModelId.INVALID, width: int = 0, height: int = 0,
                 params: Optional[List[float]] = None, has_prior_focal_length: bool = False,
                 principal_point: Optional[np.ndarray] = None, focal_length: Optional[np.ndarray] = None):
        self.id = id
        self.model_id = model_id
        self.width = width
        self.height = height
        self.has_prior_focal_length = has_prior_focal_length
        self.principal_point = principal_point if principal_point is not None else np.zeros(2)
        self.focal_length = focal_length if focal_length is not None else np.zeros(2)
        self.k: List[float] = [0.0]
        self.p: np.ndarray = np.zeros(2)
        self.omega: float = 0.0
        self.sx: np.ndarray = np.zeros(2)
        if params is not None:
            self.set_params(params)
        else:
            self.params: List[float] = []

    def focal(self) -> float:
        return float(np.mean(self.focal_length))

    def set_params(self, params) -> None:
        """defs.py:161-228: same length assertions and field unpacking."""
        info = _MODEL_INFO.get(self.model_id)
        if info is None:
            raise NotImplementedError
        assert len(params) == info['num_params']
        self.params = params
        f = info['focal']
        self.focal_length = np.array([params[f[0]], params[f[-1]]])
        self.principal_point = np.array([params[info['pp'][0]], params[info['pp'][1]]])
        if info.get('k'):
            self.k = [params[i] for i in info['k']]
        if info.get('p'):  # OPENCV_FISHEYE's info has no 'p' key (defs.py:129)
            self.p = np.array([params[i] for i in info['p']])
        if info.get('omega'):
            self.omega = params[info['omega'][0]]
        if info.get('sx'):
            self.sx = np.array([params[i] for i in info['sx']])

    def get_K(self):
        return np.array([[self.focal_length[0], 0, self.principal_point[0]],
                         [0, self.focal_length[1], self.principal_point[1]],
                         [0, 0, 1]])


class Track:
    """defs.py:414-423."""

    def __init__(self, **kwargs):
        self.id = -1
        self.xyz = np.zeros(3)
        self.color = np.zeros(3)
        self.is_initialized = False
        self.observations = np.zeros(0)
        for key, val in kwargs.items():
            setattr(self, key, val)
