"""COLMAP database reader -- drop-in for ``instantsfm/controllers/data_reader.py:11-120`` (``PathInfo``, ``ReadData``,
``ReadColmapDatabase``).  Host code over sqlite3 (stdlib): the same query, the same filters (invalid match indices,
NULL match blobs, invalid two-view configurations), the same id remapping to list indices and the same return value
``(view_graph, cameras, images, feature_name)``.  ``ReadDepthsIntoFeatures`` / ``ReadDepths`` (:122-144) read
ScanNet-style 16-bit depth PNGs with the framework's own PNG reader (``utils.png``; the reference uses cv2) and
sample them at the features (``utils.depth_sample``).
"""
import glob
import os
import time

import numpy as np

from ..scene.defs import (Camera, CameraModelId, ConfigurationType, Ids2PairId, Image, ImagePair, PairId2IdsInversed,
                          ViewGraph)
from ..utils.database import COLMAPDatabase, blob_to_array
from ..utils.depth_sample import sample_depths
from ..utils.png import read_png_gray

_INVALID_CONFIGS = (ConfigurationType.UNDEFINED, ConfigurationType.DEGENERATE, ConfigurationType.WATERMARK,
                    ConfigurationType.MULTIPLE)


class PathInfo:
    """data_reader.py:11-18."""

    def __init__(self):
        self.image_path = ""
        self.database_path = ""
        self.output_path = ""
        self.database_exists = False
        self.depth_path = ""
        self.record_path = ""


def ReadData(path) -> PathInfo:
    """data_reader.py:20-36: COLMAP (images/) or ScanNet (color/) layout."""
    info = PathInfo()
    if os.path.exists(os.path.join(path, 'images')):
        info.image_path = os.path.join(path, 'images')
    elif os.path.exists(os.path.join(path, 'color')):
        info.image_path = os.path.join(path, 'color')
    info.database_path = os.path.join(path, 'database.db')
    info.output_path = os.path.join(path, 'sparse')
    info.database_exists = os.path.exists(info.database_path)
    if os.path.exists(os.path.join(path, 'depth')):
        info.depth_path = os.path.join(path, 'depth')
    info.record_path = os.path.join(path, 'record')
    return info


def ReadColmapDatabase(path):
    """data_reader.py:38-120."""
    start_time = time.time()
    view_graph = ViewGraph()
    db = COLMAPDatabase.connect(path)

    images = {image_id: Image(id=image_id, filename=name, cam_id=cam_id)
              for image_id, name, cam_id in db.execute("SELECT image_id, name, camera_id FROM images")}
    cameras = {}
    for cam_id, model, width, height, params, prior in db.execute("SELECT * FROM cameras"):
        cameras[cam_id] = Camera(id=cam_id, model_id=CameraModelId(model), width=width, height=height,
                                 params=blob_to_array(params, np.float64), has_prior_focal_length=prior > 0)
    for cam in cameras.values():
        cam.set_params(cam.params)

    for image_id, cols, data in db.execute("SELECT image_id, cols, data FROM keypoints"):
        if data is not None:
            images[image_id].features = blob_to_array(data, np.float32, (-1, cols))[:, :2]

    rows = db.execute("SELECT m.pair_id, m.data, t.config, t.F, t.E, t.H FROM matches AS m "
                      "INNER JOIN two_view_geometries AS t ON m.pair_id = t.pair_id")
    image_pairs = {}
    invalid_count = 0
    for pair_id, data, config, F_blob, E_blob, H_blob in rows:
        if data is None:
            invalid_count += 1
            continue
        m = blob_to_array(data, np.uint32, (-1, 2))
        id1, id2 = PairId2IdsInversed(pair_id)
        pair = ImagePair(image_id1=id1, image_id2=id2)
        image_pairs[pair_id] = pair
        # (idx != -1) is always true for uint32 under numpy 1.26's value-based comparison (pyproject.toml:17)
        ok = (m[:, 0] < len(images[id1].features)) & (m[:, 1] < len(images[id2].features))
        pair.matches = m[ok]
        pair.config = ConfigurationType(config)
        if pair.config in _INVALID_CONFIGS:
            pair.is_valid = False
            invalid_count += 1
            continue
        pair.F = blob_to_array(F_blob, np.float64).reshape(3, 3)
        pair.E = blob_to_array(E_blob, np.float64).reshape(3, 3)
        pair.H = blob_to_array(H_blob, np.float64).reshape(3, 3)

    view_graph.image_pairs = {pid: p for pid, p in image_pairs.items() if p.is_valid}
    print(f'Pairs read done. {invalid_count} / {len(image_pairs)+invalid_count} are invalid')

    cam_id2idx = {cam_id: idx for idx, cam_id in enumerate(cameras.keys())}
    img_id2idx = {img_id: idx for idx, img_id in enumerate(images.keys())}
    cameras = list(cameras.values())
    images = list(images.values())
    for cam in cameras:
        cam.id = cam_id2idx[cam.id]
    for image in images:
        image.id = img_id2idx[image.id]
        image.cam_id = cam_id2idx[image.cam_id]
    for pair in view_graph.image_pairs.values():
        pair.image_id1 = img_id2idx[pair.image_id1]
        pair.image_id2 = img_id2idx[pair.image_id2]
    view_graph.image_pairs = {Ids2PairId(p.image_id1, p.image_id2): p for p in view_graph.image_pairs.values()}
    print(f'Reading database took: {time.time() - start_time:.2f}')

    try:
        feature_name = db.execute("SELECT feature_name FROM feature_name").fetchone()[0]
    except Exception:
        feature_name = 'colmap'  # no (or an empty) feature_name table: a COLMAP-produced database
    return view_graph, cameras, images, feature_name


def ReadDepthsIntoFeatures(path, cameras, images, depths=None):
    """data_reader.py:122-134: the depth maps of ``path`` (``ReadDepths``), sampled at every feature of every image
    (nearest, ``utils.depth_sample``) into ``image.depths`` (float32, 0 where the feature lies outside the image);
    returns the [N, H, W] float32 maps, which ``SolveGlobalMapper(..., depths=...)`` takes.  Image i uses map i (the
    sorted file order) and its camera's width / height.  ``depths``: maps already in memory (skips the file read).
    One vectorized sample per image instead of the reference's per-feature loop; same values (tests/test_depth.py)."""
    if depths is None:
        depths = ReadDepths(path)
    for image in images:
        camera = cameras[image.cam_id]
        feats = np.asarray(image.features).reshape(-1, 2)
        d, _ = sample_depths(depths[image.id], feats, camera.width, camera.height)
        image.depths = d.astype(np.float32)
    return depths


def ReadDepths(path):
    """data_reader.py:136-144: every ``*.png`` of ``path`` in sorted order, 16-bit millimetres -> float32 metres,
    stacked [N, H, W] (the maps must share one size, as ``np.array`` requires in the reference)."""
    maps = [read_png_gray(f).astype(np.float32) / 1000.0 for f in sorted(glob.glob(os.path.join(path, '*.png')))]
    return np.array(maps, dtype=np.float32)
