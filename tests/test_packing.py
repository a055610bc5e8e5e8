"""TorchBA.Solve packing (bundle_adjustment.py:66-126) vs golden vectors captured from the reference itself
(tools/gen_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from instantsfm_amd.processors.bundle_adjustment import _pose_matrices, pack, update
from instantsfm_amd.scene.defs import Camera, CameraModelId, Image, Track

OPTS = dict(optimize_poses=True, optimize_points=True, min_num_view_per_track=2, thres_loss_function=1.0,
            max_num_iterations=200, function_tolerance=5e-4)


def scene_from_fixture(g, params_kind):
    """params_kind: 'pyfloat' (list of Python floats), 'np64list' (list of np.float64), 'array' (float64 ndarray)."""
    model = CameraModelId(int(g["model"]))
    cams = []
    for i, p in enumerate(g["cam_params"]):
        params = {"pyfloat": [float(x) for x in p], "np64list": list(p), "array": np.array(p)}[params_kind]
        cams.append(Camera(id=i, model_id=model, params=params))
    imgs = []
    fp = g["img_feat_ptr"]
    for i in range(len(g["img_cam_id"])):
        imgs.append(Image(id=i, cam_id=int(g["img_cam_id"][i]), is_registered=bool(g["img_registered"][i]),
                          world2cam=g["img_world2cam"][i], features=g["img_feats"][fp[i]:fp[i + 1]]))
    tracks = {}
    tp = g["track_obs_ptr"]
    for k, key in enumerate(g["track_keys"]):
        tracks[int(key)] = Track(id=int(key), xyz=g["track_xyz"][k], observations=g["track_obs"][tp[k]:tp[k + 1]])
    return cams, imgs, tracks


def quat_equal_up_to_sign(a, b, tol):
    return np.all(np.minimum(np.abs(a - b).max(-1), np.abs(a + b).max(-1)) < tol)


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("name", ["packing_config1", "packing_edge", "packing_edge_points_only"])
def test_pack_matches_reference(golden_dir, name, native):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    # rebuild the scene with the parameter types tools/gen_golden.py used for that fixture
    kind = "np64list" if name == "packing_config1" else "pyfloat"
    cams, imgs, tracks = scene_from_fixture(g, kind)
    opts = dict(OPTS, optimize_poses=bool(g["out_optimize_poses"]))
    pk = pack(cams, imgs, tracks, opts, native=native)
    np.testing.assert_array_equal(pk.points_2d, g["out_points_2d"])
    np.testing.assert_array_equal(pk.camera_indices, g["out_camera_indices"])
    np.testing.assert_array_equal(pk.point_indices, g["out_point_indices"])
    np.testing.assert_array_equal(pk.camera_pps, g["out_camera_pps"])
    np.testing.assert_array_equal(pk.points_3d, g["out_points_3d"])
    pose = g["out_pose"]
    np.testing.assert_allclose(pk.camera_params[:, :3], pose[:, :3], rtol=0, atol=1e-12)
    assert quat_equal_up_to_sign(pk.camera_params[:, 3:7], pose[:, 3:7], 1e-12)
    # intrinsics: bit-exact, including the reference's float32 rounding of list-typed params
    np.testing.assert_array_equal(pk.camera_params[:, 7:], pose[:, 7:])
    assert np.all(np.diff(pk.point_indices) >= 0), "track-major order"


def test_pack_float64_params_not_rounded(golden_dir):
    g = np.load(os.path.join(golden_dir, "packing_edge.npz"))
    cams, imgs, tracks = scene_from_fixture(g, "array")
    pk = pack(cams, imgs, tracks, OPTS)
    # numpy float64 params (what the COLMAP database reader produces, data_reader.py:44) stay float64
    expect = np.asarray(g["cam_params"])[:, [0, 1, 4, 5, 6, 7]]
    assert np.array_equal(pk.camera_params[0, 7:], expect[int(g["img_cam_id"][0])])


def test_unsupported_models_raise():
    for m in (CameraModelId.FOV, CameraModelId.THIN_PRISM_FISHEYE):
        n = 5 if m == CameraModelId.FOV else 12
        cams = [Camera(id=0, model_id=m, params=[100.0] * n)]
        imgs = [Image(id=0, cam_id=0, is_registered=True, features=np.zeros((1, 2)))]
        tracks = {0: Track(xyz=np.zeros(3), observations=np.array([[0, 0], [0, 0]]))}
        with pytest.raises(NotImplementedError):
            pack(cams, imgs, tracks, OPTS)


def test_update_writes_back(golden_dir):
    """update() (reference :18-36): pp re-inserted, SE3 -> 4x4, last image of a shared camera wins."""
    g = np.load(os.path.join(golden_dir, "packing_edge.npz"))
    cams, imgs, tracks = scene_from_fixture(g, "array")
    pk = pack(cams, imgs, tracks, OPTS)
    cp = pk.camera_params.copy()
    cp[:, 7] += np.arange(cp.shape[0])  # distinct fx per packed image
    pts = pk.points_3d + 1.0
    update(cams, imgs, tracks, pk, cp, pts)
    for i, orig in enumerate(pk.unique_points):
        np.testing.assert_array_equal(tracks[pk.track_keys[orig]].xyz, pts[i])
    M = _pose_matrices(cp[:, :7])
    for i, image_id in enumerate(pk.unique_cameras):
        np.testing.assert_allclose(imgs[image_id].world2cam, M[i], atol=1e-15)
        np.testing.assert_allclose(imgs[image_id].world2cam[:3, :3] @ imgs[image_id].world2cam[:3, :3].T, np.eye(3), atol=1e-12)
    # images 0, 2, 4 share camera 0: the last packed one of them wins
    last = max(i for i, image_id in enumerate(pk.unique_cameras) if imgs[image_id].cam_id == 0)
    assert cams[0].params[0] == cp[last, 7]
    assert cams[0].params[2] == pk.camera_pps[last, 0]  # principal point re-inserted


def _fields(pk):
    return [pk.points_2d, pk.camera_indices, pk.point_indices, pk.camera_pps, pk.camera_params, pk.points_3d,
            pk.unique_cameras, pk.unique_points]


def test_native_pack_is_built_and_matches_numpy_path():
    """The C packer (csrc/packx.c) is what pack() runs, and it gives bit-identical arrays and dtypes to the numpy
    path on a synthetic scene with unregistered images, short tracks, points behind cameras, int32 observations and
    float32 xyz (the layouts the reference's DB reader and TrackEngine produce); Track attributes it does not take
    (a Python list) fall back to the numpy path."""
    from instantsfm_amd.processors import bundle_adjustment as BA
    from instantsfm_amd.synth import make_problem, to_scene
    assert BA.packx() is not None, "instantsfm_amd/_lib/_packx*.so not built (instantsfm_amd.build.build_packx)"
    prob = make_problem(30, 1500, seed=3)
    cams, imgs, tracks = to_scene(prob)
    rng = np.random.default_rng(0)
    for i in rng.choice(len(imgs), 3, replace=False):
        imgs[i].is_registered = False
    keys = list(tracks)
    for k in rng.choice(len(keys), 40, replace=False):       # length-1 tracks
        tracks[keys[k]].observations = tracks[keys[k]].observations[:1]
    for k in rng.choice(len(keys), 40, replace=False):       # points behind the cameras
        tracks[keys[k]].xyz = tracks[keys[k]].xyz * -50.0
    for k in rng.choice(len(keys), 100, replace=False):      # int32 observations, float32 xyz
        tracks[keys[k]].observations = tracks[keys[k]].observations.astype(np.int32)
        tracks[keys[k]].xyz = tracks[keys[k]].xyz.astype(np.float32)
    a, b = pack(cams, imgs, tracks, OPTS, native=True), pack(cams, imgs, tracks, OPTS, native=False)
    assert a.points_2d.shape[0] < prob.n_obs
    for x, y in zip(_fields(a), _fields(b)):
        assert x.dtype == y.dtype and x.shape == y.shape
        np.testing.assert_array_equal(x, y)
    # the int32 index copies insfm_ba_create takes: written by the C packer, made on demand on the numpy path
    assert a.indices_i32 is not None and b.indices_i32 is None
    for x, y in zip(a.indices32(), b.indices32()):
        assert x.dtype == np.int32 and y.dtype == np.int32
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.indices32()[0], a.camera_indices)
    np.testing.assert_array_equal(a.indices32()[1], a.point_indices)
    assert BA.packx().collect(list(tracks.values()), 2) is not None
    tracks[keys[0]].observations = tracks[keys[0]].observations.tolist()
    assert BA.packx().collect(list(tracks.values()), 2) is None
    c = pack(cams, imgs, tracks, OPTS)
    for x, y in zip(_fields(c), _fields(b)):
        np.testing.assert_array_equal(x, y)


def test_assign_xyz_writes_in_place_only_when_unobservable():
    """packx.assign_xyz (update()'s track.xyz write-back, bundle_adjustment.py:18-36): an xyz array nothing else can
    see -- an exact float64 [3] ndarray owning its writable buffer, held only by the track -- gets the point written
    into it; any other xyz (held elsewhere, a view, weak-referenced, another dtype or shape, a subclass, a list, absent)
    is replaced by a new owned float64 [3] array and the old object keeps its values."""
    import weakref
    from instantsfm_amd.processors import bundle_adjustment as BA
    px = BA.packx()
    assert px is not None
    n = 9
    tracks = [Track() for _ in range(n)]
    held = np.array([7.0, 7.0, 7.0])
    base = np.arange(30.0)
    tracks[1].xyz = held                       # referenced elsewhere
    tracks[2].xyz = base[3:6]                  # a view
    tracks[3].xyz = np.zeros(3)
    wr = weakref.ref(tracks[3].xyz)            # weak-referenced
    tracks[4].xyz = np.zeros(3, np.float32)    # another dtype
    tracks[5].xyz = np.zeros(4)                # another shape
    tracks[6].xyz = np.zeros(3).view(np.matrix)  # a subclass
    tracks[7].xyz = [0.0, 0.0, 0.0]            # not an array
    del tracks[8].xyz                          # absent
    own_id = id(tracks[0].xyz)
    pts = np.arange(3.0 * n).reshape(n, 3) + 0.5
    order = np.arange(n - 1, -1, -1, dtype=np.int64)   # point i -> track n - 1 - i
    px.assign_xyz(tracks, order, pts)
    for i in range(n):
        x = tracks[n - 1 - i].xyz
        assert type(x) is np.ndarray and x.dtype == np.float64 and x.shape == (3,) and x.flags.owndata
        assert np.array_equal(x, pts[i])
    assert id(tracks[0].xyz) == own_id        # written in place
    assert np.array_equal(held, [7.0, 7.0, 7.0]) and tracks[1].xyz is not held
    assert np.array_equal(base, np.arange(30.0))
    assert wr() is None                         # replaced (not written in place) and released
    pts[:] = 0.0                                 # the tracks own their values
    assert np.array_equal(tracks[n - 1].xyz, np.arange(3.0) + 0.5)
