"""TorchGP.Optimize packing (global_positioning.py:85-170) vs golden vectors captured from the reference itself
(tools/gen_golden.py --only gp).  CPU only."""
import os

import numpy as np
import pytest

from instantsfm_amd.processors.global_positioning import TorchGP, pack_gp
from instantsfm_amd.engine import GP_DEFAULTS
from instantsfm_amd.scene.defs import Camera, CameraModelId, Image, Track

OPTS = dict(min_num_view_per_track=3, thres_loss_function=1e-1, max_num_iterations=100, function_tolerance=5e-4)
NAMES = ["gp_packing_plain", "gp_packing_depth", "gp_packing_depth_only", "gp_packing_edge", "gp_packing_depth_f32"]


def scene_from_fixture(g):
    cams = [Camera(id=i, model_id=CameraModelId.SIMPLE_RADIAL, params=[1000.0, 500.0, 400.0, 0.0],
                   has_prior_focal_length=bool(f)) for i, f in enumerate(g["cam_prior_focal"])]
    fp = g["img_feat_ptr"]
    imgs = []
    for i in range(len(g["img_cam_id"])):
        imgs.append(Image(id=i, cam_id=int(g["img_cam_id"][i]), is_registered=bool(g["img_registered"][i]),
                          world2cam=g["img_world2cam"][i].copy(), features_undist=g["img_feats_undist"][fp[i]:fp[i + 1]],
                          depths=g["img_depths"][fp[i]:fp[i + 1]]))
    tp = g["track_obs_ptr"]
    tracks = {int(k): Track(id=int(k), xyz=g["track_xyz"][j].copy(), observations=g["track_obs"][tp[j]:tp[j + 1]])
              for j, k in enumerate(g["track_keys"])}
    depths = g["img_depths"] if bool(g["has_depths"]) else None
    return cams, imgs, tracks, depths


@pytest.mark.parametrize("name", NAMES)
def test_gp_pack_matches_reference(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    cams, imgs, tracks, depths = scene_from_fixture(g)
    pk = pack_gp(cams, imgs, tracks, depths, OPTS, depth_only=bool(g["out_depth_only"]))
    np.testing.assert_allclose(pk.translations, g["out_translations"], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(pk.camera_indices, g["out_camera_indices"])
    np.testing.assert_array_equal(pk.point_indices, g["out_point_indices"])
    np.testing.assert_array_equal(pk.is_calibrated, g["out_is_calibrated"])
    np.testing.assert_array_equal(pk.camera_translations, g["out_positions"])
    np.testing.assert_array_equal(pk.points_3d, g["out_points_3d"])
    np.testing.assert_array_equal(pk.scales, g["out_scales"])
    # fixed scales: the complement of scales.optimize_indices (none optimized in depth-only mode)
    if bool(g["out_has_optimize_indices"]):
        np.testing.assert_array_equal(np.flatnonzero(pk.scale_free), g["out_optimize_indices"])
    elif bool(g["out_depth_only"]):
        assert not pk.scale_free.any()
    else:
        assert pk.scale_free.all()
    # the scene mutations the reference performs before building the LM
    np.testing.assert_array_equal(np.array(list(tracks.keys())), g["out_track_keys_after"])
    np.testing.assert_array_equal(np.array([im.is_registered for im in imgs]), g["out_img_registered_after"])
    assert np.all(np.diff(pk.point_indices) >= 0), "track-major order"


def test_gp_lm_options_match_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "gp_packing_plain.npz"))
    radius, rmax, up, down = g["out_tr"]
    assert (radius, rmax, up, down) == (GP_DEFAULTS["tr_radius"], GP_DEFAULTS["tr_max"], GP_DEFAULTS["tr_up"],
                                        GP_DEFAULTS["tr_down"])
    assert float(g["out_huber"]) == OPTS["thres_loss_function"]
    assert float(g["out_pcg_tol"]) == GP_DEFAULTS["pcg_tol"]
    assert int(g["out_reject"]) == GP_DEFAULTS["max_rejects"]


def test_convert_results_and_random_init():
    imgs = [Image(id=0, world2cam=np.eye(4)), Image(id=1, world2cam=np.eye(4))]
    from scipy.spatial.transform import Rotation
    imgs[1].world2cam[:3, :3] = Rotation.from_rotvec([0.1, 0.2, 0.3]).as_matrix()
    tracks = {5: Track(id=5), 9: Track(id=9)}
    gp = TorchGP(device="cpu")
    np.random.seed(0)
    gp.InitializeRandomPositions([], imgs, tracks, depths=np.array([0.0, 2.0, 4.0]))
    np.random.seed(0)
    exp = [12.0 * np.random.uniform(-1, 1, 3) for _ in range(4)]   # scene_scale = mean(2, 4) * 4
    np.testing.assert_array_equal(imgs[0].world2cam[:3, 3], exp[0])
    np.testing.assert_array_equal(tracks[9].xyz, exp[3])
    assert tracks[5].is_initialized
    c = imgs[1].world2cam[:3, 3].copy()
    gp.ConvertResults(imgs)
    np.testing.assert_allclose(imgs[1].world2cam[:3, 3], -imgs[1].world2cam[:3, :3] @ c)


def test_random_init_matches_per_track_draws():
    """InitializeRandomPositions draws all tracks' positions in one call of the global RNG: the same doubles, in the
    same order, as the reference's uniform(-1, 1, 3) per image then per track (global_positioning.py:23-39)."""
    rng = np.random.default_rng(1)
    imgs = [Image(id=i, world2cam=np.eye(4)) for i in range(7)]
    tracks = {int(k): Track(id=int(k)) for k in rng.permutation(5000)[:600]}
    gp = TorchGP(device="cpu")
    np.random.seed(3)
    gp.InitializeRandomPositions([], imgs, tracks)
    np.random.seed(3)
    exp_img = [100 * np.random.uniform(-1, 1, 3) for _ in imgs]
    exp_trk = [100 * np.random.uniform(-1, 1, 3) for _ in tracks]
    for im, e in zip(imgs, exp_img):
        np.testing.assert_array_equal(im.world2cam[:3, 3], e)
    for t, e in zip(tracks.values(), exp_trk):
        assert t.xyz.shape == (3,) and t.xyz.dtype == np.float64 and t.is_initialized
        np.testing.assert_array_equal(t.xyz, e)


@pytest.mark.parametrize("name", NAMES)
def test_gp_pack_native_matches_numpy_path(golden_dir, name):
    """The C collect path of pack_gp (observations and xyz read in one loop) gives the numpy path's arrays and the
    same scene mutations, also when one Track's observations are an array layout collect does not take (int16,
    Fortran order: the numpy path for the whole call)."""
    from instantsfm_amd.processors.bundle_adjustment import packx
    assert packx() is not None
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    outs = []
    for native in (True, False):
        cams, imgs, tracks, depths = scene_from_fixture(g)
        pk = pack_gp(cams, imgs, tracks, depths, OPTS, depth_only=bool(g["out_depth_only"]), native=native)
        outs.append((pk, list(tracks.keys()), [im.is_registered for im in imgs]))
    (a, ka, ra), (b, kb, rb) = outs
    assert ka == kb and ra == rb
    for f in ("translations", "camera_indices", "point_indices", "is_calibrated", "camera_translations", "points_3d",
              "scales", "scale_free", "image_idx2id"):
        x, y = getattr(a, f), getattr(b, f)
        assert x.dtype == y.dtype and x.shape == y.shape, f
        np.testing.assert_array_equal(x, y)
    assert [t.id for t in a.track_list] == [t.id for t in b.track_list]
    cams, imgs, tracks, depths = scene_from_fixture(g)
    k0 = next(iter(tracks))
    tracks[k0].observations = np.asfortranarray(tracks[k0].observations.astype(np.int16))  # numpy path for the call
    c = pack_gp(cams, imgs, tracks, depths, OPTS, depth_only=bool(g["out_depth_only"]))
    np.testing.assert_array_equal(c.point_indices, b.point_indices)
