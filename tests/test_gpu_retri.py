"""RetriangulateTracks' passes on the HIP path (csrc/passes.hip: k_filter_reproj_pixel, k_reproj_candidates) vs the
CPU restatement (oracle/passes.py) and the reference's own outputs (tests/golden/retri_*.npz).  Needs an MI355X."""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from instantsfm_amd import passes  # noqa: E402
from instantsfm_amd.config.colmap import BUNDLE_ADJUSTER_OPTIONS, TRIANGULATOR_OPTIONS  # noqa: E402
from instantsfm_amd.processors import track_filter as TF  # noqa: E402
from instantsfm_amd.processors import track_retriangulation as TR  # noqa: E402
from instantsfm_amd.synth import make_retri_scene  # noqa: E402
from oracle import passes as OP  # noqa: E402

import retri_scene as RS  # noqa: E402


@pytest.mark.parametrize("model", list(range(11)))
def test_cam2img_kernel_matches_reference(golden_dir, model):
    """k_filter_reproj_pixel with world2cam = I and the point at the golden (u, v, 1): the error against the
    reference's Camera.cam2img output is the kernel's cam2img deviation."""
    g = np.load(f"{golden_dir}/camera_models_golden.npz")
    uv = g[f"m{model}_uv"]
    n = uv.shape[0]
    xyz = np.concatenate([uv, np.ones((n, 1))], 1)
    valid, err = passes.filter_reproj_pixel(np.zeros(n), np.arange(n), np.arange(n), g[f"m{model}_cam2img"],
                                            np.zeros(1), [model], [g[f"m{model}_params"]], np.eye(4)[None], xyz,
                                            1e-6, with_err=True)
    assert valid.all()
    assert err.max() <= 1e-9, err.max()


@pytest.mark.parametrize("name", RS.NAMES)
@pytest.mark.parametrize("thr", [3.0, 0.8])
def test_filter_reproj_pixel_kernel_vs_oracle(name, thr):
    g = RS.load(name)
    cameras, images, tracks, _ = RS.scene(g)
    ov, counts, counter, oerr = OP.filter_reproj_pixel(cameras, images, tracks, thr)
    obs = np.concatenate([t.observations for t in tracks.values()])
    foff = g["feat_ptr"]
    trow = np.repeat(np.arange(len(tracks)), counts)
    v, err = passes.filter_reproj_pixel(obs[:, 0], trow, foff[obs[:, 0]] + obs[:, 1], g["feats"], g["img_cam"],
                                        g["cam_model"], g["cam_params"], g["w2c"], g["track_xyz"], thr, with_err=True)
    np.testing.assert_allclose(err, oerr, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(v, ov)


@pytest.mark.parametrize("name", RS.NAMES)
@pytest.mark.parametrize("thr", [3.0, 0.8])
def test_FilterTracksByReprojection_matches_reference(name, thr):
    g = RS.load(name)
    cameras, images, tracks, _ = RS.scene(g)
    cnt = TF.FilterTracksByReprojection(cameras, images, tracks, thr)
    keys, ptr, obs = RS.flat(tracks)
    np.testing.assert_array_equal(keys, g[f"filter_{thr:g}_keys"])
    np.testing.assert_array_equal(ptr, g[f"filter_{thr:g}_ptr"])
    np.testing.assert_array_equal(obs, g[f"filter_{thr:g}_obs"])
    assert cnt == int(g[f"filter_{thr:g}_counter"])


@pytest.mark.parametrize("name", RS.NAMES)
def test_reproj_candidates_kernel_vs_oracle(name):
    g = RS.load(name)
    cameras, images, tracks, tracks_orig = RS.scene(g)
    obs, rows, opass, oerr = OP.complete_candidates(cameras, images, tracks, tracks_orig, 3.0)
    from instantsfm_amd.scene.defs import get_camera_model_info
    rows_img, pps = TR._image_rows(cameras, images, get_camera_model_info(cameras[0].model_id)['pp'])
    v, err = passes.reproj_candidates(int(g["cam_model"][0]), obs[:, 0], rows, g["feat_ptr"][obs[:, 0]] + obs[:, 1],
                                      g["feats"], rows_img, pps, g["track_xyz"], 3.0, with_err=True)
    np.testing.assert_allclose(err, oerr, rtol=1e-10, atol=1e-9)
    np.testing.assert_array_equal(v, opass)


@pytest.mark.parametrize("name", RS.NAMES)
def test_complete_tracks_matches_reference(name):
    g = RS.load(name)
    cameras, images, tracks, tracks_orig = RS.scene(g)
    n = TR.complete_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS)
    assert n == int(g["complete_num"])
    keys, ptr, obs = RS.flat(tracks)
    np.testing.assert_array_equal(keys, g["complete_keys"])
    np.testing.assert_array_equal(ptr, g["complete_ptr"])
    np.testing.assert_array_equal(obs, g["complete_obs"])
    assert str(np.asarray(next(iter(tracks.values())).observations).dtype) == str(g["complete_dtype"])


def test_complete_tracks_unsupported_model():
    cameras, images, tracks, tracks_orig = make_retri_scene(model=2, n_cams=12, n_points=20, seed=4)
    from instantsfm_amd.scene.defs import CameraModelId
    cameras[0].model_id = CameraModelId.FOV
    with pytest.raises(NotImplementedError):
        TR.complete_tracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS)


@pytest.mark.parametrize("model", [2, 4])
def test_RetriangulateTracks_end_to_end(model):
    """Completion, points-only BA rounds and filtering: registration flags restored, poses unchanged (up to the
    quaternion round trip of the write-back), every remaining
    observation inside the filter threshold (the last round ends with filter_points), no track left with a
    triangulation angle under the minimum, and the reprojection error of the kept observations goes down."""
    cameras, images, tracks, tracks_orig = make_retri_scene(model=model, n_cams=20, n_points=600, seed=11,
                                                            point_sigma=0.05)
    images[3].is_registered = False
    w2c0 = [im.world2cam.copy() for im in images]
    _, _, _, err0 = OP.filter_reproj_pixel(cameras, images, tracks, 1e9)
    TR.RetriangulateTracks(cameras, images, tracks, tracks_orig, TRIANGULATOR_OPTIONS, BUNDLE_ADJUSTER_OPTIONS)
    assert images[3].is_registered is False and all(im.is_registered for i, im in enumerate(images) if i != 3)
    for im, w in zip(images, w2c0):  # poses are written back through the quaternion (update(), :18-36): 1e-15 level
        np.testing.assert_allclose(im.world2cam, w, rtol=0, atol=1e-12)
    valid, _, _, err1 = OP.filter_reproj_pixel(cameras, images, tracks, TRIANGULATOR_OPTIONS['filter_max_reproj_error'])
    assert valid.all()
    assert OP.filter_tri_angle(images, copy.deepcopy(tracks), TRIANGULATOR_OPTIONS['filter_min_tri_angle']) == []
    assert np.sqrt(np.mean(err1 ** 2)) < 0.8 * np.sqrt(np.mean(np.minimum(err0, 3.0) ** 2))
    assert len(tracks) > 500
