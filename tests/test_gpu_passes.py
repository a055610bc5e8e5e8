"""Between-round passes on the HIP path (csrc/passes.hip) vs the CPU restatement (oracle/passes.py) and the reference's
golden vectors (tools/gen_golden.py --only passes).  Needs an MI355X."""
import copy
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from instantsfm_amd import passes  # noqa: E402
from instantsfm_amd.processors.image_undistortion import UndistortImages  # noqa: E402
from instantsfm_amd.processors import track_filter as TF  # noqa: E402
from instantsfm_amd.scene.defs import Camera, CameraModelId, Image  # noqa: E402
from oracle import passes as OP  # noqa: E402

from test_passes_oracle import kept_obs, load_scene  # noqa: E402

EXACT = (0, 1, 2, 3, 4, 6)  # no transcendental functions on the path: bit-exact


@pytest.fixture(scope="module")
def golden(golden_dir):
    with np.load(os.path.join(golden_dir, "passes_golden.npz")) as z:
        return dict(z)


@pytest.fixture(scope="module")
def cams(golden_dir):
    with np.load(os.path.join(golden_dir, "camera_models_golden.npz")) as z:
        return dict(z)


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("model", list(range(11)))
def test_undistort_kernel_matches_oracle(cams, model, f32):
    rng = np.random.default_rng(model)
    prm = cams[f"m{model}_params"]
    xy = rng.uniform([0, 0], [1000, 800], (5000, 2))
    xy[0] = [prm[1], prm[2]] if model in (0, 2, 3, 8, 9) else [prm[2], prm[3]]  # the principal point itself
    if f32:
        xy = xy.astype(np.float32)
    got = passes.undistort(xy, np.zeros(len(xy), np.int32), np.array([model], np.int32), [prm])
    exp = OP.undistort_rays(model, prm, xy)
    if model in EXACT:
        np.testing.assert_array_equal(got, exp)
    else:
        ok = np.isfinite(exp).all(1)
        np.testing.assert_allclose(got[ok], exp[ok], rtol=0, atol=2e-6 if f32 else 1e-13)


def test_undistort_images_processor_mixed_cameras(cams):
    rng = np.random.default_rng(3)
    cameras, images = [], []
    for c, m in enumerate((2, 4, 6, 1, 2)):
        cameras.append(Camera(id=c, model_id=CameraModelId(m), params=list(cams[f"m{m}_params"])))
    for i in range(12):
        c = i % len(cameras)
        n = int(rng.integers(0, 300))
        f = rng.uniform([0, 0], [1000, 800], (n, 2))
        images.append(Image(id=i, cam_id=c, features=f.astype(np.float32) if i % 3 == 0 else f))
    UndistortImages(cameras, images)
    for im in images:
        cam = cameras[im.cam_id]
        exp = OP.undistort_rays(cam.model_id.value, np.asarray(cam.params), np.asarray(im.features).reshape(-1, 2)) \
            if len(im.features) else np.zeros((0, 3))
        np.testing.assert_array_equal(im.features_undist, exp)


@pytest.mark.parametrize("thr", [1e-2, 3e-2])
def test_filter_reproj_normalized_processor_matches_reference(golden, thr):
    imgs, tracks = load_scene(golden)
    tracks = {k: t for k, t in tracks.items() if len(t.observations)}
    counter = TF.FilterTracksByReprojectionNormalized(None, imgs, tracks, thr)
    assert counter == int(golden[f"reproj_{thr:g}_counter"])
    exp = kept_obs(golden, f"reproj_{thr:g}_")
    assert list(tracks) == list(exp)
    for k, t in tracks.items():
        np.testing.assert_array_equal(t.observations, exp[k])


def test_filter_angle_processor_matches_reference(golden):
    imgs, tracks = load_scene(golden)
    tracks = {k: t for k, t in tracks.items() if len(t.observations)}
    out = TF.FilterTracksByAngle(None, imgs, tracks, 1.0)
    assert out is tracks
    exp = kept_obs(golden, "angle_")
    for k, t in tracks.items():
        np.testing.assert_array_equal(t.observations, exp[k])


def test_filter_tri_angle_processor_matches_reference(golden):
    imgs, tracks = load_scene(golden)
    counter = TF.FilterTracksTriangulationAngle(None, imgs, tracks, 1.5)
    assert counter == int(golden["tri_counter"])
    assert list(tracks) == [int(k) for k in golden["tri_keys"]]


def test_filter_errors_match_oracle_at_scale():
    """2M observations (config-3 size): GPU reprojection errors vs the vectorized oracle arithmetic; masks agree
    everywhere except within 1e-11 of the threshold."""
    rng = np.random.default_rng(0)
    M, T, L = 1000, 200000, 10
    w2c = np.tile(np.eye(4), (M, 1, 1))
    from scipy.spatial.transform import Rotation
    w2c[:, :3, :3] = Rotation.from_rotvec(rng.normal(0, 0.3, (M, 3))).as_matrix()
    w2c[:, :3, 3] = rng.normal(0, 1, (M, 3)) + [0, 0, 10]
    xyz = rng.normal(0, 3, (T, 3))
    img = rng.integers(0, M, T * L).astype(np.int32)
    trk = np.repeat(np.arange(T), L).astype(np.int32)
    pc = np.einsum('ijk,ik->ij', w2c[img], np.hstack([xyz[trk], np.ones((T * L, 1))]))[:, :3]
    rays = pc / np.linalg.norm(pc, axis=1, keepdims=True) + rng.normal(0, 3e-3, (T * L, 3))
    v, err = passes.filter_reproj_normalized(img, trk, np.arange(T * L), w2c, xyz, rays, 1e-2, with_err=True)
    fr = rays[:, :2] / (rays[:, 2:] + 1e-10)
    e_ref = np.linalg.norm(pc[:, :2] / (pc[:, 2:] + 1e-10) - fr, axis=1)
    np.testing.assert_allclose(err, e_ref, rtol=1e-10, atol=1e-15)  # einsum order; points near a camera plane amplify it
    v_ref = (pc[:, 2] > 1e-10) & (e_ref < 1e-2)
    near = np.abs(e_ref - 1e-2) < 1e-11
    assert np.array_equal(v[~near], v_ref[~near])
    assert 0.05 < v.mean() < 0.99 and (~v).sum() > 10000  # both outcomes well represented
