"""Between-round passes: the CPU restatement (oracle/passes.py) and the host-side pieces of the
processors against golden vectors captured from the reference itself (tools/gen_golden.py --only passes).  CPU only."""
import os

import numpy as np
import pytest

from oracle import passes as OP
from instantsfm_amd.processors.reconstruction_normalizer import NormalizeReconstruction
from instantsfm_amd.processors.track_filter import quirk_counter
from instantsfm_amd.scene.defs import Image, Track


def load_scene(g):
    fp = g["feat_ptr"]
    imgs = [Image(id=i, cam_id=i, is_registered=True, world2cam=g["w2c"][i].copy(),
                  features_undist=g["feats_undist"][fp[i]:fp[i + 1]], depths=g["depths"][fp[i]:fp[i + 1]])
            for i in range(g["w2c"].shape[0])]
    tp = g["track_ptr"]
    tracks = {int(k): Track(id=int(k), xyz=g["track_xyz"][j].copy(), observations=g["track_obs"][tp[j]:tp[j + 1]].copy())
              for j, k in enumerate(g["track_keys"])}
    return imgs, tracks


def kept_obs(g, prefix):
    return {int(k): g[prefix + "obs"][g[prefix + "ptr"][j]:g[prefix + "ptr"][j + 1]] for j, k in enumerate(g[prefix + "keys"])}


@pytest.fixture(scope="module")
def golden(golden_dir):
    with np.load(os.path.join(golden_dir, "passes_golden.npz")) as z:
        return dict(z)  # decompress once


@pytest.mark.parametrize("thr", [1e-2, 3e-2])
def test_oracle_filter_reproj_normalized_matches_reference(golden, thr):
    imgs, tracks = load_scene(golden)
    tracks = {k: t for k, t in tracks.items() if len(t.observations)}
    valid, counts, counter, _ = OP.filter_reproj_normalized(imgs, tracks, thr)
    exp = kept_obs(golden, f"reproj_{thr:g}_")
    starts = np.concatenate([[0], np.cumsum(counts)])
    for j, (k, t) in enumerate(tracks.items()):
        np.testing.assert_array_equal(t.observations[valid[starts[j]:starts[j + 1]]], exp[k])
    assert counter == int(golden[f"reproj_{thr:g}_counter"])
    assert quirk_counter(valid, counts) == counter


def test_oracle_filter_angle_matches_reference(golden):
    imgs, tracks = load_scene(golden)
    tracks = {k: t for k, t in tracks.items() if len(t.observations)}
    valid, counts, _ = OP.filter_angle(imgs, tracks, 1.0)
    exp = kept_obs(golden, "angle_")
    starts = np.concatenate([[0], np.cumsum(counts)])
    for j, (k, t) in enumerate(tracks.items()):
        np.testing.assert_array_equal(t.observations[valid[starts[j]:starts[j + 1]]], exp[k])


def test_oracle_filter_tri_angle_matches_reference(golden):
    imgs, tracks = load_scene(golden)
    removed = set(OP.filter_tri_angle(imgs, tracks, 1.5))
    assert set(tracks) - removed == set(int(k) for k in golden["tri_keys"])
    assert len(removed) == int(golden["tri_counter"])


@pytest.mark.parametrize("depths,f32", [(None, False), (np.ones(3), False), (np.ones(3), True)])
def test_normalize_reconstruction_matches_reference(golden, depths, f32):
    """f32: float32 depth maps (data_reader.py:132) -- the reference's log runs in float32 then."""
    imgs, tracks = load_scene(golden)
    if f32:
        for im in imgs:
            im.depths = np.asarray(im.depths).astype(np.float32)
    NormalizeReconstruction(imgs, tracks, depths)
    pre = "norm_" if depths is None else ("normdepth32_" if f32 else "normdepth_")
    np.testing.assert_allclose(np.stack([im.world2cam for im in imgs]), golden[pre + "w2c"], rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(np.stack([t.xyz for t in tracks.values()]), golden[pre + "xyz"], rtol=1e-13, atol=1e-12)


@pytest.fixture(scope="module")
def cams(golden_dir):
    with np.load(os.path.join(golden_dir, "camera_models_golden.npz")) as z:
        return dict(z)


@pytest.mark.parametrize("model", [0, 1, 7])
def test_oracle_img2cam_matches_reference(cams, model):
    prm = cams[f"m{model}_params"]
    np.testing.assert_array_equal(OP.img2cam(model, prm, cams[f"m{model}_xy"]), cams[f"m{model}_img2cam"])
    got32 = OP.img2cam(model, prm, cams[f"m{model}_xy32"])
    exp32 = cams[f"m{model}_img2cam32"]
    assert got32.dtype == exp32.dtype
    np.testing.assert_allclose(got32, exp32, rtol=1e-6)


@pytest.mark.parametrize("model", [2, 3, 4, 5, 6, 8, 9])
def test_oracle_undistort_inverts_reference_forward_model(cams, model):
    """cv2 is absent: the restated cv2.undistortPoints must invert the reference's own cam2img (golden) -- five
    fixed-point iterations converge on these mild distortions.  THIN_PRISM_FISHEYE (10) is excluded: the reference's
    img2cam passes its sx as cv2's (s1, s2) -- x-only r^2 and r^4 terms -- while its cam2img adds sx * r^2 to (x, y), so
    the reference's own pair is not mutually inverse (test_thin_prism_reference_pair_is_not_inverse)."""
    prm = cams[f"m{model}_params"]
    uv = OP.img2cam(model, prm, cams[f"m{model}_cam2img"])
    np.testing.assert_allclose(uv, cams[f"m{model}_uv"], atol=5e-7)


def test_quirk_counter_reads_the_next_tracks_slice():
    valid = np.array([True, True, False, True, True, True], bool)
    counts = np.array([2, 1, 3])
    # track 0 -> slice [2, 4) has a False -> counted; track 1 -> [3, 4) all True; track 2 -> [6, 9) empty
    assert quirk_counter(valid, counts) == 1


def test_thin_prism_reference_pair_is_not_inverse(cams):
    uv = OP.img2cam(10, cams["m10_params"], cams["m10_cam2img"])
    assert np.abs(uv - cams["m10_uv"]).max() > 1e-5  # the documented reference inconsistency
