"""Oracle restatements of RetriangulateTracks' passes against the reference's own outputs
(tests/golden/retri_*.npz, tools/gen_golden.py gen_retri): Camera.cam2img for every model, FilterTracksByReprojection,
complete_tracks.  CPU only."""
import numpy as np
import pytest

from oracle import passes as OP
import retri_scene as RS


@pytest.mark.parametrize("model", list(range(11)))
def test_cam2img_matches_reference(golden_dir, model):
    g = np.load(f"{golden_dir}/camera_models_golden.npz")
    uv = g[f"m{model}_uv"]
    uvw = np.concatenate([uv, np.ones((uv.shape[0], 1))], 1)
    out = OP.cam2img(model, g[f"m{model}_params"], uvw)
    np.testing.assert_allclose(out, g[f"m{model}_cam2img"], rtol=1e-14, atol=1e-10)


@pytest.mark.parametrize("name", RS.NAMES)
@pytest.mark.parametrize("thr", [3.0, 0.8])
def test_filter_reproj_pixel_oracle(name, thr):
    g = RS.load(name)
    cameras, images, tracks, _ = RS.scene(g)
    valid, counts, counter, err = OP.filter_reproj_pixel(cameras, images, tracks, thr)
    starts = np.concatenate([[0], np.cumsum(counts)])
    for j, t in enumerate(tracks.values()):
        t.observations = t.observations[valid[starts[j]:starts[j + 1]]]
    keys, ptr, obs = RS.flat(tracks)
    np.testing.assert_array_equal(keys, g[f"filter_{thr:g}_keys"])
    np.testing.assert_array_equal(ptr, g[f"filter_{thr:g}_ptr"])
    np.testing.assert_array_equal(obs, g[f"filter_{thr:g}_obs"])
    assert counter == int(g[f"filter_{thr:g}_counter"])


@pytest.mark.parametrize("name", RS.NAMES)
def test_complete_tracks_oracle(name):
    g = RS.load(name)
    cameras, images, tracks, tracks_orig = RS.scene(g)
    obs, rows, passing, err = OP.complete_candidates(cameras, images, tracks, tracks_orig, 3.0)
    # no candidate sits within 1e-9 px of the threshold, so the mask is not a rounding accident
    assert np.min(np.abs(err - 3.0)) > 1e-9
    n = RS.apply_completion(tracks, obs, rows, passing)
    assert n == int(g["complete_num"])
    keys, ptr, o = RS.flat(tracks)
    np.testing.assert_array_equal(keys, g["complete_keys"])
    np.testing.assert_array_equal(ptr, g["complete_ptr"])
    np.testing.assert_array_equal(o, g["complete_obs"])
    assert str(g["complete_dtype"]) in ("int32", "int64")
