"""COLMAP database reader and the track-establishment oracle against the reference's own outputs
(tests/golden/tracks_db*.npz: the reference's ReadColmapDatabase and TrackEngine on databases written by the build's
writer).  CPU only."""
import numpy as np
import pytest

from oracle import tracks as OT

import tracks_scene as TS


@pytest.mark.parametrize("name", TS.NAMES)
def test_read_colmap_database_matches_reference(name):
    g = TS.load(name)
    vg, cams, imgs, fname = TS.read(g, with_inliers=False)
    assert fname == str(g["feature_name"])
    np.testing.assert_array_equal([im.id for im in imgs], g["img_id"])
    np.testing.assert_array_equal([im.cam_id for im in imgs], g["img_cam"])
    np.testing.assert_array_equal([im.filename for im in imgs], g["img_name"])
    feats = [np.asarray(im.features).reshape(-1, 2) for im in imgs]
    assert all(f.dtype == np.float32 for f in feats if f.size)
    np.testing.assert_array_equal(np.concatenate([[0], np.cumsum([f.shape[0] for f in feats])]), g["feat_ptr"])
    np.testing.assert_array_equal(np.concatenate(feats), g["feats"])
    np.testing.assert_array_equal([c.id for c in cams], g["cam_id"])
    np.testing.assert_array_equal([c.model_id.value for c in cams], g["cam_model"])
    np.testing.assert_array_equal([[c.width, c.height] for c in cams], g["cam_wh"])
    np.testing.assert_array_equal(np.stack([c.params for c in cams]), g["cam_params"])
    np.testing.assert_array_equal([c.has_prior_focal_length for c in cams], g["cam_prior"])
    pairs = list(vg.image_pairs.items())
    np.testing.assert_array_equal([k for k, _ in pairs], g["pair_key"])
    np.testing.assert_array_equal([[p.image_id1, p.image_id2] for _, p in pairs], g["pair_ids"])
    np.testing.assert_array_equal([p.config.value for _, p in pairs], g["pair_config"])
    np.testing.assert_array_equal([p.is_valid for _, p in pairs], g["pair_valid"])
    np.testing.assert_array_equal(np.stack([np.stack([p.F, p.E, p.H]) for _, p in pairs]), g["pair_FEH"])
    np.testing.assert_array_equal(np.concatenate([[0], np.cumsum([len(p.matches) for _, p in pairs])]), g["pair_mptr"])
    np.testing.assert_array_equal(np.concatenate([p.matches for _, p in pairs]), g["pair_matches"])
    assert str(pairs[0][1].matches.dtype) == str(g["pair_mdtype"])


@pytest.mark.parametrize("name", TS.NAMES)
def test_track_oracle_matches_reference(name):
    g = TS.load(name)
    vg, cams, imgs, _ = TS.read(g)
    full, discarded = OT.establish_full_tracks(vg, imgs, TS.OPTS["thres_inconsistency"])
    assert discarded == int(g["discarded"])
    keys, ptr, obs = TS.flat(full)
    np.testing.assert_array_equal(keys, g["full_keys"])
    np.testing.assert_array_equal(ptr, g["full_ptr"])
    np.testing.assert_array_equal(obs, g["full_obs"])
    for i, im in enumerate(imgs):
        im.is_registered = bool(g["registered"][i])
    prob = OT.find_tracks_for_problem(full, imgs, TS.OPTS)
    keys, ptr, obs = TS.flat(prob)
    np.testing.assert_array_equal(keys, g["prob_keys"])
    np.testing.assert_array_equal(ptr, g["prob_ptr"])
    np.testing.assert_array_equal(obs, g["prob_obs"])


def test_union_find_root_depends_on_order():
    """The reference's root is order dependent (Union(x, y) hangs root(x) under root(y)); the oracle keeps that."""
    uf = OT.UnionFind()
    uf.Union(5, 1)
    uf.Union(3, 2)
    uf.Union(5, 3)
    assert uf.Find(1) == 2 and uf.Find(5) == 2
