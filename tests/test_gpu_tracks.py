"""Track establishment on the HIP path (csrc/tracks.hip via TrackEngine) vs the reference's own outputs
(tests/golden/tracks_db*.npz) and the CPU restatement (oracle/tracks.py).  Needs an MI355X."""
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from instantsfm_amd.processors.track_establishment import TrackEngine  # noqa: E402
from instantsfm_amd.scene.defs import ImagePair, ViewGraph  # noqa: E402
from instantsfm_amd.synth import assign_inliers, write_match_database  # noqa: E402
from instantsfm_amd.controllers.data_reader import ReadColmapDatabase  # noqa: E402
from oracle import tracks as OT  # noqa: E402

import tracks_scene as TS  # noqa: E402


def _discarded(out):
    return int(re.search(r"Discarded (\d+) features", out).group(1))


@pytest.mark.parametrize("name", TS.NAMES)
def test_track_engine_matches_reference(name, capsys):
    g = TS.load(name)
    vg, cams, imgs, _ = TS.read(g)
    eng = TrackEngine(vg, imgs)
    capsys.readouterr()
    full = eng.EstablishFullTracks(TS.OPTS)
    assert _discarded(capsys.readouterr().out) == int(g["discarded"])
    keys, ptr, obs = TS.flat(full)
    np.testing.assert_array_equal(keys, g["full_keys"])
    np.testing.assert_array_equal(ptr, g["full_ptr"])
    np.testing.assert_array_equal(obs, g["full_obs"])
    assert str(next(iter(full.values())).dtype) == str(g["full_dtype"])
    for i, im in enumerate(imgs):
        im.is_registered = bool(g["registered"][i])
    prob = eng.FindTracksForProblem(full, TS.OPTS)
    keys, ptr, obs = TS.flat(prob)
    np.testing.assert_array_equal(keys, g["prob_keys"])
    np.testing.assert_array_equal(ptr, g["prob_ptr"])
    np.testing.assert_array_equal(obs, g["prob_obs"])


def _vs_oracle(vg, imgs, capsys, thres=10.0):
    capsys.readouterr()
    full = TrackEngine(vg, imgs).EstablishFullTracks(dict(TS.OPTS, thres_inconsistency=thres))
    disc = _discarded(capsys.readouterr().out)
    ofull, odisc = OT.establish_full_tracks(vg, imgs, thres)
    assert disc == odisc
    for a, b in zip(TS.flat(full), TS.flat(ofull)):
        np.testing.assert_array_equal(a, b)
    return full


@pytest.mark.parametrize("seed,kw", [
    (2, dict(n_images=40, n_points=5000, wrong_frac=0.02)),
    (3, dict(n_images=20, n_points=3000, wrong_frac=0.4, dup_frac=0.2)),   # wrong matches chain tracks together
    (4, dict(n_images=64, n_points=12000, track_len=8, window=7, dup_frac=0.1, distractors=200)),
])
def test_track_engine_vs_oracle(tmp_path, capsys, seed, kw):
    path = str(tmp_path / "database.db")
    write_match_database(path, seed=seed, **kw)
    vg, cams, imgs, _ = ReadColmapDatabase(path)
    assign_inliers(vg, seed=seed, frac=0.85)
    full = _vs_oracle(vg, imgs, capsys)
    assert len(full) > 0


def test_track_engine_float64_features_and_thresholds(tmp_path, capsys):
    path = str(tmp_path / "database.db")
    write_match_database(path, seed=5, n_images=24, n_points=2000, wrong_frac=0.2, dup_frac=0.3)
    vg, cams, imgs, _ = ReadColmapDatabase(path)
    assign_inliers(vg, seed=5)
    for thres in (0.5, 2.0, 50.0):
        _vs_oracle(vg, imgs, capsys, thres)
    for im in imgs:
        im.features = np.asarray(im.features, dtype=np.float64).reshape(-1, 2) * 1.000001
    _vs_oracle(vg, imgs, capsys, 2.0)


def test_track_engine_no_matches(capsys):
    vg = ViewGraph()
    vg.image_pairs = {1: ImagePair(0, 1, is_valid=False), 2: ImagePair(0, 2)}
    vg.image_pairs[1].matches = np.zeros((5, 2), np.uint32)
    vg.image_pairs[1].inliers = np.arange(5)
    vg.image_pairs[2].matches = np.zeros((0, 2), np.uint32)

    class Im:
        features = np.zeros((3, 2), np.float32)
    assert TrackEngine(vg, [Im(), Im(), Im()]).EstablishFullTracks(TS.OPTS) == {}


def test_track_engine_long_chain(capsys):
    """One component built from a long chain of matches (a worst case for the per-component replay)."""
    rng = np.random.default_rng(9)
    n_img, nf = 50, 400

    class Im:
        def __init__(self):
            self.features = rng.uniform(0, 1000, (nf, 2)).astype(np.float32)
    imgs = [Im() for _ in range(n_img)]
    vg = ViewGraph()
    for i in range(n_img - 1):
        p = ImagePair(i, i + 1)
        perm = rng.permutation(nf)
        p.matches = np.stack([np.arange(nf), perm], 1).astype(np.uint32)
        p.inliers = np.arange(nf)
        vg.image_pairs[i * 1000 + i + 1] = p
    p = ImagePair(0, n_img - 1)  # close the loop with shifted features: everything merges
    p.matches = np.stack([np.arange(nf), (np.arange(nf) + 1) % nf], 1).astype(np.uint32)
    p.inliers = np.arange(nf)
    vg.image_pairs[n_img - 1] = p
    _vs_oracle(vg, imgs, capsys)
