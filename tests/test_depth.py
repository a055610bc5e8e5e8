"""Depth-map input path (data_reader.py:122-144, depth_sample.py:3-44): the product's vectorized sampling and PNG
reader vs the reference's own outputs (tests/golden/depth_sample.npz, tools/gen_golden.py gen_depth) and vs the
per-pixel restatement in oracle/depth.py.  Bit-exact throughout (float32 outputs compared with array_equal)."""
import os
import struct
import types
import zlib

import numpy as np
import pytest

from instantsfm_amd.controllers.data_reader import ReadDepths, ReadDepthsIntoFeatures
from instantsfm_amd.utils.depth_sample import sample_depth_at_pixel, sample_depths
from instantsfm_amd.utils.png import read_png_gray
from oracle import depth as OD

GOLD = os.path.join(os.path.dirname(__file__), "golden", "depth_sample.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _split(g):
    p = g["feat_ptr"]
    return [g["feats"][p[i]:p[i + 1]] for i in range(len(p) - 1)]


def _scene(g):
    cams = [types.SimpleNamespace(width=int(w), height=int(h)) for w, h in g["cam_wh"]]
    imgs = [types.SimpleNamespace(id=i, cam_id=int(c), features=f.astype(np.float32))
            for i, (c, f) in enumerate(zip(g["img_cam"], _split(g)))]
    return cams, imgs


def _png(path, img, filters=(0, 1, 2, 3, 4)):
    """Minimal grayscale PNG encoder (8/16-bit), row r filtered with filters[r % len(filters)]."""
    img = np.asarray(img)
    depth = 16 if img.dtype == np.uint16 else 8
    bpp = depth // 8
    rows = img.astype(">u2").view(np.uint8) if depth == 16 else img.astype(np.uint8)
    rows = rows.reshape(img.shape[0], -1).astype(np.int64)
    out, prev = bytearray(), np.zeros(rows.shape[1], dtype=np.int64)
    for r, cur in enumerate(rows):
        ft = filters[r % len(filters)]
        a = np.concatenate([np.zeros(bpp, np.int64), cur[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int64), prev[:-bpp]])
        if ft == 0:
            pred = np.zeros_like(cur)
        elif ft == 1:
            pred = a
        elif ft == 2:
            pred = prev
        elif ft == 3:
            pred = (a + prev) >> 1
        else:
            p = a + prev - c
            pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - c)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
        out.append(ft)
        out += bytes(((cur - pred) & 255).astype(np.uint8))
        prev = cur

    def chunk(k, b):
        return struct.pack(">I", len(b)) + k + b + struct.pack(">I", zlib.crc32(k + b) & 0xFFFFFFFF)
    ihdr = struct.pack(">IIBBBBB", img.shape[1], img.shape[0], depth, 0, 0, 0, 0)
    z = zlib.compress(bytes(out))
    with open(path, "wb") as f:  # IDAT split in two chunks: the reader must concatenate them
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", z[:len(z) // 2])
                + chunk(b"IDAT", z[len(z) // 2:]) + chunk(b"IEND", b""))


def test_oracle_matches_reference_golden(gold):
    """The restatement reproduces the reference's ReadDepthsIntoFeatures and bilinear samples exactly."""
    near = OD.depths_into_features(gold["ref_maps"], gold["cam_wh"], gold["img_cam"], _split(gold))
    assert np.array_equal(np.concatenate(near), gold["nearest"])
    bil = []
    for i, f in enumerate(_split(gold)):
        w, h = gold["cam_wh"][gold["img_cam"][i]]
        bil += [OD.sample_one(gold["ref_maps"][i], x, y, int(w), int(h), "bilinear")[0] for x, y in f]
    assert np.array_equal(np.array(bil), gold["bilinear"])
    assert np.array_equal(gold["ref_maps"], gold["maps_u16"].astype(np.float32) / 1000.0)


def test_read_depths_into_features_matches_reference(gold):
    cams, imgs = _scene(gold)
    maps = ReadDepthsIntoFeatures("", cams, imgs, depths=gold["ref_maps"])
    assert maps is gold["ref_maps"]
    got = np.concatenate([im.depths for im in imgs])
    assert got.dtype == np.float32 and np.array_equal(got, gold["nearest"])
    assert (got == 0).sum() > 0 and (got > 0).sum() > 0  # both invalid maps pixels and outside features present


def test_bilinear_and_scalar_api_match_reference(gold):
    feats = _split(gold)
    got, avail = [], []
    for i, f in enumerate(feats):
        w, h = gold["cam_wh"][gold["img_cam"][i]]
        d, a = sample_depths(gold["ref_maps"][i], f.astype(np.float32), int(w), int(h), method="bilinear")
        got.append(d)
        avail.append(a)
    assert np.array_equal(np.concatenate(got), gold["bilinear"])
    assert np.array_equal(np.concatenate(avail), gold["bilinear_avail"])
    w, h = gold["cam_wh"][0]
    for x, y in feats[0][-8:]:  # the edge cases, one call each through the drop-in scalar API
        for m in ("nearest", "bilinear"):
            d, a = sample_depth_at_pixel(gold["ref_maps"][0], np.array([x, y], np.float32), int(w), int(h), m)
            do, ao = OD.sample_one(gold["ref_maps"][0], x, y, int(w), int(h), m)
            assert d == do and a == ao and isinstance(a, bool)


def test_border_pixel_raises_like_the_reference(gold):
    it = iter(gold["border_raises"])
    for m in ("nearest", "bilinear"):
        for x, y in ((640.0, 10.0), (10.0, 480.0)):
            expect = bool(next(it))
            assert expect
            with pytest.raises(IndexError):
                sample_depth_at_pixel(gold["ref_maps"][0], np.array([x, y]), 640, 480, method=m)
            with pytest.raises(IndexError):
                OD.sample_one(gold["ref_maps"][0], x, y, 640, 480, m)


def test_random_against_oracle():
    rng = np.random.default_rng(3)
    m = rng.random((37, 53)).astype(np.float32) - 0.1
    f = np.stack([rng.uniform(-20, 700, 3000), rng.uniform(-20, 500, 3000)], 1).astype(np.float32)
    f = f[(f[:, 0] != 640) & (f[:, 1] != 480)]
    for meth in ("nearest", "bilinear"):
        d, a = sample_depths(m, f, 640, 480, meth)
        ref = [OD.sample_one(m, x, y, 640, 480, meth) for x, y in f]
        assert np.array_equal(d.astype(np.float64), np.array([r[0] for r in ref]))
        assert np.array_equal(a, np.array([r[1] for r in ref]))
    d, a = sample_depths(m, np.zeros((0, 2)), 640, 480)
    assert d.shape == (0,) and a.shape == (0,)


@pytest.mark.parametrize("filters", [(0,), (1,), (2,), (3,), (4,), (0, 1, 2, 3, 4)])
@pytest.mark.parametrize("dtype", [np.uint16, np.uint8])
def test_png_reader_round_trip(tmp_path, filters, dtype):
    rng = np.random.default_rng(11)
    img = rng.integers(0, np.iinfo(dtype).max + 1, size=(19, 23)).astype(dtype)
    img[:, 5] = img[:, 4]  # smooth runs exercise the predictors' ties
    p = str(tmp_path / "d.png")
    _png(p, img, filters)
    got = read_png_gray(p)
    assert got.dtype == dtype and np.array_equal(got, img)


def test_png_reader_rejects_colour(tmp_path):
    p = tmp_path / "c.png"
    ihdr = struct.pack(">IIBBBBB", 2, 2, 8, 2, 0, 0, 0)
    with open(p, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + struct.pack(">I", 13) + b"IHDR" + ihdr + b"\0\0\0\0"
                + struct.pack(">I", 0) + b"IDAT" + b"\0\0\0\0")
    with pytest.raises(ValueError):
        read_png_gray(str(p))


def test_read_depths_from_png_directory(tmp_path, gold):
    """ReadDepths + ReadDepthsIntoFeatures from files: the maps written as 16-bit PNGs in the reference's layout
    (sorted *.png, millimetres) give the reference's maps and feature depths."""
    for i, m in enumerate(gold["maps_u16"]):
        _png(str(tmp_path / f"{i:06d}.png"), m)
    (tmp_path / "notes.txt").write_text("ignored")
    maps = ReadDepths(str(tmp_path))
    assert maps.dtype == np.float32 and np.array_equal(maps, gold["ref_maps"])
    cams, imgs = _scene(gold)
    ReadDepthsIntoFeatures(str(tmp_path), cams, imgs)
    assert np.array_equal(np.concatenate([im.depths for im in imgs]), gold["nearest"])
