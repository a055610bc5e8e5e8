"""Golden COLMAP databases (tools/gen_golden.py gen_tracks): regenerate the database with the build's writer and
read it with the build's reader."""
import ast
import os
import tempfile

import numpy as np

from instantsfm_amd.controllers.data_reader import ReadColmapDatabase
from instantsfm_amd.synth import assign_inliers, write_match_database

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ("tracks_db0", "tracks_db1")
OPTS = dict(thres_inconsistency=10.0, min_num_view_per_track=3, max_num_view_per_track=9)


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def read(g, with_inliers=True):
    kw = ast.literal_eval(str(g["db_args"]))
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "database.db")
        write_match_database(path, **kw)
        vg, cams, imgs, fname = ReadColmapDatabase(path)
    if with_inliers:
        assign_inliers(vg, seed=kw["seed"])
    return vg, cams, imgs, fname


def flat(tracks):
    keys = np.array([int(k) for k in tracks.keys()], dtype=np.int64)
    vals = [np.asarray(getattr(v, "observations", v)) for v in tracks.values()]
    ptr = np.concatenate([[0], np.cumsum([len(v) for v in vals])])
    obs = np.concatenate(vals).astype(np.int64) if vals else np.zeros((0, 2), np.int64)
    return keys, ptr, obs
