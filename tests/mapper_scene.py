"""Small config-5-shaped mapper scenes shared by the CPU and GPU mapper tests: a seeded COLMAP database read back
through ReadColmapDatabase, with the stand-in for the out-of-scope stages applied."""
import contextlib
import io

from instantsfm_amd.controllers.config import Config
from instantsfm_amd.controllers.data_reader import ReadColmapDatabase
from instantsfm_amd.synth import stand_in_rotation_averaging, write_mapper_database

SMALL = dict(n_images=40, n_points=3000, track_len=6, window=6, reach=2, images_per_camera=10, distractors=50)


def make_db(path, seed=0, **kw):
    return write_mapper_database(str(path), seed=seed, **dict(SMALL, **kw))


def load(path, scene, seed=0):
    """A fresh scene (view graph, cameras, images) from the database, ready for SolveGlobalMapper."""
    with contextlib.redirect_stdout(io.StringIO()):
        vg, cams, ims, fn = ReadColmapDatabase(str(path))
    stand_in_rotation_averaging(vg, ims, scene, seed=seed)
    return vg, cams, ims, Config.for_ba_half(fn)
