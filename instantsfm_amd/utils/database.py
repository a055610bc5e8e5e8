"""COLMAP ``database.db`` on-disk format: the schema of ``instantsfm/utils/database.py:42-122``
and the blob conventions its reader relies on, plus a writer used to build test and benchmark databases.

Tables and columns are COLMAP's: ``cameras(camera_id, model, width, height, params BLOB f64, prior_focal_length)``,
``images(image_id, name, camera_id)``, ``keypoints(image_id, rows, cols, data BLOB f32 [rows, cols])``,
``matches(pair_id, rows, cols, data BLOB u32 [rows, 2])``, ``two_view_geometries(pair_id, rows, cols, data, config,
F, E, H, qvec, tvec)`` (F/E/H/qvec/tvec f64), ``feature_name(feature_name)`` and the unused ``descriptors`` /
``pose_priors``.  A pair id is ``min(id) * (2^31 - 1) + max(id)``; matches are stored with the smaller image id's
feature index first (database.py:125-135, 292-303).
"""
import sqlite3

import numpy as np

MAX_IMAGE_ID = 2 ** 31 - 1

_TABLES = {
    "cameras": "camera_id INTEGER PRIMARY KEY AUTOINCREMENT NOT NULL, model INTEGER NOT NULL, width INTEGER NOT NULL, "
               "height INTEGER NOT NULL, params BLOB, prior_focal_length INTEGER NOT NULL",
    "images": "image_id INTEGER PRIMARY KEY AUTOINCREMENT NOT NULL, name TEXT NOT NULL UNIQUE, camera_id INTEGER NOT NULL, "
              f"CONSTRAINT image_id_check CHECK(image_id >= 0 and image_id < {MAX_IMAGE_ID}), "
              "FOREIGN KEY(camera_id) REFERENCES cameras(camera_id)",
    "pose_priors": "image_id INTEGER PRIMARY KEY NOT NULL, position BLOB, coordinate_system INTEGER NOT NULL, "
                   "FOREIGN KEY(image_id) REFERENCES images(image_id) ON DELETE CASCADE",
    "keypoints": "image_id INTEGER PRIMARY KEY NOT NULL, rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB, "
                 "FOREIGN KEY(image_id) REFERENCES images(image_id) ON DELETE CASCADE",
    "descriptors": "image_id INTEGER PRIMARY KEY NOT NULL, rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB, "
                   "FOREIGN KEY(image_id) REFERENCES images(image_id) ON DELETE CASCADE",
    "matches": "pair_id INTEGER PRIMARY KEY NOT NULL, rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB",
    "two_view_geometries": "pair_id INTEGER PRIMARY KEY NOT NULL, rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB, "
                           "config INTEGER NOT NULL, F BLOB, E BLOB, H BLOB, qvec BLOB, tvec BLOB",
    "feature_name": "feature_name TEXT PRIMARY KEY NOT NULL",
}


def image_ids_to_pair_id(image_id1, image_id2):
    a, b = (image_id1, image_id2) if image_id1 <= image_id2 else (image_id2, image_id1)
    return a * MAX_IMAGE_ID + b


def pair_id_to_image_ids(pair_id):
    return pair_id // MAX_IMAGE_ID, pair_id % MAX_IMAGE_ID


def array_to_blob(array):
    return np.ascontiguousarray(array).tobytes()


def blob_to_array(blob, dtype, shape=(-1,)):
    return np.frombuffer(blob, dtype=dtype).reshape(*shape)


class COLMAPDatabase(sqlite3.Connection):
    """sqlite3 connection with the COLMAP schema helpers."""

    @staticmethod
    def connect(database_path):
        return sqlite3.connect(database_path, factory=COLMAPDatabase)

    def create_tables(self):
        self.executescript("; ".join(f"CREATE TABLE IF NOT EXISTS {t} ({cols})" for t, cols in _TABLES.items())
                           + "; CREATE UNIQUE INDEX IF NOT EXISTS index_name ON images(name)")

    def add_camera(self, model, width, height, params, prior_focal_length=False, camera_id=None):
        params = np.asarray(params, np.float64)
        cur = self.execute("INSERT INTO cameras VALUES (?, ?, ?, ?, ?, ?)",
                           (camera_id, int(model), int(width), int(height), array_to_blob(params),
                            int(prior_focal_length)))
        return cur.lastrowid

    def add_image(self, name, camera_id, image_id=None):
        cur = self.execute("INSERT INTO images VALUES (?, ?, ?)", (image_id, name, int(camera_id)))
        return cur.lastrowid

    def add_keypoints(self, image_id, keypoints):
        kp = np.asarray(keypoints, np.float32)
        assert kp.ndim == 2 and kp.shape[1] in (2, 4, 6)
        self.execute("INSERT INTO keypoints VALUES (?, ?, ?, ?)", (int(image_id),) + kp.shape + (array_to_blob(kp),))

    def _pair_blob(self, image_id1, image_id2, matches):
        m = np.asarray(matches)
        assert m.ndim == 2 and m.shape[1] == 2
        if image_id1 > image_id2:
            m = m[:, ::-1]
        m = np.ascontiguousarray(m, np.uint32)
        return image_ids_to_pair_id(image_id1, image_id2), m

    def add_matches(self, image_id1, image_id2, matches):
        pid, m = self._pair_blob(image_id1, image_id2, matches)
        self.execute("INSERT INTO matches VALUES (?, ?, ?, ?)", (pid,) + m.shape + (array_to_blob(m),))

    def add_null_matches(self, image_id1, image_id2):
        """A matches row whose data is NULL (the reader counts it as invalid, data_reader.py:66-68)."""
        self.execute("INSERT INTO matches VALUES (?, 0, 2, NULL)", (image_ids_to_pair_id(image_id1, image_id2),))

    def add_two_view_geometry(self, image_id1, image_id2, matches, F=np.eye(3), E=np.eye(3), H=np.eye(3),
                              qvec=np.array([1.0, 0.0, 0.0, 0.0]), tvec=np.zeros(3), config=2):
        pid, m = self._pair_blob(image_id1, image_id2, matches)
        blobs = [array_to_blob(np.asarray(x, np.float64)) for x in (F, E, H, qvec, tvec)]
        self.execute("INSERT INTO two_view_geometries VALUES (?, ?, ?, ?, ?, ?, ?, ?, ?, ?)",
                     (pid,) + m.shape + (array_to_blob(m), int(config), *blobs))

    def add_feature_name(self, feature_name):
        self.execute("INSERT INTO feature_name VALUES (?)", (feature_name,))
