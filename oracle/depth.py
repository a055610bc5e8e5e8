"""TEST INFRASTRUCTURE ONLY -- restatement of the reference's depth sampling, one pixel at a time in plain Python
floats, as the checker of ``instantsfm_amd.utils.depth_sample`` / ``controllers.data_reader.ReadDepthsIntoFeatures``.
Only tests/ may import it.  Pinned by ``tests/golden/depth_sample.npz`` (the reference's own functions, see
tools/gen_golden.py ``gen_depth``).

Follows ``instantsfm/utils/depth_sample.py:3-44`` and ``instantsfm/controllers/data_reader.py:122-134`` under the
numpy the reference pins (1.26.4): a float32 coordinate over the integer image width is computed in float64 there
(scalar-by-scalar promotion), which Python floats reproduce.
"""
import math

import numpy as np


def sample_one(depth_map, x, y, w, h, method="nearest"):
    """depth_sample.py:11-44 for one pixel -> (depth as float, available); IndexError where numpy would raise."""
    H, W = depth_map.shape
    x, y = float(x), float(y)
    xp, yp = x / w, y / h                                          # :13
    if xp < 0 or xp > 1 or yp < 0 or yp > 1:                       # :14-16
        return 0.0, False
    xc, yc = xp * W, yp * H                                        # :18

    def at(r, c):
        if not (0 <= r < H and 0 <= c < W):
            raise IndexError(f"({r}, {c}) outside a {H} x {W} depth map")
        return float(depth_map[r, c])

    if method == "nearest":                                        # :20-23
        d = at(int(yc), int(xc))
    else:                                                          # :24-40
        x0, y0 = math.floor(xc), math.floor(yc)
        x1, y1 = min(max(x0 + 1, 0), W - 1), min(max(y0 + 1, 0), H - 1)
        wx, wy = xc - x0, yc - y0
        d00, d01, d10, d11 = at(y0, x0), at(y1, x0), at(y0, x1), at(y1, x1)
        d = d00 * (1 - wx) * (1 - wy) + d10 * wx * (1 - wy) + d01 * (1 - wx) * wy + d11 * wx * wy
    return d, d > 0.0                                              # :42-43


def depths_into_features(depths, cam_wh, img_cam, feats_per_image):
    """data_reader.py:125-132: image i samples map i at each feature with its camera's (width, height)."""
    out = []
    for i, feats in enumerate(feats_per_image):
        w, h = cam_wh[img_cam[i]]
        out.append(np.array([sample_one(depths[i], f[0], f[1], int(w), int(h))[0] for f in np.asarray(feats)],
                            dtype=np.float32))
    return out
