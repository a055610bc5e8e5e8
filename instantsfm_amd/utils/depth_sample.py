"""Depth sampling at feature pixels -- drop-in for ``instantsfm/utils/depth_sample.py:3-44``
(``sample_depth_at_pixel``), plus ``sample_depths``, the same arithmetic over all features of an image at once, which
``ReadDepthsIntoFeatures`` (controllers/data_reader.py) uses instead of the reference's per-feature Python loop
(data_reader.py:128-131).

Arithmetic follows the reference under the numpy it pins (1.26.4, pyproject.toml:17).  There a float32 feature
coordinate divided by the camera's integer width is a scalar-by-scalar operation, which numpy 1.x promotes with
``promote_types(float32, int64) = float64``; the coordinates are therefore converted to float64 first here (under
numpy 2's NEP 50 rules the reference's own expression would stay float32).  Per pixel (x, y) of an image w x h and a
depth map H x W:
  outside: x / w or y / h outside [0, 1]            -> depth 0.0, not available
  nearest: map[int(y / h * H), int(x / w * W)]      (truncation)
  bilinear: x0 = floor(x / w * W), x1 = min(x0 + 1, W - 1) (same in y), weights from the fractional parts, the four
            taps summed in the reference's order (d00 (1-wx)(1-wy) + d10 wx (1-wy) + d01 (1-wx) wy + d11 wx wy)
  available = depth > 0.
A pixel exactly on the right or bottom border (x == w) passes the range check and then indexes column W of the map:
the reference raises IndexError there, and so does this module.
"""
import numpy as np

__all__ = ["sample_depth_at_pixel", "sample_depths"]


def _taps(idx, n, axis):
    if idx.size and (idx.min() < 0 or idx.max() >= n):
        bad = idx[(idx < 0) | (idx >= n)][0]
        raise IndexError(f"index {bad} is out of bounds for axis {axis} with size {n}")
    return idx


def _sample(depth_map, pixels, w, h, method):
    depth_map = np.asarray(depth_map)
    if depth_map.ndim != 2:
        raise ValueError(f"depth_map must be [H, W], got shape {depth_map.shape}")
    H, W = depth_map.shape
    p = np.asarray(pixels, dtype=np.float64).reshape(-1, 2)
    xp, yp = p[:, 0] / w, p[:, 1] / h
    inside = ~((xp < 0) | (xp > 1) | (yp < 0) | (yp > 1))
    xc, yc = xp[inside] * W, yp[inside] * H
    if method == "nearest":
        out = np.zeros(len(p), dtype=depth_map.dtype if depth_map.dtype.kind == "f" else np.float64)
        xi = _taps(xc.astype(np.int64), W, 1)
        yi = _taps(yc.astype(np.int64), H, 0)
        out[inside] = depth_map[yi, xi]
    else:  # bilinear (the reference's `else` branch takes any other method string)
        out = np.zeros(len(p), dtype=np.float64)
        x0 = _taps(np.floor(xc).astype(np.int64), W, 1)
        y0 = _taps(np.floor(yc).astype(np.int64), H, 0)
        x1 = np.clip(x0 + 1, 0, W - 1)
        y1 = np.clip(y0 + 1, 0, H - 1)
        wx, wy = xc - x0, yc - y0
        d00 = depth_map[y0, x0].astype(np.float64)
        d01 = depth_map[y1, x0].astype(np.float64)
        d10 = depth_map[y0, x1].astype(np.float64)
        d11 = depth_map[y1, x1].astype(np.float64)
        out[inside] = d00 * (1 - wx) * (1 - wy) + d10 * wx * (1 - wy) + d01 * (1 - wx) * wy + d11 * wx * wy
    return out, inside


def sample_depths(depth_map, pixels, w, h, method="nearest"):
    """Depth at every row of ``pixels`` ([N, 2] x, y in image pixels) of an image ``w`` x ``h``.

    Returns ``(depth, available)``: ``depth`` [N] in the map's float dtype for ``nearest`` (0 outside the image),
    float64 for ``bilinear``; ``available`` [N] bool = depth > 0.  Raises IndexError where the reference does."""
    out, _ = _sample(depth_map, pixels, w, h, method)
    return out, out > 0.0


def sample_depth_at_pixel(depth_map, pixel_coords, w, h, method="nearest"):
    """depth_sample.py:3-44: ``(depth, available)`` at one pixel; ``(0.0, False)`` outside the image."""
    out, inside = _sample(depth_map, pixel_coords, w, h, method)
    if not inside[0]:
        return 0.0, False
    return out[0], bool(out[0] > 0.0)
