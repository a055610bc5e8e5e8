"""Device wrappers of the between-round passes (include/insfm_passes.h): numpy in, numpy out, HIP kernels in between.

torch only provides device memory and the current stream; there is no CPU path (``_require_gpu`` raises without a
ROCm GPU, ``_capi.load`` without the built library).
"""
import ctypes

import numpy as np
import torch

from . import _capi
from .engine import _require_gpu


def _dev(a, dev, dtype=None):
    # (np.require: C-contiguous and writable -- a read-only input is copied, torch.from_numpy needs a writable array)
    t = torch.from_numpy(np.require(a if dtype is None else np.asarray(a, dtype=dtype), requirements=("C", "W")))
    return t.to(dev, non_blocking=False).contiguous()


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    with torch.cuda.device(dev):
        return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise _capi.BAError(rc, what)


def undistort(xy, feat_cam, cam_model, cam_params, device="cuda:0"):
    """Rays [n,3] of features ``xy`` [n,2] (float32 or float64) through their cameras (Camera.img2cam + normalize)."""
    dev = _require_gpu(device)
    L = _capi.load()
    xy = np.asarray(xy)
    f32 = xy.dtype == np.float32
    xy = xy.astype(np.float32 if f32 else np.float64, copy=False).reshape(-1, 2)
    n = xy.shape[0]
    out = torch.empty((n, 3), dtype=torch.float64, device=dev)
    if n == 0:
        return out.cpu().numpy()
    params = np.zeros((len(cam_model), 12))
    for i, p in enumerate(cam_params):
        p = np.asarray(p, dtype=np.float64).reshape(-1)
        params[i, :p.size] = p
    args = [_dev(xy, dev), _dev(feat_cam, dev, np.int32), _dev(cam_model, dev, np.int32), _dev(params, dev)]
    _check(L.insfm_undistort(n, _p(args[0]), int(f32), _p(args[1]), _p(args[2]), _p(args[3]), _p(out), _stream(dev)),
           "insfm_undistort")
    return out.cpu().numpy()


def _obs_args(dev, obs_img, obs_track, obs_ray, world2cam, track_xyz, rays):
    return [_dev(obs_img, dev, np.int32), _dev(obs_track, dev, np.int32), _dev(obs_ray, dev, np.int64),
            _dev(np.asarray(world2cam, dtype=np.float64).reshape(-1, 16), dev), _dev(track_xyz, dev, np.float64),
            _dev(rays, dev, np.float64)]


def filter_reproj_normalized(obs_img, obs_track, obs_ray, world2cam, track_xyz, rays, max_err, device="cuda:0",
                             with_err=False):
    dev = _require_gpu(device)
    L = _capi.load()
    n = int(np.asarray(obs_img).shape[0])
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.float64, device=dev) if with_err else None
    if n:
        a = _obs_args(dev, obs_img, obs_track, obs_ray, world2cam, track_xyz, rays)
        _check(L.insfm_filter_reproj_normalized(n, *[_p(t) for t in a], float(max_err), _p(valid), _p(err), _stream(dev)),
               "insfm_filter_reproj_normalized")
    v = valid.cpu().numpy().astype(bool)
    return (v, err.cpu().numpy()) if with_err else v


def filter_angle(obs_img, obs_track, obs_ray, world2cam, track_xyz, rays, cos_thres, device="cuda:0"):
    dev = _require_gpu(device)
    L = _capi.load()
    n = int(np.asarray(obs_img).shape[0])
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    if n:
        a = _obs_args(dev, obs_img, obs_track, obs_ray, world2cam, track_xyz, rays)
        _check(L.insfm_filter_angle(n, *[_p(t) for t in a], float(cos_thres), _p(valid), _stream(dev)), "insfm_filter_angle")
    return valid.cpu().numpy().astype(bool)


def filter_tri_angle(track_ptr, obs_img, centers, track_xyz, cos_thres, device="cuda:0"):
    dev = _require_gpu(device)
    L = _capi.load()
    nt = int(np.asarray(track_ptr).shape[0]) - 1
    remove = torch.zeros(max(nt, 0), dtype=torch.uint8, device=dev)
    if nt > 0:
        a = [_dev(track_ptr, dev, np.int64), _dev(obs_img, dev, np.int32) if len(obs_img) else torch.zeros(1, dtype=torch.int32, device=dev),
             _dev(centers, dev, np.float64), _dev(track_xyz, dev, np.float64)]
        _check(L.insfm_filter_tri_angle(nt, *[_p(t) for t in a], float(cos_thres), _p(remove), _stream(dev)),
               "insfm_filter_tri_angle")
    return remove.cpu().numpy().astype(bool)


def _feats(feats, dev):
    """Concatenated features [F,2]: float32 stays float32 (the database's keypoint type), anything else float64."""
    a = np.asarray(feats)
    f32 = a.dtype == np.float32
    a = a.astype(np.float32 if f32 else np.float64, copy=False).reshape(-1, 2)
    if a.shape[0] == 0:
        a = np.zeros((1, 2), a.dtype)
    return _dev(a, dev), int(f32)


def filter_reproj_pixel(obs_img, obs_track, obs_feat, feats, img_cam, cam_model, cam_params, world2cam, track_xyz,
                        max_err, device="cuda:0", with_err=False):
    """FilterTracksByReprojection's per-observation test (track_filter.py:68-113) on the GPU."""
    dev = _require_gpu(device)
    L = _capi.load()
    n = int(np.asarray(obs_img).shape[0])
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.float64, device=dev) if with_err else None
    if n:
        params = np.zeros((len(cam_model), 12))
        for i, p in enumerate(cam_params):
            p = np.asarray(p, dtype=np.float64).reshape(-1)
            params[i, :p.size] = p
        ft, f32 = _feats(feats, dev)
        a = [_dev(obs_img, dev, np.int32), _dev(obs_track, dev, np.int32), _dev(obs_feat, dev, np.int64)]
        b = [_dev(img_cam, dev, np.int32), _dev(cam_model, dev, np.int32), _dev(params, dev),
             _dev(np.asarray(world2cam, dtype=np.float64).reshape(-1, 16), dev), _dev(track_xyz, dev, np.float64)]
        _check(L.insfm_filter_reproj_pixel(n, *[_p(t) for t in a], _p(ft), f32, *[_p(t) for t in b], float(max_err),
                                           _p(valid), _p(err), _stream(dev)), "insfm_filter_reproj_pixel")
    v = valid.cpu().numpy().astype(bool)
    return (v, err.cpu().numpy()) if with_err else v


def reproj_candidates(cam_model, cand_img, cand_track, cand_feat, feats, image_rows, image_pps, track_xyz, max_err,
                      device="cuda:0", with_err=False):
    """complete_tracks' candidate test (track_retriangulation.py:58-90) on the GPU."""
    dev = _require_gpu(device)
    L = _capi.load()
    n = int(np.asarray(cand_img).shape[0])
    valid = torch.zeros(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.float64, device=dev) if with_err else None
    ft, f32 = _feats(feats, dev)
    a = [_dev(cand_img, dev, np.int32), _dev(cand_track, dev, np.int32), _dev(cand_feat, dev, np.int64)]
    b = [_dev(image_rows, dev, np.float64), _dev(image_pps, dev, np.float64), _dev(track_xyz, dev, np.float64)]
    _check(L.insfm_reproj_candidates(n, int(cam_model), *[_p(t) for t in a], _p(ft), f32, *[_p(t) for t in b],
                                     float(max_err), _p(valid), _p(err), _stream(dev)), "insfm_reproj_candidates")
    v = valid.cpu().numpy().astype(bool)
    return (v, err.cpu().numpy()) if with_err else v
