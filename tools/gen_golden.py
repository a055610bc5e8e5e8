#!/usr/bin/env python3
"""Generate golden vectors from the reference itself (run in the build container only).

The reference (``/root/reference``) imports five modules that are absent from this image
(pyceres, cv2, pypose@bae, bae.*).  Following SURVEY.md Appendix B, this script writes tiny shim
modules into a temporary directory OUTSIDE the repository, imports the reference's own
``instantsfm.utils.cost_function`` / ``instantsfm.processors.bundle_adjustment`` through them and
records:

* ``projection_golden.npz`` -- ``reproject_funcs[m]`` (cost_function.py:32-208) for the 9 implemented
  models, 256 random observations each (seed 0).  The only restated piece inside is
  ``bae.utils.ba.rotate_quat`` (R(q) p + t, pypose [t, q_xyzw] layout).
* ``gp_packing_<name>.npz`` -- what ``TorchGP.Optimize`` (global_positioning.py:85-170) hands to the LM: rays,
  indices, calibration flags, initial positions / points / scales, the fixed-scale set, the LM options, and the
  scene mutations (dropped tracks, unregistered images), together with the scene that produced them.
* ``packing_<name>.npz`` -- what ``TorchBA.Solve`` (bundle_adjustment.py:66-126) hands to the LM:
  ``points_2d``, ``camera_indices``, ``point_indices``, ``camera_pps`` and the model's ``pose`` /
  ``points_3d`` parameters, together with the scene that produced them.  The LM shim raises after
  capturing its input, so nothing past bundle_adjustment.py:132 runs.

Only data leaves this script: no reference source is copied into the repository.
Usage:  python tools/gen_golden.py [--out tests/golden]
"""
import argparse
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

import numpy as np  # noqa: E402
import torch  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


class _Captured(Exception):
    pass


def install_shims():
    """Register in-memory shim modules for the absent dependencies (Appendix B)."""
    from scipy.spatial.transform import Rotation

    def mod(name):
        m = types.ModuleType(name)
        sys.modules[name] = m
        return m

    pyceres = mod("pyceres")

    class CostFunction:  # pragma: no cover - only subclassed at import time
        def __init__(self, *a, **k):
            pass
    pyceres.CostFunction = CostFunction
    mod("cv2")

    # --- bae ---------------------------------------------------------------------------------
    bae = mod("bae")
    bae_utils = mod("bae.utils")
    bae_ba = mod("bae.utils.ba")
    bae_solvers = mod("bae.utils.pysolvers")
    bae_optim = mod("bae.optim")
    bae_autograd = mod("bae.autograd")
    bae_fn = mod("bae.autograd.function")
    bae.utils, bae.optim, bae.autograd = bae_utils, bae_optim, bae_autograd
    bae_utils.ba, bae_utils.pysolvers, bae_autograd.function = bae_ba, bae_solvers, bae_fn

    def rotate_quat(points, pose):
        t, qv, w = pose[..., 0:3], pose[..., 3:6], pose[..., 6:7]
        uv = torch.cross(qv, points, dim=-1)
        uuv = torch.cross(qv, uv, dim=-1)
        return points + 2.0 * (w * uv + uuv) + t
    bae_ba.rotate_quat = rotate_quat
    bae_fn.TrackingTensor = lambda x: x
    bae_fn.map_transform = lambda f: f

    class PCG:
        def __init__(self, tol=None, **kw):
            self.tol = tol
    bae_solvers.PCG = PCG

    class LM:
        last = None

        def __init__(self, model, **kwargs):
            self.model, self.kwargs = model, kwargs

        def step(self, inp):
            LM.last = (self.model, self.kwargs, inp)
            raise _Captured()
    bae_optim.LM = LM

    # --- pypose ------------------------------------------------------------------------------
    pp = mod("pypose")
    pp_optim = mod("pypose.optim")
    pp_kernel = mod("pypose.optim.kernel")
    pp_strategy = mod("pypose.optim.strategy")
    pp.optim, pp_optim.kernel, pp_optim.strategy = pp_optim, pp_kernel, pp_strategy

    class _SE3:
        def __init__(self, data):
            self.data = torch.as_tensor(data, dtype=torch.float64)

        def tensor(self):
            return self.data

        def matrix(self):
            d = self.data.detach().cpu().numpy().reshape(-1, 7)
            out = np.tile(np.eye(4), (d.shape[0], 1, 1))
            out[:, :3, :3] = Rotation.from_quat(d[:, 3:7]).as_matrix()
            out[:, :3, 3] = d[:, :3]
            return torch.from_numpy(out.reshape(self.data.shape[:-1] + (4, 4)))

    def mat2SE3(m):
        m = np.asarray(m, dtype=np.float64)
        q = Rotation.from_matrix(m[:3, :3]).as_quat()
        return _SE3(np.concatenate([m[:3, 3], q]))
    pp.mat2SE3 = mat2SE3
    pp.identity_SE3 = lambda: _SE3([0, 0, 0, 0, 0, 0, 1.0])
    pp.SE3 = _SE3

    class _Rec:
        def __init__(self, *a, **k):
            self.args, self.kwargs = a, k
    pp_strategy.TrustRegion = _Rec
    pp_kernel.Huber = _Rec
    pp_kernel.Cauchy = _Rec
    return LM


def gen_projection(out_dir):
    from instantsfm.utils.cost_function import reproject_funcs
    sys.path.insert(0, REPO)
    from oracle.projection_ref import N_INTR
    rng = np.random.default_rng(0)
    res = {}
    n = 256
    base = {0: [900.0], 1: [900.0, 950.0], 2: [900.0, -0.05], 3: [900.0, -0.05, 0.01],
            4: [900.0, 950.0, -0.05, 0.01, 1e-3, -2e-3], 5: [900.0, 950.0, -0.02, 0.004, -1e-3, 5e-4],
            6: [900.0, 950.0, -0.05, 0.01, 1e-3, -2e-3, 3e-3, 0.02, -0.004, 6e-4],
            8: [900.0, -0.03], 9: [900.0, -0.03, 0.006]}
    for m, ni in N_INTR.items():
        q = rng.normal(size=(n, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        t = rng.normal(0, 0.5, (n, 3))
        intr = np.asarray(base[m])[None, :] * (1 + rng.normal(0, 0.1, (n, ni)))
        cam = np.concatenate([t, q, intr], axis=1)
        # points in front of the camera: p = R^T (pc - t) with pc at depth 2..10
        from scipy.spatial.transform import Rotation
        R = Rotation.from_quat(q).as_matrix()
        pc = np.stack([rng.uniform(-1.5, 1.5, n), rng.uniform(-1.2, 1.2, n), np.ones(n)], 1) * rng.uniform(2, 10, (n, 1))
        X = np.einsum('nji,nj->ni', R, pc - t)
        ppt = rng.uniform(200, 1200, (n, 2))
        out = reproject_funcs[m](torch.from_numpy(X), torch.from_numpy(cam), torch.from_numpy(ppt))
        res[f"m{m}_points"] = X
        res[f"m{m}_cam"] = cam
        res[f"m{m}_pp"] = ppt
        res[f"m{m}_out"] = out.numpy()
    for m in (7, 10):  # FOV / THIN_PRISM_FISHEYE raise in the reference
        try:
            reproject_funcs[m](torch.zeros(1, 3), torch.zeros(1, 19), torch.zeros(1, 2))
            res[f"m{m}_raises"] = np.array(0)
        except NotImplementedError:
            res[f"m{m}_raises"] = np.array(1)
    np.savez_compressed(os.path.join(out_dir, "projection_golden.npz"), **res)
    print("projection_golden.npz", len(res), "arrays")


def _scene_arrays(cameras, images, tracks, model):
    """Serialise a reference-class scene into plain arrays (inputs of the fixture)."""
    keys = list(tracks.keys())
    obs = [np.asarray(tracks[k].observations, dtype=np.int64).reshape(-1, 2) for k in keys]
    feats = [np.asarray(im.features, dtype=np.float64).reshape(-1, 2) for im in images]
    return dict(
        model=np.array(model),
        cam_params=np.stack([np.asarray(c.params, dtype=np.float64) for c in cameras]),
        img_cam_id=np.array([im.cam_id for im in images]),
        img_registered=np.array([im.is_registered for im in images]),
        img_world2cam=np.stack([np.asarray(im.world2cam, dtype=np.float64) for im in images]),
        img_feat_ptr=np.concatenate([[0], np.cumsum([len(f) for f in feats])]),
        img_feats=np.concatenate(feats) if feats else np.zeros((0, 2)),
        track_keys=np.array(keys, dtype=np.int64),
        track_xyz=np.stack([np.asarray(tracks[k].xyz, dtype=np.float64) for k in keys]),
        track_obs_ptr=np.concatenate([[0], np.cumsum([len(o) for o in obs])]),
        track_obs=np.concatenate(obs) if obs else np.zeros((0, 2), np.int64),
    )


def _run_solve(LM, cameras, images, tracks, opts):
    from instantsfm.processors.bundle_adjustment import TorchBA
    try:
        TorchBA(device="cpu").Solve(cameras, images, tracks, opts)
    except _Captured:
        pass
    model, kwargs, inp = LM.last
    return dict(
        out_points_2d=inp["points_2d"].numpy(),
        out_camera_indices=inp["camera_indices"].numpy(),
        out_point_indices=inp["point_indices"].numpy(),
        out_camera_pps=inp["camera_pps"].numpy(),
        out_pose=model.pose.detach().numpy(),
        out_points_3d=model.points_3d.detach().numpy(),
        out_optimize_poses=np.array(bool(model.pose.requires_grad)),
        out_reject=np.array(kwargs.get("reject", -1)),
    )


def gen_packing(out_dir, LM):
    from instantsfm.scene.defs import Camera, CameraModelId, Image, Track
    sys.path.insert(0, REPO)
    from instantsfm_amd.synth import make_config, full_params, quat_to_matrix
    opts = dict(optimize_poses=True, optimize_points=True, min_num_view_per_track=2, thres_loss_function=1.0,
                max_num_iterations=200, function_tolerance=5e-4)

    # (1) config-1 synthetic scene (20 cams / 2k points / 20k obs), SIMPLE_RADIAL
    prob = make_config(1, seed=0)
    cams, imgs, trks = [], [], {}
    C = prob.n_cams
    order = np.argsort(prob.cam_idx, kind="stable")
    counts = np.bincount(prob.cam_idx, minlength=C)
    starts = np.concatenate([[0], np.cumsum(counts)])
    feat_id = np.empty(prob.n_obs, np.int64)
    feat_id[order] = np.arange(prob.n_obs) - np.repeat(starts[:-1], counts)
    for c in range(C):
        cams.append(Camera(id=c, model_id=CameraModelId(prob.model), width=2000, height=1500,
                           params=list(full_params(prob.model, prob.cams_init[c, 7:], prob.pp[c]))))
        w2c = np.eye(4)
        w2c[:3, :3] = quat_to_matrix(prob.cams_init[c, 3:7])
        w2c[:3, 3] = prob.cams_init[c, :3]
        imgs.append(Image(id=c, cam_id=c, is_registered=True, world2cam=w2c,
                          features=prob.uv[order[starts[c]:starts[c + 1]]].copy()))
    ptr = np.concatenate([[0], np.cumsum(np.bincount(prob.pt_idx, minlength=prob.n_points))])
    pairs = np.stack([prob.cam_idx.astype(np.int64), feat_id], 1)
    for p in range(prob.n_points):
        trks[p] = Track(id=p, xyz=prob.points_init[p].copy(), observations=pairs[ptr[p]:ptr[p + 1]].copy())
    res = _scene_arrays(cams, imgs, trks, prob.model)
    res.update(_run_solve(LM, cams, imgs, trks, opts))
    np.savez_compressed(os.path.join(out_dir, "packing_config1.npz"), **res)
    print("packing_config1.npz", res["out_points_2d"].shape)

    # (2) hand-built edge cases, OPENCV (pp at columns 2,3): unregistered image, length-1 track,
    #     point behind a camera (z <= 0.1), two images sharing one camera, non-contiguous track keys
    rng = np.random.default_rng(1)
    model = CameraModelId.OPENCV
    cams = [Camera(id=0, model_id=model, params=[800.0, 810.0, 500.0, 400.0, -0.01, 0.001, 1e-4, -1e-4]),
            Camera(id=1, model_id=model, params=[900.0, 905.0, 520.0, 390.0, 0.02, -0.002, -2e-4, 3e-4])]
    imgs = []
    for i in range(5):
        w2c = np.eye(4)
        ang = 0.1 * i
        w2c[:3, :3] = np.array([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]])
        w2c[:3, 3] = [0.3 * i, -0.1 * i, 4.0]
        imgs.append(Image(id=i, cam_id=0 if i in (0, 2, 4) else 1, is_registered=(i != 3), world2cam=w2c,
                          features=rng.uniform(0, 1000, (6, 2))))
    pts = {17: ([0.1, 0.2, 0.5], [[0, 0], [1, 1], [2, 2]]),
           3: ([0.0, 0.0, 0.0], [[1, 0]]),                      # length 1 -> dropped
           9: ([-0.3, 0.1, 1.0], [[0, 1], [3, 2], [4, 3]]),      # obs in unregistered image 3 skipped
           42: ([0.0, 0.0, -5.0], [[0, 2], [2, 3], [4, 4]]),     # z_cam ~ -1 < 0.1 -> all filtered
           5: ([0.2, -0.2, 0.3], [[3, 4], [2, 5]]),              # one registered obs survives
           11: ([0.05, 0.0, 0.2], [[4, 0], [1, 3], [0, 5], [2, 1]])}
    trks = {k: Track(id=k, xyz=np.array(v[0]), observations=np.array(v[1])) for k, v in pts.items()}
    res = _scene_arrays(cams, imgs, trks, model.value)
    res.update(_run_solve(LM, cams, imgs, trks, opts))
    np.savez_compressed(os.path.join(out_dir, "packing_edge.npz"), **res)
    print("packing_edge.npz", res["out_points_2d"].shape)

    # (3) points-only variant (track_retriangulation.py:247-249 passes optimize_poses=False)
    opts2 = dict(opts, optimize_poses=False)
    trks = {k: Track(id=k, xyz=np.array(v[0]), observations=np.array(v[1])) for k, v in pts.items()}
    res = _scene_arrays(cams, imgs, trks, model.value)
    res.update(_run_solve(LM, cams, imgs, trks, opts2))
    np.savez_compressed(os.path.join(out_dir, "packing_edge_points_only.npz"), **res)
    print("packing_edge_points_only.npz", res["out_points_2d"].shape)


def _gp_scene_arrays(cameras, images, tracks):
    keys = list(tracks.keys())
    obs = [np.asarray(tracks[k].observations, dtype=np.int64).reshape(-1, 2) for k in keys]
    fu = [np.asarray(im.features_undist, dtype=np.float64).reshape(-1, 3) for im in images]
    dep = [np.asarray(im.depths).reshape(-1) for im in images]   # kept in their dtype (float32 depth maps)
    return dict(
        cam_prior_focal=np.array([c.has_prior_focal_length for c in cameras]),
        img_cam_id=np.array([im.cam_id for im in images]),
        img_registered=np.array([im.is_registered for im in images]),
        img_world2cam=np.stack([np.asarray(im.world2cam, dtype=np.float64) for im in images]),
        img_feat_ptr=np.concatenate([[0], np.cumsum([len(f) for f in fu])]),
        img_feats_undist=np.concatenate(fu),
        img_depths=np.concatenate(dep),
        track_keys=np.array(keys, dtype=np.int64),
        track_xyz=np.stack([np.asarray(tracks[k].xyz, dtype=np.float64) for k in keys]),
        track_obs_ptr=np.concatenate([[0], np.cumsum([len(o) for o in obs])]),
        track_obs=np.concatenate(obs),
    )


def _run_gp(LM, cameras, images, tracks, depths, opts, depth_only):
    from instantsfm.processors.global_positioning import TorchGP
    try:
        TorchGP(device="cpu").Optimize(cameras, images, tracks, depths, opts, depth_only=depth_only)
    except _Captured:
        pass
    model, kwargs, inp = LM.last
    scales = inp["scales"] if depth_only else model.scales
    opt_idx = getattr(model.scales, "optimize_indices", None) if not depth_only else None
    strat = kwargs["strategy"].kwargs
    return dict(
        out_translations=inp["translations"].numpy(),
        out_camera_indices=inp["camera_indices"].numpy(),
        out_point_indices=inp["point_indices"].numpy(),
        out_is_calibrated=inp["is_calibrated"].numpy(),
        out_positions=model.translations.detach().numpy(),
        out_points_3d=model.points_3d.detach().numpy(),
        out_scales=scales.detach().numpy().reshape(-1),
        out_has_optimize_indices=np.array(opt_idx is not None),
        out_optimize_indices=(opt_idx.numpy() if opt_idx is not None else np.zeros(0, np.int64)),
        out_track_keys_after=np.array(list(tracks.keys()), dtype=np.int64),
        out_img_registered_after=np.array([im.is_registered for im in images]),
        out_tr=np.array([strat["radius"], strat["max"], strat["up"], strat["down"]]),
        out_huber=np.array(kwargs["kernel"].args[0]),
        out_pcg_tol=np.array(kwargs["solver"].tol),
        out_reject=np.array(kwargs.get("reject", -1)),
        out_depth_only=np.array(bool(depth_only)),
    )


def gen_gp_cost(out_dir):
    """pairwise_cost (cost_function.py:23-29) on random inputs: 512 observations, mixed calibration flags."""
    from instantsfm.utils.cost_function import pairwise_cost
    rng = np.random.default_rng(11)
    n, C, P = 512, 16, 100
    cams = rng.normal(0, 10, (C, 3))
    pts = rng.normal(0, 10, (P, 3))
    ci = rng.integers(0, C, n)
    pi = np.sort(rng.integers(0, P, n))
    t = rng.normal(size=(n, 3))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    s = rng.uniform(0.02, 0.2, (n, 1))
    calib = rng.uniform(size=C) < 0.6
    out = pairwise_cost(torch.from_numpy(pts[pi]), torch.from_numpy(cams[ci]), torch.from_numpy(s), torch.from_numpy(t),
                        torch.from_numpy(calib[ci]))
    np.savez_compressed(os.path.join(out_dir, "gp_cost_golden.npz"), cams=cams, pts=pts, cam_idx=ci, pt_idx=pi, trans=t,
                        scales=s.reshape(-1), calibrated=calib, out=out.numpy())
    print("gp_cost_golden.npz", out.shape)


def gen_gp_packing(out_dir, LM):
    """TorchGP.Optimize packing: a small synthetic scene (no depths / some depths / depth-only) and edge cases."""
    from instantsfm.scene.defs import Camera, CameraModelId, Image, Track
    sys.path.insert(0, REPO)
    from instantsfm_amd.synth import make_gp_problem
    opts = dict(min_num_view_per_track=3, thres_loss_function=1e-1, max_num_iterations=100, function_tolerance=5e-4)
    rng = np.random.default_rng(7)

    def build(prob, with_depth, extra, f32=False):
        C = prob.n_cams
        cams = [Camera(id=c, model_id=CameraModelId.SIMPLE_RADIAL, params=[1000.0, 500.0, 400.0, 0.0],
                       has_prior_focal_length=bool(prob.fcam[c] == 1.0)) for c in range(C)]
        Rs = []
        imgs = []
        order = np.argsort(prob.cam_idx, kind="stable")
        counts = np.bincount(prob.cam_idx, minlength=C)
        starts = np.concatenate([[0], np.cumsum(counts)])
        feat_id = np.empty(prob.n_obs, np.int64)
        feat_id[order] = np.arange(prob.n_obs) - np.repeat(starts[:-1], counts)
        for c in range(C):
            from scipy.spatial.transform import Rotation
            R = Rotation.from_rotvec(rng.normal(0, 0.5, 3)).as_matrix()
            Rs.append(R)
            w2c = np.eye(4)
            w2c[:3, :3] = R
            w2c[:3, 3] = prob.cams_init[c]
            rays_world = prob.trans[order[starts[c]:starts[c + 1]]]
            fu = rays_world @ R.T  # features_undist = R t  so that  R^T fu = t
            dep = np.where(rng.uniform(size=fu.shape[0]) < 0.5, rng.uniform(1, 20, fu.shape[0]), 0.0) if with_depth \
                else np.zeros(fu.shape[0])
            if f32:
                dep = dep.astype(np.float32)   # depth maps are float32 (controllers/data_reader.py:132)
            imgs.append(Image(id=c, cam_id=c, is_registered=True, world2cam=w2c, features=np.zeros((fu.shape[0], 2)),
                              features_undist=fu, depths=dep))
        ptr = np.concatenate([[0], np.cumsum(np.bincount(prob.pt_idx, minlength=prob.n_points))])
        pairs = np.stack([prob.cam_idx.astype(np.int64), feat_id], 1)
        trks = {}
        for p in range(prob.n_points):
            trks[3 * p + 1] = Track(id=3 * p + 1, xyz=prob.points_init[p].copy(), observations=pairs[ptr[p]:ptr[p + 1]].copy())
        if extra:
            # an extra image observed by nothing (-> unregistered), an unregistered image with observations, a
            # 2-view track (-> dropped)
            imgs.append(Image(id=C, cam_id=0, is_registered=True, world2cam=np.eye(4), features=np.zeros((2, 2)),
                              features_undist=np.array([[0, 0, 1.0], [0, 1.0, 0]]), depths=np.array([3.0, 0.0])))
            imgs[1].is_registered = False
            trks[1000] = Track(id=1000, xyz=np.ones(3), observations=np.array([[0, 0], [2, 0]]))
        return cams, imgs, trks

    cases = [("gp_packing_plain", dict(seed=3), False, False, False),
             ("gp_packing_depth", dict(seed=4), True, False, False),
             ("gp_packing_depth_only", dict(seed=5), True, True, False),
             ("gp_packing_edge", dict(seed=6), True, False, True),
             ("gp_packing_depth_f32", dict(seed=8), True, False, False)]
    for name, kw, with_depth, depth_only, extra in cases:
        prob = make_gp_problem(8, 40, track_len=4, window=3, init="perturbed", **kw)
        cams, imgs, trks = build(prob, with_depth, extra, f32=name.endswith("_f32"))
        res = _gp_scene_arrays(cams, imgs, trks)
        depths = np.concatenate([np.asarray(im.depths) for im in imgs]) if with_depth else None
        res["has_depths"] = np.array(depths is not None)
        res.update(_run_gp(LM, cams, imgs, trks, depths, opts, depth_only))
        np.savez_compressed(os.path.join(out_dir, name + ".npz"), **res)
        print(name + ".npz", res["out_translations"].shape)


def gen_passes(out_dir):
    """Between-round passes: the reference's own track filters and NormalizeReconstruction on a
    perturbed config-1 scene, img2cam for the models that do not call cv2, cam2img (the forward model) for all."""
    import copy
    from scipy.spatial.transform import Rotation
    from instantsfm.scene.defs import Camera, CameraModelId, Image, Track
    from instantsfm.processors import track_filter as TF
    from instantsfm.processors.reconstruction_normalizer import NormalizeReconstruction
    sys.path.insert(0, REPO)
    from instantsfm_amd.synth import make_config, quat_to_matrix
    rng = np.random.default_rng(21)
    prob = make_config(1, seed=3)
    C, P = prob.n_cams, prob.n_points
    order = np.argsort(prob.cam_idx, kind="stable")
    counts = np.bincount(prob.cam_idx, minlength=C)
    starts = np.concatenate([[0], np.cumsum(counts)])
    feat_id = np.empty(prob.n_obs, np.int64)
    feat_id[order] = np.arange(prob.n_obs) - np.repeat(starts[:-1], counts)
    imgs = []
    w2cs = []
    for c in range(C):
        w2c = np.eye(4)
        w2c[:3, :3] = quat_to_matrix(prob.cams_gt[c, 3:7])
        w2c[:3, 3] = prob.cams_gt[c, :3]
        w2cs.append(w2c)
    # rays: ground-truth camera-frame directions, small noise, 5% outliers, a few rays pointing backwards
    fu_all = np.zeros((prob.n_obs, 3))
    for o in range(prob.n_obs):
        W = w2cs[prob.cam_idx[o]]
        pc = W[:3, :3] @ prob.points_gt[prob.pt_idx[o]] + W[:3, 3]
        fu_all[o] = pc / np.linalg.norm(pc)
    fu_all += rng.normal(0, 2e-3, fu_all.shape) * (rng.uniform(size=(prob.n_obs, 1)) < 0.95)
    fu_all += rng.normal(0, 5e-2, fu_all.shape) * (rng.uniform(size=(prob.n_obs, 1)) >= 0.95)
    fu_all /= np.linalg.norm(fu_all, axis=1, keepdims=True)
    depth_all = np.where(rng.uniform(size=prob.n_obs) < 0.7, rng.uniform(5, 60, prob.n_obs), 0.0)
    for c in range(C):
        sl = order[starts[c]:starts[c + 1]]
        W = w2cs[c].copy()
        W[:3, :3] = W[:3, :3] @ Rotation.from_rotvec(rng.normal(0, 2e-3, 3)).as_matrix()
        imgs.append(Image(id=c, cam_id=c, is_registered=True, world2cam=W, features=prob.uv[sl].copy(),
                          features_undist=fu_all[sl].copy(), depths=depth_all[sl].copy()))
    ptr = np.concatenate([[0], np.cumsum(np.bincount(prob.pt_idx, minlength=P))])
    pairs = np.stack([prob.cam_idx.astype(np.int64), feat_id], 1)
    tracks = {}
    for p in range(P):
        xyz = prob.points_gt[p] + rng.normal(0, 0.02, 3)
        ob = pairs[ptr[p]:ptr[p + 1]].copy()
        if p % 97 == 5:
            ob = ob[:1]                                # single-view track
        if p % 89 == 7:
            ob = np.concatenate([ob, ob[:1]])          # duplicate observation of one image
        if p % 83 == 11:
            xyz = -3.0 * prob.cams_gt[prob.cam_idx[ptr[p]], :3]  # far away / behind some cameras
        tracks[5 * p + 2] = Track(id=5 * p + 2, xyz=xyz, observations=ob)
    tracks[10 ** 6] = Track(id=10 ** 6, xyz=np.zeros(3), observations=np.zeros((0, 2), np.int64))  # empty track
    res = dict(
        w2c=np.stack([im.world2cam for im in imgs]), feat_ptr=starts, feats_undist=np.concatenate([im.features_undist for im in imgs]),
        depths=np.concatenate([im.depths for im in imgs]),
        track_keys=np.array(list(tracks.keys())), track_xyz=np.stack([t.xyz for t in tracks.values()]),
        track_ptr=np.concatenate([[0], np.cumsum([len(t.observations) for t in tracks.values()])]),
        track_obs=np.concatenate([t.observations for t in tracks.values()]).astype(np.int64))

    def run(fn, *a):
        ims, trs = copy.deepcopy(imgs), copy.deepcopy(tracks)
        out = fn(ims, trs, *a)
        return ims, trs, out

    def tracks_out(trs, prefix):
        return {prefix + "keys": np.array(list(trs.keys())),
                prefix + "ptr": np.concatenate([[0], np.cumsum([len(t.observations) for t in trs.values()])]),
                prefix + "obs": (np.concatenate([np.asarray(t.observations).reshape(-1, 2) for t in trs.values()])
                                 if trs else np.zeros((0, 2))).astype(np.int64)}
    # FilterTracksByReprojectionNormalized needs at least one observation per concatenation -> drop the empty track
    for thr in (1e-2, 3e-2):
        ims, trs = copy.deepcopy(imgs), copy.deepcopy({k: v for k, v in tracks.items() if len(v.observations)})
        cnt = TF.FilterTracksByReprojectionNormalized(None, ims, trs, thr)
        res.update(tracks_out(trs, f"reproj_{thr:g}_"))
        res[f"reproj_{thr:g}_counter"] = np.array(cnt)
    ims, trs = copy.deepcopy(imgs), copy.deepcopy({k: v for k, v in tracks.items() if len(v.observations)})
    TF.FilterTracksByAngle(None, ims, trs, 1.0)
    res.update(tracks_out(trs, "angle_"))
    ims, trs = copy.deepcopy(imgs), copy.deepcopy(tracks)
    cnt = TF.FilterTracksTriangulationAngle(None, ims, trs, 1.5)
    res.update(tracks_out(trs, "tri_"))
    res["tri_counter"] = np.array(cnt)
    for name, dep in (("norm_", None), ("normdepth_", np.ones(3)), ("normdepth32_", np.ones(3))):
        ims, trs = copy.deepcopy(imgs), copy.deepcopy(tracks)
        if name == "normdepth32_":
            for im in ims:
                im.depths = im.depths.astype(np.float32)   # float32 depth maps (data_reader.py:132)
        NormalizeReconstruction(ims, trs, dep)
        res[name + "w2c"] = np.stack([im.world2cam for im in ims])
        res[name + "xyz"] = np.stack([t.xyz for t in trs.values()])
    np.savez_compressed(os.path.join(out_dir, "passes_golden.npz"), **res)
    print("passes_golden.npz", len(res), "arrays")

    # camera models: img2cam where it is numpy-only (0, 1, 7), cam2img (forward) for every model
    cam_res = {}
    base = {0: [900.0, 500.0, 400.0], 1: [900.0, 950.0, 500.0, 400.0], 2: [900.0, 500.0, 400.0, -0.05],
            3: [900.0, 500.0, 400.0, -0.05, 0.01], 4: [900.0, 950.0, 500.0, 400.0, -0.05, 0.01, 1e-3, -2e-3],
            5: [900.0, 950.0, 500.0, 400.0, -0.02, 0.004, -1e-3, 5e-4],
            6: [900.0, 950.0, 500.0, 400.0, -0.05, 0.01, 1e-3, -2e-3, 3e-3, 0.02, -0.004, 6e-4],
            7: [900.0, 950.0, 500.0, 400.0, 0.9], 8: [900.0, 500.0, 400.0, -0.03], 9: [900.0, 500.0, 400.0, -0.03, 0.006],
            10: [900.0, 950.0, 500.0, 400.0, -0.02, 0.004, 1e-3, -2e-3, 1e-3, 5e-4, 2e-4, -3e-4]}
    for m, prm in base.items():
        cam = Camera(id=0, model_id=CameraModelId(m), params=list(prm))
        uvw = np.stack([rng.uniform(-0.6, 0.6, 300), rng.uniform(-0.45, 0.45, 300), np.ones(300)], 1)
        cam_res[f"m{m}_params"] = np.array(prm)
        cam_res[f"m{m}_uv"] = uvw[:, :2].copy()
        cam_res[f"m{m}_cam2img"] = cam.cam2img(uvw.copy())
        if m in (0, 1, 7):
            xy = rng.uniform([0, 0], [1000, 800], (300, 2))
            cam_res[f"m{m}_xy"] = xy
            cam_res[f"m{m}_img2cam"] = cam.img2cam(xy.copy())
            cam_res[f"m{m}_xy32"] = xy.astype(np.float32)
            cam_res[f"m{m}_img2cam32"] = cam.img2cam(xy.astype(np.float32))
    np.savez_compressed(os.path.join(out_dir, "camera_models_golden.npz"), **cam_res)
    print("camera_models_golden.npz", len(cam_res), "arrays")


def _retri_arrays(cameras, images, tracks, tracks_orig):
    """Flat arrays of a retriangulation scene (rebuilt into scene objects by the tests)."""
    feats = [np.asarray(im.features).reshape(-1, 2) for im in images]
    return dict(
        cam_model=np.array([c.model_id.value for c in cameras]), cam_params=np.stack([np.asarray(c.params) for c in cameras]),
        img_cam=np.array([im.cam_id for im in images]), w2c=np.stack([im.world2cam for im in images]),
        feat_ptr=np.concatenate([[0], np.cumsum([f.shape[0] for f in feats])]), feats=np.concatenate(feats),
        track_keys=np.array(list(tracks.keys())), track_xyz=np.stack([t.xyz for t in tracks.values()]),
        track_ptr=np.concatenate([[0], np.cumsum([len(t.observations) for t in tracks.values()])]),
        track_obs=np.concatenate([t.observations for t in tracks.values()]).astype(np.int64),
        orig_keys=np.array(list(tracks_orig.keys())),
        orig_ptr=np.concatenate([[0], np.cumsum([len(o) for o in tracks_orig.values()])]),
        orig_obs=np.concatenate(list(tracks_orig.values())).astype(np.int64))


def _to_ref_scene(cameras, images, tracks):
    from instantsfm.scene.defs import Camera, CameraModelId, Image, Track
    cams = [Camera(id=c.id, model_id=CameraModelId(c.model_id.value), width=c.width, height=c.height,
                   params=np.asarray(c.params, dtype=np.float64)) for c in cameras]
    ims = [Image(id=im.id, cam_id=im.cam_id, is_registered=im.is_registered, world2cam=im.world2cam.copy(),
                 features=np.asarray(im.features).copy()) for im in images]
    trs = {k: Track(id=t.id, xyz=t.xyz.copy(), observations=t.observations.copy()) for k, t in tracks.items()}
    return cams, ims, trs


def gen_retri(out_dir):
    """RetriangulateTracks' passes: the reference's complete_tracks and FilterTracksByReprojection
    on seeded scenes (SIMPLE_RADIAL; OPENCV; RADIAL_FISHEYE).  The points-only BA between them is TorchBA's LM
    (parity-tested on its own)."""
    import copy
    sys.path.insert(0, REPO)
    from instantsfm.processors.track_retriangulation import complete_tracks
    from instantsfm.processors.track_filter import FilterTracksByReprojection
    from instantsfm_amd.synth import make_retri_scene
    opts = dict(complete_max_reproj_error=3.0)

    def tracks_out(trs, prefix):
        return {prefix + "keys": np.array(list(trs.keys())),
                prefix + "ptr": np.concatenate([[0], np.cumsum([len(t.observations) for t in trs.values()])]),
                prefix + "obs": np.concatenate([np.asarray(t.observations).reshape(-1, 2) for t in trs.values()]).astype(np.int64),
                prefix + "dtype": np.array(str(np.asarray(next(iter(trs.values())).observations).dtype))}

    for name, model, seed in (("retri_simple_radial", 2, 0), ("retri_opencv", 4, 1), ("retri_radial_fisheye", 9, 2)):
        cameras, images, tracks, tracks_orig = make_retri_scene(model=model, seed=seed)
        res = _retri_arrays(cameras, images, tracks, tracks_orig)
        cams, ims, trs = _to_ref_scene(cameras, images, tracks)
        n = complete_tracks(cams, ims, trs, copy.deepcopy(tracks_orig), opts)
        res.update(tracks_out(trs, "complete_"))
        res["complete_num"] = np.array(n)
        for thr in (3.0, 0.8):
            cams, ims, trs = _to_ref_scene(cameras, images, tracks)
            cnt = FilterTracksByReprojection(cams, ims, trs, thr)
            res.update(tracks_out(trs, f"filter_{thr:g}_"))
            res[f"filter_{thr:g}_counter"] = np.array(cnt)
        np.savez_compressed(os.path.join(out_dir, name + ".npz"), **res)
        print(name + ".npz", "completed", n)


TRACK_DBS = {  # write_match_database() arguments of the golden databases
    "tracks_db0": dict(n_images=24, n_points=1500, seed=0),
    "tracks_db1": dict(n_images=30, n_points=2500, seed=1, kp_cols=2, feature_name=None, wrong_frac=0.08,
                       dup_frac=0.06, distractors=10),
}


def gen_tracks(out_dir):
    """COLMAP database reader + TrackEngine: databases written by the build's own writer
    (instantsfm_amd.synth.write_match_database, the reference's schema), read by the reference's ReadColmapDatabase,
    then the reference's TrackEngine.EstablishFullTracks / FindTracksForProblem on seeded inlier subsets.
    The reference pins numpy 1.26 (pyproject.toml:17), where ``(image_id << 32) | np.uint32`` promotes to int64; under
    this image's numpy 2 it overflows, so the captured pairs' matches are widened to int64 first (same values)."""
    import contextlib
    import io
    import re
    sys.path.insert(0, REPO)
    from instantsfm.controllers.data_reader import ReadColmapDatabase
    from instantsfm.processors.track_establishment import TrackEngine
    from instantsfm_amd.synth import write_match_database, assign_inliers
    for name, kw in TRACK_DBS.items():
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "database.db")
            write_match_database(path, **kw)
            vg, cams, imgs, fname = ReadColmapDatabase(path)
        res = dict(db_args=np.array(repr(kw)), feature_name=np.array(fname))
        res["img_id"] = np.array([im.id for im in imgs])
        res["img_cam"] = np.array([im.cam_id for im in imgs])
        res["img_name"] = np.array([im.filename for im in imgs])
        feats = [np.asarray(im.features).reshape(-1, 2) for im in imgs]
        res["feat_ptr"] = np.concatenate([[0], np.cumsum([f.shape[0] for f in feats])])
        res["feats"] = np.concatenate(feats).astype(np.float32)
        res["cam_id"] = np.array([c.id for c in cams])
        res["cam_model"] = np.array([c.model_id.value for c in cams])
        res["cam_wh"] = np.array([[c.width, c.height] for c in cams])
        res["cam_params"] = np.stack([np.asarray(c.params) for c in cams])
        res["cam_prior"] = np.array([c.has_prior_focal_length for c in cams])
        pairs = list(vg.image_pairs.items())
        res["pair_key"] = np.array([k for k, _ in pairs], dtype=np.int64)
        res["pair_ids"] = np.array([[p.image_id1, p.image_id2] for _, p in pairs])
        res["pair_config"] = np.array([p.config.value for _, p in pairs])
        res["pair_valid"] = np.array([p.is_valid for _, p in pairs])
        res["pair_FEH"] = np.stack([np.stack([p.F, p.E, p.H]) for _, p in pairs])
        res["pair_mptr"] = np.concatenate([[0], np.cumsum([len(p.matches) for _, p in pairs])])
        res["pair_matches"] = np.concatenate([np.asarray(p.matches).reshape(-1, 2) for _, p in pairs]).astype(np.int64)
        res["pair_mdtype"] = np.array(str(pairs[0][1].matches.dtype))
        assign_inliers(vg, seed=kw["seed"])
        for _, p in pairs:
            p.matches = np.asarray(p.matches).astype(np.int64)
        opts = dict(thres_inconsistency=10.0, min_num_view_per_track=3, max_num_view_per_track=9)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            eng = TrackEngine(vg, imgs)
            full = eng.EstablishFullTracks(opts)
        res["discarded"] = np.array(int(re.search(r"Discarded (\d+) features", out.getvalue()).group(1)))
        res["full_keys"] = np.array([int(k) for k in full.keys()], dtype=np.int64)
        res["full_ptr"] = np.concatenate([[0], np.cumsum([len(v) for v in full.values()])])
        res["full_obs"] = np.concatenate(list(full.values())).astype(np.int64)
        res["full_dtype"] = np.array(str(next(iter(full.values())).dtype))
        for i, im in enumerate(imgs):
            im.is_registered = (i % 5) != 2
        res["registered"] = np.array([im.is_registered for im in imgs])
        prob = eng.FindTracksForProblem(full, opts)
        res["prob_keys"] = np.array([int(k) for k in prob.keys()], dtype=np.int64)
        res["prob_ptr"] = np.concatenate([[0], np.cumsum([len(t.observations) for t in prob.values()])])
        res["prob_obs"] = np.concatenate([t.observations for t in prob.values()]).astype(np.int64)
        np.savez_compressed(os.path.join(out_dir, name + ".npz"), **res)
        print(name + ".npz", len(full), "tracks,", int(res["discarded"]), "discarded,", len(pairs), "pairs")


def gen_depth(out_dir):
    """Depth sampling (VERDICT r2 missing #4): the reference's ReadDepthsIntoFeatures (data_reader.py:122-134) over
    three synthetic 16-bit depth maps, with ``cv2.imread`` (absent here) answered from memory by the shim, and its
    ``sample_depth_at_pixel`` (depth_sample.py:3-44) with method 'bilinear'.  Feature coordinates are float32 values
    handed over as float64: under the numpy the reference pins (1.26) a float32 scalar over the integer width
    promotes to float64, which float64 inputs reproduce under this image's numpy 2."""
    import glob as _glob
    import types as _types
    from instantsfm.controllers import data_reader as ref_dr
    from instantsfm.utils.depth_sample import sample_depth_at_pixel
    rng = np.random.default_rng(7)
    H, W = 120, 160
    maps = rng.integers(300, 9000, size=(3, H, W)).astype(np.uint16)
    maps[rng.random(maps.shape) < 0.15] = 0  # invalid (zero) depth
    cam_wh = np.array([[640, 480], [320, 240]])
    img_cam = np.array([0, 1, 0])
    feats = []
    for i in range(3):
        w, h = cam_wh[img_cam[i]]
        f = np.stack([rng.uniform(0, w, 400), rng.uniform(0, h, 400)], 1)
        edge = np.array([[0, 0], [w * (1 - 2 ** -20), h * (1 - 2 ** -20)], [-0.5, 10], [w + 3, 10], [10, -1e-3],
                         [10, h + 1], [w / 2, h / 2], [np.nextafter(np.float32(w), 0), 5]])
        feats.append(np.concatenate([f, edge]).astype(np.float32).astype(np.float64))
    sys.modules["cv2"].IMREAD_UNCHANGED = -1
    with tempfile.TemporaryDirectory() as d:
        files = {}
        for i in range(3):
            fp = os.path.join(d, f"{i:06d}.png")
            open(fp, "wb").close()
            files[fp] = maps[i]
        sys.modules["cv2"].imread = lambda fp, flag: files[fp]
        assert sorted(_glob.glob(os.path.join(d, "*.png"))) == sorted(files)
        cams = [_types.SimpleNamespace(width=int(w), height=int(h)) for w, h in cam_wh]
        imgs = [_types.SimpleNamespace(id=i, cam_id=int(img_cam[i]), features=feats[i]) for i in range(3)]
        ref_maps = ref_dr.ReadDepthsIntoFeatures(d, cams, imgs)
    res = dict(maps_u16=maps, ref_maps=ref_maps, cam_wh=cam_wh, img_cam=img_cam,
               feat_ptr=np.concatenate([[0], np.cumsum([len(f) for f in feats])]), feats=np.concatenate(feats),
               nearest=np.concatenate([im.depths for im in imgs]))
    bil, bav = [], []
    for i in range(3):
        w, h = cam_wh[img_cam[i]]
        for f in feats[i]:
            dv, av = sample_depth_at_pixel(ref_maps[i], f, int(w), int(h), method="bilinear")
            bil.append(float(dv))
            bav.append(bool(av))
    res["bilinear"], res["bilinear_avail"] = np.array(bil), np.array(bav)
    raised = []  # pixels on the right / bottom border: the reference indexes column W (row H) and raises
    for mth in ("nearest", "bilinear"):
        for x, y in ((640.0, 10.0), (10.0, 480.0)):
            try:
                sample_depth_at_pixel(ref_maps[0], np.array([x, y]), 640, 480, method=mth)
                raised.append(False)
            except IndexError:
                raised.append(True)
    res["border_raises"] = np.array(raised)
    np.savez_compressed(os.path.join(out_dir, "depth_sample.npz"), **res)
    print("depth_sample.npz", len(res["feats"]), "features; border raises", raised)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    ap.add_argument("--only", choices=("projection", "packing", "gp", "passes", "retri", "tracks", "depth"), default=None)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    with tempfile.TemporaryDirectory():
        LM = install_shims()
        sys.path.insert(0, REF)
        if args.only in (None, "projection"):
            gen_projection(args.out)
        if args.only in (None, "packing"):
            gen_packing(args.out, LM)
        if args.only in (None, "gp"):
            gen_gp_cost(args.out)
            gen_gp_packing(args.out, LM)
        if args.only in (None, "passes"):
            gen_passes(args.out)
        if args.only in (None, "retri"):
            gen_retri(args.out)
        if args.only in (None, "tracks"):
            gen_tracks(args.out)
        if args.only in (None, "depth"):
            gen_depth(args.out)


if __name__ == "__main__":
    main()
