"""TorchGP -- drop-in for ``instantsfm/processors/global_positioning.py`` (reference :17-206).

Same constructor, ``InitializeRandomPositions``, ``ConvertResults`` and ``Optimize(cameras, images, tracks, depths,
GLOBAL_POSITIONER_OPTIONS, depth_only=False)``: same track / image filters (they mutate ``tracks`` and
``images[*].is_registered`` like the reference), same packing order, stop rule and write-back.  The LM underneath is
the MI355X HIP library (``engine.GlobalPositioner``, include/insfm_gp.h) instead of bae/pypose; the packing loop
(reference :114-152, Python over tracks x observations) is vectorized.
"""
import time

import numpy as np
import torch

from ..engine import GlobalPositioner
from .bundle_adjustment import packx


class PackedGP:
    """What TorchGP.Optimize hands the LM (reference :101-161)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def pack_gp(cameras, images, tracks, depths, options, depth_only=False, native=True):
    """Vectorized restatement of global_positioning.py:85-152.  Mutates ``tracks`` (drops short tracks) and
    ``images[*].is_registered`` (images left without tracks) exactly like the reference.  With the native extension
    (csrc/packx.c ``collect``, as in the BA pack) every Track's observations and xyz are read in one C loop; Track
    attributes that are not plain ndarrays (or ``native=False``) take the numpy path, which gives the same arrays."""
    min_len = options['min_num_view_per_track']
    keys, vals = list(tracks.keys()), list(tracks.values())
    got = packx().collect(vals, 0) if (native and packx() is not None) else None
    if got is not None:
        lengths = np.frombuffer(got[0], np.int64)
        short = lengths < min_len
        for k in np.flatnonzero(short).tolist():                                                # :86-89
            del tracks[keys[k]]
        obs = np.frombuffer(got[1], np.int64).reshape(-1, 2)
        xyz_all = np.frombuffer(got[2], np.float64).reshape(-1, 3)
        if short.any():
            track_list = [v for v, sh in zip(vals, short.tolist()) if not sh]
            obs = obs[np.repeat(~short, lengths)]
            counts, points_3d = lengths[~short], np.ascontiguousarray(xyz_all[~short])
        else:
            track_list, counts, points_3d = vals, lengths, xyz_all
    else:
        short = [k for k, t in tracks.items() if t.observations.shape[0] < min_len]
        for track_id in short:                                                                  # :86-89
            del tracks[track_id]
        track_list = list(tracks.values())
        raw = [t.observations for t in track_list]
        if raw and all(isinstance(o, np.ndarray) and o.ndim == 2 for o in raw):  # one concatenation over the arrays
            counts = np.fromiter((o.shape[0] for o in raw), dtype=np.int64, count=len(raw))
            obs = np.concatenate(raw).astype(np.int64, copy=False).reshape(-1, 2)
        else:
            obs = [np.asarray(o, dtype=np.int64).reshape(-1, 2) for o in raw]
            counts = np.fromiter(map(len, obs), dtype=np.int64, count=len(obs))
            obs = np.concatenate(obs) if obs else np.zeros((0, 2), np.int64)
        xyz = [t.xyz for t in track_list]                                                       # :110-111
        try:
            points_3d = np.concatenate(xyz).astype(np.float64, copy=False).reshape(-1, 3)
            if points_3d.shape[0] != len(xyz):
                raise ValueError
        except ValueError:
            points_3d = np.stack([np.asarray(x, dtype=np.float64).reshape(3) for x in xyz])
    image_used = np.zeros(len(images), dtype=bool)                                              # :91-99
    image_used[obs[:, 0]] = True  # the union over all tracks (the reference's early exit does not change it)
    for image_id, image in enumerate(images):
        if not image_used[image_id]:
            image.is_registered = False

    registered = np.array([img.is_registered for img in images], dtype=bool)                    # :101-107
    image_idx2id = np.nonzero(registered)[0]
    image_id2idx = -np.ones(len(images), dtype=np.int64)
    image_id2idx[image_idx2id] = np.arange(image_idx2id.size)
    w2c = np.array([np.asarray(im.world2cam, dtype=np.float64) for im in images]).reshape(-1, 4, 4)
    camera_translations = np.ascontiguousarray(w2c[image_idx2id, :3, 3])                        # :108-109

    tid = np.repeat(np.arange(len(track_list)), counts)                                         # :120-138
    img_id, feat_id = obs[:, 0], obs[:, 1]
    keep = registered[img_id]
    if not keep.all():
        img_id, feat_id, tid = img_id[keep], feat_id[keep], tid[keep]
    if depths is not None:
        # image.depths[feature_id] keeps the depth map's dtype (float32 from data_reader.py:132), and so does the
        # reference's 1 / depth (:133); the list becomes float64 only in the final np.array
        dep_img = [np.asarray(im.depths).reshape(-1) for im in images]
        dep_off = np.concatenate([[0], np.cumsum([d.shape[0] for d in dep_img])]).astype(np.int64)
        dep_all = np.concatenate(dep_img) if dep_img else np.zeros(0)
        dep = dep_all[dep_off[img_id] + feat_id]
        if depth_only:                                                                          # :129-130
            m = dep != 0
            img_id, feat_id, tid, dep = img_id[m], feat_id[m], tid[m], dep[m]
        available = dep != 0                                                                    # :131-134
        safe = np.where(available, dep, np.ones(1, dtype=dep.dtype))
        scales = np.where(available, (1 / safe), 1.0).astype(np.float64)
    else:
        available = np.zeros(img_id.size, dtype=bool)
        scales = np.ones(img_id.size)                                                           # :146-147
    rot = w2c[:, :3, :3]
    fu_list = [np.asarray(im.features_undist, dtype=np.float64).reshape(-1, 3) if len(im.features_undist) else
               np.zeros((0, 3)) for im in images]
    foff = np.concatenate([[0], np.cumsum([f.shape[0] for f in fu_list])]).astype(np.int64)
    fu_all = np.concatenate(fu_list) if fu_list else np.zeros((0, 3))
    fu = fu_all[foff[img_id] + feat_id]
    translations = np.einsum('nki,nk->ni', rot[img_id], fu)                                     # :135  R^T f
    is_calibrated = np.array([bool(cameras[images[i].cam_id].has_prior_focal_length) for i in image_idx2id])
    # depth_only: the scales are inputs, none optimized (PairwiseNonBatchedDepthOnly, :73-83); otherwise the
    # observations with a valid depth keep theirs (scales.optimize_indices, :57-59, :150-152)
    scale_free = np.zeros(img_id.size, np.int32) if depth_only else (~available).astype(np.int32)
    return PackedGP(translations=np.ascontiguousarray(translations), camera_indices=image_id2idx[img_id],
                    point_indices=tid.astype(np.int64), is_calibrated=is_calibrated,
                    camera_translations=np.ascontiguousarray(camera_translations),
                    points_3d=np.ascontiguousarray(points_3d), scales=np.ascontiguousarray(scales),
                    scale_free=scale_free, image_idx2id=image_idx2id, track_list=track_list)


class TorchGP:
    """global_positioning.py:17-206 with the HIP engine underneath."""

    def __init__(self, visualizer=None, device='cuda:0'):
        self.device = device
        self.visualizer = visualizer
        self.loss_history = []
        self.last_stats = None
        self.timings = {}

    def InitializeRandomPositions(self, cameras, images, tracks, depths=None):
        """global_positioning.py:23-39 (same draws from numpy's global RNG, in the same order)."""
        scene_scale = 100
        if depths is not None:
            valid_depths = depths[depths > 0]
            if len(valid_depths):
                scene_scale = np.mean(valid_depths) * 4.0
        for image in images:
            image.world2cam[:3, 3] = scene_scale * np.random.uniform(-1, 1, 3)
        # the tracks' draws in one call: the legacy global RNG yields the same doubles in the same order as one
        # uniform(-1, 1, 3) per track (tests/test_gp_packing.py), and each track gets its own row
        vals = list(tracks.values())
        xyz = scene_scale * np.random.uniform(-1, 1, 3 * len(vals)).reshape(-1, 3)
        if packx() is not None and xyz.dtype == np.float64 and vals:
            packx().assign_xyz(vals, np.arange(len(vals), dtype=np.int64), np.ascontiguousarray(xyz))
        else:
            for track, row in zip(vals, xyz):
                track.xyz = row
        for track in vals:
            track.is_initialized = True
        if self.visualizer:
            self.visualizer.add_step(cameras, images, tracks)

    def ConvertResults(self, images):
        """global_positioning.py:41-43: position c -> translation t = -R c (every image, like the reference)."""
        for image in images:
            image.world2cam[:3, 3] = -(image.world2cam[:3, :3] @ image.world2cam[:3, 3])

    def Optimize(self, cameras, images, tracks, depths, GLOBAL_POSITIONER_OPTIONS, depth_only=False, progress=True):
        opts = GLOBAL_POSITIONER_OPTIONS
        if depth_only and depths is None:                                                       # :46-48
            print("Warning: No depth maps provided, skip depth-only optimization.")
            return
        t0 = time.perf_counter()
        pk = pack_gp(cameras, images, tracks, depths, opts, depth_only)
        t1 = time.perf_counter()
        C, P = pk.camera_translations.shape[0], pk.points_3d.shape[0]
        eng = GlobalPositioner(pk.translations, pk.camera_indices, pk.point_indices,
                               np.where(pk.is_calibrated, 1.0, 0.5), pk.scale_free, C, P, device=self.device,
                               huber_delta=opts['thres_loss_function'], deterministic=opts.get('deterministic', False),
                               **{k: opts[k] for k in ('pcg_max_iter', 'pcg_tol', 'precond') if k in opts})
        dev = torch.device(self.device)
        # (np.require: a read-only pack array -- a broadcast or a mapped buffer -- is copied, torch needs a writable one)
        pos_t = torch.from_numpy(np.require(pk.camera_translations, requirements='W')).to(dev).contiguous()
        pts_t = torch.from_numpy(np.require(pk.points_3d, requirements='W')).to(dev).contiguous()
        scl_t = torch.from_numpy(np.require(pk.scales, requirements='W')).to(dev).contiguous()
        t2 = time.perf_counter()
        window_size = 4                                                                         # :172-186
        loss_history = []
        it = range(opts['max_num_iterations'])
        bar = None
        if progress:
            try:
                import tqdm
                bar = tqdm.trange(opts['max_num_iterations'])
                it = bar
            except ImportError:
                pass
        for _ in it:
            loss, stats = eng.step(pos_t, pts_t, scl_t)
            self.last_stats = stats
            loss_history.append(loss)
            if len(loss_history) >= 2 * window_size:
                avg_recent = np.mean(loss_history[-window_size:])
                avg_previous = np.mean(loss_history[-2 * window_size:-window_size])
                improvement = (avg_previous - avg_recent) / avg_previous
                if abs(improvement) < opts['function_tolerance']:
                    break
            if bar is not None:
                bar.set_postfix({"loss": loss})
            if self.visualizer:
                self._write_back(images, pk, pos_t, pts_t)
                self.ConvertResults(images)
                self.visualizer.add_step(cameras, images, tracks, "global_positioning")
        if bar is not None:
            bar.close()
        self.loss_history = loss_history
        t3 = time.perf_counter()
        self.final_loss, self.final_rmse = eng.cost(pos_t, pts_t, scl_t)
        self.scales = scl_t.cpu().numpy()
        self._write_back(images, pk, pos_t, pts_t)                                              # :199-206
        self.ConvertResults(images)
        eng.close()
        t4 = time.perf_counter()
        self.timings = dict(pack_s=t1 - t0, create_s=t2 - t1, steps_s=t3 - t2, update_s=t4 - t3, total_s=t4 - t0,
                            steps=len(loss_history), n_cams=C, n_points=P, n_obs=int(pk.translations.shape[0]))

    @staticmethod
    def _write_back(images, pk, pos_t, pts_t):
        pts = pts_t.detach().cpu().numpy()
        pos = pos_t.detach().cpu().numpy()
        if packx() is not None and pts.dtype == np.float64 and pts.flags.c_contiguous and pts.ndim == 2 and len(pts):
            packx().assign_xyz(pk.track_list, np.arange(len(pk.track_list), dtype=np.int64), pts)
        else:
            for track, xyz in zip(pk.track_list, pts):
                track.xyz = xyz
        for idx, image_id in enumerate(pk.image_idx2id.tolist()):
            images[image_id].world2cam[:3, 3] = pos[idx]
