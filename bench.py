#!/usr/bin/env python3
"""LM-BA iterations/sec + final reprojection RMSE on the synthetic 1k-camera / 200k-point / 2M-observation scene
(BASELINE.json configs[2]; configs[3] when run on N GPUs: the same scene track-sharded, strong scaling).

A "step" is one LM step (bae.optim.LM.step semantics: linearize, damped Schur solve with PCG (two-level by default, --precond 0 for
the reference's block-Jacobi), trial,
TrustRegion accept/reject) over the whole scene.  Inputs are resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL all-reduce of the camera system)
    python bench.py --path gp ...   global positioning (TorchGP.Optimize's LM) on the same scene geometry
    python bench.py --path tracks|passes|mapper   track establishment, the between-round passes, the config-5 mapper


Rank 0 prints one JSON line.  The CPU baseline (rank 0, N=1 only) is the build's C/OpenMP restatement of the same LM
(oracle/ba_oracle.c; the reference has no CPU BA) run to convergence on the same scene.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6   # MI355X dense FP64 (MFMA = vector rate on gfx950)
# ds_add_f64 issue cost in k_schur's pattern (8 groups of 8 lanes, each group 8 contiguous doubles of its own block):
# 8.5 CU clocks per wave-instruction at 8 and at 16 waves per CU (tools/lds_atomic_bench.hip mode 1,
# profiles/r6_v20/lds_bench.txt; the microarchitecture guide gives no rate for LDS f64 atomics)
LDS_ADD_F64_CLK = 8.5


def w_record_doubles(D):
    """Doubles per stored W record: [3][D]."""
    return 3 * D


def algorithmic_bytes(kernel, C, P, N, D, nnzb, extra=None):
    """Compulsory HBM bytes of one launch (every input byte read once, every output byte written once)."""
    if kernel == "k_schur":
        return (N * w_record_doubles(D) * 8  # W_o records
                + N * 4 * 3            # cam_obs, ptl, cam
                + (P + 1) * 4          # pt_ptr
                + P * 9 * 8            # V^-1 (6) + y (3)
                + C * (D * D + D) * 8  # U, g_c
                + nnzb * D * D * 8     # S (upper blocks) written
                + C * D * 8)           # b written
    if kernel == "k_cg_iter":
        off = nnzb - C                 # off-diagonal upper blocks (diagonal blocks of S~ are I and never read)
        return (off * D * D * 8        # S~ read once (the kernel streams a full copy: 2x this)
                + C * D * D * 8        # L_i (true-residual norm)
                + (C + 1) * 4 + 2 * off * 4   # nbr_ptr, nbr_j
                + 10 * C * D * 8)      # r, w, s, p, x read + written
    if kernel == "k_tl_pspmv":
        off = nnzb - C
        return (off * D * D * 8        # S~ read once (the kernel streams the full-row copy: 2x this)
                + (C + 1) * 4 + 2 * off * 4   # nbr_ptr, nbr_j
                + 9 * C * D * 8        # m (neighbour gathers counted once), u, w, r, z, q, s, p, x read
                + 8 * C * D * 8        # z, q, s, p, x, r, u, w written
                + C * D * D * 8        # L_i (true-residual norm)
                + 3 * C * 8 + C * (D + 1) * 8)  # row partials and restriction partials written
    if kernel == "k_tl_cgp":
        # one launch = one whole two-level PCG solve (csrc/ba_cgp.h): S~'s unique off-diagonal blocks once (the kernel
        # holds each row's blocks of both triangles in registers, i.e. reads 2x this), Z~ and L_i once, the row vectors
        # in and out once; per iteration the coarse rows of E^-1 once (y = E^-1 R), the exchanged w written and
        # gathered once, and the per-cluster partials / tagged y granules (written and read once)
        off = nnzb - C
        m, nc, iters = extra["m"], extra["nc"], extra["iters"]
        return (off * D * D * 8 + C * D * (D + 1) * 8 + C * D * D * 8 + 16 * C * D * 8
                + iters * (m * m * 8 + 2 * C * D * 8 + 2 * 16 * m + 2 * 8 * (3 * nc + m)))
    if kernel == "k_lin_points":
        return (N * 2 * 8              # observed uv
                + N * 4 * 2            # cam, ptl
                + (P + 1) * 4          # pt_ptr
                + C * (D + 1 + 2) * 8  # camera rows and principal points (each read once)
                + P * 3 * 8            # points
                + N * w_record_doubles(D) * 8  # W records written
                + P * 9 * 8)           # V (6) + g_p (3) written
    raise ValueError(kernel)


def cpu_baseline(prob, max_steps, min_seconds=10.0, max_runs=8, cluster_size=24, precond=2):
    """The oracle's LM to convergence on the same scene, repeated until >= min_seconds of CPU work (a bounded sample)."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    dt, steps, runs = 0.0, 0, 0
    while runs < max_runs and (runs == 0 or dt < min_seconds):
        t0 = time.perf_counter()
        cams, pts, hist, rmse = O.solve_to_convergence(prob, max_iters=max_steps, threads=threads,
                                                       cluster_size=cluster_size, precond=precond)
        dt += time.perf_counter() - t0
        steps += len(hist)
        runs += 1
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return dict(value=steps / dt, unit="LM it/s", cores=threads, kind="port",
                sample=f"oracle/ba_oracle.c (C/OpenMP f64 restatement of the same LM incl. the two-level PCG, precond {precond}), same "
                       f"scene, {runs} runs to the reference stop rule ({len(hist)} LM steps each), {steps} steps in "
                       f"{dt:.2f} s incl. setup; CPU: {model}",
                final_rmse_px=rmse, steps=len(hist))


def cpu_baseline_gp(prob, max_steps, min_seconds=10.0, max_runs=8):
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    dt, steps, runs = 0.0, 0, 0
    while runs < max_runs and (runs == 0 or dt < min_seconds):
        t0 = time.perf_counter()
        _, _, _, hist = O.gp_solve_to_convergence(prob, max_iters=max_steps, threads=threads)
        dt += time.perf_counter() - t0
        steps += len(hist)
        runs += 1
    return dict(value=steps / dt, unit="LM it/s", cores=threads, kind="port",
                sample=f"oracle/ba_oracle.c ora_gp_* (C/OpenMP f64 restatement of TorchGP's LM), same scene, {runs} "
                       f"runs of up to {max_steps} LM steps ({len(hist)} each), {steps} steps in {dt:.2f} s",
                final_loss=hist[-1], steps=len(hist))


def run_gp(args):
    """Global positioning (TorchGP.Optimize, global_positioning.py:158-186): LM it/s on a synthetic scene with the
    geometry of config 3 (1k cameras / 200k tracks / 2M rays), random initial positions as InitializeRandomPositions."""
    import numpy as np
    import torch
    from instantsfm_amd.engine import GlobalPositioner
    from instantsfm_amd.shard import shard_ranges
    from instantsfm_amd.synth import make_gp_problem

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # INSFM_DIST_BACKEND=gloo rehearses the N-rank path on a box with fewer GPUs (ranks share devices, the reduced
    # system goes through host memory); the measured configuration is RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("INSFM_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local if backend == "nccl" else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    prob = make_gp_problem(1000, 200000, track_len=10, seed=args.seed, init="random")
    shards = shard_ranges(prob.pt_idx, prob.n_points, world)
    eng = GlobalPositioner(prob.trans, prob.cam_idx, prob.pt_idx, prob.fcam, prob.sfree, prob.n_cams, prob.n_points,
                           device=dev, deterministic=args.deterministic, world_size=world, rank=rank, shard=shards[rank],
                           precond=args.precond)
    init = [torch.from_numpy(a).to(dev) for a in (prob.cams_init, prob.points_init, prob.scales_init)]
    par = [a.clone() for a in init]

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.step(*par)
    eng.reset()
    for a, b in zip(par, init):
        a.copy_(b)
    barrier()
    t0 = time.perf_counter()
    stats, losses = [], []
    for _ in range(args.steps):
        loss, st = eng.step(*par)
        losses.append(loss)
        stats.append(st)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    final_loss, rmse = eng.cost(*par)
    tl = args.precond >= 1
    us_cg = eng.debug_time_kernel(3 if tl else 0, 100)
    us_schur = eng.debug_time_kernel(1, 5)
    C, P, N, D = prob.n_cams, prob.n_points, prob.n_obs, 3
    Pl = shards[rank][1] - shards[rank][0]
    Nl = int(np.sum((prob.pt_idx >= shards[rank][0]) & (prob.pt_idx < shards[rank][1])))
    nnzb = eng.nnzb()
    trials = sum(s["trials"] for s in stats)
    cg_launches = sum(s["cg_launches"] for s in stats)
    kcg = "k_tl_pspmv" if tl else "k_cg_iter"
    kern = {kcg: (us_cg * cg_launches, cg_launches, us_cg, algorithmic_bytes(kcg, C, Pl, Nl, D, nnzb)),
            "k_schur": (us_schur * trials, trials, us_schur, algorithmic_bytes("k_schur", C, Pl, Nl, D, nnzb))}
    name = max(kern, key=lambda k: kern[k][0])
    _, launches, avg_us, nbytes = kern[name]
    achieved = nbytes / (avg_us * 1e-6) / 1e9 if avg_us > 0 else 0.0
    out = {
        "metric": "LM-GP iterations/sec (global positioning, TorchGP.Optimize)",
        "value": round(args.steps / dt, 4), "unit": "LM it/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (instantsfm_amd/synth.py make_gp_problem, random initial positions)",
        "config": {"workload": f"global positioning: {C} cameras / {P} tracks / {N} rays (config-3 geometry), "
                               f"LM steps of the full scene from random initial positions",
                   "cams": C, "points": P, "obs": N, "camera_block_dim": D, "schur_blocks": nnzb,
                   "parallelism": f"track-shard x{world}" if world > 1 else "single GPU"},
        "final_loss": final_loss, "final_rmse": rmse, "loss_history": [round(x, 6) for x in losses],
        "pcg_iters": [s["pcg_iters"] for s in stats], "trials": trials,
        "kernel_us": {kcg: round(us_cg, 3), "k_schur": round(us_schur, 2)},
        "roofline": {"kernel": name, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "avg_launch_us": round(avg_us, 3), "algorithmic_bytes_per_launch": int(nbytes),
                     "launches_per_run": int(launches)},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baseline_gp(prob, args.cpu_max_steps)
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
        out["cpu_final_loss"] = cb["final_loss"]
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def run_tracks(args):
    """Track establishment (TrackEngine.EstablishFullTracks, track_establishment.py:14-86) on a config-5-sized match
    graph (500 images, ~8M inlier matches, synth.make_match_graph): matches/s of the device pipeline
    (insfm_tracks_establish) with the flattened matches already in HBM; the end-to-end EstablishFullTracks time (host
    flattening + device + building the reference's dict) is reported beside it.  N GPUs: independent replicas."""
    import ctypes
    import numpy as np
    import torch
    from instantsfm_amd import _capi
    from instantsfm_amd.processors.track_establishment import TrackEngine, flatten_matches
    from instantsfm_amd.synth import make_match_graph

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
    vg, images = make_match_graph(seed=args.seed)
    ea, eb, off, xy = flatten_matches(vg, images)
    ne, nn = int(ea.shape[0]), int(off[-1])
    node_img = np.repeat(np.arange(len(images), dtype=np.int32), np.diff(off))
    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
    t_img, t_xy, t_a, t_b = d(node_img, np.int32), d(xy, np.float32), d(ea, np.int32), d(eb, np.int32)
    outs = [torch.empty(ne, dtype=torch.int32, device=dev), torch.empty(ne, dtype=torch.uint8, device=dev),
            torch.empty(ne, dtype=torch.int32, device=dev), torch.empty(2 * ne, dtype=torch.int32, device=dev),
            torch.empty(2 * ne, dtype=torch.int32, device=dev)]
    counts = (ctypes.c_int64 * 2)()
    L = _capi.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def call():
        rc = L.insfm_tracks_establish(nn, p(t_img), p(t_xy), 1, ne, p(t_a), p(t_b), 10.0, *[p(o) for o in outs],
                                      counts, stream)
        if rc != 0:
            raise RuntimeError(f"insfm_tracks_establish: {rc}")

    for _ in range(args.warmup):
        call()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    n_tracks, n_rows = int(counts[0]), int(counts[1])
    avg_s = dt / args.steps
    # compulsory bytes of one call: read the two edge arrays and every node's image and (float32) coordinates once,
    # write the per-track and per-row outputs once
    nbytes = 8 * ne + 12 * nn + 9 * n_tracks + 8 * n_rows
    achieved = nbytes / avg_s / 1e9
    t0 = time.perf_counter()
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        full = TrackEngine(vg, images, device=dev).EstablishFullTracks({'thres_inconsistency': 10.0})
    e2e = time.perf_counter() - t0
    out = {
        "metric": "track establishment: inlier matches/s (TrackEngine.EstablishFullTracks core)",
        "value": round(world * ne / dt * args.steps, 1), "unit": "matches/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(avg_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak" if world > 1 else "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (instantsfm_amd/synth.py make_match_graph)",
        "config": {"workload": f"config-5-sized match graph: {len(images)} images / {nn} features / {len(vg.image_pairs)} "
                               f"pairs / {ne} inlier matches -> {n_tracks} tracks", "images": len(images),
                   "features": nn, "pairs": len(vg.image_pairs), "matches": ne, "tracks": n_tracks,
                   "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
        "tracks_kept": len(full), "end_to_end_s": round(e2e, 3),
        "roofline": {"kernel": "insfm_tracks_establish (whole device pipeline, 15 launches incl. 2 radix sorts)",
                     "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "avg_launch_us": round(avg_s * 1e6, 1), "algorithmic_bytes_per_launch": int(nbytes),
                     "launches_per_run": args.steps},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import tracks as OT
        from instantsfm_amd.scene.defs import ViewGraph
        sub = ViewGraph()
        n = 0
        for k, pair in vg.image_pairs.items():
            sub.image_pairs[k] = pair
            n += len(pair.inliers)
            if n >= args.cpu_edges:
                break
        t0 = time.perf_counter()
        OT.establish_full_tracks(sub, images, 10.0)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / cdt, 1), "unit": "matches/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/tracks.py (the reference's TrackEngine restated loop for loop, "
                                         f"pure Python) on the first {len(sub.image_pairs)} pairs = {n} matches, "
                                         f"{cdt:.2f} s; CPU: {_cpu_model()}"}
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_passes(args):
    """Between-round and retriangulation passes on the config-3 scene (1000 images,
    200k tracks, 2M observations), inputs resident in HBM: one "step" = the six per-item kernels once each --
    undistortion of every feature (UndistortImages), FilterTracksByReprojectionNormalized, FilterTracksByAngle,
    FilterTracksTriangulationAngle, FilterTracksByReprojection (pixel) and complete_tracks' candidate test.
    value = observations / s through the whole set; per-kernel device times from HIP events on the library stream."""
    import ctypes
    import numpy as np
    import torch
    from scipy.spatial.transform import Rotation
    from instantsfm_amd import _capi
    from instantsfm_amd.synth import make_config, full_params, quat_to_matrix

    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    prob = make_config(3, seed=args.seed)
    C, P, N = prob.n_cams, prob.n_points, prob.n_obs
    w2c = np.tile(np.eye(4), (C, 1, 1))
    for c in range(C):
        w2c[c, :3, :3] = quat_to_matrix(prob.cams_gt[c, 3:7])
        w2c[c, :3, 3] = prob.cams_gt[c, :3]
    params = np.zeros((C, 12))
    params[:, :4] = np.stack([full_params(2, prob.cams_gt[c, 7:], prob.pp[c]) for c in range(C)])
    feats = prob.uv.astype(np.float32)
    pc = np.einsum('nij,nj->ni', w2c[prob.cam_idx, :3, :3], prob.points_gt[prob.pt_idx]) + w2c[prob.cam_idx, :3, 3]
    rays = pc / np.linalg.norm(pc, axis=1, keepdims=True)
    centers = -np.einsum('cji,cj->ci', w2c[:, :3, :3], w2c[:, :3, 3])
    rows = np.concatenate([w2c[:, :3, 3], Rotation.from_matrix(w2c[:, :3, :3]).as_quat(), prob.cams_gt[:, 7:]], 1)
    d = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a if dt is None else np.asarray(a, dt))).to(dev)  # noqa
    t = dict(img=d(prob.cam_idx, np.int32), trk=d(prob.pt_idx, np.int32), row=d(np.arange(N), np.int64),
             cam=d(np.zeros(C) + np.arange(C), np.int32), model=d(np.full(C, 2), np.int32), params=d(params),
             feats=d(feats), w2c=d(w2c.reshape(C, 16)), xyz=d(prob.points_gt), rays=d(rays), centers=d(centers),
             ptr=d(np.arange(0, N + 1, 10), np.int64), rows=d(rows), pps=d(prob.pp),
             valid=torch.empty(N, dtype=torch.uint8, device=dev), out=torch.empty((N, 3), dtype=torch.float64, device=dev))
    L = _capi.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda k: ctypes.c_void_p(t[k].data_ptr())  # noqa: E731
    calls = {
        "k_undistort": (lambda: L.insfm_undistort(N, p("feats"), 1, p("img"), p("model"), p("params"), p("out"), stream),
                        N * (8 + 4 + 24)),
        "k_filter_reproj": (lambda: L.insfm_filter_reproj_normalized(N, p("img"), p("trk"), p("row"), p("w2c"), p("xyz"),
                                                                     p("rays"), 1e-2, p("valid"), None, stream),
                            N * 65),
        "k_filter_angle": (lambda: L.insfm_filter_angle(N, p("img"), p("trk"), p("row"), p("w2c"), p("xyz"), p("rays"),
                                                        0.99985, p("valid"), stream), N * 65),
        "k_filter_tri_angle": (lambda: L.insfm_filter_tri_angle(P, p("ptr"), p("img"), p("centers"), p("xyz"), 0.99966,
                                                                p("valid"), stream), P * (8 + 24 + 1) + N * 4),
        "k_filter_reproj_pixel": (lambda: L.insfm_filter_reproj_pixel(N, p("img"), p("trk"), p("row"), p("feats"), 1,
                                                                      p("cam"), p("model"), p("params"), p("w2c"),
                                                                      p("xyz"), 3.0, p("valid"), None, stream), N * 49),
        "k_reproj_candidates": (lambda: L.insfm_reproj_candidates(N, 2, p("img"), p("trk"), p("row"), p("feats"), 1,
                                                                  p("rows"), p("pps"), p("xyz"), 3.0, p("valid"), None,
                                                                  stream), N * 49),
    }
    for fn, _ in calls.values():
        for _ in range(max(args.warmup, 1)):
            if fn() != 0:
                raise RuntimeError("pass kernel failed")
    torch.cuda.synchronize(dev)
    kern = {}
    for name, (fn, nbytes) in calls.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.steps
        kern[name] = dict(avg_launch_us=round(us, 2), algorithmic_bytes_per_launch=int(nbytes),
                          achieved_gbs=round(nbytes / (us * 1e-6) / 1e9, 1))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for fn, _ in calls.values():
            fn()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    name = max(kern, key=lambda k: kern[k]["avg_launch_us"])
    kk = kern[name]
    out = {
        "metric": "between-round + retriangulation passes: observations/s (6 per-item kernels per step)",
        "value": round(N * args.steps / dt, 1), "unit": "obs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (config-3 scene, instantsfm_amd/synth.py; float32 features as a database holds them)",
        "config": {"workload": f"config 3 scene: {C} images / {P} tracks / {N} observations, one pass of each filter",
                   "images": C, "tracks": P, "obs": N, "parallelism": "single GPU"},
        "kernel_us": {k: v["avg_launch_us"] for k, v in kern.items()}, "kernels": kern,
        "roofline": {"kernel": name, "bound": "hbm", "achieved": kk["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(kk["achieved_gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
                     "avg_launch_us": kk["avg_launch_us"], "algorithmic_bytes_per_launch": kk["algorithmic_bytes_per_launch"],
                     "launches_per_run": args.steps,
                     "timing": "torch.cuda.Event on the current stream, which the library launches on"},
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_passes(args.seed)
    print(json.dumps(out), flush=True)


def cpu_baseline_passes(seed):
    """The oracle restatements of the six passes (oracle/passes.py; numpy where the reference is numpy, its Python
    loops where it loops) on a 400-image / 40k-track / 400k-observation sample of the same generator."""
    import copy
    import numpy as np
    from oracle import passes as OP
    from instantsfm_amd.synth import make_problem, to_scene
    prob = make_problem(400, 40000, seed=seed)
    cameras, images, tracks = to_scene(prob, use_init=False, image_features_dtype=np.float32)
    t0 = time.perf_counter()
    for c, im in enumerate(images):
        im.features_undist = OP.undistort_rays(2, cameras[c].params, im.features)
    OP.filter_reproj_normalized(images, tracks, 1e-2)
    OP.filter_angle(images, tracks, 1.0)
    OP.filter_tri_angle(images, tracks, 1.5)
    OP.filter_reproj_pixel(cameras, images, tracks, 3.0)
    OP.complete_candidates(cameras, images, tracks, {k: t.observations for k, t in tracks.items()}, 3.0)
    dt = time.perf_counter() - t0
    return {"value": round(prob.n_obs / dt, 1), "unit": "obs/s", "cores": 1, "kind": "port",
            "sample": f"oracle/passes.py restatements of the six passes on a 400-image / 40000-track / {prob.n_obs}-obs "
                      f"scene of the same generator, {dt:.2f} s; CPU: {_cpu_model()}"}


def solve_end_to_end(prob, dev):
    """TorchBA.Solve (bundle_adjustment.py:44-154) on the scene objects of the same problem (cameras, images, a
    dict of Track; built untimed): the wall-time split of one converged Solve -- host packing, engine creation
    (H2D copies + insfm_ba_create's host sort / pattern / clustering), the LM steps to the reference stop rule, the
    write-back -- as the reference's callers see it (global_mapper.py:114-116)."""
    from instantsfm_amd.config.colmap import BUNDLE_ADJUSTER_OPTIONS
    from instantsfm_amd.processors.bundle_adjustment import TorchBA
    from instantsfm_amd.synth import to_scene
    # Four Solves on fresh copies of the scene: the first of a process maps fresh device memory and loads code objects
    # (reported as first_*); the others are the steady state a caller that solves repeatedly (the mapper) sees, its
    # engine taking the device buffers the previous one parked in the library's cache -- the median of those three by
    # total time is reported (the host phases vary by several ms from Solve to Solve on a shared host).
    runs = []
    for rep in range(4):
        cams, ims, tracks = to_scene(prob)
        ba = TorchBA(device=str(dev))
        ba.Solve(cams, ims, tracks, BUNDLE_ADJUSTER_OPTIONS, progress=False)
        runs.append(dict(ba.timings))
        del cams, ims, tracks, ba
    first = runs[0]
    t = sorted(runs[1:], key=lambda r: r["total_s"])[1]
    host = t["pack_s"] + t["create_s"] + t["update_s"]
    return {"first_solve_total_s": round(first["total_s"], 4), "first_create_s": round(first["create_s"], 4),
            "first_update_s": round(first["update_s"], 4),
            "solve_total_s": round(t["total_s"], 4), "pack_s": round(t["pack_s"], 4),
            "create_s": round(t["create_s"], 4), "steps_s": round(t["steps_s"], 4),
            "ms_per_step": round(1e3 * t["steps_s"] / max(1, t["steps"]), 3),
            "step_ms": [round(x, 3) for x in t.get("step_ms", [])],
            "first_solve_step_ms": [round(x, 3) for x in first.get("step_ms", [])],
            "update_s": round(t["update_s"], 4), "steps": t["steps"], "host_frac": round(host / t["total_s"], 4),
            "pack_phases_ms": {k: round(1e3 * v, 2) for k, v in t.get("pack_phases", {}).items()},
            "update_phases_ms": {k: round(1e3 * v, 2) for k, v in t.get("update_phases", {}).items()},
            "final_rmse_px": t.get("final_rmse")}


def _run_mapper_once(db_path, scene, device, seed):
    import contextlib
    import io
    import numpy as np
    from instantsfm_amd.controllers.data_reader import ReadColmapDatabase
    from instantsfm_amd.controllers.config import Config
    from instantsfm_amd.controllers.global_mapper import SolveGlobalMapper
    from instantsfm_amd.synth import stand_in_rotation_averaging
    T = {}
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        vg, cams, ims, fn = ReadColmapDatabase(db_path)
    T['read_database_s'] = time.perf_counter() - t0
    stand_in_rotation_averaging(vg, ims, scene, seed=seed)
    np.random.seed(seed)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        SolveGlobalMapper(vg, cams, ims, Config.for_ba_half(fn), device=device, timings=T)
    T['mapper_s'] = time.perf_counter() - t0
    return T, ims


def run_mapper(args):
    """Config 5: COLMAP database.db -> ReadColmapDatabase -> SolveGlobalMapper from track establishment on
    (global_mapper.py:80-146: TrackEngine, GP, 3 x [BA, undistort, filter], filters, normalize, RetriangulateTracks,
    BA, filters) on a seeded ~500-image database (synth.write_mapper_database).  The stages before track
    establishment are out of scope; their outputs come from synth.stand_in_rotation_averaging.  One "step" = one
    whole mapper run; the value is the wall time of the run (host + device), per-stage times beside it.
    N GPUs: independent replicas (the mapper itself does not shard)."""
    import tempfile
    import numpy as np
    import torch
    from instantsfm_amd.synth import write_mapper_database

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
    tmp = tempfile.mkdtemp(prefix="insfm_mapper_")
    db = os.path.join(tmp, f"database_{rank}.db")
    t0 = time.perf_counter()
    scene = write_mapper_database(db, n_images=args.mapper_images, n_points=args.mapper_points, seed=args.seed)
    gen_s = time.perf_counter() - t0
    if args.warmup:
        small = os.path.join(tmp, f"warm_{rank}.db")
        sc = write_mapper_database(small, n_images=40, n_points=3000, track_len=6, window=6, reach=2,
                                   images_per_camera=10, distractors=50, seed=args.seed)
        _run_mapper_once(small, sc, dev, args.seed)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    runs = []
    t0 = time.perf_counter()
    for _ in range(args.mapper_runs):
        T, ims = _run_mapper_once(db, scene, dev, args.seed)
        runs.append(T)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    T = runs[-1]
    C = np.array([im.center() for im in ims])
    G = scene.centers_gt
    mc, mg = C.mean(0), G.mean(0)
    U, sv, Vt = np.linalg.svd((G - mg).T @ (C - mc))
    sc_ = sv.sum() / np.sum((C - mc) ** 2)
    center_err = float(np.linalg.norm(sc_ * (C - mc) @ (U @ Vt).T + mg - G, axis=1).max())
    r3 = lambda x: round(float(x), 4)  # noqa: E731
    stages = {k: r3(T[k]) for k in ('read_database_s', 'track_establishment_s', 'global_positioning_s',
                                    'bundle_adjustment_s', 'retriangulation_s') if k in T}
    ba = [{k: (r3(v) if isinstance(v, float) else v) for k, v in b.items()} for b in T['ba']]
    ba_host = sum(b['pack_s'] + b['create_s'] + b['update_s'] for b in T['ba'])
    ba_total = sum(b['total_s'] for b in T['ba'])
    per_run = dt / args.mapper_runs
    out = {
        "metric": "config-5 mapper (BA half: tracks -> GP -> 3x BA + filters -> retriangulation -> BA) wall time",
        "value": round(per_run, 3), "unit": "s per mapper run", "n_gpus": world, "steps": args.mapper_runs,
        "warmup": args.warmup, "ms_per_step": round(per_run * 1e3, 1), "higher_is_better": False,
        "scaling": "weak" if world > 1 else "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic COLMAP database.db (instantsfm_amd/synth.py write_mapper_database), rotations = GT + "
                "0.1 deg (stand-in for the out-of-scope rotation averaging)",
        "config": {"workload": f"config 5: {scene.n_images} images / {scene.n_points} points / {scene.n_pairs} pairs / "
                               f"{scene.n_matches} matches -> {T.get('tracks_problem')} tracks",
                   "images": scene.n_images, "matches": scene.n_matches, "pairs": scene.n_pairs,
                   "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
        "stages_s": stages, "gp": {k: (r3(v) if isinstance(v, float) else v) for k, v in T['gp'].items()},
        "ba_solves": ba, "ba_host_s": r3(ba_host), "ba_total_s": r3(ba_total),
        "ba_host_frac": r3(ba_host / ba_total) if ba_total else None,
        "trace": [[t[0], t[1], t[2], None if t[3] is None else float(t[3])] for t in T['trace']],
        "camera_center_err_max": round(center_err, 5), "db_generation_s": round(gen_s, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_mapper(args, tmp, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline_mapper(args, tmp, dev):
    """The oracle-stage pipeline (oracle/mapper.py: the reference's union-find and passes restated in numpy / Python,
    the C/OpenMP LM restatement for GP and BA) on a 100-image / 20k-point database of the same generator, beside the
    GPU mapper on the same sample."""
    import contextlib
    import io
    import numpy as np
    from instantsfm_amd.controllers.data_reader import ReadColmapDatabase
    from instantsfm_amd.controllers.config import Config
    from instantsfm_amd.synth import stand_in_rotation_averaging, write_mapper_database
    from oracle import mapper as OM
    path = os.path.join(tmp, "cpu_sample.db")
    scene = write_mapper_database(path, n_images=100, n_points=20000, seed=args.seed)
    Tg, _ = _run_mapper_once(path, scene, dev, args.seed)
    with contextlib.redirect_stdout(io.StringIO()):
        vg, cams, ims, fn = ReadColmapDatabase(path)
    stand_in_rotation_averaging(vg, ims, scene, seed=args.seed)
    np.random.seed(args.seed)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        OM.solve_global_mapper(vg, cams, ims, Config.for_ba_half(fn))
    dt = time.perf_counter() - t0
    return {"value": round(dt, 2), "unit": "s per mapper run", "cores": int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0)), "kind": "port",
            "sample": f"oracle/mapper.py on a 100-image / 20000-point / {scene.n_matches}-match database of the same "
                      f"generator: {dt:.2f} s; the GPU mapper on the same sample: {Tg['mapper_s']:.2f} s; "
                      f"CPU: {_cpu_model()}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-solve", action="store_true", help="skip the end-to-end TorchBA.Solve split")
    ap.add_argument("--cpu-max-steps", type=int, default=30)
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--precond", type=int, default=2,
                    help="2 (default, TorchBA's) two-level with the A-DEF2 coarse correction, 1 the additive two-level "
                         "form, 0 block-Jacobi (the reference's)")
    ap.add_argument("--cluster-size", type=int, default=24, help="two-level: target cameras per coarse cluster")
    ap.add_argument("--path", choices=("ba", "gp", "tracks", "passes", "mapper"), default="ba")
    ap.add_argument("--mapper-images", type=int, default=500, help="--path mapper: images in the database")
    ap.add_argument("--mapper-points", type=int, default=100_000, help="--path mapper: scene points")
    ap.add_argument("--mapper-runs", type=int, default=1, help="--path mapper: timed mapper runs")
    ap.add_argument("--cpu-edges", type=int, default=1_500_000, help="--path tracks: matches in the CPU sample")
    args = ap.parse_args()
    if args.path == "gp":
        return run_gp(args)
    if args.path == "tracks":
        return run_tracks(args)
    if args.path == "passes":
        return run_passes(args)
    if args.path == "mapper":
        return run_mapper(args)

    import numpy as np
    import torch
    from instantsfm_amd.engine import BundleAdjuster
    from instantsfm_amd.shard import shard_ranges
    from instantsfm_amd.synth import CONFIGS, make_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    # INSFM_DIST_BACKEND=gloo rehearses the N-rank path on a box with fewer GPUs (ranks share devices, the reduced
    # system goes through host memory); the measured configuration is RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("INSFM_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local if backend == "nccl" else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    prob = make_config(args.config, seed=args.seed)
    shards = shard_ranges(prob.pt_idx, prob.n_points, world)
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                         deterministic=args.deterministic, world_size=world, rank=rank, shard=shards[rank],
                         precond=args.precond, cluster_size=args.cluster_size)
    cams0 = torch.from_numpy(prob.cams_init).to(dev)
    pts0 = torch.from_numpy(prob.points_init).to(dev)
    cams, pts = cams0.clone(), pts0.clone()

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.step(cams, pts)
    eng.reset()
    cams.copy_(cams0)
    pts.copy_(pts0)
    barrier()
    t0 = time.perf_counter()
    stats = []
    losses = []
    for _ in range(args.steps):
        loss, st = eng.step(cams, pts)
        losses.append(loss)
        stats.append(st)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    final_loss, rmse = eng.cost(cams, pts)

    # stop rule of bundle_adjustment.py:134-141 applied to the timed loss history
    conv_step = None
    for k in range(8, len(losses) + 1):
        h = losses[:k]
        a, b = np.mean(h[-4:]), np.mean(h[-8:-4])
        if abs((b - a) / b) < 5e-4 or h[-1] == h[-2]:
            conv_step = k
            break

    # ---- outside the timed region: per-phase breakdown (instrumented replay) and per-kernel device times ----
    eng.reset()
    ci, pi = cams0.clone(), pts0.clone()
    eng.set_timing(True)
    istats = []
    rmse_conv = None  # RMSE where the reference stop rule fires: like-for-like with the CPU run's final RMSE
    for k in range(args.steps):
        istats.append(eng.step(ci, pi)[1])
        if conv_step is not None and k + 1 == conv_step:
            rmse_conv = eng.cost(ci, pi)[1]
    eng.set_timing(False)
    tl = args.precond >= 1
    C, P, N, D = prob.n_cams, prob.n_points, prob.n_obs, eng.D
    Pl = shards[rank][1] - shards[rank][0]
    Nl = int(np.sum((prob.pt_idx >= shards[rank][0]) & (prob.pt_idx < shards[rank][1])))
    nnzb = eng.nnzb()
    ph = np.sum([s["time_ms"] for s in istats], axis=0)
    trials = sum(s["trials"] for s in stats)
    cg_launches = sum(s["cg_launches"] for s in stats)
    # which CG the default path runs: the persistent k_tl_cgp (one launch per solve) when this handle is eligible
    cgp = eng.debug_time_cgp(10) if tl else None
    us_schur = eng.debug_time_kernel(1, 5)
    us_lin = eng.debug_time_kernel(5, 20)
    us_gj = eng.debug_time_kernel(6, 10) if tl else None     # the coarse inverse (k_gj_pinv0 + nB k_gj_step)
    us_erow = eng.debug_time_kernel(7, 10) if tl else None   # the E build (k_tl_erow + k_tl_ereduce)
    kern = {}  # name -> (device us per step, launches per step, us per launch, algorithmic bytes per launch, extra)
    steps_k = float(args.steps)
    if cgp is not None:
        us_cgp, us_pc0, it_cgp = cgp
        m = eng.coarse_dim()
        ext = {"m": m, "nc": m // (D + 1), "iters": it_cgp}
        kern["k_tl_cgp"] = (us_cgp * cg_launches / steps_k, cg_launches / steps_k, us_cgp,
                            algorithmic_bytes("k_tl_cgp", C, Pl, Nl, D, nnzb, ext), ext)
    else:
        kcg = "k_tl_pspmv" if tl else "k_cg_iter"
        us_cg = eng.debug_time_kernel(3 if tl else 0, 100)
        kern[kcg] = (us_cg * cg_launches / steps_k, cg_launches / steps_k, us_cg,
                     algorithmic_bytes(kcg, C, Pl, Nl, D, nnzb), None)
    kern["k_schur"] = (us_schur * trials / steps_k, trials / steps_k, us_schur,
                       algorithmic_bytes("k_schur", C, Pl, Nl, D, nnzb), None)
    kern["k_lin_points"] = (us_lin, 1.0, us_lin, algorithmic_bytes("k_lin_points", C, Pl, Nl, D, nnzb), None)
    # the dominant kernel: the most device time per LM step on the default path (launches per step x hipEvent-timed
    # average launch)
    name = max(kern, key=lambda k: kern[k][0])
    traffic_tab, traffic_it = {}, {}
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
            tr = json.load(f)
        if tr.get("config") == args.config:
            traffic_tab = {k: v["hbm_bytes_per_launch"] for k, v in tr.get("kernels", {}).items()}
            traffic_it = {k: v.get("iterations") for k, v in tr.get("kernels", {}).items()}
    except (OSError, ValueError):
        pass

    def roof_entry(kname):
        per_step, lps, avg_us, nbytes, ext = kern[kname]
        ach = nbytes / (avg_us * 1e-6) / 1e9 if avg_us > 0 else 0.0
        e = {"kernel": kname, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic_tab.get(kname),
             "avg_launch_us": round(avg_us, 3), "algorithmic_bytes_per_launch": int(nbytes),
             "launches_per_step": round(lps, 3), "device_us_per_step": round(per_step, 2),
             "timing": "hipEvents on the library stream (insfm_ba_debug_time_kernel / insfm_ba_debug_time_cgp)"}
        if kname == "k_tl_cgp":
            # (the PMC traffic was taken at its own iteration count; its ratio to the algorithmic
            # bytes is only meaningful at the same count)
            tit = traffic_it.get(kname)
            if tit and traffic_tab.get(kname):
                nb_t = algorithmic_bytes("k_tl_cgp", C, Pl, Nl, D, nnzb, dict(ext, iters=tit))
                e.update(algorithmic_bytes_at_traffic_iterations=int(nb_t),
                         traffic_over_algorithmic_at_traffic_iterations=round(traffic_tab[kname] / nb_t, 3))
            e.update(iterations_per_solve=round(ext["iters"], 2), traffic_iterations=traffic_it.get(kname),
                     us_per_iteration_incl_setup_share=round(avg_us / max(ext["iters"], 1.0), 3),
                     bytes_formula="8*[(nnzb-C)*D^2 + C*D*(D+1) + C*D^2 + 16*C*D + iters*(m^2 + 2*C*D + 4*m + 2*(3*nc+m))]",
                     timing="hipEvents around the k_tl_cgp launch of a solve re-run from its rhs "
                            "(insfm_ba_debug_time_cgp; the coarse solve of r0 runs inside it since round 5)")
        if kname == "k_lin_points":
            e["timing"] = ("back-to-back launches (hipEvents): the sustained rate of its 384-MB record write; in the step "
                           "it overlaps the previous solve's coarse-inverse chain")
        if kname == "k_schur" and avg_us > 0:
            # the kernel's other ceiling: its LDS f64 accumulation.  Every (own observation, upper partner incl.
            # itself) pair of a track adds one D x D block: D*D lane-adds = D*D/64 ds_add_f64 wave-instructions
            lt = np.bincount(prob.pt_idx[(prob.pt_idx >= shards[rank][0]) & (prob.pt_idx < shards[rank][1])])
            pairs = int(np.sum(lt * (lt + 1) // 2))
            winstr = pairs * D * D / 64.0
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            clk_per = avg_us * 2400.0 / (winstr / ncu)  # CU clocks per wave-instruction at 2.4 GHz
            e["roofline_lds"] = {
                "bound": "lds", "unit": "ds_add_f64 wave-instructions per CU clock",
                "achieved": round(1.0 / clk_per, 5), "peak": round(1.0 / LDS_ADD_F64_CLK, 5),
                "frac": round(LDS_ADD_F64_CLK / clk_per, 4), "wave_instructions_per_launch": int(winstr),
                "pairs_per_launch": pairs, "cus": ncu,
                "peak_source": "tools/lds_atomic_bench.hip mode 1: 8.5 clocks per wave-instruction per CU "
                               "(profiles/r6_v20/lds_bench.txt)",
                "note": "the accumulation alone would take frac x the kernel time; the gather floor (loads only, "
                        "SCHUR_PROBE=2) is ~77 % of it (DESIGN.md section 8)"}
        return e
    roof = roof_entry(name)
    roof["timing"] = roof["timing"] + "; dominant = most device time per LM step on the default path"
    others = [roof_entry(k) for k in sorted(kern, key=lambda k: -kern[k][0]) if k != name]

    # the side chain of the two-level preconditioner (runs on the side stream, overlapping the next linearization /
    # Schur build): the Gauss-Jordan inversion of E against the FP64 matrix peak (2 m^3 flops; its tile products are
    # v_mfma_f64_16x16x4f64), the E build against HBM
    chain_situ_ms = float(ph[6]) / args.steps if len(ph) > 6 else None
    if tl:
        m = eng.coarse_dim()
        nb_gj = (m + 31) // 32
        flops = 2.0 * m ** 3
        tfs = flops / (us_gj * 1e-6) / 1e12 if us_gj else 0.0
        others.append({"kernel": f"k_gj_pinv0 + {nb_gj} x k_gj_step (coarse inverse, m = {m})", "bound": "mfma",
                       "achieved": round(tfs, 3), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                       "frac": round(tfs / FP64_PEAK_TFS, 4), "avg_launch_us": round(us_gj / (nb_gj + 1), 3),
                       "chain_us": round(us_gj, 2), "algorithmic_flops_per_chain": int(flops),
                       "chain_in_situ_us_per_step": None if chain_situ_ms is None else round(1e3 * chain_situ_ms, 2),
                       "timing": "chain_us: back-to-back chains (hipEvents), main stream alone; chain_in_situ_us_per_step: "
                                 "the side stream's E build + inversion per LM step in the instrumented replay (events "
                                 "on the side stream around each chain), overlapping the next linearization / Schur"})
        nbe = 2 * (nnzb - C) * D * (D + (D & 1)) * 8 + C * D * (D + 1) * 8
        ach = nbe / (us_erow * 1e-6) / 1e9 if us_erow else 0.0
        others.append({"kernel": "k_tl_erow + k_tl_ereduce (E build; behind k_tl_cgp only k_tl_ereduce runs)",
                       "bound": "hbm", "achieved": round(ach, 2),
                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                       "avg_launch_us": round(us_erow, 3), "algorithmic_bytes_per_launch": int(nbe),
                       "timing": "back-to-back builds with the full grid on the main stream (hipEvents); on the default "
                                 "path k_tl_cgp writes the segments and only k_tl_ereduce runs"})

    out = {
        "metric": "LM-BA iterations/sec (+ final reprojection RMSE)",
        "value": round(args.steps / dt, 4),
        "unit": "LM it/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded scene generator instantsfm_amd/synth.py, SURVEY.md 8(d))",
        "config": {"workload": f"config {args.config}: synthetic {C}-cam / {P}-point / {N}-obs SIMPLE_RADIAL BA, "
                               f"LM steps of the full scene" + (", track-sharded" if world > 1 else ""),
                   "cams": C, "points": P, "obs": N, "camera_block_dim": D, "schur_blocks": nnzb,
                   "parallelism": f"track-shard x{world}" if world > 1 else "single GPU"},
        "final_loss": final_loss,
        "final_rmse_px": rmse_conv,
        "converged_at_step": conv_step,
        "rmse_after_timed_steps_px": rmse,
        "pcg_iters": [s["pcg_iters"] for s in stats],
        "trials": trials,
        "phase_ms_per_step": {k: round(float(v) / args.steps, 3) for k, v in
                              zip(["linearize", "k_schur", "linear_solve", "backsub_update", "trial_cost",
                                   "cg_iterations", "coarse_chain_side_stream"], ph)},
        "kernel_us": dict({k: round(v[2], 3) for k, v in kern.items()},
                          **({"k_tl_cgp_iterations": round(cgp[2], 2)}
                             if cgp is not None else {})),
        "preconditioner": ("block-Jacobi" if not tl else "two-level (block-Jacobi + camera-cluster similarity coarse space"
                           + (", A-DEF2 coarse correction from the coarse initial guess)" if args.precond == 2 else ", additive)")),
        "cg_path": eng.cg_info()[0],
        "roofline": roof,
        "roofline_next_kernels": others,
    }
    if world > 1 or eng.exchange_calls[0]:
        from instantsfm_amd.engine import CG_PATHS
        xspan = float(ph[7]) / args.steps if len(ph) > 7 else 0.0
        out["dist"] = {"backend": dist.get_backend() if dist is not None else None, "world_size": world,
                       "rank0_shard_points": Pl, "rank0_shard_obs": Nl,
                       "cg_path": CG_PATHS.get(eng.cg_path, str(eng.cg_path)), "cg_path_code": eng.cg_path,
                       "ranks_per_device": getattr(eng, "ranks_per_device", 1),
                       "exchange_calls": eng.exchange_calls[0],
                       "exchange_callback_host_ms_per_step": round(1e3 * eng.exchange_calls[1] / (2 * args.steps), 4),
                       "exchange_span_ms_per_step": round(xspan, 4),
                       "note": "exchange_span: the chunked [S | b] all-reduce's span on the exchange stream per LM step "
                               "in the instrumented replay (first chunk issued -> b reduced; overlaps the Schur build); "
                               "callback host ms: time inside the synchronous callbacks ([U | g_c], trial scalars) over "
                               "the timed + replayed steps"}
    if rank == 0 and world == 1 and not args.no_solve:
        out["solve_end_to_end"] = solve_end_to_end(prob, dev)
    if rank == 0 and not args.no_cpu:
        cb = cpu_baseline(prob, args.cpu_max_steps, cluster_size=args.cluster_size, precond=args.precond)
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
        out["cpu_final_rmse_px"] = cb["final_rmse_px"]
        out["cpu_steps_to_converge"] = cb["steps"]
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
