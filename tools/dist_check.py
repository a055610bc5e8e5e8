#!/usr/bin/env python3
"""Track-sharded multi-rank LM vs the single-GPU LM on the same scene.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        tools/dist_check.py --backend gloo --config 1 --steps 6

Every rank builds the same seeded scene, owns a contiguous range of tracks (instantsfm_amd.shard.shard_ranges) and
steps the shared LM; the camera system is summed across ranks through the engine's all-reduce callback.  Rank 0 then
re-runs the problem on one GPU and prints the largest relative differences as one JSON line.  With --backend gloo the
ranks may share one GPU (the 1-GPU test box); with nccl (RCCL) each rank needs its own GPU.
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from instantsfm_amd.engine import LM_DEFAULTS, BundleAdjuster, GlobalPositioner, effective_precond  # noqa: E402
from instantsfm_amd.shard import shard_ranges  # noqa: E402
from instantsfm_amd.synth import make_config, make_gp_problem, make_problem  # noqa: E402


def allsum(t, backend):
    if backend == "gloo" and t.is_cuda:
        host = t.cpu()
        dist.all_reduce(host)
        return host
    dist.all_reduce(t)
    return t.cpu()


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def run_gp(args, rank, world, dev):
    """Global positioning: the same check for insfm_gp (points and per-observation scales are rank-local)."""
    prob = make_gp_problem(24, 900, seed=9, init="random", depth_frac=0.2)
    shards = shard_ranges(prob.pt_idx, prob.n_points, world)
    mk = lambda **kw: GlobalPositioner(prob.trans, prob.cam_idx, prob.pt_idx, prob.fcam, prob.sfree, prob.n_cams,  # noqa: E731
                                       prob.n_points, device=dev, deterministic=True, **kw)
    eng = mk(world_size=world, rank=rank, shard=shards[rank])
    par = [torch.from_numpy(a.copy()).to(dev) for a in (prob.cams_init, prob.points_init, prob.scales_init)]
    losses = [eng.step(*par)[0] for _ in range(args.steps)]
    rmse = eng.cost(*par)[1]  # collective (the cost partials are all-reduced): every rank calls it
    p0, p1 = shards[rank]
    pm = torch.zeros_like(par[1])
    pm[p0:p1] = 1.0
    om = torch.from_numpy(((prob.pt_idx >= p0) & (prob.pt_idx < p1)).astype(np.float64)).to(dev)
    pts = allsum((par[1] * pm).contiguous(), args.backend)
    scl = allsum((par[2] * om).contiguous(), args.backend)
    cams_all = [torch.zeros_like(par[0]).cpu() for _ in range(world)]
    if args.backend == "gloo":
        dist.all_gather(cams_all, par[0].cpu())
    if rank == 0:
        ref = mk()
        rpar = [torch.from_numpy(a.copy()).to(dev) for a in (prob.cams_init, prob.points_init, prob.scales_init)]
        ref_losses = [ref.step(*rpar)[0] for _ in range(args.steps)]
        out = dict(world=world, backend=args.backend, path="gp",
                   loss_rel=max(abs(a - b) / b for a, b in zip(losses, ref_losses)),
                   cams_rel=rel(par[0].cpu().numpy(), rpar[0].cpu().numpy()),
                   points_rel=rel(pts.numpy(), rpar[1].cpu().numpy()), scales_rel=rel(scl.numpy(), rpar[2].cpu().numpy()),
                   rmse=rmse, ref_rmse=ref.cost(*rpar)[1],
                   cams_equal_across_ranks=all(bool(torch.equal(c, cams_all[0])) for c in cams_all))
        print(json.dumps(out), flush=True)
    dist.barrier()
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0")
    ap.add_argument("--gp", action="store_true", help="global positioning (insfm_gp) instead of BA")
    ap.add_argument("--force-exchange", action="store_true",
                    help="install the all-reduce callback even with one rank (drives the RCCL branch on one GPU)")
    ap.add_argument("--cg-partition", action="store_true",
                    help="row-partitioned CG (each rank applies S~ to its own rows, partials exchanged over IPC windows)")
    ap.add_argument("--exchange-chunks", type=int, default=4,
                    help="row chunks of the [S | b] exchange behind the Schur build (1: one all-reduce after it)")
    ap.add_argument("--diag-rank", type=int, default=-1, help="set INSFM_DIAG=--diag on this rank only")
    ap.add_argument("--diag", default="")
    ap.add_argument("--cluster-size", type=int, default=0,
                    help="coarse cluster target of every handle, the single-GPU reference included (0: the default)")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if rank == args.diag_rank:  # (read by the library once, at its first diagnostic query)
        os.environ["INSFM_DIAG"] = args.diag
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", 0 if args.same_device else local)
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(args.backend)
    if args.gp:
        run_gp(args, rank, world, dev)
        dist.destroy_process_group()
        return
    prob = make_problem(24, 900, seed=9) if args.small else make_config(args.config)
    # every handle -- the ranks' and the single-GPU reference's -- runs the same cluster target (default or --cluster-size)
    ckw = {"cluster_size": args.cluster_size} if args.cluster_size > 0 else {}
    shards = shard_ranges(prob.pt_idx, prob.n_points, world)
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                         world_size=world, rank=rank, shard=shards[rank], deterministic=True,
                         force_exchange=args.force_exchange, exchange_chunks=args.exchange_chunks,
                         **ckw)
    rows = eng.partition_cg() if args.cg_partition else None
    path0 = eng.cg_info()[0]  # the CG every rank agreed on at create (engine.agree_cg_path)
    cams = torch.from_numpy(prob.cams_init.copy()).to(dev)
    pts = torch.from_numpy(prob.points_init.copy()).to(dev)
    losses, iters, launches, trials = [], [], [], []
    for _ in range(args.steps):
        loss, st = eng.step(cams, pts)
        losses.append(loss)
        iters.append(int(st["pcg_total"]))
        launches.append(int(st["cg_launches"]))
        trials.append(int(st["trials"]))
    xchg_us = eng.debug_time_exchange(200) if args.cg_partition else None
    loss, rmse = eng.cost(cams, pts)
    # every rank updated only its own tracks: assemble the full point array
    p0, p1 = shards[rank]
    mask = torch.zeros_like(pts)
    mask[p0:p1] = 1.0
    full = (pts * mask).contiguous()
    if args.backend == "gloo" and full.is_cuda:
        host = full.cpu()
        dist.all_reduce(host)
        full = host
    else:
        dist.all_reduce(full)
        full = full.cpu()
    if args.backend == "gloo":
        cams_all = [torch.zeros_like(cams).cpu() for _ in range(world)]
        dist.all_gather(cams_all, cams.cpu())
    else:
        cams_all = [torch.zeros_like(cams) for _ in range(world)]
        dist.all_gather(cams_all, cams)
        cams_all = [c.cpu() for c in cams_all]
    paths = [None] * world  # (agreed at create, after the steps) per rank
    dist.all_gather_object(paths, (path0, eng.cg_info()[0]))
    # the preconditioner the ranks ran: A-DEF2 on the persistent CG, the additive form on the launch path (ranks that
    # share a GPU, an ineligible rank, after an abort); the single-GPU reference runs the same
    eff = effective_precond(LM_DEFAULTS["precond"], eng.cg_info()[0])
    if rank == 0:
        os.environ.pop("INSFM_DIAG", None)
        ref = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                             device=dev, deterministic=True, precond=eff, **ckw)
        rc = torch.from_numpy(prob.cams_init.copy()).to(dev)
        rp = torch.from_numpy(prob.points_init.copy()).to(dev)
        ref_losses = [ref.step(rc, rp)[0] for _ in range(args.steps)]
        _, ref_rmse = ref.cost(rc, rp)
        rcn, rpn = rc.cpu().numpy(), rp.cpu().numpy()
        out = dict(world=world, backend=args.backend, shards=shards,
                   loss_rel=max(abs(a - b) / b for a, b in zip(losses, ref_losses)),
                   cams_rel=rel(cams.cpu().numpy(), rcn), points_rel=rel(full.numpy(), rpn),
                   rmse=rmse, ref_rmse=ref_rmse, exchange_calls=eng.exchange_calls[0], n_obs=int(prob.n_obs),
                   clusters=eng.clusters()[1], ref_clusters=ref.clusters()[1], precond_effective=eff,
                   ref_cg_path=ref.cg_info()[0],
                   labels_equal=bool(np.array_equal(eng.clusters()[0], ref.clusters()[0])),
                   cg_partition=bool(args.cg_partition), rows=rows, pcg_iters=iters, xchg_us=xchg_us,
                   ranks_per_device=getattr(eng, "ranks_per_device", 1), cg_launches=launches, trials=trials,
                   losses_hex=[float(x).hex() for x in losses], cg_paths=paths,
                   params_sha=hashlib.sha256(cams.cpu().numpy().tobytes() + full.numpy().tobytes()).hexdigest(),
                   cams_equal_across_ranks=all(bool(torch.equal(c, cams_all[0])) for c in cams_all) if cams_all else None)
        print(json.dumps(out), flush=True)
        ok = out["loss_rel"] < 1e-9 and out["cams_rel"] < 1e-7 and out["points_rel"] < 1e-7
        if not ok:
            print("MISMATCH", file=sys.stderr)
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
