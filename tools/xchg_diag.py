#!/usr/bin/env python3
"""Exchange-path vs plain handle on one GPU: the same scene stepped by a plain single-rank handle
and by a 1-rank handle with the all-reduce callbacks forced on (gloo group of one), side by side with the oracle.

    python tools/xchg_diag.py --out gpurun_out/xchg.json [--cluster-size 24] [--steps 5] [--chunks 4]

Prints / writes per handle: clusters, nnzb, cg_info, per step (loss, trials, PCG iterations), and after one
debug_linearize + debug_solve the first-solve arrays (U, g_c, b, S~, dc) against the oracle's.
"""
import argparse
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_problem  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--cluster-size", type=int, default=24)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--precond", type=int, default=1)
    ap.add_argument("--nondet", action="store_true")
    ap.add_argument("--order", default="xchg,plain", help="handle order (comma list of plain / xchg)")
    ap.add_argument("--overlap", action="store_true", help="keep every handle alive until the end (as dist_check does)")
    args = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    prob = make_problem(24, 900, seed=9)
    kw = dict(cluster_size=args.cluster_size, precond=args.precond, deterministic=not args.nondet)
    ora = O.OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                     precond=args.precond, cluster_size=args.cluster_size)
    res = {"oracle": {"clusters": ora.clusters()[1], "nnzb": ora.nnzb()}}
    co, po = prob.cams_init.copy(), prob.points_init.copy()
    res["oracle"]["steps"] = []
    for _ in range(args.steps):
        lo = ora.step(co, po)
        so = ora.stats()
        res["oracle"]["steps"].append([lo, so["trials"], so["pcg_iters"]])
    first = {}
    alive = []
    variants = {"plain": {}, "xchg": dict(force_exchange=True, exchange_chunks=args.chunks)}
    for name in args.order.split(","):
        extra = variants[name]
        eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                             device=dev, **kw, **extra)
        lab, nc = eng.clusters()
        r = {"clusters": nc, "labels": lab.tolist(), "nnzb": eng.nnzb(), "cg_info": eng.cg_info()}
        cg = torch.from_numpy(prob.cams_init.copy()).to(dev)
        pg = torch.from_numpy(prob.points_init.copy()).to(dev)
        r["steps"] = []
        for _ in range(args.steps):
            loss, st = eng.step(cg, pg)
            r["steps"].append([loss, int(st["trials"]), int(st["pcg_iters"])])
        r["cams_final"] = cg.cpu().numpy()
        # one linearization + one solve at the first trial's damping, arrays against the oracle
        C, P, D = prob.n_cams, prob.n_points, eng.D
        eng.debug_linearize(torch.from_numpy(prob.cams_init.copy()).to(dev),
                            torch.from_numpy(prob.points_init.copy()).to(dev))
        it = eng.debug_solve(1.0 + 1e-4)
        arrs = {"U": eng.debug_get(3, (C, D, D)), "gc": eng.debug_get(4, (C, D)), "b": eng.debug_get(6, (C, D)),
                "S": eng.debug_get(5, (eng.nnzb(), D, D)), "dc": eng.debug_get(7, (C, D)),
                "dp": eng.debug_get(8, (P, 3))}
        r["solve_iters"] = it
        first[name] = arrs
        if args.overlap:
            alive.append(eng)
        else:
            eng.close()
        res[name] = r
    o2 = O.OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points,
                    precond=args.precond, cluster_size=args.cluster_size)
    o2.linearize(prob.cams_init, prob.points_init)
    res["oracle"]["solve_iters"] = o2.solve(1.0 + 1e-4)
    oarr = {"U": o2.get(O.U), "gc": o2.get(O.GC), "b": o2.get(O.B), "S": o2.get(O.S), "dc": o2.get(O.DC),
            "dp": o2.get(O.DP)}
    cmp = {}
    for k in oarr:
        cmp[k] = {"plain_vs_oracle": rel(first["plain"][k], oarr[k]), "xchg_vs_oracle": rel(first["xchg"][k], oarr[k]),
                  "plain_vs_xchg": rel(first["plain"][k], first["xchg"][k]),
                  "plain_eq_xchg": bool(np.array_equal(first["plain"][k], first["xchg"][k]))}
    res["first_solve"] = cmp
    res["cams_final_plain_vs_xchg"] = rel(res["plain"].pop("cams_final"), res["xchg"].pop("cams_final"))
    res["steps_rel"] = {n: [abs(a[0] - b[0]) / b[0] for a, b in zip(res[n]["steps"], res["oracle"]["steps"])]
                        for n in ("plain", "xchg")}
    txt = json.dumps(res)
    print(txt, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
