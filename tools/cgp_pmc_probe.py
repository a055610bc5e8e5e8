#!/usr/bin/env python3
"""k_tl_cgp launches at a known state for the PMC passes: config 3, `--steps` LM steps from the
initial scene (bench.py's replay: the same 10 steps), then `insfm_ba_debug_time_cgp` re-runs the last solve's
k_tl_cgp `--reps` times -- the launch bench.py times for its roofline entry.  Run under
`rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`; tools/pmc_traffic.py takes the last `--reps`
k_tl_cgp records.  Prints {"iterations": ..., "reps": ..., "us": ...}.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- python3 tools/cgp_pmc_probe.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from instantsfm_amd.engine import BundleAdjuster  # noqa: E402
from instantsfm_amd.synth import make_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precond", type=int, default=2, help="2: the A-DEF2 k_tl_cgp that bench.py's roofline times")
    a = ap.parse_args()
    prob = make_config(3)
    dev = torch.device("cuda:0")
    eng = BundleAdjuster(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, device=dev,
                         precond=a.precond)
    cams = torch.from_numpy(prob.cams_init).to(dev)
    pts = torch.from_numpy(prob.points_init).to(dev)
    iters = [eng.step(cams, pts)[1]["pcg_iters"] for _ in range(a.steps)]
    us, _, it = eng.debug_time_cgp(a.reps)
    torch.cuda.synchronize()
    print(json.dumps({"iterations": it, "reps": a.reps, "us": us, "step_pcg_iters": iters}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
