"""Traffic model for the row-band Schur build VERDICT r1 asked about: partner W records fetched per trial when one
workgroup owns a band of B consecutive camera rows (rows in cluster order, so co-visible cameras are adjacent) and
fetches each partner record once per band, against the current one-row-per-workgroup k_schur (each row fetches its
own records and the upper tail of every track it observes).  CPU only; uses the oracle's clustering (test
infrastructure, not the product path)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from instantsfm_amd.synth import make_config  # noqa: E402
from oracle import oracle as O  # noqa: E402

prob = make_config(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
C = prob.n_cams
ora = O.OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points, threads=8)
lab, _ = ora.clusters()
order = np.lexsort((np.arange(C), lab))          # cluster order (cameras ascending within a cluster)
pos = np.empty(C, np.int64)
pos[order] = np.arange(C)
ci, pi = prob.cam_idx.astype(np.int64), prob.pt_idx.astype(np.int64)
o = np.lexsort((ci, pi))
ci_s, pi_s = ci[o], pi[o]
starts = np.r_[0, np.flatnonzero(np.diff(pi_s)) + 1]
lens = np.diff(np.r_[starts, len(pi_s)])
# current kernel: per own observation, its record + the upper tail of its track (cameras after it)
rank_in_track = np.arange(len(pi_s)) - np.repeat(starts, lens)
row_fetch = len(pi_s) + int(np.sum(np.repeat(lens, lens) - 1 - rank_in_track))
print(f"records per trial, one row per workgroup: {row_fetch} ({row_fetch / len(pi_s):.2f} per observation)")
for B in (2, 4, 8, 16):
    band = pos[ci_s] // B
    total = 0
    for s0, L in zip(starts, lens):
        cams = ci_s[s0:s0 + L]          # track sorted by camera id (the partner order of k_schur)
        b = band[s0:s0 + L]
        for bb in np.unique(b):
            first = np.flatnonzero(b == bb)[0]
            # the band fetches its own records and every record after its first observation once
            total += L - first
    print(f"band of {B:2d} rows (cluster order): {total} records ({row_fetch / total:.2f}x fewer), LDS for the band's "
          f"S rows {B * 31} KB")
