"""Multi-rank path on CPU (gloo, world_size 2): track sharding, the all-reduce callback the C ABI calls, and the
decomposition the GPU ranks rely on (per-shard camera blocks sum to the full system; point blocks are shard-local)."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from instantsfm_amd.shard import shard_ranges
from instantsfm_amd.synth import make_config, make_problem


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, world, *args):
    port = _free_port()
    mp.spawn(fn, args=(world, port) + args, nprocs=world, join=True)


def _init(rank, world, port):
    os.environ["OMP_NUM_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_ranges_cover_and_balance(world):
    prob = make_problem(40, 3000, seed=1)
    # uneven tracks: drop every third observation of the first half of the points
    keep = np.ones(prob.n_obs, bool)
    keep[: prob.n_obs // 2][::3] = False
    pt = prob.pt_idx[keep]
    rng = shard_ranges(pt, prob.n_points, world)
    assert rng[0][0] == 0 and rng[-1][1] == prob.n_points
    assert all(rng[r][1] == rng[r + 1][0] for r in range(world - 1))
    counts = [int(np.sum((pt >= a) & (pt < b))) for a, b in rng]
    assert sum(counts) == pt.size
    assert max(counts) - min(counts) <= 2 * 10 + 1  # within a couple of tracks of perfect balance


def _cb_worker(rank, world, port):
    _init(rank, world, port)
    from instantsfm_amd import _capi
    from instantsfm_amd.engine import make_allreduce_callback
    buf = torch.arange(20, dtype=torch.float64) * (rank + 1)
    errors = []
    cb = _capi.ALLREDUCE_FN(make_allreduce_callback(lambda: buf, None, errors))
    ptr = ctypes.cast(buf.data_ptr() + 5 * 8, ctypes.POINTER(ctypes.c_double))
    assert cb(None, ptr, 7) == 0
    expect = torch.arange(20, dtype=torch.float64) * (rank + 1)
    expect[5:12] = torch.arange(5, 12, dtype=torch.float64) * sum(range(1, world + 1))
    assert torch.equal(buf, expect), (buf, expect)
    bad = ctypes.cast(buf.data_ptr() + 18 * 8, ctypes.POINTER(ctypes.c_double))
    assert cb(None, bad, 7) == -1 and errors  # outside the exchange buffer -> error code, no collective issued
    dist.destroy_process_group()


def test_allreduce_callback_gloo():
    _run(_cb_worker, 2)


def _shard_worker(rank, world, port, cfg):
    _init(rank, world, port)
    from oracle.oracle import GC, GP, U, V, OracleBA
    prob = make_config(cfg) if cfg else make_problem(30, 1500, seed=4)
    p0, p1 = shard_ranges(prob.pt_idx, prob.n_points, world)[rank]
    sel = (prob.pt_idx >= p0) & (prob.pt_idx < p1)
    ora = OracleBA(prob.model, prob.uv[sel], prob.cam_idx[sel], prob.pt_idx[sel] - p0, prob.pp, prob.n_cams, p1 - p0)
    ora.linearize(prob.cams_init, np.ascontiguousarray(prob.points_init[p0:p1]))
    Ur, gcr = torch.from_numpy(ora.get(U)), torch.from_numpy(ora.get(GC))
    dist.all_reduce(Ur)
    dist.all_reduce(gcr)
    full = OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points)
    full.linearize(prob.cams_init, prob.points_init)
    Uf, gcf = full.get(U), full.get(GC)
    assert np.max(np.abs(Ur.numpy() - Uf)) <= 1e-12 * np.max(np.abs(Uf))
    assert np.max(np.abs(gcr.numpy() - gcf)) <= 1e-11 * np.max(np.abs(gcf))
    # point blocks are shard-local and identical to the full problem's
    assert np.array_equal(ora.get(V), full.get(V)[p0:p1])
    assert np.array_equal(ora.get(GP), full.get(GP)[p0:p1])
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [0, 1])
def test_track_sharding_decomposes_camera_system(cfg):
    _run(_shard_worker, 2, cfg)


class _Props:
    def __init__(self, bus):
        self.pci_domain_id, self.pci_bus_id, self.pci_device_id = 0, bus, 0


def _rpd_worker(rank, world, port, buses, expect):
    _init(rank, world, port)
    from instantsfm_amd import engine
    torch.cuda.get_device_properties = lambda device: _Props(buses[rank])  # (no GPU here: the rank's PCI address)
    got = engine.ranks_per_device(None)
    assert got == expect, (rank, got, expect)
    dist.destroy_process_group()


@pytest.mark.parametrize("buses,expect", [([3, 3, 3, 3], 4), ([1, 2, 3, 4], 1), ([1, 1, 2, 3], 2)])
def test_ranks_per_device(buses, expect):
    """engine.ranks_per_device: the most ranks on one GPU, from every rank's (host name, PCI address) -- the count the
    engine passes to insfm_ba_set_ranks_per_device (the persistent CG stays on only if that many grids fit on a GPU;
    every rank gets the same count, so every rank takes the same CG path)."""
    _run(_rpd_worker, len(buses), buses, expect)


@pytest.mark.parametrize("infos,expect", [
    # (bus, path, grid, slots) per rank -> (ranks per device, keep k_tl_cgp)
    ([(1, 2, 250, 256), (2, 2, 250, 256)], (1, True)),       # one rank per GPU, fixed-order everywhere
    ([(1, 2, 50, 256), (1, 2, 50, 256)], (2, True)),         # two config-2 grids fit one GPU
    ([(1, 2, 250, 256), (1, 2, 250, 256)], (2, False)),      # two config-3 grids do not
    ([(1, 2, 250, 256), (2, 0, 250, 256)], (1, False)),      # one rank ineligible (e.g. INSFM_DIAG=no_cgp there)
    ([(1, 2, 250, 256), (2, 2, 250, 240)], (1, False)),      # one GPU with fewer CUs (a partition mode)
    ([(1, 1, 250, 256), (2, 2, 250, 256)], (1, False)),      # a rank on the atomic (non-deterministic) form
    ([(1, 5, 250, 256), (2, 5, 250, 256)], (1, True)),       # the fixed-order A-DEF2 form everywhere (round 6)
    ([(1, 5, 50, 256), (1, 5, 50, 256)], (2, True)),
    ([(1, 5, 250, 256), (2, 2, 250, 256)], (1, False)),      # A-DEF2 on one rank, additive on another
    ([(1, 4, 250, 256), (2, 4, 250, 256)], (1, False)),      # the atomic A-DEF2 form is not replicable
])
def test_cg_path_decision(infos, expect):
    """engine.cg_path_decision: the replicated multi-rank CG keeps k_tl_cgp only when every rank runs its
    fixed-order form and every GPU holds all the grids placed on it; otherwise every rank takes the launch path."""
    from instantsfm_amd import engine
    allv = [(("h", 0, bus, 0), path, grid, slots) for bus, path, grid, slots in infos]
    assert engine.cg_path_decision(allv) == expect


class _FakeLib:
    def __init__(self, info):
        self.info, self.off = list(info), False

    def insfm_ba_cg_info(self, h, out):
        for k, v in enumerate(self.info):
            out[k] = v
        return 0

    def insfm_ba_set_persistent_cg(self, h, on):
        if not on:
            self.off = True
            self.info[0] = 0
        return 0


def _agree_worker(rank, world, port, infos, expect_path):
    _init(rank, world, port)
    from instantsfm_amd import _capi, engine
    bus, path, grid, slots = infos[rank]
    fake = _FakeLib([path, grid, slots, 64])
    _capi.load = lambda: fake
    _capi.check = lambda h, rc: rc
    torch.cuda.get_device_properties = lambda device: _Props(bus)
    rpd, got = engine.agree_cg_path(None, None)
    assert got == expect_path, (rank, got, expect_path)
    dist.destroy_process_group()


@pytest.mark.parametrize("infos,expect_path", [
    ([(1, 2, 50, 256), (1, 2, 50, 256), (2, 2, 50, 256), (2, 2, 50, 256)], 2),
    ([(1, 2, 50, 256), (1, 2, 50, 256), (2, 0, 50, 256), (2, 2, 50, 256)], 0),   # rank 2 ineligible: all launch path
])
def test_agree_cg_path_world4(infos, expect_path):
    """agree_cg_path over 4 gloo ranks: one rank that cannot run k_tl_cgp turns it off on every rank."""
    _run(_agree_worker, len(infos), infos, expect_path)
