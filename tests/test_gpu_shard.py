"""Sharded windows on the GPU against the CPU oracle.

Two ranks share the box's one GPU through the host transport (gloo all-reduces); a 1-rank
RCCL communicator exercises the RCCL transport and its capture into the step graph. With two or
more GPUs visible, two processes on two GPUs run the RCCL transport for real (rank-ordered
ncclAllGather of the reduced camera system, all-reduces of the iteration/decision terms)."""
import numpy as np
import pytest

import dist_workers as dw
import oracle_api as oa
from parity import EST_RTOL, assert_parity, compare
from plba import synth

pytestmark = pytest.mark.gpu


def _check(out, ref):
    m = compare(out, ref)
    assert m["pt_level_diff"] == 0 and m["ln_level_diff"] == 0, m
    assert_parity(m)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    np.testing.assert_array_equal(out["ept_depth_ok"], ref["ept_depth_ok"])


@pytest.mark.parametrize("cfg", ["C1L", "C2", "C5"])
def test_two_ranks_host_transport_match_oracle(tmp_path, cfg):
    """C5 is BASELINE configs[4], the window the driver's multi-GPU bench shards (two BCR
    factorisations of 129 super-rows then share the one GPU: the ticket order of plba_bcr.hpp
    keeps that deadlock-free)."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(tmp_path), cfg, "host"), nprocs=world,
             join=True)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    g = synth.generate(cfg)
    # each rank kept part of the window, and all ranks return the identical full result
    assert 0 < int(r[0]["local_landmarks"]) < g.n_pt + g.n_ln
    assert int(r[0]["local_landmarks"]) + int(r[1]["local_landmarks"]) == g.n_pt + g.n_ln
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "iters", "trace_chi2"):
        assert np.array_equal(r[0][k], r[1][k]), k
    assert bool(r[0]["rerun_equal"]) and bool(r[1]["rerun_equal"])
    # the device build's ownership is plba_shard_plan's: same landmarks and edges per rank
    for x in r:
        assert int(x["local_landmarks"]) == int(x["plan_landmarks"]), (int(x["local_landmarks"]), int(x["plan_landmarks"]))
        assert int(x["local_edges"]) == int(x["plan_edges"]), (int(x["local_edges"]), int(x["plan_edges"]))
    _check(r[0], oa.lba_plucker(g))


def test_two_ranks_allreduce_exchange_matches_oracle(tmp_path, monkeypatch):
    """PLBA_SHARD_XCHG=allreduce: the reduced camera system summed by one all-reduce of the whole
    system (the round-3 exchange) instead of the all-gather of each rank's block-row runs."""
    import torch.multiprocessing as mp
    world = 2
    monkeypatch.setenv("PLBA_SHARD_XCHG", "allreduce")
    mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(tmp_path), "C2", "host"), nprocs=world,
             join=True)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "iters"):
        assert np.array_equal(r[0][k], r[1][k]), k
    _check(r[0], oa.lba_plucker(synth.generate("C2")))


def test_two_ranks_device_build_equals_host_build(tmp_path):
    """The sharded device window build (k_b_owner + the device sorts) against the host build with
    plba_shard_plan on two ranks: every output bitwise equal."""
    import torch.multiprocessing as mp
    world = 2
    res = {}
    for host in (False, True):
        d = tmp_path / ("host" if host else "dev")
        d.mkdir()
        mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(d), "C2", "host", host), nprocs=world,
                 join=True)
        res[host] = [dict(np.load(d / f"rank{i}.npz")) for i in range(world)]
    for i in range(world):
        for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "iters", "trace_chi2",
                  "local_landmarks", "local_edges"):
            assert np.array_equal(res[False][i][k], res[True][i][k]), (i, k)


def test_two_ranks_bcr_timeout_fall_back_together(tmp_path, monkeypatch):
    """PLBA_DIAG bit 64 makes every BCR hand-off wait time out: both ranks must agree on the
    error, restore their starting state and re-solve with the column-lane factorisation together
    (no rank left waiting in a collective), matching the oracle."""
    import torch.multiprocessing as mp
    world = 2
    monkeypatch.setenv("PLBA_FACTOR", "bcr")
    monkeypatch.setenv("PLBA_DIAG", "64")
    mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(tmp_path), "C2", "host"), nprocs=world,
             join=True)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    assert all(int(x["bcr_fallbacks"]) == 1 for x in r), [int(x["bcr_fallbacks"]) for x in r]
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "iters"):
        assert np.array_equal(r[0][k], r[1][k]), k
    _check(r[0], oa.lba_plucker(synth.generate("C2")))


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_four_ranks_host_transport_match_oracle(tmp_path, cfg):
    """configs[3]'s 4-way landmark sharding, the 4 ranks sharing the box's GPU (host transport)."""
    import torch.multiprocessing as mp
    world = 4
    mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(tmp_path), cfg, "host"), nprocs=world,
             join=True)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    g = synth.generate(cfg)
    loc = [int(x["local_landmarks"]) for x in r]
    assert all(0 < n < g.n_pt + g.n_ln for n in loc) and sum(loc) == g.n_pt + g.n_ln, loc
    for i in range(1, world):
        for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "iters", "trace_chi2"):
            assert np.array_equal(r[0][k], r[i][k]), (i, k)
    assert all(bool(x["rerun_equal"]) for x in r)
    for x in r:
        assert int(x["local_landmarks"]) == int(x["plan_landmarks"]) and int(x["local_edges"]) == int(x["plan_edges"])
    _check(r[0], oa.lba_plucker(g))


def _visible_gpus() -> int:
    import torch
    return torch.cuda.device_count()  # (does not initialise the GPU on this image)


@pytest.mark.skipif(_visible_gpus() < 2, reason="needs two GPUs (one RCCL rank per GPU)")
@pytest.mark.parametrize("cfg", ["C2", "C5"])
def test_two_ranks_rccl_two_gpus_match_oracle(tmp_path, cfg):
    """One process per GPU over the library's RCCL communicator: the rank-ordered all-gather
    exchange (k_rcs_blockpart -> ncclAllGather -> k_rcs_xunpack) that the host transport only
    emulates by a zero-padded sum. Every rank must return the identical result, equal to the oracle
    and bitwise equal to the same window over the host transport."""
    import torch.multiprocessing as mp
    world = 2
    res = {}
    for transport in ("rccl", "host"):
        d = tmp_path / transport
        d.mkdir()
        mp.spawn(dw.sharded_gpu_worker, args=(world, dw.free_port(), str(d), cfg, transport, False,
                                              transport == "rccl"), nprocs=world, join=True)
        res[transport] = [dict(np.load(d / f"rank{i}.npz")) for i in range(world)]
    r = res["rccl"]
    for k in ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "iters", "trace_chi2"):
        assert np.array_equal(r[0][k], r[1][k]), k
        assert np.array_equal(r[0][k], res["host"][0][k]), ("rccl vs host", k)
    assert all(bool(x["rerun_equal"]) for x in r)
    _check(r[0], oa.lba_plucker(synth.generate(cfg)))


@pytest.mark.parametrize("cfg,params", [("C1", {"lambda0": 1e-24}), ("C1", {"lambda0": 1e-24, "err_per_obs": 1}),
                                        ("C2", {})])
def test_two_ranks_hand_rolled_lm_match_oracle(tmp_path, cfg, params):
    """The hand-rolled LM on a sharded window (host transport). At λ0 = 1e-24 on C1 an exactly zero
    landmark pivot fails the solve on the rank that owns the landmark only: the ranks sum their
    failures in the decision all-reduce, so every rank rejects the step and stops together (ADVICE
    r5; before, the other rank applied it and waited in the next collective)."""
    import torch.multiprocessing as mp
    from plba import capi
    from plba.hlm import hlm_window
    from test_gpu_hlm import _compare
    world = 2
    mp.spawn(dw.sharded_hlm_worker, args=(world, dw.free_port(), str(tmp_path), cfg, params), nprocs=world,
             join=True)
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    for k in ("kf_x", "kf_Tcw", "pt_xyz", "ln_orth", "linearizations", "solves", "accepted", "trace"):
        assert np.array_equal(r[0][k], r[1][k]), k
    assert [list(x["info"]) for x in r] == [[world, 0, 0], [world, 1, 0]]
    win = hlm_window(synth.generate(cfg))
    ref = oa.hlm_lba(win, capi.hlm_params(**params))
    out = {k: (v.item() if v.ndim == 0 else v) for k, v in r[0].items()}
    _compare(out, ref, win)


def test_one_rank_rccl_transport_matches_oracle():
    from plba.lib import Solver, comm_unique_id
    g = synth.generate("C1L")
    s = Solver()
    s.comm_init_rccl(1, 0, comm_unique_id())
    ci = s.comm_info()
    assert ci["transport"] == "rccl" and ci["ranks"] == 1 and ci["rank"] == 0, ci
    assert ci["comm_device"] == ci["hip_device"] == 0 and ci["pci"], ci
    s.upload(g)
    out = s.lba_plucker()
    s.reset()
    out2 = s.lba_plucker()
    st = s.structure_stats()
    s.close()
    assert st["sharded"] == 1
    assert st["graph"] == 1, "RCCL all-reduces were not captured into the step graph"
    _check(out, oa.lba_plucker(g))
    for k in ("kf_Tcw", "pt_xyz", "ln_orth"):
        assert np.array_equal(out[k], out2[k]), k
