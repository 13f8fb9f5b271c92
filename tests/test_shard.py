"""Sharded windows on the CPU: the landmark partition and the exchange step,
with two gloo ranks (world_size 2) summing partial reduced camera systems through the
product's host all-reduce hook."""
import numpy as np
import pytest

import dist_workers as dw
from plba import synth
from plba.lib import shard_plan


@pytest.mark.parametrize("R", [1, 2, 3, 8])
def test_plan_is_a_balanced_partition_by_first_keyframe(R):
    g = synth.generate("C2")
    po, lo = shard_plan(g, R)
    assert po.shape == (g.n_pt,) and lo.shape == (g.n_ln,)
    assert po.min() >= 0 and po.max() < R and (lo.size == 0 or lo.max() < R)
    # edges per rank within one landmark's worth of the even split
    cnt = np.bincount(np.r_[po[g.ept_lm], lo[g.eln_lm]], minlength=R)
    tot = g.n_ept + g.n_eln
    assert np.all(np.abs(cnt - tot / R) <= 8 + 1), cnt
    # ranks own contiguous ranges of first-observation keyframes
    first = {}
    for kind, lm, kf, own in (("p", g.ept_lm, g.ept_kf, po), ("l", g.eln_lm, g.eln_kf, lo)):
        for e in range(len(lm)):
            first.setdefault((kind, lm[e]), (g.kf_id[kf[e]], own[lm[e]]))
    keys = sorted(first.values())
    ranks = [r for _, r in keys]
    assert ranks == sorted(ranks)
    # deterministic
    po2, lo2 = shard_plan(g, R)
    assert np.array_equal(po, po2) and np.array_equal(lo, lo2)


def test_plan_rejects_bad_graph():
    g = synth.generate("C1")
    g.ept_lm = g.ept_lm.copy()
    g.ept_lm[0] = g.n_pt + 5
    with pytest.raises(Exception):
        shard_plan(g, 2)


def test_two_gloo_ranks_sum_partial_reduced_camera_systems(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(dw.plan_and_schur_worker, args=(world, dw.free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    # both ranks computed the same plan, and it covers every landmark exactly once
    assert np.array_equal(r[0]["po"], r[1]["po"]) and np.array_equal(r[0]["lo"], r[1]["lo"])
    assert set(np.unique(r[0]["po"])) == {0, 1}
    # both received the same sum, equal to the unsharded system
    assert np.array_equal(r[0]["sum"], r[1]["sum"])
    g = synth.generate("C1L", fixed_frac=0.2)
    S, bs = dw.dense_schur_part(g, np.ones(g.n_pt, bool), np.ones(g.n_ln, bool))
    full = np.concatenate([S.ravel(), bs])
    np.testing.assert_allclose(r[0]["sum"], full, rtol=1e-10, atol=1e-8 * np.abs(full).max())


def test_two_gloo_ranks_gather_the_transport_report(tmp_path):
    """bench.py --mode shard records what the transport reports on every rank (plba_comm_info):
    gathered over gloo, every rank holds the same summary, naming ranks 0..N-1 once each, the rank
    count RCCL reported and the number of distinct GPUs (HIP ordinal + PCI location)."""
    import json
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(dw.comm_info_worker, args=(world, dw.free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    assert r[0] == r[1]
    s = r[0]
    assert s["rank_set_ok"] and s["rccl_ranks"] == [world]
    assert s["distinct_hip_devices"] == world and s["distinct_pci"] == world
    assert [c["rank"] for c in s["ranks"]] == [0, 1] and [c["hip_device"] for c in s["ranks"]] == [0, 1]


def test_comm_summary_flags_ranks_on_one_device():
    """Two ranks that report the same device (the one-GPU host-transport rehearsal) count as one
    distinct GPU; a rank set with a hole is not a valid N-rank communicator."""
    from plba.dist import comm_summary
    same = [dict(transport="host", ranks=2, rank=r, comm_device=0, hip_device=0, pci="0000:75:00") for r in (0, 1)]
    s = comm_summary(same)
    assert s["rank_set_ok"] and s["distinct_hip_devices"] == 1
    bad = [dict(transport="rccl", ranks=3, rank=r, comm_device=r, hip_device=r, pci=f"0000:{r:02x}:00") for r in (0, 2)]
    assert not comm_summary(bad)["rank_set_ok"]
