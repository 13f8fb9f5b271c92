"""Speculative damped trials (DESIGN §2 "Speculative trials"; g2o OptimizationAlgorithmLevenberg::
solve, the trial loop src/mapHandler.cpp:6122,6152 drives): a step evaluates λ, λ·ν, λ·ν·2ν, ... of
one linearisation in parallel trial slots and k_decide consumes them in the order the sequential
loop meets them. Every trial's arithmetic is the sequential one, so every output must be BITWISE
the one-slot solve's — estimates, per-edge χ² (stale-χ² semantics included), levels, depth flags,
iteration counts and the per-iteration trace — for every slot count and policy."""
import os

import numpy as np
import pytest

import graph_mut as gm
import oracle_api as oa
from parity import assert_parity, compare
from plba import synth
from plba.hlm import hlm_window

pytestmark = pytest.mark.gpu

KEYS = ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "eln_level", "ept_depth_ok", "iters",
        "chi2")
# (slots, policy): policy 1 always, 2 after a rejection within the iteration, 3 after the first
# rejection of the optimize() call
SETTINGS = [(2, 1), (2, 2), (2, 3), (3, 3), (4, 1)]


class _Env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _solve(g, slots, policy, diag=0, tau=None, **kw):
    from plba.lib import Solver
    with _Env(PLBA_SPEC=slots, PLBA_SPEC_POLICY=policy, PLBA_DIAG=diag):
        with Solver(**({} if tau is None else {"tau": tau})) as s:
            s.upload(g)
            out = s.lba_plucker(**kw)
            st = s.structure_stats()
            s.reset()  # a second schedule from the uploaded window: graphs replayed, buffers rotated
            out2 = s.lba_plucker(**kw)
    return out, out2, st


def _bits(x):
    x = np.ascontiguousarray(np.asarray(x))
    return x.shape, x.dtype, x.tobytes()  # bitwise (NaN χ² of a failed trial's state included)


def _assert_same(a, b, what):
    for k in KEYS:
        assert _bits(a[k]) == _bits(b[k]), (what, k)
    ta, tb = a["trace"], b["trace"]
    assert len(ta) == len(tb), (what, len(ta), len(tb))
    assert _bits(ta) == _bits(tb), (what, ta, tb)


@pytest.mark.parametrize("cfg", ["C1L", "C2", "C3"])
def test_speculative_slots_are_bitwise_the_sequential_solve(cfg):
    g = synth.generate(cfg)
    base, base2, st0 = _solve(g, 1, 0)
    assert st0["spec_slots"] == 1
    _assert_same(base, base2, "rerun")
    for slots, pol in SETTINGS:
        out, out2, st = _solve(g, slots, pol)
        assert st["column_lane"] == 1 and st["spec_slots"] == slots and st["spec_policy"] == pol, st
        _assert_same(base, out, (slots, pol))
        _assert_same(base, out2, (slots, pol, "second schedule"))
        # never more steps than the sequential loop (fewer once a rejection was speculated past)
        assert st["device_steps"] <= st0["device_steps"], (slots, pol, st, st0)
    if cfg == "C3":  # the window's stage 2 rejects trials: speculation must save steps there
        _, _, st = _solve(g, 2, 1)
        assert st["device_steps"] < st0["device_steps"], (st, st0)
    # and the sequential result is the oracle's (parity bar of tests/parity.py)
    if cfg != "C3":
        assert_parity(compare(base, oa.lba_plucker(g)))


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_speculative_failed_solves_follow_the_sequential_loop(cfg):
    """Solves forced to fail by a deterministic function of λ (PLBA_DIAG bit 128): a failed trial is
    rejected and applies the last successful solve's x (A13); a slot failing after an earlier
    slot of the same step succeeded is evaluated again alone. Bitwise the one-slot run (C2 and C3:
    the two-sided column-lane factorisation)."""
    g = synth.generate(cfg)
    base, _, _ = _solve(g, 1, 0, diag=128)
    assert any(t["trials"] > 1 for t in base["trace"]), base["trace"]
    for slots, pol in SETTINGS:
        out, out2, _ = _solve(g, slots, pol, diag=128)
        _assert_same(base, out, (slots, pol))
        _assert_same(base, out2, (slots, pol, "second schedule"))


def test_speculative_slot_width_changes_on_an_oversubscribed_grid():
    """The folded decision (last k_lm_solve workgroup) changes the next step's slot count inside
    the launch. With far more k_lm_solve workgroups than the device holds at once (C4: ~1.5k per
    slot), late workgroups of the idle slot run after the decision: they must neither run as a live
    slot nor skew the arrival count. The sticky policy goes 1 -> 2 slots at the first
    rejection; the result must stay bitwise the one-slot solve, twice in a row."""
    g = synth.generate("C4")
    with _Env(PLBA_FACTOR="cl"):
        base, _, st0 = _solve(g, 1, 0)
        assert st0["column_lane"] == 1 and st0["bcr_rows"] == 0, st0
        for slots, pol in ((2, 3), (3, 2)):
            out, out2, st = _solve(g, slots, pol)
            assert st["spec_slots"] == slots, st
            _assert_same(base, out, (slots, pol))
            _assert_same(base, out2, (slots, pol, "second schedule"))


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_speculative_slots_on_block_cyclic_reduction_are_bitwise(cfg):
    """Trial slots on BCR windows (on by default when the slots' super-rows fit the device): each
    slot runs its own ticketed BCR launch
    (records, flags, tickets and epochs per slot, grid.y = slot). Bitwise the one-slot solve, with
    forced solve failures too (C2: BCR forced on a short window; C4: its natural choice)."""
    with _Env(PLBA_FACTOR="bcr", PLBA_SPEC_BCR=1):
        g = synth.generate(cfg)
        for diag in (0, 128):
            base, base2, st0 = _solve(g, 1, 0, diag=diag)
            assert st0["bcr_rows"] > 0 and st0["spec_slots"] == 1, st0
            _assert_same(base, base2, "rerun")
            for slots, pol in ((2, 1), (2, 3), (3, 2)):
                out, out2, st = _solve(g, slots, pol, diag=diag)
                assert st["bcr_rows"] > 0 and st["spec_slots"] == slots, st
                _assert_same(base, out, (slots, pol, diag))
                _assert_same(base, out2, (slots, pol, diag, "second schedule"))
                assert st["device_steps"] <= st0["device_steps"], (st, st0)


@pytest.mark.parametrize("cfg,kw", [("C2R", {}), ("C1", dict(n_kf=30, n_pt=400, seed=35, track_max=30))])
def test_speculative_slots_on_the_band_window_kernels_are_bitwise(cfg, kw):
    """Trial slots on the band kernels with the register-resident window (grid.y = slot; per-slot
    band, factors and separator windows): C2R runs the two-sided kernel at bw 20, the 30-KF window
    the one-sided kernel at bw 21. Bitwise the one-slot solve, with forced solve failures too."""
    g = synth.generate(cfg, **kw)
    for diag in (0, 128):
        base, base2, st0 = _solve(g, 1, 0, diag=diag)
        assert st0["banded"] == 1 and st0["column_lane"] == 0 and st0["bcr_rows"] == 0, st0
        _assert_same(base, base2, "rerun")
        for slots, pol in ((2, 1), (3, 3), (4, 2)):
            out, out2, st = _solve(g, slots, pol, diag=diag)
            assert st["spec_slots"] == slots, st
            _assert_same(base, out, (slots, pol, diag))
            _assert_same(base, out2, (slots, pol, diag, "second schedule"))
            assert st["device_steps"] <= st0["device_steps"], (st, st0)


def test_speculative_zero_pivot_window():
    """τ = 0 and a keyframe with zero information: every solve fails (λ stays 0), every slot's
    trial is rejected with the previous x and optimize(5) terminates after maxTrials."""
    g = gm.zero_information_keyframe(synth.generate("C1L", track_min=3, seed=41))
    base, _, _ = _solve(g, 1, 0, tau=0.0)
    for slots, pol in SETTINGS:
        out, out2, _ = _solve(g, slots, pol, tau=0.0)
        _assert_same(base, out, (slots, pol))
        _assert_same(base, out2, (slots, pol, "second schedule"))


def test_speculative_window_runs_the_g2o_call_sequence_and_handrolled_lm():
    """The g2o call sequence (initializeOptimization / optimize(n) twice with levels set between)
    and the hand-rolled LM (one slot, rotated buffers) on a window uploaded with trial slots."""
    from plba.lib import Solver
    g = synth.generate("C1L")
    res = {}
    for slots in (1, 3):
        with _Env(PLBA_SPEC=slots, PLBA_SPEC_POLICY=1):
            with Solver() as s:
                s.upload(g)
                s.set_robust(True)
                s.initialize_optimization(0)
                a = s.optimize(5)
                pc, pd, lc = s.edge_chi2()
                s.set_edge_levels((pc > 5.991).astype(np.uint8), (lc > 5.991).astype(np.uint8))
                s.set_robust(False)
                s.initialize_optimization(0)
                b = s.optimize(10)
                T, P, O = s.download()
                pc2, _, lc2 = s.edge_chi2()
                # the hand-rolled LM on the same context: a new window, one slot, rotated buffers
                win = hlm_window(g)
                s.upload(win.graph)
                h = s.hlm_lba(win)
        res[slots] = (a, b, T, P, O, pc, lc, pc2, lc2, h)
    r1, r3 = res[1], res[3]
    for i in range(9):
        assert _bits(r1[i]) == _bits(r3[i]), i
    for k in r1[9]:
        if isinstance(r1[9][k], np.ndarray):
            assert _bits(r1[9][k]) == _bits(r3[9][k]), k
