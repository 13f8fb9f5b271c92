"""Per-call paths of the drop-in use (SURVEY.md §8d end-to-end, §8f row 2): several windows solved
concurrently on one GPU (one context and stream each, one host thread each — the
`concurrent_windows` line of bench.py), and the separate g2o-style read-back calls
(`plba_download` ≈ estimate(), `plba_get_edge_chi2` ≈ chi2()/isDepthPositive()) against the
outputs `plba_lba_plucker` scatters on the device (k_out_scatter)."""
import threading

import numpy as np
import pytest

import oracle_api as oa
from parity import assert_parity, compare
from plba import synth

pytestmark = pytest.mark.gpu

KEYS = ("kf_Tcw", "pt_xyz", "ln_orth", "ept_chi2", "eln_chi2", "ept_level", "eln_level", "ept_depth_ok", "iters",
        "chi2")


def test_concurrent_windows_equal_sequential_solves():
    """Three windows (column-lane C2, C1L and a BCR C4) solved at the same time from three host
    threads on one GPU: each result is bitwise the sequential solve of the same window."""
    from plba.lib import Solver
    gs = [synth.generate("C2", seed=synth.CONFIGS["C2"][3] + 7), synth.generate("C1L"), synth.generate("C4")]
    seq = []
    for g in gs:
        with Solver() as s:
            s.upload(g)
            seq.append(s.lba_plucker(with_trace=False))
    solvers = [Solver() for _ in gs]
    for s, g in zip(solvers, gs):
        s.upload(g)
    outs = [None] * len(gs)
    errs = []
    go = threading.Barrier(len(gs))

    def run(i):
        try:
            go.wait()
            for _ in range(2):  # twice: the second solve replays the captured graphs
                solvers[i].reset()
                outs[i] = solvers[i].lba_plucker(with_trace=False)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(gs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for s in solvers:
        s.close()
    assert not errs, errs
    for o, r in zip(outs, seq):
        for k in KEYS:
            assert np.array_equal(o[k], r[k]), k


def test_readback_calls_equal_scattered_outputs():
    """plba_download / plba_get_edge_chi2 after a solve without outputs return exactly what the
    solve's own output scatter returns (and both match the oracle)."""
    from plba.lib import Solver
    g = synth.generate("C1L")
    ref = oa.lba_plucker(g)
    with Solver() as s:
        s.upload(g)
        full = s.lba_plucker(with_trace=False)
        s.reset()
        s.lba_plucker(want_outputs=False, with_trace=False)
        T, P, O = s.download()
        pc, pd, lc = s.edge_chi2()
    np.testing.assert_array_equal(T, full["kf_Tcw"])
    np.testing.assert_array_equal(P, full["pt_xyz"])
    np.testing.assert_array_equal(O, full["ln_orth"])
    np.testing.assert_array_equal(pc, full["ept_chi2"])
    np.testing.assert_array_equal(pd, full["ept_depth_ok"])
    np.testing.assert_array_equal(lc, full["eln_chi2"])
    assert_parity(compare(full, ref))


def test_concurrent_windows_of_different_sizes_regrow_while_capturing():
    """contexts that GROW (arena, window-build scratch, pinned download
    block) while another context of the process captures its step graphs. Three host threads,
    each a sequence of windows of increasing size (C1L -> C2 -> C3, C2 -> C3, C1L -> C2 -> C4) on its
    own context, started together: every solve equals the sequential solve of the same window on a
    fresh context, bitwise (arena / scratch growth is stream-ordered: hipMallocAsync / hipFreeAsync,
    no device-synchronising call that a concurrent capture would refuse)."""
    from plba.lib import Solver
    seqs = [["C1L", "C2", "C3"], ["C2", "C3"], ["C1L", "C2", "C4"]]
    gs = [[synth.generate(c, seed=synth.CONFIGS[c][3] + 31 * t) for c in seq] for t, seq in enumerate(seqs)]
    ref = []
    for row in gs:
        r = []
        for g in row:
            with Solver() as s:
                s.upload(g)
                r.append(s.lba_plucker(with_trace=False))
        ref.append(r)
    solvers = [Solver() for _ in seqs]
    outs = [[None] * len(row) for row in gs]
    errs = []
    go = threading.Barrier(len(seqs))

    def run(t):
        try:
            go.wait()
            for i, g in enumerate(gs[t]):
                solvers[t].upload(g)  # grows the context's arena while the others capture / solve
                outs[t][i] = solvers[t].lba_plucker(with_trace=False)
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(t,)) for t in range(len(seqs))]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    for s in solvers:
        s.close()
    assert not errs, errs
    for t in range(len(seqs)):
        for o, r in zip(outs[t], ref[t]):
            for k in KEYS:
                assert np.array_equal(o[k], r[k]), (t, k)
