"""Index arithmetic of the register-resident band window (csrc/plba_kernels.hpp band_forward),
restated step by step in numpy and checked against a dense solve: blocks owned per diagonal ring
slot (diagonal w has W-w+1 slots, row i in slot i mod (W-w+1)), the slot offset o = (slot-k-w) mod
(W-w+1) that says whether a slot holds a pivot-column block (o = 0), a trailing block (pair w+o, o)
or the spare slot of the entering row, the two pivot-column buffers, the pivot blocks written two
steps ahead, the entering rows (diagonal-BW block into the next pivot column one step early, the
rest into the owners at the top of the step that first updates them) and the right-hand-side ring.
CPU only: this is the kernel's bookkeeping, not its arithmetic (the GPU tests check that)."""
import numpy as np
import pytest


def _band_solve(A, b, nf, BW):
    W = BW + 1
    Bd = np.zeros((nf, W, 6, 6))
    for i in range(nf):
        for w in range(W):
            if i - w >= 0:
                Bd[i, w] = A[6 * i:6 * i + 6, 6 * (i - w):6 * (i - w) + 6]
    bs = b.reshape(nf, 6)
    cap = lambda w: W - w + 1  # noqa: E731
    t, oo = {}, {}
    for w in range(W):
        for p in range(cap(w)):
            o = (p - w) % cap(w)
            oo[(w, p)] = o
            i = w + o
            t[(w, p)] = Bd[i, w].copy() if (o != cap(w) - 1 and i < nf) else np.zeros((6, 6))
    col = np.zeros((2, W, 6, 6))
    piv = np.zeros((2, 6, 6))
    for (w, p), o in oo.items():
        if w >= 1 and o == 0:
            col[0][w] = t[(w, p)]
        elif w == 0 and o <= 1:
            piv[o] = t[(w, p)]
    bwin = np.zeros((W, 6))
    for r in range(min(W, nf)):
        bwin[r] = bs[r]
    Kv, ys = [np.linalg.inv(piv[0]), None], [bwin[0].copy(), None]
    Lst, zst = {}, {0: Kv[0] @ ys[0]}
    for k in range(nf):
        kb, wmax, sk = k & 1, min(BW, nf - 1 - k), k % W
        slot = lambda w: (sk + w) % W  # noqa: E731
        if k > 0:  # top of step: row k+BW into its owners, its rhs into its slot
            r = min(k + BW, nf - 1)
            for (w, p), o in oo.items():
                if o == cap(w) - 2:
                    t[(w, p)] = Bd[r, w].copy()
                    if BW == 1 and w == 0:
                        piv[kb ^ 1] = Bd[r, w].copy()
            bwin[slot(BW)] = bs[k + BW] if k + BW < nf else 0
        Lcol = {w: col[kb][w] @ Kv[kb] for w in range(1, wmax + 1)}  # phase 1
        for w, L in Lcol.items():
            Lst[(k + w, w)] = L
        if k + 1 < nf:  # wave 0: the next pivot
            M = piv[kb ^ 1] - Lcol[1] @ col[kb][1].T
            y = bwin[slot(1)] - Lcol[1] @ ys[kb]
            piv[kb ^ 1], bwin[slot(1)] = M, y
            Kv[kb ^ 1], ys[kb ^ 1] = np.linalg.inv(M), y
            zst[k + 1] = Kv[kb ^ 1] @ y
        for (w, p), o in oo.items():  # trailing updates of the owned blocks
            wi = w + o
            if 1 <= o != cap(w) - 1 and wi <= wmax and not (w == 0 and o == 1):
                t[(w, p)] = t[(w, p)] - Lcol[wi] @ col[kb][o].T
                if w >= 1 and o == 1:
                    col[kb ^ 1][w] = t[(w, p)].copy()
                if w == 0 and o == 2:
                    piv[kb] = t[(w, p)].copy()
        col[kb ^ 1][BW] = Bd[min(k + W, nf - 1), BW]  # next pivot column's diagonal-BW entry
        for wr in range(2, wmax + 1):
            bwin[slot(wr)] = bwin[slot(wr)] - Lcol[wr] @ ys[kb]
        for key in oo:
            oo[key] = cap(key[0]) - 1 if oo[key] == 0 else oo[key] - 1
    x = np.zeros((nf, 6))
    for k in range(nf - 1, -1, -1):
        v = zst[k].copy()
        for w in range(1, BW + 1):
            if k + w < nf:
                v -= Lst[(k + w, w)].T @ x[k + w]
        x[k] = v
    return x.reshape(-1)


@pytest.mark.parametrize("nf,BW", [(30, 4), (40, 10), (11, 10), (24, 23), (5, 1), (60, 27)])
def test_band_window_bookkeeping_solves_the_band(nf, BW):
    rng = np.random.default_rng(nf * 100 + BW)
    n = 6 * nf
    A = np.zeros((n, n))
    for i in range(nf):
        for j in range(max(0, i - BW), i + 1):
            A[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.standard_normal((6, 6)) * 0.1
    A = A + A.T + np.eye(n) * 20
    b = rng.standard_normal(n)
    np.testing.assert_allclose(_band_solve(A, b, nf, BW), np.linalg.solve(A, b), rtol=0, atol=1e-12)
