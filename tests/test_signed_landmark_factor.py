"""CPU restatement of the hand-rolled LM's signed landmark factor (csrc/plba_kernels.hpp lm_chol
with sgn, and k_lm_solve's solve): (H + λ·diag H) = M S Mᵀ with S = diag(±1), M lower triangular
stored with reciprocal diagonals. Checked against a dense solve and against the oracle's unpivoted
LDLᵀ (oracle/refhlm.cpp ldlt_solve): both factor the same matrix, so they solve it alike, and a
pivot that is exactly zero in one is exactly zero in the other's exact arithmetic (DESIGN.md §8,
tiny-λ breakdown). No GPU."""
import numpy as np
import pytest


def signed_factor(A):
    """lm_chol(sgn=true): returns (L with reciprocal diagonal, S, zero_pivot)."""
    n = A.shape[0]
    L = np.zeros_like(A)
    S = np.ones(n)
    zero = False
    for j in range(n):
        sj = A[j, j]
        for p in range(j):
            sj -= (L[j, p] * S[p]) * L[j, p]
        sg = -1.0 if sj < 0.0 else 1.0
        S[j] = sg
        zero |= sj == 0.0
        djj = 1.0 / np.sqrt(sg * sj) if sj != 0.0 else np.inf
        L[j, j] = djj
        for i in range(j + 1, n):
            t = A[i, j]
            for p in range(j):
                t -= L[i, p] * (L[j, p] * S[p])
            L[i, j] = (t * djj) * sg
    return L, S, zero


def signed_solve(L, S, b):
    """k_lm_solve: y = M⁻¹ b (reciprocal diagonal), y *= S, x = M⁻ᵀ y."""
    n = len(b)
    y = np.zeros(n)
    for i in range(n):
        t = b[i]
        for p in range(i):
            t -= L[i, p] * y[p]
        y[i] = t * L[i, i]
    y *= S
    x = np.zeros(n)
    for i in range(n - 1, -1, -1):
        t = y[i]
        for p in range(i + 1, n):
            t -= L[p, i] * x[p]
        x[i] = t * L[i, i]
    return x


def ldlt_pivots(A):
    """oracle/refhlm.cpp ldlt_solve's pivots D_j (unpivoted)."""
    n = A.shape[0]
    Lw = A.copy()
    D = np.zeros(n)
    for j in range(n):
        dj = Lw[j, j] - sum(Lw[j, k] * Lw[j, k] * D[k] for k in range(j))
        D[j] = dj
        for i in range(j + 1, n):
            Lw[i, j] = (Lw[i, j] - sum(Lw[i, k] * Lw[j, k] * D[k] for k in range(j))) / dj
    return D


@pytest.mark.parametrize("dim", [3, 4])
def test_signed_factor_solves_indefinite_blocks(dim):
    rng = np.random.default_rng(7 + dim)
    for _ in range(200):
        Q, _r = np.linalg.qr(rng.standard_normal((dim, dim)))
        ev = rng.uniform(0.2, 3.0, dim) * rng.choice([-1.0, 1.0], dim)
        A = (Q * ev) @ Q.T
        if np.min(np.abs(ldlt_pivots(A))) < 1e-3:   # keep the unpivoted factor well conditioned
            continue
        L, S, zero = signed_factor(A)
        assert not zero
        # the signs are the LDLᵀ pivots' signs (Sylvester: same inertia as A)
        np.testing.assert_array_equal(S, np.sign(ldlt_pivots(A)))
        assert int((S < 0).sum()) == int((ev < 0).sum())
        b = rng.standard_normal(dim)
        np.testing.assert_allclose(signed_solve(L, S, b), np.linalg.solve(A, b), rtol=1e-9, atol=1e-9)
        # M S Mᵀ reproduces A (M = L with the reciprocal diagonal inverted)
        M = L.copy()
        np.fill_diagonal(M, 1.0 / np.diag(L))
        np.testing.assert_allclose((M * S) @ M.T, A, rtol=1e-10, atol=1e-10)


def test_positive_definite_blocks_keep_the_cholesky_form():
    """S = +1 everywhere on an SPD block: the g2o path's lm_chol (sgn = false) is the same factor."""
    rng = np.random.default_rng(3)
    for _ in range(50):
        J = rng.standard_normal((6, 4))
        A = J.T @ J + 1e-3 * np.eye(4)
        L, S, zero = signed_factor(A)
        assert not zero and np.all(S == 1.0)
        np.testing.assert_allclose(np.linalg.inv(np.diag(np.diag(L))) + np.tril(L, -1),
                                   np.linalg.cholesky(A), rtol=1e-10, atol=1e-12)


def test_rank_one_block_meets_a_zero_pivot_like_the_oracle():
    """A single-observation point (H = w·JᵀJ, rank 1) with a structurally exact cancellation: both
    factorisations see the same exactly zero second pivot, which fails the solve (X unchanged)."""
    J = np.array([[2.0, 4.0, 1.0]])   # powers of two: every product and difference is exact
    A = J.T @ J
    with np.errstate(divide="ignore", invalid="ignore"):   # the rows past the zero pivot
        L, S, zero = signed_factor(A)
        D = ldlt_pivots(A)
    assert zero
    assert D[1] == 0.0
