"""Algorithmic bytes per kernel launch: the bytes a launch must move at
minimum — each input array read once, each output written once, per-landmark / per-pose
state counted once (not once per edge). Re-reads through L2/MALL and padding are *not*
counted; PMC traffic above these figures is waste.

Units (f64 = 8 B, index = 4 B), with E = E_p + E_l, E_f = edges whose pose is free,
n_lm = N_p + N_l, nf = free poses, T = Schur triples, nblk = RCS blocks, nch = chunks,
bw = envelope bandwidth in pose blocks.
"""
from __future__ import annotations

from .synth import Graph

F = 8
I = 4


def state_bytes(g: Graph) -> int:
    """pose (12 f64), point (3 f64), line orth (4 f64) — read once."""
    return g.n_kf * 12 * F + g.n_pt * 3 * F + g.n_ln * 4 * F


def kernel_bytes(g: Graph, name: str, st: dict) -> float:
    E, Ep, El = g.n_ept + g.n_eln, g.n_ept, g.n_eln
    Ef = st.get("free_edges", E)
    n_lm = g.n_pt + g.n_ln
    nf = st.get("nf", int((g.kf_fixed == 0).sum()))
    bw = st.get("bw", 7)
    T = st.get("triples", 0)
    nblk = st.get("nblk", 0)
    nch = st.get("chunks", 0)
    blk = 36 * F
    if name == "k_linearize":
        # read: 2 indices, obs (2|4 f64), info, active flag, pose index; states once
        # write: A (12), c (2), B (8), χ² (1) per edge
        rd = Ep * (2 * I + 2 * F + F + 1 + I) + El * (2 * I + 4 * F + F + 1 + I) + state_bytes(g)
        return rd + E * (12 + 2 + 8 + 1) * F
    if name == "k_iter_reduce":
        # pose role: per free edge its index, A (12), c (2); 4 parts x 27 partial sums per pose
        # landmark role: per edge B (8), c (2); per landmark offset, Hll (10) + b_l (4) out
        return (Ef * (I + 14 * F) + nf * 4 * 27 * F
                + E * (8 + 2) * F + n_lm * (I + (10 + 4) * F))
    if name == "k_iter_init":
        # the pose parts in, Hpp (36) + b_p (6) out
        return nf * 4 * 27 * F + nf * (36 + 6) * F
    if name == "k_edge_schur":
        # per edge: landmark index, B (8) in; Z (8), q (2) out; per landmark Hll (10) + b_l (4) once
        return E * (I + 8 * F + 10 * F) + n_lm * (10 + 4) * F
    if name == "k_rcs_chunk":
        # every edge's A (12) and Z (8), q (2) read once; the triple list; 42 partials per chunk
        return E * (12 + 8 + 2) * F + T * 2 * I + nch * 42 * F
    if name == "k_rcs_finalize":
        return nch * 42 * F + nf * (36 + 6) * F + nblk * blk + nf * 6 * F
    if name in ("k_rcs_factor", "k_rcs_factor_band", "k_rcs_factor_twisted"):
        # band in (nf·(bw+1) blocks) + b_s; L band, S⁻¹, z, x_p out; then the pose update:
        # current poses in, trial poses out, b_p in
        return (nf * (bw + 1) * blk + nf * 6 * F + nf * bw * blk + nf * (36 + 6 + 6) * F
                + g.n_kf * (12 + 12) * F + nf * 6 * F)
    if name == "k_rcs_factor_bcr":
        # block cyclic reduction over N = ceil(nf/bw) super-rows of S = 6·bw: band + b_s in once;
        # every non-root super-row writes one Schur record (36·NG Gram-tile values, NG = lower
        # triangle of (2bw+1)² blocks minus the (b,b) corner) read by its two neighbours; each
        # solution record (S) written once and read by up to two neighbours; x_p and the poses
        S = 6 * bw
        N = -(-nf // max(bw, 1))
        NG = (2 * bw + 1) * (2 * bw + 2) // 2 - 1
        return (nf * (bw + 1) * blk + nf * 6 * F + (N - 1) * 36 * NG * F * 3 + N * S * F * 3
                + nf * 6 * F + g.n_kf * (12 + 12) * F + nf * 6 * F)
    if name == "k_pose_update":
        return g.n_kf * (12 + 12) * F + nf * 12 * F
    if name == "k_lm_solve":
        # per landmark: X (4), b_l (4), Hll (10) in, X_trial (4), x_l (4) out; per free edge the
        # back-substitution reads A (12) and B (8); x_p once; then the trial evaluation of every
        # edge: pose index, active flag, obs (2|4), info in, χ² out; trial poses once
        ev = Ep * (I + 1 + 2 * F + F) + El * (I + 1 + 4 * F + F) + E * F + g.n_kf * 12 * F
        return n_lm * (4 + 4 + 10 + 4 + 4) * F + n_lm * I + Ef * (I + (12 + 8) * F) + nf * 6 * F + ev
    return 0.0
