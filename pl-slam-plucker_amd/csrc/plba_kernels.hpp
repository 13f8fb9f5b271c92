// plba_kernels.hpp — HIP kernels of the LM solve (gfx950, FP64, wave64).
//
// Per LM outer iteration (OptimizationAlgorithmLevenberg::solve):
//   k_linearize        edge-parallel: error, χ², Huber weight, weighted Jacobians
//                      (computeActiveErrors + linearizeOplus + constructQuadraticForm, A5/A6/A9/A10)
//   k_iter_reduce      one launch, two roles: pose-parallel partial sums of Hpp, b_p
//                      (kPoseParts workgroups per pose) and landmark-parallel Hll, b_l,
//                      max|diag| partials
//   k_iter_init        Hpp, b_p from the pose parts, χ²_cur, λ init (τ·max|H_jj|, iteration 0)
// Stage switch (initializeOptimization): folded into the iteration kernels of the first step
// of a stage — k_linearize classifies and activates edges, k_iter_reduce activates
// landmarks, k_iter_init advances the stage (or skips it when nothing is active).
// Per damped trial (TRIAL_GUARD):
//   k_edge_schur       edge-parallel: (Hll+λI) = LLᵀ of its landmark, Z_e = B_e L⁻ᵀ, q_e = Z_e L⁻¹b_l
//   k_rcs_chunk        one wave per chunk of <=128 (e1,e2) triples of one RCS block:
//                      Σ A₁ᵀ(Z₁Z₂ᵀ)A₂ (and Σ A_eᵀq_e on diagonal blocks)
//   k_rcs_finalize     per block entry: Hpp+λI − Σ chunks into the band (or dense) matrix, b_s
//   k_rcs_factor_twisted<BW>  two workgroups: two-sided block-banded LDLᵀ meeting at a
//                      bw-block separator, forward/backward solve (LinearSolverEigen);
//                      k_rcs_factor_band<BW> (one sweep) and the dense k_rcs_factor (bw>20)
//                      are the fallbacks
//                      ... each ending with the pose oplus of the free poses (pose_update_wg)
//   k_lm_solve         landmark-parallel: x_l = L⁻ᵀL⁻¹(b_l − Σ_e B_eᵀA_e x_p), oplus, Σx(λx+b)
//                      partials, then the landmark's edges' χ² at the trial state (robust partials)
//   k_decide           ρ, accept/reject, λ/ν update, optimize() loop control (g2o Levenberg)
//                      (accepting flips Ctrl::cur: the trial buffer becomes the current state)
// After the schedule: k_refresh (level-1 computeError) and k_depth (isDepthPositive).
// All reductions are fixed-order trees: results are bitwise reproducible run to run.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/plba.h"
#include "plba_math.hpp"

namespace plba {

constexpr int kBlock = 256;
constexpr int kLmBlock = 64;  // landmark-parallel kernels: 24k landmarks at C3 -> 375 workgroups, not 94
#ifndef PLBA_CHUNK
#define PLBA_CHUNK 256
#endif
constexpr int kChunk = PLBA_CHUNK;  // Schur triples per assembly wave (4 per lane)
constexpr int kTraceCap = 64;
constexpr int kTile = 32;   // RCS factorisation tile (dense fallback)
constexpr int kBandMax = 27; // widest envelope (in pose blocks) the register-window factorisation holds
#ifndef PLBA_BAND_NT
#define PLBA_BAND_NT 768
#endif
constexpr int kBandNT = PLBA_BAND_NT; // threads of the banded factorisation workgroup (bw <= 24)
// rows of a band block one worker owns in registers (plba_kernels.hpp band_forward): whole 6x6
// blocks at 512 threads (256 VGPRs), half blocks when more, smaller waves are configured
// Bandwidths 25..27 need more owned blocks than 704 worker threads hold at three rows each: they
// run 512-thread workgroups owning whole blocks (256 VGPRs, no scratch; at bw 23 that form was 6 %
// slower than 768 threads at half blocks)
__host__ __device__ constexpr int band_nt(int bw) { return bw <= 24 ? kBandNT : 512; }
__host__ __device__ constexpr int band_ur(int bw) { return band_nt(bw) <= 512 ? 6 : 3; }
// Speculative trials (DESIGN §2 "Speculative trials"): a step may evaluate up to kMaxSpec damped
// trials of one linearisation at once — λ, λ·ν, λ·ν·2ν, ... (exactly the λ sequence g2o's
// Levenberg loop walks after rejections) — in trial slots 0..W-1 (blockIdx.y of the trial
// kernels); k_decide consumes them in order, as the sequential loop would have evaluated them.
// State-like arrays rotate through kNB buffers so that no slot overwrites the current state,
// the last consumed χ² or the last successful solve.
constexpr int kMaxSpec = 4;
constexpr int kNB = kMaxSpec + 1;

// Device-resident LM control block: the g2o optimize()/solve() loop runs as a state machine
// advanced by k_decide, so the host only replays a captured "step" graph and polls this block.
struct Ctrl {
    double lambda, ni, currentChi, tempChi, rho, scale, maxdiag;
    double chi2_start, lambda_start;
    double chi2_final[2];
    int32_t qmax, accept, broke;
    int32_t solve_ok[kMaxSpec];                        // per trial slot: the factorisation succeeded
    int32_t last_ok, chi_src;                          // xp/xl buffer of the last successful consumed solve,
                                                       // χ² buffer of the last consumed trial (or linearisation)
    int32_t spec_w, spec_sticky;                       // trial slots of the next step; a rejection seen in
                                                       // this optimize() call
    int32_t stage, n_stages, iter, need_iter;        // schedule position
    int32_t all_done, switch_pending, robust, level;
    int32_t max_iters[2], iters_done[2];
    int32_t stage_robust[2], stage_level[2], stage_classify[2];
    int32_t max_trials, ntrace, any_active, cur;      // cur: which state buffer is current
    int32_t steps;                                     // step graphs that did work (diagnostic)
    int32_t dev_error;                                 // a bounded in-kernel wait timed out
    // hand-rolled LM (plba_hlm_lba, src/mapHandler.cpp:1618-2332): the same step graph with the
    // scalar-residual linearisation, Marquardt damping, se(3) pose update and its own decision
    int32_t hlm;                                       // 0: g2o Levenberg, 1: levMarquardtOptimizationLBAForPluker
    int32_t hlm_lin, hlm_solves, hlm_acc;              // linearisations, solves, applied updates
    int32_t pad[2];
    double hlm_lambda0, hlm_k, hlm_homog, hlm_minerr, hlm_minchg;
    double hlm_nobs;                                   // err divisor (0 = the reference's Npt_obs+Nls_obs)
    double err_prev, dx2;                              // err of the previous linearisation, ‖DX‖² of the last solve
};

// All device pointers of one window (passed by value to every kernel).
struct Dev {
    int32_t n_kf, n_pt, n_ln, n_lm, Ep, El, E, nf, n;
    int32_t corrected, n_lin_blocks, n_lm_blocks, n_kf_blocks, nblk, ntiles;
    int32_t solve_lds_n;                // dense solve: y in LDS up to this n (kSolveLdsN; tests lower it)
    int32_t n_lms_blocks;               // k_lm_solve workgroups (kLmLanes lanes per landmark)
    Cam cam;
    double huber_pt, huber_ln, tau;
    // state
    // state buffers: Tb[ctrl->cur] is the current estimate; trial slot s writes Tb[(cur+1+s) % nbs];
    // accepting slot s moves ctrl->cur there (g2o's push/pop/discardTop without a copy)
    double *Tb[kNB], *T_init;           // [n_kf][12]
    double *Xb[kNB], *X_init;           // [n_lm][4]
    double *xk[kNB];                    // [n_kf][6] se(3) pose vectors X_i of the hand-rolled LM
    double *XL[kNB];                    // [n_ln_g][6] GBA line3D endpoints, reference (global) line order
    double *Hl6, *bl6;                  // [n_ln][21], [n_ln][6] GBA line blocks (packed lower 6x6)
    int32_t *ln_gidx;                   // [n_ln] device line -> reference (global) line index
    double *Lpb[kNB];                   // [n_ln][8]: Plücker vector (6) of each line at Xb[i]
                                        //   (k_line_pluker at schedule start, then k_lm_solve)
    // solve / χ² buffers: slot s writes xpb/xlb[(last_ok+1+s) % nbx] and chi2b[(chi_src+1+s) % nbx]
    // (nbx = 1 without speculation: one buffer, as g2o's _x and the edges' _error)
    double *xpb[kNB], *xlb[kNB], *chi2b[kNB];
    int32_t nbs, nbx;                   // state buffers (spec_max + 1), solve / χ² buffers
    int32_t spec_max, spec_policy;      // trial slots captured per step; when to use them (kSpec*)
    // ---- resolved per trial slot by slot_view() (trial kernels) / cur_view() (others)
    int32_t slot;
    double lam;                         // λ of this slot
    double *Tc, *Tt, *Xc, *Xt, *Lpc, *Lpt, *xkc, *xkt, *XLc, *XLt;  // current / trial state of the slot
    double *xp_prev, *xl_prev;          // solution of the last successful solve (used when this one fails)
    int32_t *solve_okp;                 // &ctrl->solve_ok[slot]
    int32_t *cnt_rcs;                   // [spec_max][nblk] arrival counters of the RCS blocks
    int32_t *kf_hidx;                   // [n_kf]
    // edges, landmark-major CSR order (points first, then lines)
    int32_t *e_lm, *e_kf, *e_hidx;      // [E]
    double *e_obs;                      // [E][4]
    double *e_info;                     // [E]
    uint8_t *e_level, *e_active;        // [E]
    int32_t *lm_off;                    // [n_lm+1]
    uint8_t *lm_active;                 // [n_lm]
    int32_t *pe_off, *pe_list;          // free-pose-major edge lists [nf+1], [..]
    // linearisation
    double *A, *cvec, *B, *chi2_last;   // [E][12], [E][2], [E][8], [E] (chi2_last: this slot's χ² buffer)
    double *Hpp, *bp;                   // [nf][36], [nf][6]
    double *Hll, *bl;                   // [n_lm][10], [n_lm][4]
    // Schur
    double *Z, *q, *xl;                 // [E][8], [E][2], [n_lm][4]
    // reduced camera system
    int32_t *blk_i1, *blk_i2, *blk_off; // [nblk], [nblk], [nblk+1]
    int32_t *trip;                      // [T][2]
    int32_t nch;                        // triple chunks (<= kChunk triples, one block each)
    int32_t *ch_blk, *ch_off;           // [nch], [nch+1] (triple range)
    int32_t *blk_ch;                    // [nblk+1] chunk range of each block
    double *ch_part;                    // [nch][42]  partial block sums (36) + b_s sums (6)
    double *Ad, *bs, *xp, *Wbuf;        // [n*n], [n], [n], [n*(kTile+1)] (W, then y of the dense path)
    int32_t *tile_first;                // [ntiles] first nonzero column tile of each row tile
    int32_t *tile_last;                 // [ntiles] last row tile whose envelope reaches column tile K
    // block-band storage (used when the envelope bandwidth bw <= kBandMax)
    int32_t bw, band_mode;              // bandwidth in pose blocks; 1 = banded factorisation
    int32_t dense_mfma;                 // dense RCS on many workgroups + MFMA (plba_dense.hpp)
    int32_t ring;                       // steps of L / S^-1 / z staged in LDS between global flushes
    unsigned long long *stamps;         // diagnostic build only (PLBA_STAMPS): per-phase cycle sums
    int32_t *first_blk;                 // [nf] first block column of each block row (lower)
    double *Bd;                         // [nf][bw+1][36]  block (i, i-w), row-major 6x6
    double *Lband;                      // [nf][bw+1][36]  L_{i,i-w} (w >= 1)
    double *Kinv;                       // [nf][36]        S_k^{-1}
    double *zb;                         // [nf][6]         z = D_B^{-1} y
    // reductions
    double *part_chi2;                  // [n_lin_blocks]
    double *wg_red, *grp_red;           // folded init: [nred][3], [ceil(nred/64)][3] (χ², max, any)
    int32_t *part_any;                  // [n_lm_blocks] block has an active landmark
    double *part_max;                   // [nf + n_lm_blocks] (landmark part from nf on)
    double *part_lm, *part_lms;         // [n_lms_blocks] trial χ² partials, scale partials (k_lm_solve)
    double *part_ps;                    // [n_ps] pose part of Σx(λx+b) (one slot per factorisation workgroup)
    int32_t n_ps;                       // max(n_kf_blocks, bcr_N)
    int32_t fold;                       // 1: k_rcs_finalize / k_decide run as the tails of the
                                        //    preceding launch (last arriver); 0 when sharded
    int32_t fold_init;                  // 1: k_iter_init runs as the tail of k_iter_reduce
    int32_t *cnt;                       // [2 + nblk + nf] arrival counters: lm_solve, iter_reduce, per RCS block, per pose
    int32_t *h_kf;                      // [nf] keyframe of each free-pose Hessian index
    Ctrl *ctrl;
    plba_iter_trace *trace;             // [kTraceCap] per-iteration records written by k_decide
    // sharded windows: the arrays the ranks sum with one all-reduce each
    int32_t sharded, nranks, rank;
    int32_t n_lm_g, E_g;                // whole-window landmark / edge counts
    // Out-of-place (send *_loc -> receive) so that replaying a step whose kernels were guarded
    // off re-reduces unchanged partials and leaves the totals intact.
    double *red_iter, *red_iter_loc;    // [nf*43 + 2 + nranks] (sharded [nf*13 + ...], see Hdg): Hpp | b_p | #active edges | χ² | active | lm max per rank
    double *red_rcs, *red_rcs_loc;      // [nblk*36 + nf*6]: Σ A₁ᵀZ₁Z₂ᵀA₂ per block | Σ A_eᵀq_e per pose
    // sharded, all-gather exchange (xg_P > 0): each rank's partial RCS is nonzero only on the
    // block rows of its keyframe range; xg_rng[4r..4r+3] = rank r's two runs of red_rcs
    // (block run start, length | right-hand-side run start, length, in doubles), xg_send = this
    // rank's runs packed (P doubles; host transport: its slot of an R x P array), xg_recv = R x P
    double *xg_send, *xg_recv;
    int64_t *xg_rng;
    int64_t xg_P;
    int32_t xg_host;
    double *red_dec, *red_dec_loc;      // [3]: trial χ² | landmark part of Σx(λx+b) | failed solves (sharded)
    double *Hpp_w, *bp_w;               // where pose_combine writes (== Hpp, bp unless sharded)
    // sharded: the iteration all-reduce carries only diag(Hpp) | b_p | active counts | scalars
    // (nf·13 + 2 + R); this rank's full partial Hpp (Hpp_w, local) rides in the RCS exchange inside
    // its diagonal blocks (k_rcs_blockpart), so Hpp is nullptr and Hdg holds the summed diagonals
    double *Hdg, *Hdg_w;                // [nf][6] (sharded only)
    double *pose_part;                  // [nf][kPoseParts][kPP] partial Σ AᵀA (upper), Σ Aᵀc, #active edges
    double *pact, *pact_w;              // [nf] active edges of each free pose (0 = vertex inactive in g2o)
    int32_t *lm_gpos, *e_gpos;          // local landmark / edge -> whole-window position
    double *gat;                        // [n_lm_g*4 + 3*E_g] final gather buffer
    // two-sided banded factorisation (k_rcs_factor_twisted)
    int32_t cl;                         // column-lane factorisation (plba_band_cl.hpp)
    int32_t diag;                       // PLBA_DIAG timing-experiment bits (0 in every real run)
    int32_t twisted, tw_m;              // enabled; rows 0..tw_m-1 top-down, separator tw_m..tw_m+bw-1
    double *Bd2, *bs2;                  // block-reversed band / rhs (row r' = nf-1-i)
    double *Lband2, *Kinv2, *zb2;       // factors of the bottom segment (reversed numbering)
    double *tw_sep;                     // [2][bw][bw+1][36] + [2][bw][6] separator windows
    int32_t *tw_fail, *tw_count;        // [2] per-segment failure, arrival counter
    // block cyclic reduction over super-rows of bw pose blocks (plba_bcr.hpp)
    int32_t bcr, bcr_N;                 // enabled; super-rows (= workgroups of the launch)
    int32_t bcr_fused;                  // back substitution + pose update in the forward launch (1) or
                                        // a second launch, k_rcs_bcr_back (0: PLBA_BCR_SPLIT=1)
    double *bcr_pub;                    // [N][bcr_pub_doubles(bw)] Schur contributions + coupling
    double *bcr_x;                      // [N][6 bw] solution of each super-row
    double *bcr_X;                      // [N][6 bw][12 bw + 1] X = D_m⁻¹[U | V | b] (forward -> backward)
    uint32_t *bcr_flag;                 // [N][2] forward / backward hand-off flags (epoch)
    uint32_t *bcr_ctl;                  // [kBcrCtl] epoch, forward arrivals / tickets, backward arrivals / tickets
    unsigned long long *bcr_stamps;     // [N][32] phase timestamps (PLBA_DIAG bit 8 only)
    int64_t bcr_sl[6];                  // per trial slot strides of bcr_pub, _x, _X, _flag, _ctl, _stamps
};


// current state, read straight from the kernel arguments (kernels outside the trial: the index is
// dynamic, so these must not be applied to a local copy of Dev)
__device__ __forceinline__ double *Tcur(const Dev &d) { return d.Tb[d.ctrl->cur]; }
__device__ __forceinline__ double *Xcur(const Dev &d) { return d.Xb[d.ctrl->cur]; }
// per-edge χ² as g2o's edges hold it (the last consumed trial's, or the last linearisation's)
__device__ __forceinline__ double *chi2cur(const Dev &d) { return d.chi2b[d.ctrl->chi_src]; }

// element counts of the per-slot arrays (each allocated spec_max times back to back; the host
// allocation in plba.hip uses the same functions)
__host__ __device__ __forceinline__ size_t sl_band(const Dev &d) { return d.band_mode ? (size_t)d.nf * (d.bw + 1) * 36 : 1; }
__host__ __device__ __forceinline__ size_t sl_tw(const Dev &d) { return (size_t)d.nf * (d.bw + 1) * 36; }
__host__ __device__ __forceinline__ size_t sl_sep(const Dev &d) {
    return 2 * ((size_t)d.bw * (d.bw + 1) * 36 + (size_t)d.bw * 6);
}
__host__ __device__ __forceinline__ size_t sl_chp(const Dev &d) { return (size_t)(d.nch > 1 ? d.nch : 1) * 42; }
__host__ __device__ __forceinline__ size_t sl_lms(const Dev &d) { return (size_t)(d.n_lms_blocks > 1 ? d.n_lms_blocks : 1); }

// The window as trial slot s sees it: λ_s (g2o's λ after s rejections: λ *= ν, ν *= 2 — the same
// operations in the same order, so bitwise the λ the sequential loop would use), the state it
// starts from and the buffers it writes, and its own copies of every λ-dependent array.
// Returns a copy of Dev whose rotating-buffer arrays (Tb, Xb, ...) must not be indexed: only the
// resolved pointers are valid in it.
__device__ __forceinline__ Dev slot_view(const Dev &d0, int s) {
    Dev d = d0;
    const Ctrl *c = d0.ctrl;
    double lam = c->lambda, ni = c->ni;
    for (int k = 0; k < s; ++k) {
        lam *= ni;
        ni *= 2.0;
    }
    d.slot = s;
    d.lam = lam;
    const int cur = c->cur, ts = (cur + 1 + s) % d0.nbs;
    d.Tc = d0.Tb[cur]; d.Tt = d0.Tb[ts];
    d.Xc = d0.Xb[cur]; d.Xt = d0.Xb[ts];
    d.Lpc = d0.Lpb[cur]; d.Lpt = d0.Lpb[ts];
    d.xkc = d0.xk[cur]; d.xkt = d0.xk[ts];
    d.XLc = d0.XL[cur]; d.XLt = d0.XL[ts];
    const int lo = c->last_ok, xw = (lo + 1 + s) % d0.nbx;
    d.xp = d0.xpb[xw]; d.xl = d0.xlb[xw];
    d.xp_prev = d0.xpb[lo]; d.xl_prev = d0.xlb[lo];
    d.chi2_last = d0.chi2b[(c->chi_src + 1 + s) % d0.nbx];
    d.solve_okp = const_cast<int32_t *>(c->solve_ok) + s;
    if (s) {
        const size_t E = (size_t)d0.E, nf = (size_t)d0.nf, ss = (size_t)s;
        d.Z += ss * E * 8;
        d.q += ss * E * 2;
        d.ch_part += ss * sl_chp(d0);
        d.Bd += ss * sl_band(d0);
        d.Lband += ss * sl_band(d0);
        d.bs += ss * (size_t)d0.n;
        d.Kinv += ss * nf * 36;
        d.zb += ss * nf * 6;
        if (d0.twisted) {
            d.Bd2 += ss * sl_tw(d0);
            d.Lband2 += ss * sl_tw(d0);
            d.bs2 += ss * nf * 6;
            d.Kinv2 += ss * nf * 36;
            d.zb2 += ss * nf * 6;
            d.tw_sep += ss * sl_sep(d0);
            d.tw_fail += 2 * ss;
            d.tw_count += ss;
        }
        if (d0.bcr) {
            d.bcr_pub += ss * d0.bcr_sl[0];
            d.bcr_x += ss * d0.bcr_sl[1];
            d.bcr_X += ss * d0.bcr_sl[2];
            d.bcr_flag += ss * d0.bcr_sl[3];
            d.bcr_ctl += ss * d0.bcr_sl[4];
            d.bcr_stamps += ss * d0.bcr_sl[5];
        }
        d.part_lm += ss * sl_lms(d0);
        d.part_lms += ss * sl_lms(d0);
        d.part_ps += ss * (size_t)d0.n_ps;
        d.cnt_rcs += ss * (size_t)d0.nblk;
    }
    return d;
}

// ---------------------------------------------------------------- block reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v = fmax(v, __shfl_xor(v, m, 64));
    return v;
}
// deterministic block sum: xor-butterfly inside each wave, then waves in index order.
// `sh` needs NT/64 doubles. Every thread receives the result.
template <int NT>
__device__ __forceinline__ double block_sum(double v, double *sh) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) r += sh[w];
    __syncthreads();
    return r;
}
template <int NT>
__device__ __forceinline__ double block_max(double v, double *sh) {
    v = wave_max(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) r = fmax(r, sh[w]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ bool is_point_lm(const Dev &d, int lm) { return lm < d.n_pt; }

// ---------------------------------------------------------------- in-launch hand-offs
// Write-through (sc1) stores / loads: MI355X_MICROARCH.md "Valid forms" row 1 — data stored sc1,
// every storing wave drained, one lane per workgroup adds to an agent-scope counter, the
// workgroup whose add returns total-1 is last and reads the others' data with sc1 loads.
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Every thread calls it after its sc1 stores; true in the last of `total` arriving workgroups,
// which resets the counter for the next launch (exactly `total` arrivals per launch).
__device__ __forceinline__ bool arrive_last(int32_t *counter, int32_t total) {
    __shared__ int s_last_arrival;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int32_t old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last_arrival = old == total - 1 ? 1 : 0;
        if (s_last_arrival) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return s_last_arrival != 0;
}

#ifdef PLBA_STAMPS
#define STAMP(slot)                                                                         \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        unsigned long long _t;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if ((threadIdx.x & 63) == 0) { st_acc[slot] += _t - st_last; }                      \
        st_last = _t;                                                                       \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

// Wave-level LDS ordering: this wave's LDS writes are complete and visible to its other lanes.
// Unlike a wavefront fence it does not wait for global loads/stores (vmcnt), so prefetches and
// result stores stay in flight across it.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Workgroup barrier that orders LDS only: global stores/prefetch loads stay in flight across it
// (__syncthreads() would drain vmcnt and put an L2 round trip on every step of a serial chain).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------- linearisation
// iteration kernels run for a new outer iteration and for the first one of a stage (the stage
// switch — SparseOptimizer::initializeOptimization — is folded into them)
// (a bounded in-kernel wait that timed out — Ctrl::dev_error — stops every later kernel of the
// batch; the host then re-solves the window with another factorisation)
#define ITER_GUARD                                                                             \
    {                                                                                          \
        const Ctrl *cg = d.ctrl;                                                               \
        if (cg->all_done || cg->dev_error || !(cg->need_iter || cg->switch_pending)) return;   \
    }
constexpr double kChi2Thr = 5.991;  // src/mapHandler.cpp:6129,6142
// a stage skipped by k_iter_init (no active edge) leaves switch_pending set: no trial
// PLBA_DIAG bit 128 (tests only): the column-lane factorisation reports a failed solve whenever
// bits 20.. of λ's representation are ≡ 0 (mod 3) — a deterministic function of the trial's λ, so
// runs with and without speculative slots fail the same trials (exercises A13's failure path).
__device__ __forceinline__ bool diag_fail(const Dev &d) {
    return (d.diag & 128) && ((unsigned long long)__double_as_longlong(d.lam) >> 20) % 3 == 0;
}
#define TRIAL_GUARD_OF(dd)                                                   \
    {                                                                        \
        const Ctrl *cg = (dd).ctrl;                                          \
        if (cg->all_done || cg->switch_pending || cg->dev_error) return;     \
    }
#define TRIAL_GUARD TRIAL_GUARD_OF(d)
// Trial kernels take the window as d0 and work on slot_view(d0, S): slots at or above this
// step's width (Ctrl::spec_w) exit at once.
#define TRIAL_SLOT(S)                                   \
    TRIAL_GUARD_OF(d0)                                  \
    if ((int)(S) >= d0.ctrl->spec_w) return;            \
    const Dev d = slot_view(d0, (int)(S));

__global__ __launch_bounds__(kBlock) void k_linearize(Dev d) {
    ITER_GUARD
    __shared__ double sh[kBlock / 64];
    const int e = blockIdx.x * kBlock + threadIdx.x;
    double rc = 0.0;
    const Ctrl *cc = d.ctrl;
    const bool sw = cc->switch_pending;
    const int nxt = cc->stage + 1;
    const int robust = sw ? cc->stage_robust[nxt] : cc->robust;
    double *chi2e = chi2cur(d);  // this iteration's χ² go where the last consumed trial's are
#ifndef PLBA_LIN_DIRECT
    // A/c/B rows are staged in LDS and written out as contiguous 1-KB pieces per store instruction:
    // written per lane (96/16/64-B rows at a lane stride) every store instruction of a wave touched
    // ~48 cache lines, and the stores of the long line-edge waves were the kernel's tail
    __shared__ __attribute__((aligned(16))) double stA[kBlock * 12], stc[kBlock * 2], stB[kBlock * 8];
#endif
    if (e < d.E) {
#ifndef PLBA_LIN_DIRECT
        double *A = stA + threadIdx.x * 12, *c = stc + threadIdx.x * 2, *B = stB + threadIdx.x * 8;
#else
        double *A = d.A + (size_t)e * 12, *c = d.cvec + (size_t)e * 2, *B = d.B + (size_t)e * 8;
#endif
        if (sw) {
            const double stale = chi2e[e];
            // every χ² buffer starts the stage with the stale values: an edge the new stage leaves
            // inactive keeps its χ² whichever buffer the stage's last trial writes
            for (int b = 0; b < d.nbx; ++b)
                if (d.chi2b[b] != chi2e) d.chi2b[b][e] = stale;
            // stage switch: classify on the stale χ² and the current depth (src/mapHandler.cpp:
            // 6125-6147), then activate the edges of the optimised level
            if (cc->stage_classify[nxt]) {
                bool bad = stale > kChi2Thr;
                if (e < d.Ep) {
                    double Pc[3];
                    point_pc(Tcur(d) + (size_t)d.e_kf[e] * 12, Xcur(d) + (size_t)d.e_lm[e] * 4, Pc);
                    bad = bad || !(Pc[2] > 0.0);
                }
                if (bad) d.e_level[e] = 1;
            }
            d.e_active[e] = d.e_level[e] == cc->stage_level[nxt] ? 1 : 0;
        }
        if (d.e_active[e] && cc->hlm) {
            // hand-rolled LM (src/mapHandler.cpp:1909-2103): one scalar residual r = ‖e‖ with
            // Cauchy weight w; row 0 of A/B holds √w·J, c = (√w·r, 0), so Σ AᵀA = Σ w JᵀJ and
            // Σ Aᵀc = Σ w J r = g. Point observations read the current pose (the map pose of
            // fixed KFs and, before the first update, of every KF); line observations always
            // read the map pose T_init (:2010-2012) and the current NDw (the map's on the first
            // linearisation, uploaded into Lpb by plba_hlm_lba).
            const int lm = d.e_lm[e], kf = d.e_kf[e];
            const double *obs = d.e_obs + (size_t)e * 4;
            double r, w, Jp[6], Jl[4];
            double Jl6[6] = {0, 0, 0, 0, 0, 0};
            if (e < d.Ep) {
                hlm_point(Tcur(d) + (size_t)kf * 12, Xcur(d) + (size_t)lm * 4, obs, d.cam, cc->hlm_homog, r, w, Jp, Jl);
            } else if (cc->hlm == 2) {
                // GBA: map pose, endpoints line3D on the first linearisation, then both read from
                // the aliased X.block(6Nkf+3Npt+3·j) (src/mapHandler.cpp:3547-3548)
                const int j = d.ln_gidx[lm - d.n_pt];
                const double *XLc = d.XL[cc->cur];
                const bool first = cc->iter == 0;
                const double *P = XLc + (first ? (size_t)j * 6 : (size_t)j * 3);
                const double *Q = XLc + (first ? (size_t)j * 6 + 3 : (size_t)j * 3);
                gba_line(d.T_init + (size_t)kf * 12, P, Q, obs, d.cam, cc->hlm_homog, r, w, Jp, Jl6);
            } else {
                const double *Lc = d.Lpb[cc->cur] + (size_t)(lm - d.n_pt) * 8;
                double L[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) L[k] = Lc[k];
                hlm_line(d.T_init + (size_t)kf * 12, L, obs, d.cam, cc->hlm_homog, r, w, Jp, Jl);
            }
            chi2e[e] = r * r;
            rc = r * r * w;
            const double sw = sqrt(w);
            const bool pose_free = d.e_hidx[e] >= 0;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                A[k] = pose_free ? sw * Jp[k] : 0.0;
                A[6 + k] = 0.0;
            }
            c[0] = sw * r;
            c[1] = 0.0;
            if (e >= d.Ep && cc->hlm == 2) {  // 6-dim landmark row, flat in B
#pragma unroll
                for (int k = 0; k < 6; ++k) B[k] = sw * Jl6[k];
                B[6] = B[7] = 0.0;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    B[k] = sw * Jl[k];
                    B[4 + k] = 0.0;
                }
            }
        } else if (d.e_active[e]) {
            const int lm = d.e_lm[e], kf = d.e_kf[e];
            const double *T = Tcur(d) + (size_t)kf * 12;
            const double *X = Xcur(d) + (size_t)lm * 4;
            const double *obs = d.e_obs + (size_t)e * 4;
            double err[2], Jl[8], Jp[12];
            double delta;
            if (e < d.Ep) {
                double z;
                point_error(T, X, obs, d.cam, err, z);
                point_jac(T, X, d.cam, Jl, Jp);
                // widen 2x3 -> 2x4
                Jl[7] = 0; Jl[6] = Jl[5]; Jl[5] = Jl[4]; Jl[4] = Jl[3]; Jl[3] = 0;
                delta = d.huber_pt;
            } else {
                // changeOrthToPluker of the current state, evaluated once per line (Lpb)
                const double *Lc = d.Lpb[cc->cur] + (size_t)(lm - d.n_pt) * 8;
                double L[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) L[k] = Lc[k];
                line_jac(T, X, L, obs, d.cam, d.corrected, err, Jl, Jp);
                delta = d.huber_ln;
            }
            const double info = d.e_info[e];
            const double chi = err[0] * (info * err[0]) + err[1] * (info * err[1]);
            chi2e[e] = chi;
            double rho0 = chi, rho1 = 1.0;
            if (robust) huber(chi, delta, rho0, rho1);
            rc = rho0;
            const double s = sqrt(rho1 * info);
            const bool pose_free = d.e_hidx[e] >= 0;
#pragma unroll
            for (int k = 0; k < 12; ++k) A[k] = pose_free ? s * Jp[k] : 0.0;
            c[0] = -s * err[0];
            c[1] = -s * err[1];
#pragma unroll
            for (int k = 0; k < 8; ++k) B[k] = s * Jl[k];
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) A[k] = 0.0;
            c[0] = c[1] = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) B[k] = 0.0;
        }
    }
#ifndef PLBA_LIN_DIRECT
    __syncthreads();
    {
        const int e0 = blockIdx.x * kBlock, n = min(kBlock, d.E - e0);
        auto copy_out = [&](const double *src, double *dst, int cnt) {  // cnt doubles, even
            const double2 *s2 = reinterpret_cast<const double2 *>(src);
            double2 *d2 = reinterpret_cast<double2 *>(dst);
            for (int t = threadIdx.x; t < cnt / 2; t += kBlock) d2[t] = s2[t];
        };
        copy_out(stA, d.A + (size_t)e0 * 12, n * 12);
        copy_out(stc, d.cvec + (size_t)e0 * 2, n * 2);
        copy_out(stB, d.B + (size_t)e0 * 8, n * 8);
    }
#endif
    double s = block_sum<kBlock>(rc, sh);
    if (threadIdx.x == 0) d.part_chi2[blockIdx.x] = s;
}

// The iteration's two reductions in ONE launch of 64-thread workgroups (they are independent
// and each alone leaves most of the chip idle):
//   workgroups [0, kPoseParts·nf): pose h, part j sums A_eᵀA_e and A_eᵀc_e over the pose's
//     edges p ≡ 64j + lane (mod 64·kPoseParts) into pose_part[h][j][kPP]; the parts are added in
//     j order by pose_combine (k_iter_init / k_iter_pack) — the same per-lane sets and order
//     as one 256-thread workgroup per pose, so the sums are deterministic;
//   workgroups [kPoseParts·nf, ...): 64 landmarks each, Hll = Σ B_eᵀB_e, b_l = Σ B_eᵀc_e
//     (and, on a stage switch, the landmark activation).
#ifndef PLBA_POSE_PARTS
#define PLBA_POSE_PARTS 4
#endif
constexpr int kPoseParts = PLBA_POSE_PARTS;
#ifndef PLBA_POSE_KU
#define PLBA_POSE_KU 4  // pose-part edges with loads in flight per pass
#endif
constexpr int kPP = 28;        // per pose part: 21 (upper Σ AᵀA) + 6 (Σ Aᵀc) + active-edge count
constexpr int kInitNT = 1024;  // k_iter_init / k_iter_pack: one wide workgroup (the pose combine)

// packed lower-triangular index for 4x4 symmetric
__device__ __forceinline__ constexpr int pk(int r, int c) { return r * (r + 1) / 2 + c; }

// returns max|Hpp_jj| of pose h in the workgroup that combined it (folded init), else 0
__device__ __forceinline__ double pose_partial(const Dev &d, int h, int part) {
    double acc[kPP];
#pragma unroll
    for (int k = 0; k < kPP; ++k) acc[k] = 0.0;
    // kU edges per pass with all their loads issued before the arithmetic (the per-thread
    // chains are edge-index -> A/c misses; one edge at a time leaves them serialised)
    constexpr int S = kPoseParts * 64, kU = PLBA_POSE_KU;
    const int pend = d.pe_off[h + 1];
    for (int p0 = d.pe_off[h] + part * 64 + threadIdx.x; p0 < pend; p0 += kU * S) {
        int ei[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j) ei[j] = p0 + j * S < pend ? d.pe_list[p0 + j * S] : -1;
        double a[kU][12], cv[kU][2];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const int e = ei[j] < 0 ? ei[0] : ei[j];  // in-range address; masked below
            const double *A = d.A + (size_t)e * 12;
#pragma unroll
            for (int k = 0; k < 12; ++k) a[j][k] = A[k];
            cv[j][0] = d.cvec[(size_t)e * 2];
            cv[j][1] = d.cvec[(size_t)e * 2 + 1];
        }
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            if (ei[j] < 0) break;
            acc[27] += d.e_active[ei[j]] ? 1.0 : 0.0;
            const double *a0 = a[j], *a1 = a[j] + 6;
            int idx = 0;
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int cc = r; cc < 6; ++cc) acc[idx++] += a0[r] * a0[cc] + a1[r] * a1[cc];
#pragma unroll
            for (int r = 0; r < 6; ++r) acc[21 + r] += a0[r] * cv[j][0] + a1[r] * cv[j][1];
        }
    }
#ifdef PLBA_POSE_WAVESUM
#pragma unroll
    for (int k = 0; k < kPP; ++k) acc[k] = wave_sum(acc[k]);
    if (threadIdx.x == 0) {
        double *o = d.pose_part + ((size_t)h * kPoseParts + part) * kPP;
#pragma unroll
        for (int k = 0; k < kPP; ++k) st_sc1(o + k, acc[k]);  // read by the pose's combine below
    }
#else
    {
        // the 28 sums as a reduce-scatter: each butterfly step halves the values a lane carries
        // (~220 instead of ~500 instructions); value k ends in lane 2k. The same pairwise
        // additions as wave_sum (a + b in the same butterfly order), so bitwise the same sums.
        const int lane = threadIdx.x;
        double v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = k < kPP ? acc[k] : 0.0;
#pragma unroll
        for (int n = 16; n >= 1; n >>= 1) {
            const int m = 2 * n;  // lane bit of this step: 32, 16, 8, 4, 2
            const bool hi = (lane & m) != 0;
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const double keep = hi ? v[n + i] : v[i], send = hi ? v[i] : v[n + i];
                v[i] = keep + __shfl_xor(send, m, 64);
            }
        }
        v[0] += __shfl_xor(v[0], 1, 64);
        if ((lane & 1) == 0 && lane / 2 < kPP)
            st_sc1(d.pose_part + ((size_t)h * kPoseParts + part) * kPP + lane / 2, v[0]);  // read by the combine below
    }
#endif
    // folded iteration init: the last of the pose's kPoseParts workgroups adds the parts (in part
    // order, as pose_combine does) into Hpp / b_p / active count and publishes max|Hpp_jj|
    // (sharded windows too: the combine then writes this rank's partial Hpp / b_p into the
    // all-reduce source, and k_iter_pack only packs χ² and the landmark maxima)
    if ((d.fold_init || d.sharded) && arrive_last(d.cnt + 2 + d.nblk + h, kPoseParts)) {
        const int k = threadIdx.x;
        double v = 0.0;
        if (k < kPP) {
            const double *src = d.pose_part + (size_t)h * kPoseParts * kPP + k;
            double p[kPoseParts];
#pragma unroll
            for (int j = 0; j < kPoseParts; ++j) p[j] = ld_sc1(src + j * kPP);
            v = p[0];
#pragma unroll
            for (int j = 1; j < kPoseParts; ++j) v += p[j];
            if (k < 21) {
                int r = 0, rem = k;
                while (rem >= 6 - r) { rem -= 6 - r; ++r; }
                const int cc = r + rem;
                d.Hpp_w[(size_t)h * 36 + r * 6 + cc] = v;
                d.Hpp_w[(size_t)h * 36 + cc * 6 + r] = v;
                if (r == cc && d.Hdg_w) d.Hdg_w[(size_t)h * 6 + r] = v;
                if (r != cc) v = 0.0;
            } else if (k < 27) {
                d.bp_w[(size_t)h * 6 + (k - 21)] = v;
                v = 0.0;
            } else {
                d.pact_w[h] = v;
                v = 0.0;
            }
        }
        const double m = wave_max(fabs(v));  // kLmBlock = one wave
        if (threadIdx.x == 0) st_sc1(d.part_max + h, m);
        return m;
    }
    return 0.0;
}

// returns (block max|H_ll diag|, block has an active landmark) through mx_out / any_out
__device__ __forceinline__ void landmark_reduce(const Dev &d, int lb, double &mx_out, int &any_out) {
    __shared__ double sh[kLmBlock / 64];
    const int l = lb * kLmBlock + threadIdx.x;
    const bool sw = d.ctrl->switch_pending;
    double mx = 0.0;
    bool any = false;
    if (l < d.n_lm) {
        if (sw) {  // a landmark is active iff it has an active edge
            bool act = false;
            for (int e = d.lm_off[l]; e < d.lm_off[l + 1]; ++e) act = act || d.e_active[e];
            d.lm_active[l] = act ? 1 : 0;
        }
        any = d.lm_active[l] != 0;
        if (l >= d.n_pt && d.ctrl->hlm == 2) {  // GBA line: 6x6 block (flat 6-vector rows in B)
            double H6[21], b6[6];
#pragma unroll
            for (int k = 0; k < 21; ++k) H6[k] = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) b6[k] = 0.0;
            for (int e = d.lm_off[l]; e < d.lm_off[l + 1]; ++e) {
                double bb[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) bb[k] = d.B[(size_t)e * 8 + k];
                const double c0 = d.cvec[(size_t)e * 2];
#pragma unroll
                for (int r = 0; r < 6; ++r) {
#pragma unroll
                    for (int cc = 0; cc <= r; ++cc) H6[pk(r, cc)] += bb[r] * bb[cc];
                    b6[r] += bb[r] * c0;
                }
            }
            const int li = l - d.n_pt;
#pragma unroll
            for (int k = 0; k < 21; ++k) d.Hl6[(size_t)li * 21 + k] = H6[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) d.bl6[(size_t)li * 6 + k] = b6[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) mx = fmax(mx, fabs(H6[pk(k, k)]));
        } else {
        double H[10], b[4];
#pragma unroll
        for (int k = 0; k < 10; ++k) H[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = 0.0;
        const int e1 = d.lm_off[l + 1];
        for (int e0 = d.lm_off[l]; e0 < e1; e0 += 2) {  // two edges' loads in flight per pass
            double bb[2][8], cc2[2][2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int e = e0 + j < e1 ? e0 + j : e0;
#pragma unroll
                for (int k = 0; k < 8; ++k) bb[j][k] = d.B[(size_t)e * 8 + k];
                cc2[j][0] = d.cvec[(size_t)e * 2];
                cc2[j][1] = d.cvec[(size_t)e * 2 + 1];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (e0 + j >= e1) break;
                const double *b0 = bb[j], *b1 = bb[j] + 4;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
#pragma unroll
                    for (int cc = 0; cc <= r; ++cc) H[pk(r, cc)] += b0[r] * b0[cc] + b1[r] * b1[cc];
                    b[r] += b0[r] * cc2[j][0] + b1[r] * cc2[j][1];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 10; ++k) d.Hll[(size_t)l * 10 + k] = H[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) d.bl[(size_t)l * 4 + k] = b[k];
        mx = fmax(fmax(fabs(H[pk(0, 0)]), fabs(H[pk(1, 1)])), fmax(fabs(H[pk(2, 2)]), fabs(H[pk(3, 3)])));
        }
    }
    double m = block_max<kLmBlock>(mx, sh);
    const int anyb = __syncthreads_or(any ? 1 : 0);
    if (threadIdx.x == 0) {
        st_sc1(d.part_max + d.nf + lb, m);
        __hip_atomic_store(d.part_any + lb, anyb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    mx_out = m;
    any_out = anyb;
}


// Hpp, b_p from the pose parts (added in part order); returns this thread's max |Hpp_jj|
template <int NT, bool SC1 = false>
__device__ __forceinline__ double pose_combine(const Dev &d, double *H, double *bp) {
    double m = 0.0;
    for (int i = threadIdx.x; i < d.nf * kPP; i += NT) {
        const int h = i / kPP, k = i % kPP;
        const double *src = d.pose_part + (size_t)h * kPoseParts * kPP + k;
        double v = SC1 ? ld_sc1(src) : src[0];
#pragma unroll
        for (int j = 1; j < kPoseParts; ++j) v += SC1 ? ld_sc1(src + j * kPP) : src[j * kPP];
        if (k < 21) {
            int r = 0, rem = k;
            while (rem >= 6 - r) { rem -= 6 - r; ++r; }
            const int cc = r + rem;
            H[(size_t)h * 36 + r * 6 + cc] = v;
            H[(size_t)h * 36 + cc * 6 + r] = v;
            if (r == cc) m = fmax(m, fabs(v));
        } else if (k < 27) {
            bp[(size_t)h * 6 + (k - 21)] = v;
        } else {
            d.pact_w[h] = v;
        }
    }
    return m;
}

// sharded windows: this rank's χ² and landmark max|diag| into the all-reduced iteration array
// (Hpp and b_p already sit in it). The rank's max goes to its own slot: the sum over ranks of
// one-hot slots is the list of maxima, reduced with max by k_iter_init.
__global__ __launch_bounds__(kInitNT) void k_iter_pack(Dev d) {
    ITER_GUARD
    __shared__ double sh[kInitNT / 64];
    // (Hpp / b_p / active counts: combined per pose by the last of its k_iter_reduce parts)
    double s = 0.0;
    for (int i = threadIdx.x; i < d.n_lin_blocks; i += kInitNT) s += d.part_chi2[i];
    const double chi = block_sum<kInitNT>(s, sh);
    double m = 0.0;
    for (int i = threadIdx.x; i < d.n_lm_blocks; i += kInitNT) m = fmax(m, d.part_max[d.nf + i]);
    const double mx = block_max<kInitNT>(m, sh);
    int any = 0;
    for (int i = threadIdx.x; i < d.n_lm_blocks; i += kInitNT) any |= d.part_any[i];
    any = __syncthreads_or(any);
    double *o = d.red_iter_loc + (size_t)d.nf * 13;  // (sharded layout: diag | b_p | active | scalars)
    if (threadIdx.x == 0) {
        o[0] = chi;
        o[1] = any ? 1.0 : 0.0;
    }
    for (int r = threadIdx.x; r < d.nranks; r += kInitNT) o[2 + r] = r == d.rank ? mx : 0.0;
}

// the iteration init (k_iter_init's work): run as its own launch (sharded windows, windows with
// nothing to reduce) or as the tail of the last-arriving k_iter_reduce workgroup (SC1: the
// partials of that launch are read write-through)
__device__ __forceinline__ void iter_init_ctrl(const Dev &d, double chi, double mx, bool any);
template <int NT>
__device__ __forceinline__ void iter_init_body(const Dev &d, double *sh) {
    double chi, mx;
    bool any;
    if (d.sharded) {  // totals from the all-reduced iteration array
        const double *o = d.red_iter + (size_t)d.nf * 13;
        double m = 0.0;
        for (int i = threadIdx.x; i < d.nf * 6; i += NT) m = fmax(m, fabs(d.Hdg[i]));
        for (int r = threadIdx.x; r < d.nranks; r += NT) m = fmax(m, o[2 + r]);
        mx = block_max<NT>(m, sh);
        chi = o[0];
        any = o[1] != 0.0;
    } else {
        double m = pose_combine<NT>(d, d.Hpp_w, d.bp_w);
        double s = 0.0;
        for (int i = threadIdx.x; i < d.n_lin_blocks; i += NT) s += d.part_chi2[i];
        chi = block_sum<NT>(s, sh);
        for (int i = threadIdx.x; i < d.n_lm_blocks; i += NT) m = fmax(m, d.part_max[d.nf + i]);
        mx = block_max<NT>(m, sh);
        int a = 0;
        for (int i = threadIdx.x; i < d.n_lm_blocks; i += NT) a |= d.part_any[i];
        any = __syncthreads_or(a) != 0;
    }
    if (threadIdx.x == 0) iter_init_ctrl(d, chi, mx, any);
}
// the control part of the iteration init (one thread): stage switch, λ init / hand-rolled stops
__device__ __forceinline__ void iter_init_ctrl(const Dev &d, double chi, double mx, bool any) {
    {
        Ctrl *c = d.ctrl;
        if (c->switch_pending) {  // initializeOptimization(level) of the next stage
            c->switch_pending = 0;
            c->stage += 1;
            c->iter = 0;
            c->robust = c->stage_robust[c->stage];
            c->level = c->stage_level[c->stage];
            if (!any) {  // _ivMap empty: optimize() returns -1 without iterating
                c->iters_done[c->stage] = -1;
                c->chi2_final[c->stage] = 0.0;
                c->need_iter = 0;
                if (c->stage + 1 < c->n_stages) c->switch_pending = 1;
                else c->all_done = 1;
                return;
            }
        }
        if (c->hlm) {  // src/mapHandler.cpp:1849-1858 (first linearisation), :2108-2112 (later)
            const double err = chi / c->hlm_nobs;  // reference: / (Npt_obs + Nls_obs) == / 0
            c->hlm_lin += 1;
            if (c->iter == 0) {
                c->maxdiag = mx;
                // GBA keeps Hmax in an int (src/mapHandler.cpp:3386): truncated toward zero
                c->lambda = c->hlm_lambda0 * (c->hlm == 2 ? (double)(long long)mx : mx);
            } else if (fabs(err - c->err_prev) < c->hlm_minchg || err < c->hlm_minerr) {
                if (c->ntrace < kTraceCap)
                    d.trace[c->ntrace++] = plba_iter_trace{c->stage, c->iter, 0, 3, err, err, c->lambda, c->lambda};
                c->currentChi = err;
                c->chi2_final[c->stage] = err;
                c->need_iter = 0;
                c->all_done = 1;
                return;
            }
            c->currentChi = err;
            c->chi2_start = err;
            c->lambda_start = c->lambda;
            c->accept = 0;
            c->need_iter = 0;
            return;
        }
        // currentChi: at iteration 0 the χ² of the linearisation; later iterations start at the
        // state of the trial just accepted, whose χ² (the same edges at the same state, summed in
        // another order) is already currentChi — kept, so the folded init can skip its global
        // reduction after the first iteration (k_iter_reduce) and every mode agrees
        if (c->iter == 0) {  // computeLambdaInit: τ·max|H_jj|, ν = 2
            c->currentChi = chi;
            c->maxdiag = mx;
            c->lambda = d.tau * mx;
            c->ni = 2.0;
        }
        c->chi2_start = c->currentChi;
        c->lambda_start = c->lambda;
        c->qmax = 0;
        c->accept = 0;
        c->rho = 0.0;
        c->broke = 0;
        c->need_iter = 0;
    }
}
__global__ __launch_bounds__(kInitNT) void k_iter_init(Dev d) {
    ITER_GUARD
    __shared__ double sh[kInitNT / 64];
    iter_init_body<kInitNT>(d, sh);
}

constexpr int kRedGrp = 256;  // k_iter_reduce workgroups per first-level group of the folded init
// an iteration after the first of its stage (g2o Levenberg, not the hand-rolled LM, unsharded,
// folded init): k_decide has already done the iteration init (decide_body), so k_iter_reduce only
// forms Hpp / b_p / Hll / b_l. Uniform: read before any workgroup can change the control block.
__device__ __forceinline__ bool iter_init_fast(const Dev &d) {
    const Ctrl *c = d.ctrl;
    return d.fold_init && !d.sharded && !c->hlm && !c->switch_pending && c->iter > 0;
}
__global__ __launch_bounds__(kLmBlock) void k_iter_reduce(Dev d) {
    ITER_GUARD
    __shared__ double sh_init[kLmBlock / 64];
    const int b = blockIdx.x, np = kPoseParts * d.nf;
    const int G = (int)gridDim.x, lane = threadIdx.x;
    // folded init: this workgroup's slice of k_linearize's χ² partials, loaded before the main
    // work so the round trip overlaps it
    double sc = 0.0;
    if (d.fold_init && !iter_init_fast(d)) {
        const int lo = (int)((long long)b * d.n_lin_blocks / G), hi = (int)((long long)(b + 1) * d.n_lin_blocks / G);
        for (int i = lo + lane; i < hi; i += kLmBlock) sc += d.part_chi2[i];
    }
    double wmax = 0.0;
    int wany = 0;
    if (b < np) wmax = pose_partial(d, b / kPoseParts, b % kPoseParts);  // workgroup-uniform branch
    else landmark_reduce(d, b - np, wmax, wany);
    if (!d.fold_init) return;
    // after the first iteration of a stage the init needs none of the global terms (λ is set, the
    // χ² is the accepted trial's, no activity change): k_decide already started the iteration
    if (iter_init_fast(d)) return;
    // folded iteration init (k_iter_init's work; the pose combine already ran per pose), reduced
    // in two levels so no single workgroup reads every partial: each workgroup adds a slice of
    // k_linearize's χ² partials to its own (max, any), the last of each group of kRedGrp
    // workgroups combines the group, the last group runs the control step. Fixed order.
    {
        sc = wave_sum(sc);  // kLmBlock = one wave
        if (lane == 0) {
            st_sc1(d.wg_red + 3 * (size_t)b, sc);
            st_sc1(d.wg_red + 3 * (size_t)b + 1, wmax);
            st_sc1(d.wg_red + 3 * (size_t)b + 2, wany ? 1.0 : 0.0);
        }
    }
    constexpr int U = kRedGrp / kLmBlock;
    const int g = b / kRedGrp, gn = min(kRedGrp, G - kRedGrp * g), ng = (G + kRedGrp - 1) / kRedGrp;
    if (!arrive_last(d.cnt + 2 + d.nblk + d.nf + g, gn)) return;
    {
        double cv[U], mv[U], av[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // lane holds members lane·U .. lane·U+U-1, all loads in flight
            const int k = lane * U + u;
            const double *w = d.wg_red + 3 * (size_t)(kRedGrp * g + min(k, gn - 1));
            cv[u] = ld_sc1(w);
            mv[u] = ld_sc1(w + 1);
            av[u] = ld_sc1(w + 2);
        }
        double c = 0.0, m = 0.0, a = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lane * U + u < gn) {
                c += cv[u];
                m = fmax(m, mv[u]);
                a = fmax(a, av[u]);
            }
        c = wave_sum(c);
        m = wave_max(m);
        a = wave_max(a);
        if (lane == 0) {
            st_sc1(d.grp_red + 3 * (size_t)g, c);
            st_sc1(d.grp_red + 3 * (size_t)g + 1, m);
            st_sc1(d.grp_red + 3 * (size_t)g + 2, a);
        }
    }
    if (!arrive_last(d.cnt + 1, ng)) return;
    double c = 0.0, m = 0.0, a = 0.0;
    for (int g0 = 0; g0 < ng; g0 += 64) {  // groups in index order, 64 at a time
        double cg = 0.0, mg = 0.0, ag = 0.0;
        if (g0 + lane < ng) {
            const double *w = d.grp_red + 3 * (size_t)(g0 + lane);
            cg = ld_sc1(w);
            mg = ld_sc1(w + 1);
            ag = ld_sc1(w + 2);
        }
        c += wave_sum(cg);
        m = fmax(m, wave_max(mg));
        a = fmax(a, wave_max(ag));
    }
    (void)sh_init;
    if (lane == 0) iter_init_ctrl(d, c, m, a != 0.0);
}

// ---------------------------------------------------------------- reduced camera system
// one entry of block b: e < 36 the 6x6 value (Hpp + λI on the diagonal minus Σ chunks), 36..41
// the right-hand side b_s = b_p - Σ A_eᵀq_e (diagonal blocks only)
__device__ __forceinline__ void rcs_finalize_entry(const Dev &d, int b, int e, double sacc) {
    const int i1 = d.blk_i1[b], i2 = d.blk_i2[b];
    const bool diag = i1 == i2;
    if (e >= 36 && !diag) return;
    const int n = d.n;
    if (e >= 36) {
        const double v = d.bp[(size_t)i1 * 6 + (e - 36)] - sacc;
        d.bs[6 * i1 + (e - 36)] = v;
        if (d.twisted) d.bs2[6 * (d.nf - 1 - i1) + (e - 36)] = v;
        return;
    }
    const int r = e / 6, c = e % 6;
    if (diag) {
        // (sharded: the exchanged sum already holds −Hpp, k_rcs_blockpart)
        double h = (d.Hpp ? d.Hpp[(size_t)i1 * 36 + e] : 0.0) - sacc;
        // a free pose with no active edge is not in g2o's system (SparseOptimizer activation,
        // SURVEY.md §8 A13); its all-zero block row becomes I (x = 0 exactly) instead of λI,
        // which would be a zero pivot at λ = 0
        // (hand-rolled LM: Marquardt damping H(i,i) += λ·H(i,i), src/mapHandler.cpp:2114-2115)
        if (r == c)
            h += d.pact[i1] == 0.0 ? 1.0
                 : d.ctrl->hlm   ? d.lam * (d.Hpp ? d.Hpp[(size_t)i1 * 36 + e] : d.Hdg[(size_t)i1 * 6 + r])
                                 : d.lam;
        if (d.band_mode) d.Bd[((size_t)i1 * (d.bw + 1)) * 36 + e] = h;
        else d.Ad[(size_t)(6 * i1 + r) + (size_t)(6 * i1 + c) * n] = h;
        if (d.twisted) d.Bd2[((size_t)(d.nf - 1 - i1) * (d.bw + 1)) * 36 + e] = h;
    } else {
        if (d.band_mode) d.Bd[((size_t)i2 * (d.bw + 1) + (i2 - i1)) * 36 + c * 6 + r] = -sacc;
        else d.Ad[(size_t)(6 * i2 + c) + (size_t)(6 * i1 + r) * n] = -sacc;
        // reversed row nf-1-i1 holds block (i1, i2) = (i1, i1 + w) in its natural orientation
        if (d.twisted) d.Bd2[((size_t)(d.nf - 1 - i1) * (d.bw + 1) + (i2 - i1)) * 36 + r * 6 + c] = -sacc;
    }
}

// Chunked reduced-camera assembly, pass 1: one wave per chunk of <= kChunk triples of one
// block; each lane accumulates A₁ᵀ(Z₁Z₂ᵀ)A₂ (36) and, for self-triples of a diagonal block,
// A_eᵀ q_e (6); the wave reduces through LDS in fixed lane order (deterministic).
// STAGED (default): the 64 triples of a batch fetch their A/Z rows cooperatively — load j of
// the wave covers rows (64j + lane)/6 of the batch's A₁ (16 B per lane, consecutive lanes on
// consecutive pieces of one 96-B row), so one load instruction touches ~8-16 cache lines
// instead of 64 (one per lane and piece); the rows land in LDS and every lane then reads its
// own row. The arithmetic per lane is unchanged (bitwise-identical sums).
typedef double dbl2 __attribute__((ext_vector_type(2)));  // register-promotable 16-B pair
template <bool STAGED>
__global__ __launch_bounds__(64) void k_rcs_chunk(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    __shared__ double smem[64 * 43];  // staging: A₁ | A₂ (64x12) | Z₁ | Z₂ (64x8); then red[64][43]
    double(*red)[43] = reinterpret_cast<double(*)[43]>(smem);
    // XCD-aware remap (blocks are dealt round-robin over the 8 XCDs): each XCD gets a contiguous
    // run of chunks = a contiguous range of RCS block rows, so the A/Z rows of the landmarks
    // they couple are re-read from that XCD's L2 instead of the fabric (speed only). The grid's x
    // extent is padded to a multiple of 8 so that every trial slot (blockIdx.y) sees the same
    // block -> XCD assignment; the padding blocks exit.
    const int nb = d.nch, per = (nb + 7) / 8, xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int full = nb - 8 * (per - 1);  // XCDs that get `per` chunks (the rest get per-1)
    if (xcd >= full && slot >= per - 1) return;  // padding
    const int ch = xcd < full ? xcd * per + slot : full * per + (xcd - full) * (per - 1) + slot;
    const int lane = threadIdx.x;
    const int hlm = d.ctrl->hlm;
    const int b = d.ch_blk[ch];
    const bool diag = d.blk_i1[b] == d.blk_i2[b];
    double acc[42];
#pragma unroll
    for (int k = 0; k < 42; ++k) acc[k] = 0.0;
    const int t0 = d.ch_off[ch], t1 = d.ch_off[ch + 1];
    // the next batch's triple indices are loaded one batch ahead, so their latency hides behind
    // this batch's row loads instead of preceding them (rows past the chunk re-read a valid triple)
    int2 nx = make_int2(0, 0);
    if (t0 < t1) nx = reinterpret_cast<const int2 *>(d.trip)[min(t0 + lane, t1 - 1)];
#pragma unroll 1
    for (int q = 0; q < kChunk / 64; ++q) {
        const int tb = t0 + 64 * q;
        if (tb >= t1) break;  // wave-uniform
        const int t = tb + lane;
        const int e1 = nx.x, e2 = nx.y;
        if (tb + 64 < t1) nx = reinterpret_cast<const int2 *>(d.trip)[min(tb + 64 + lane, t1 - 1)];
        double z1[8], z2[8], a1[12], a2[12];
        if (STAGED) {
            dbl2 *sA1 = reinterpret_cast<dbl2 *>(smem), *sA2 = sA1 + 384;
            dbl2 *sZ1 = sA2 + 384, *sZ2 = sZ1 + 256;
            dbl2 v1[6], v2[6], w1[4], w2[4];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int pc = 64 * j + lane, r = pc / 6, k = pc - 6 * r;
                const int f1 = __shfl(e1, r, 64), f2 = __shfl(e2, r, 64);
                v1[j] = reinterpret_cast<const dbl2 *>(d.A + (size_t)f1 * 12)[k];
                v2[j] = reinterpret_cast<const dbl2 *>(d.A + (size_t)f2 * 12)[k];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 16 * j + (lane >> 2), k = lane & 3;
                const int f1 = __shfl(e1, r, 64), f2 = __shfl(e2, r, 64);
                w1[j] = reinterpret_cast<const dbl2 *>(d.Z + (size_t)f1 * 8)[k];
                w2[j] = reinterpret_cast<const dbl2 *>(d.Z + (size_t)f2 * 8)[k];
            }
            __syncthreads();  // the previous batch's rows are read (one wave: a cheap barrier)
            // Bank-conflict-free row reads (ds_read_b128: 16-lane groups, bank (a/4) mod 64):
            //  Z rows (4 pieces, 64-B stride: lanes l, l+4, l+8, l+12 share a bank window) are
            //  stored rotated by ρ(r) = (r >> 2) & 3 pieces, so the lane reading its row at step k
            //  fetches piece k from position (k + ρ) mod 4; stores stay conflict-free.
            //  A rows (6 pieces, 96-B stride: lanes l and l+8 collide) are stored linearly and read
            //  rotated by ρ = (lane >> 3) & 1, the pieces put back in order with selects (rotating
            //  the stores instead would move the conflicts to the stores).
#pragma unroll
            for (int j = 0; j < 6; ++j) { sA1[64 * j + lane] = v1[j]; sA2[64 * j + lane] = v2[j]; }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 16 * j + (lane >> 2), k = lane & 3, pos = 4 * r + ((k + ((r >> 2) & 3)) & 3);
                sZ1[pos] = w1[j];
                sZ2[pos] = w2[j];
            }
            __syncthreads();
            const int ra = (lane >> 3) & 1, rz = (lane >> 2) & 3;
            dbl2 tA1[6], tA2[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int pk = k + ra < 6 ? k + ra : k + ra - 6;
                tA1[k] = sA1[6 * lane + pk];
                tA2[k] = sA2[6 * lane + pk];
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) {  // piece k sits in tA[k] (ra = 0) or tA[k - 1] (ra = 1)
                const dbl2 x = ra ? tA1[(k + 5) % 6] : tA1[k], y = ra ? tA2[(k + 5) % 6] : tA2[k];
                a1[2 * k] = x.x; a1[2 * k + 1] = x.y; a2[2 * k] = y.x; a2[2 * k + 1] = y.y;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int pos = 4 * lane + ((k + rz) & 3);
                const dbl2 x = sZ1[pos], y = sZ2[pos];
                z1[2 * k] = x.x; z1[2 * k + 1] = x.y; z2[2 * k] = y.x; z2[2 * k + 1] = y.y;
            }
        } else {
            const double *Z1 = d.Z + (size_t)e1 * 8, *Z2 = d.Z + (size_t)e2 * 8;
            const double *A1 = d.A + (size_t)e1 * 12, *A2 = d.A + (size_t)e2 * 12;
#pragma unroll
            for (int k = 0; k < 8; ++k) { z1[k] = Z1[k]; z2[k] = Z2[k]; }
#pragma unroll
            for (int k = 0; k < 12; ++k) { a1[k] = A1[k]; a2[k] = A2[k]; }
        }
        if (t < t1) {
            double m00 = 0, m01 = 0, m10 = 0, m11 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m00 = fma(z1[k], z2[k], m00);
                m01 = fma(z1[k], z2[4 + k], m01);
                m10 = fma(z1[4 + k], z2[k], m10);
                m11 = fma(z1[4 + k], z2[4 + k], m11);
            }
            // hand-rolled LM: A has one live row, so only m00 is used — and a GBA line's Z_e
            // (6 entries) spills into Z's second row: the full 8-entry product
            if (hlm == 1) m00 = m01;  // z_1 · (S z_2): row 1 of Z carries S z_0 (edge_schur_body)
            else if (hlm) m00 += m11;
            double Q[12];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                Q[k] = m00 * a2[k] + m01 * a2[6 + k];
                Q[6 + k] = m10 * a2[k] + m11 * a2[6 + k];
            }
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int c = 0; c < 6; ++c) acc[r * 6 + c] += a1[r] * Q[c] + a1[6 + r] * Q[6 + c];
            if (diag && e1 == e2) {
                const double q0 = d.q[(size_t)e1 * 2], q1 = d.q[(size_t)e1 * 2 + 1];
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[36 + r] += a1[r] * q0 + a1[6 + r] * q1;
            }
        }
    }
    if (STAGED) __syncthreads();  // the staging rows are read before red overwrites them
#pragma unroll
    for (int k = 0; k < 42; ++k) red[lane][k] = acc[k];
    __syncthreads();
    if (lane < 42) {
        double sacc = 0.0;
        for (int l = 0; l < 64; ++l) sacc += red[l][lane];
        st_sc1(d.ch_part + (size_t)ch * 42 + lane, sacc);
    }
    // the last chunk of block b to arrive assembles the block (the k_rcs_finalize entry work)
    if (d.fold && arrive_last(d.cnt_rcs + b, d.blk_ch[b + 1] - d.blk_ch[b]) && lane < 42) {
        double sacc = 0.0;
        const int c1 = d.blk_ch[b + 1];
        for (int c0 = d.blk_ch[b]; c0 < c1; c0 += 4) {  // 4 partials in flight, summed in chunk order
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = c0 + u < c1 ? ld_sc1(d.ch_part + (size_t)(c0 + u) * 42 + lane) : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) sacc += v[u];
        }
        rcs_finalize_entry(d, b, lane, sacc);
    }
}

// Chunked reduced-camera assembly with two lanes per triple, for windows with more chunks than
// k_rcs_chunk's waves can hold at once (chunk_half_min, plba.hip): lane h·32 + p takes triple p
// of a 32-triple batch and accumulates block rows 3h .. 3h+2 of A₁ᵀ(Z₁Z₂ᵀ)A₂ (18) and of A_eᵀq_e
// (3). Half the accumulators and half the staging per wave: 216 → 146 VGPRs and 22 → 11 KB of LDS,
// 3 waves per SIMD instead of 1.75 to hide the row loads, at twice the batches per wave (so a
// window whose chunks all fit at once keeps k_rcs_chunk: C3 24.9 vs 25.3 µs; C5 121.7 → 114.7 µs).
// The per-element sums run over the same triples in another lane partition (deterministic, not
// bitwise equal to k_rcs_chunk's).
#ifndef PLBA_CHH_MINB
#define PLBA_CHH_MINB 3  // waves per SIMD the register budget is sized for (4 spills: 115 -> 226 us at C5)
#endif
__global__ __launch_bounds__(64, PLBA_CHH_MINB) void k_rcs_chunk_h(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    constexpr int NB = 32, NA = 22;  // triples per batch; accumulators per lane (21) padded
    __shared__ double smem[64 * NA];  // staging: A₁ | A₂ (32x12) | Z₁ | Z₂ (32x8); then red[64][NA]
    double(*red)[NA] = reinterpret_cast<double(*)[NA]>(smem);
    // XCD-aware chunk order (as k_rcs_chunk)
    const int nb = d.nch, per = (nb + 7) / 8, xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int full = nb - 8 * (per - 1);
    if (xcd >= full && slot >= per - 1) return;  // padding
    const int ch = xcd < full ? xcd * per + slot : full * per + (xcd - full) * (per - 1) + slot;
    const int lane = threadIdx.x, p = lane & (NB - 1), h = lane >> 5;
    const int hlm = d.ctrl->hlm;
    const int b = d.ch_blk[ch];
    const bool diag = d.blk_i1[b] == d.blk_i2[b];
    double acc[21];
#pragma unroll
    for (int k = 0; k < 21; ++k) acc[k] = 0.0;
    const int t0 = d.ch_off[ch], t1 = d.ch_off[ch + 1];
    int2 nx = make_int2(0, 0);
    if (t0 < t1) nx = reinterpret_cast<const int2 *>(d.trip)[min(t0 + p, t1 - 1)];
    dbl2 *sA1 = reinterpret_cast<dbl2 *>(smem), *sA2 = sA1 + NB * 6;
    dbl2 *sZ1 = sA2 + NB * 6, *sZ2 = sZ1 + NB * 4;
#pragma unroll 1
    for (int q = 0; q < kChunk / NB; ++q) {
        const int tb = t0 + NB * q;
        if (tb >= t1) break;  // wave-uniform
        const int t = tb + p;
        const int e1 = nx.x, e2 = nx.y;
        if (tb + NB < t1) nx = reinterpret_cast<const int2 *>(d.trip)[min(tb + NB + p, t1 - 1)];
        // cooperative row loads: A pieces 64j + lane of the batch's 32 x 6, Z pieces of 32 x 4
        dbl2 v1[3], v2[3], w1[2], w2[2];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int pc = 64 * j + lane, r = pc / 6, k = pc - 6 * r;
            const int f1 = __shfl(e1, r, 64), f2 = __shfl(e2, r, 64);
            v1[j] = reinterpret_cast<const dbl2 *>(d.A + (size_t)f1 * 12)[k];
            v2[j] = reinterpret_cast<const dbl2 *>(d.A + (size_t)f2 * 12)[k];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 16 * j + (lane >> 2), k = lane & 3;
            const int f1 = __shfl(e1, r, 64), f2 = __shfl(e2, r, 64);
            w1[j] = reinterpret_cast<const dbl2 *>(d.Z + (size_t)f1 * 8)[k];
            w2[j] = reinterpret_cast<const dbl2 *>(d.Z + (size_t)f2 * 8)[k];
        }
        __syncthreads();  // the previous batch's rows are read
        // bank-conflict-free reads as k_rcs_chunk (rotated Z stores, rotated A reads)
#pragma unroll
        for (int j = 0; j < 3; ++j) { sA1[64 * j + lane] = v1[j]; sA2[64 * j + lane] = v2[j]; }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 16 * j + (lane >> 2), k = lane & 3, pos = 4 * r + ((k + ((r >> 2) & 3)) & 3);
            sZ1[pos] = w1[j];
            sZ2[pos] = w2[j];
        }
        __syncthreads();
        double m00 = 0, m01 = 0, m10 = 0, m11 = 0;
        {
            const int rz = (p >> 2) & 3;
            double z1[8], z2[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int pos = 4 * p + ((k + rz) & 3);
                const dbl2 x = sZ1[pos], y = sZ2[pos];
                z1[2 * k] = x.x; z1[2 * k + 1] = x.y; z2[2 * k] = y.x; z2[2 * k + 1] = y.y;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m00 = fma(z1[k], z2[k], m00);
                m01 = fma(z1[k], z2[4 + k], m01);
                m10 = fma(z1[4 + k], z2[k], m10);
                m11 = fma(z1[4 + k], z2[4 + k], m11);
            }
        }
        if (hlm == 1) m00 = m01;  // (as k_rcs_chunk)
        else if (hlm) m00 += m11;
        // Q = (Z₁Z₂ᵀ) A₂ from the A₂ row (read rotated as k_rcs_chunk), then this lane's A₁
        // entries 3h .. 3h+2 of both residual rows (pieces 3h/2, 3h/2 + 1 and 3 + the same)
        const int ra = (p >> 3) & 1;
        double Q[12];
        {
            dbl2 tA2[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) tA2[k] = sA2[6 * p + (k + ra < 6 ? k + ra : k + ra - 6)];
            double a2[12];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const dbl2 y = ra ? tA2[(k + 5) % 6] : tA2[k];
                a2[2 * k] = y.x; a2[2 * k + 1] = y.y;
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                Q[k] = m00 * a2[k] + m01 * a2[6 + k];
                Q[6 + k] = m10 * a2[k] + m11 * a2[6 + k];
            }
        }
        double a1[6];
        {
            const int k0 = h;  // pieces h, h+1 hold entries 2h .. 2h+3 ⊇ 3h .. 3h+2
            const dbl2 x0 = sA1[6 * p + k0], x1 = sA1[6 * p + k0 + 1];
            const dbl2 y0 = sA1[6 * p + 3 + k0], y1 = sA1[6 * p + 4 + k0];
            // h = 0: (x0.x, x0.y, x1.x); h = 1: (x0.y, x1.x, x1.y) — entries 3h + rr = 2h + (h + rr)
            a1[0] = h ? x0.y : x0.x;
            a1[1] = h ? x1.x : x0.y;
            a1[2] = h ? x1.y : x1.x;
            a1[3] = h ? y0.y : y0.x;
            a1[4] = h ? y1.x : y0.y;
            a1[5] = h ? y1.y : y1.x;
        }
        if (t < t1) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 6; ++c) acc[r * 6 + c] += a1[r] * Q[c] + a1[3 + r] * Q[6 + c];
            if (diag && e1 == e2) {
                const double q0 = d.q[(size_t)e1 * 2], q1 = d.q[(size_t)e1 * 2 + 1];
#pragma unroll
                for (int r = 0; r < 3; ++r) acc[18 + r] += a1[r] * q0 + a1[3 + r] * q1;
            }
        }
    }
    __syncthreads();  // the staging rows are read before red overwrites them
#pragma unroll
    for (int k = 0; k < 21; ++k) red[lane][k] = acc[k];
    __syncthreads();
    if (lane < 42) {
        // entry (r, c) of the block (lane < 36) or row r of the right-hand side (36..41): the 32
        // lanes of half r / 3, in lane order
        const int r = lane < 36 ? lane / 6 : lane - 36, hh = r / 3;
        const int k = lane < 36 ? (r % 3) * 6 + lane % 6 : 18 + r % 3;
        double sacc = 0.0;
        for (int l = 0; l < NB; ++l) sacc += red[hh * NB + l][k];
        st_sc1(d.ch_part + (size_t)ch * 42 + lane, sacc);
    }
    if (d.fold && arrive_last(d.cnt_rcs + b, d.blk_ch[b + 1] - d.blk_ch[b]) && lane < 42) {
        double sacc = 0.0;
        const int c1 = d.blk_ch[b + 1];
        for (int c0 = d.blk_ch[b]; c0 < c1; c0 += 4) {  // 4 partials in flight, summed in chunk order
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = c0 + u < c1 ? ld_sc1(d.ch_part + (size_t)(c0 + u) * 42 + lane) : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) sacc += v[u];
        }
        rcs_finalize_entry(d, b, lane, sacc);
    }
}

// sharded pass 2a: this rank's per-block sums (chunks in order) into the all-reduced array
__global__ __launch_bounds__(kBlock) void k_rcs_blockpart(Dev d0) {
    TRIAL_SLOT(0)
    const int gid = blockIdx.x * kBlock + threadIdx.x;
    const int b = gid / 42, e = gid % 42;
    if (b >= d.nblk) return;
    const int i1 = d.blk_i1[b];
    if (e >= 36 && i1 != d.blk_i2[b]) return;
    double sacc = 0.0;
    for (int c = d.blk_ch[b]; c < d.blk_ch[b + 1]; ++c) sacc += d.ch_part[(size_t)c * 42 + e];
    // this rank's partial Hpp into its diagonal blocks (the sum is S − Hpp: rcs_finalize_entry)
    if (e < 36 && i1 == d.blk_i2[b]) sacc -= d.Hpp_w[(size_t)i1 * 36 + e];
    const int64_t x = e < 36 ? (int64_t)b * 36 + e : (int64_t)d.nblk * 36 + 6 * i1 + (e - 36);
    if (d.xg_P > 0) {  // packed into this rank's all-gather record (outside its runs: zero by construction)
        const int64_t *rg = d.xg_rng + 4 * (size_t)d.rank;
        int64_t o;
        if (x >= rg[0] && x < rg[0] + rg[1]) o = x - rg[0];
        else if (x >= rg[2] && x < rg[2] + rg[3]) o = rg[1] + (x - rg[2]);
        else return;
        d.xg_send[(d.xg_host ? (size_t)d.rank * d.xg_P : 0) + o] = sacc;
    } else {
        d.red_rcs_loc[x] = sacc;
    }
}

// sharded pass 2b (all-gather exchange): the full red_rcs as the sum, in rank order, of every
// rank's runs — the same additions on every rank, so every rank factorises the same matrix
__global__ __launch_bounds__(kBlock) void k_rcs_xunpack(Dev d0) {
    TRIAL_SLOT(0)
    const int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (x >= (int64_t)d.nblk * 36 + (int64_t)d.nf * 6) return;
    double s = 0.0;
    for (int r = 0; r < d.nranks; ++r) {
        const int64_t *rg = d.xg_rng + 4 * (size_t)r;
        const double *rv = d.xg_recv + (size_t)r * d.xg_P;
        if (x >= rg[0] && x < rg[0] + rg[1]) s += rv[x - rg[0]];
        else if (x >= rg[2] && x < rg[2] + rg[3]) s += rv[rg[1] + (x - rg[2])];
    }
    d.red_rcs[x] = s;
}

// pass 2: per block entry, sum its chunks in order, add Hpp + λI (diagonal), write the band /
// dense matrix and b_s = b_p - Σ A_eᵀ q_e.
__global__ __launch_bounds__(kBlock) void k_rcs_finalize(Dev d0) {
    TRIAL_SLOT(0)
    const int gid = blockIdx.x * kBlock + threadIdx.x;
    const int b = gid / 42, e = gid % 42;
    if (b >= d.nblk) return;
    const int i1 = d.blk_i1[b];
    if (e >= 36 && i1 != d.blk_i2[b]) return;
    double sacc = 0.0;
    if (d.sharded) sacc = e < 36 ? d.red_rcs[(size_t)b * 36 + e] : d.red_rcs[(size_t)d.nblk * 36 + 6 * i1 + (e - 36)];
    else
        for (int c = d.blk_ch[b]; c < d.blk_ch[b + 1]; ++c) sacc += d.ch_part[(size_t)c * 42 + e];
    rcs_finalize_entry(d, b, e, sacc);
}

// oplus of every free pose with x_p (trial state; fixed poses copied), and the pose part of
// Σx(λx+b), reduced over the NT threads of one workgroup into part_ps[0] (other slots zeroed).
// `d` is a slot view; `failed`: the solve failed, x_p is the last successful solve's (A13).
template <int NT>
__device__ __forceinline__ void pose_update_wg(const Dev &d, bool failed) {
    __shared__ double sh_pu[NT / 64];
    double sc = 0.0;
    const double lam = d.lam;
    const int hlm = d.ctrl->hlm;
    const double *Tc0 = d.Tc, *xp = failed ? d.xp_prev : d.xp;
    double *Tt0 = d.Tt;
    for (int k = threadIdx.x; k < d.n_kf; k += NT) {
        const double *Tc = Tc0 + (size_t)k * 12;
        double *Tt = Tt0 + (size_t)k * 12;
        const int h = d.kf_hidx[k];
        // a free pose with no active edge has a zero RCS row: x = 0 exactly and the oplus is an
        // exact identity, so every free pose is updated
        if (h >= 0 && hlm) {  // X_i <- log(exp(X_i)·exp(DX_i)⁻¹); sc = ‖DX‖² part
            double x[6], xn[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                x[i] = xp[6 * h + i];
                sc += x[i] * x[i];
            }
            hlm_pose_update(d.xkc + (size_t)k * 6, x, xn, Tt);
#pragma unroll
            for (int i = 0; i < 6; ++i) d.xkt[(size_t)k * 6 + i] = xn[i];
        } else if (h >= 0) {
            double x[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                x[i] = xp[6 * h + i];
                sc += x[i] * (lam * x[i] + d.bp[(size_t)h * 6 + i]);
            }
            pose_oplus(Tc, x, Tt);
        } else {
#pragma unroll
            for (int i = 0; i < 12; ++i) Tt[i] = Tc[i];
            if (hlm)
#pragma unroll
                for (int i = 0; i < 6; ++i) d.xkt[(size_t)k * 6 + i] = d.xkc[(size_t)k * 6 + i];
        }
    }
    const double s = block_sum<NT>(sc, sh_pu);
    for (int i = threadIdx.x; i < d.n_ps; i += NT) d.part_ps[i] = i == 0 ? s : 0.0;
}

constexpr int kFacThreads = 1024;
constexpr int kSolveLdsN = 6144;  // y held in (dynamic) LDS up to this n (48 KiB), in Wbuf beyond
constexpr int kSolveTilesLds = 256;  // tile_first staged in LDS for the first 256 tiles
// PLBA_DIAG bit 8 (diagnostics only): phase timestamps of the dense solve (slots 12-15)
#define SOLVE_STAMP(slot)                                                                         \
    do {                                                                                         \
        if ((d.diag & 8) && d.bcr_stamps && blockIdx.x == 0 && threadIdx.x == 0)                 \
            d.bcr_stamps[slot] = __builtin_amdgcn_s_memrealtime();                              \
    } while (0)
// ---- solve L D Lᵀ x = b_s through the envelope-aware dense factor in Ad (unit L below the
// diagonal, D on it), tile by tile; one workgroup of kFacThreads. x -> xp.
// Forward: wave 0 solves the diagonal tile (its row of L in registers, y_j broadcast by
// readlane) while the other waves prefetch their rows' coefficients of the tile's columns
// (independent of y); then those rows are updated. Backward: 32 partial column sums per tile
// (lanes along rows), then wave 0 adds them and solves the tile. y lives in LDS (LY).
// y of the dense path's fused forward substitution: behind the W panel in Wbuf
__device__ __forceinline__ double *dense_yd(const Dev &d) { return d.Wbuf + (size_t)kTile * d.n; }

// FWD: y = L⁻¹b already in dense_yd (the MFMA factorisation did the forward substitution)
template <bool LY, bool FWD = false>
__device__ __forceinline__ void dense_solve_wg(const Dev &d) {
    extern __shared__ double y_lds[];
    __shared__ double red[kFacThreads / kTile][kTile + 1];
    __shared__ int tfs[kSolveTilesLds];  // tile_first in LDS (the envelope tests of every row)
    const int tid = threadIdx.x;
    const int n = d.n;
    const int nt = d.ntiles;
    const double *Ad = d.Ad;
    double *y = LY ? y_lds : d.Wbuf;
    const double *y0 = FWD ? dense_yd(d) : d.bs;
    for (int i = tid; i < n; i += kFacThreads) y[i] = y0[i];
    for (int t = tid; t < kSolveTilesLds; t += kFacThreads) tfs[t] = t < nt ? d.tile_first[t] : 0;
    auto tile_first = [&](int t) { return t < kSolveTilesLds ? tfs[t] : d.tile_first[t]; };
    __syncthreads();
    constexpr int kRowThreads = kFacThreads - 64;
    for (int K = 0; K < (FWD ? 0 : nt); ++K) {
        const int k0 = K * kTile, kb = min(kTile, n - k0);
        const int fend = min(n, (d.tile_last[K] + 1) * kTile);
        const int i1 = k0 + kb + tid - 64;  // this thread's first row of the update
        double cf[kTile];
        if (K == 5) SOLVE_STAMP(16);
        if (tid < 64) {
            double yi = (tid < kb) ? y[k0 + tid] : 0.0;
            // loads at clamped (always valid) addresses, selected after: no per-element branches
            const double *row = Ad + (size_t)(k0 + min(tid, kb - 1)) + (size_t)k0 * n;
            double l[kTile];
#pragma unroll
            for (int j = 0; j < kTile; ++j) l[j] = row[(size_t)min(j, kb - 1) * n];
#pragma unroll
            for (int j = 0; j < kTile; ++j) {
                const double yj = readlane_f64(yi, j);
                if (tid > j && tid < kb) yi -= l[j] * yj;
            }
            if (tid < kb) y[k0 + tid] = yi;
            if (K == 5) SOLVE_STAMP(17);
        } else {
            const double *row = Ad + (size_t)min(i1, n - 1) + (size_t)k0 * n;
#pragma unroll
            for (int p = 0; p < kTile; ++p) cf[p] = row[(size_t)min(p, kb - 1) * n];
        }
        __syncthreads();
        if (K == 5) SOLVE_STAMP(18);
        if (tid >= 64) {
            if (i1 < fend && tile_first(i1 / kTile) <= K) {
                double s = 0.0;
#pragma unroll
                for (int p = 0; p < kTile; ++p)
                    if (p < kb) s += cf[p] * y[k0 + p];
                y[i1] -= s;
            }
            for (int i = i1 + kRowThreads; i < fend; i += kRowThreads) {  // n > ~kFacThreads only
                if (tile_first(i / kTile) > K) continue;
                double s = 0.0;
                for (int p = 0; p < kb; ++p) s += Ad[(size_t)i + (size_t)(k0 + p) * n] * y[k0 + p];
                y[i] -= s;
            }
        }
        __syncthreads();
        if (K == 5) SOLVE_STAMP(19);
    }
    for (int i = tid; i < n; i += kFacThreads) y[i] = y[i] / Ad[(size_t)i + (size_t)i * n];
    __syncthreads();
    SOLVE_STAMP(13);
    // backward: Lᵀ x = y, tile by tile from the bottom
    for (int K = nt - 1; K >= 0; --K) {
        const int k0 = K * kTile, kb = min(kTile, n - k0);
        // y_K -= Σ_{i > tile} L[i][k] y[i]   (column k of L below the tile): 32 partial sums per
        // column (rows i ≡ part mod 32), added in part order; part runs along the lanes so a
        // wave reads two columns, 32 consecutive rows each
        const int bend = min(n, (d.tile_last[K] + 1) * kTile);
        {
            // one tile of rows per step (the stride is kTile rows): U tiles' loads in flight at
            // once, clamped valid addresses, masked after; summed in row order
            static_assert(kFacThreads / kTile == kTile, "one row of each tile per partial");
            constexpr int U = 8;
            const int part = tid % kTile, c = tid / kTile;
            double s = 0.0;
            if (c < kb) {
                const double *colp = Ad + (size_t)(k0 + c) * n;
                for (int m0 = K + 1; m0 * kTile < bend; m0 += U) {
                    double v[U], yy[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int i = (m0 + u) * kTile + part;
                        const bool ok = i < bend && tile_first(min(m0 + u, nt - 1)) <= K;
                        const int ic = min(i, n - 1);
                        v[u] = colp[ic];
                        yy[u] = ok ? y[ic] : 0.0;
                        v[u] = ok ? v[u] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) s += v[u] * yy[u];
                }
            }
            red[part][c] = s;
        }
        double l[kTile];
        if (tid < 64) {  // column of L of the diagonal tile in registers
            const double *col = Ad + (size_t)k0 + (size_t)(k0 + min(tid, kb - 1)) * n;
#pragma unroll
            for (int j = 0; j < kTile; ++j) l[j] = col[min(j, kb - 1)];
        }
        __syncthreads();
        if (tid < 64) {
            double yi = 0.0;
            if (tid < kb) {
                double s = 0.0;
                for (int p = 0; p < kFacThreads / kTile; ++p) s += red[p][tid];
                yi = y[k0 + tid] - s;
            }
#pragma unroll
            for (int j = kTile - 1; j >= 0; --j) {
                const double yj = readlane_f64(yi, j);
                if (tid < j && j < kb) yi -= l[j] * yj;
            }
            if (tid < kb) y[k0 + tid] = yi;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += kFacThreads) d.xp[i] = y[i];
}

// Envelope-aware tiled LDLᵀ of the lower triangle + solve, one workgroup of 1024 threads.
// Semantics of Eigen::SimplicialLDLT as used by LinearSolverEigen: fails iff a pivot is 0.
__global__ __launch_bounds__(kFacThreads) void k_rcs_factor(Dev d0) {
    TRIAL_SLOT(0)
    __shared__ double T[kTile][kTile + 1];
    __shared__ double Dk[kTile];
    __shared__ int s_fail;
    const int tid = threadIdx.x;
    const int n = d.n;
    double *Ad = d.Ad;
    if (tid == 0) s_fail = 0;
    const int nt = d.ntiles;
    for (int K = 0; K < nt; ++K) {
        const int k0 = K * kTile;
        const int kb = min(kTile, n - k0);
        __syncthreads();
        {   // load diagonal tile
            const int r = tid >> 5, c = tid & 31;
            if (r < kb && c <= r) T[r][c] = Ad[(size_t)(k0 + r) + (size_t)(k0 + c) * n];
        }
        __syncthreads();
        for (int j = 0; j < kb; ++j) {
            const int r = tid >> 5, c = tid & 31;
            const double djj = T[j][j];
            if (djj == 0.0) {
                if (tid == 0) s_fail = 1;
            } else if (r > j && c > j && c <= r && r < kb) {
                T[r][c] -= (T[r][j] / djj) * T[c][j];
            }
            __syncthreads();
        }
        if (s_fail) break;
        {   // L = T / D, store to global
            const int r = tid >> 5, c = tid & 31;
            if (r < kb && c < r) {
                const double l = T[r][c] / T[c][c];
                Ad[(size_t)(k0 + r) + (size_t)(k0 + c) * n] = l;
            }
            if (tid < kb) {
                Dk[tid] = T[tid][tid];
                Ad[(size_t)(k0 + tid) + (size_t)(k0 + tid) * n] = T[tid][tid];
            }
        }
        __syncthreads();
        {   // convert T strict lower to L (in LDS)
            const int r = tid >> 5, c = tid & 31;
            double l = 0.0;
            if (r < kb && c < r) l = T[r][c] / Dk[c];
            __syncthreads();
            if (r < kb && c < r) T[r][c] = l;
        }
        __syncthreads();
        // panel rows: i >= k0+kb with tile_first[tile(i)] <= K
        const int rows0 = k0 + kb;
        const int rows_end = min(n, (d.tile_last[K] + 1) * kTile);
        for (int i = rows0 + tid; i < rows_end; i += kFacThreads) {
            if (d.tile_first[i / kTile] > K) continue;
            double *w = d.Wbuf + (size_t)i * kTile;   // W = L·D for this row (re-read by the update)
            for (int c = 0; c < kb; ++c) {
                double a = Ad[(size_t)i + (size_t)(k0 + c) * n];
                for (int p = 0; p < c; ++p) a -= w[p] * T[c][p];
                w[c] = a;
                Ad[(size_t)i + (size_t)(k0 + c) * n] = a / Dk[c];
            }
        }
        __syncthreads();
        // trailing update: A[i][j] -= Σ_c W[i][c] L[j][c], for rows/cols in the panel, j <= i
        const int m = n - rows0;
        if (m > 0) {
            // iterate over trailing tiles (I, J) with K < J <= I, both in the envelope of K
            for (int I = K + 1; I <= d.tile_last[K]; ++I) {
                if (d.tile_first[I] > K) continue;
                for (int J = K + 1; J <= I; ++J) {
                    if (d.tile_first[J] > K) continue;
                    const int r = tid >> 5, c = tid & 31;
                    const int i = I * kTile + r, j = J * kTile + c;
                    if (i < n && j < n && j <= i) {
                        double s = 0.0;
                        for (int p = 0; p < kb; ++p)
                            s += d.Wbuf[(size_t)i * kTile + p] * Ad[(size_t)j + (size_t)(k0 + p) * n];
                        Ad[(size_t)i + (size_t)j * n] -= s;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (tid == 0) *d.solve_okp = s_fail ? 0 : 1;
    if (!s_fail) {  // on failure x_p keeps its previous value (g2o leaves _x untouched)
        if (n <= d.solve_lds_n) dense_solve_wg<true>(d);
        else dense_solve_wg<false>(d);
    }
    __syncthreads();
    pose_update_wg<kFacThreads>(d, s_fail != 0);  // the update is applied even after a failed solve (A13)
}


// Block-banded LDLᵀ of the reduced camera system (A = L_B D_B L_Bᵀ, 6x6 pose blocks) with an
// LDS sliding window of bw+1 block rows, forward substitution folded in (augmented column b),
// then a one-wave backward pass. One workgroup; 3 barriers per pose block.
// Failure semantics of SimplicialLDLT: a zero pivot (Gauss–Jordan pivots of S_k are the LDLᵀ
// pivots) fails the solve and x_p keeps its previous value.
// fast IEEE-accurate reciprocal: v_rcp_f64 + two Newton steps
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    r = fma(fma(-x, r, 1.0), r, r);
    return r;
}
// v_rcp_f64 + one Newton step (the estimate is good to ~2^-26, one step squares the error)
__device__ __forceinline__ double rcp_nr1(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(fma(-x, r, 1.0), r, r);
}

// Lane-local LDLᵀ of a 6x6 symmetric block held as its packed lower triangle (row-major,
// ltri(i, j) for j <= i): on return s holds the unit lower factor below the diagonal and dv the
// reciprocal pivots. zp is set if a pivot is exactly zero (SimplicialLDLT's failure condition).
__host__ __device__ constexpr int ltri(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ void ldl6_inplace(double (&s)[21], double (&dv)[6], bool &zp) {
#pragma unroll
    for (int p = 0; p < 6; ++p) {
        const double dp = s[ltri(p, p)];
        zp = zp || dp == 0.0;
        const double rp = rcp_nr1(dp);
        dv[p] = rp;
        double col[6];
#pragma unroll
        for (int i = p + 1; i < 6; ++i) col[i] = s[ltri(i, p)];
#pragma unroll
        for (int i = p + 1; i < 6; ++i) s[ltri(i, p)] = col[i] * rp;
#pragma unroll
        for (int i = p + 1; i < 6; ++i)
#pragma unroll
            for (int j = p + 1; j <= i; ++j) s[ltri(i, j)] = fma(-s[ltri(i, p)], col[j], s[ltri(i, j)]);
    }
}
// x <- (L D Lᵀ)⁻¹ x with the factors of ldl6_inplace
__device__ __forceinline__ void ldl6_solve(const double (&s)[21], const double (&dv)[6], double (&x)[6]) {
#pragma unroll
    for (int i = 1; i < 6; ++i)
#pragma unroll
        for (int m = 0; m < i; ++m) x[i] = fma(-s[ltri(i, m)], x[m], x[i]);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] *= dv[i];
#pragma unroll
    for (int i = 4; i >= 0; --i)
#pragma unroll
        for (int m = 5; m > i; --m) x[i] = fma(-s[ltri(m, i)], x[m], x[i]);
}

// Lane-local inverse of a 6x6 pivot block just published to LDS (entry (r, c) at S[r * 6 + c]; its
// lower triangle is read): every lane factors S LDLᵀ in its own registers, then lanes r*6+c
// (0..35) return (S⁻¹)[r][c] (column c of S⁻¹ solved from e_c) and lanes 36+r return (S⁻¹y)[r].
// No cross-lane traffic: replaces gj_inverse6's 6 pivot broadcasts + 18 LDS permutes, which on
// the register-window band kernel contend with the worker waves' trailing-update LDS reads.
// The LDLᵀ pivots are the system's, so a zero pivot fails the solve as SimplicialLDLT does.
// (LDS operations of one wave complete in order: the caller's stores of S and y need no wait.)
__device__ __forceinline__ double ldl_inverse6(const double *S, const double *y, int lane, bool &fail) {
    double s[21], dv[6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) s[ltri(i, j)] = S[i * 6 + j];
    bool zp = false;
    ldl6_inplace(s, dv, zp);
    if (zp) fail = true;
    const bool mat = lane < 36;
    const int r = mat ? lane / 6 : min(lane - 36, 5), c = lane % 6;
    double x[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) x[m] = mat ? (m == c ? 1.0 : 0.0) : y[m];
    ldl6_solve(s, dv, x);
    double out = x[0];
#pragma unroll
    for (int m = 1; m < 6; ++m) out = r == m ? x[m] : out;
    return out;
}
// Gauss–Jordan on [S | y] (6x7, one entry per lane): lanes r*6+c (0..35) hold S and return
// S^{-1}; lanes 36+r hold y and return z = S^{-1} y. No pivoting: the pivots are the LDLᵀ
// pivots, so a zero pivot reports failure exactly as SimplicialLDLT's NumericalIssue does.
__device__ __forceinline__ double gj_inverse6(double M, int lane, bool &fail) {
    const bool mat = lane < 36, rhs = lane >= 36 && lane < 42;
    const int r = mat ? lane / 6 : (rhs ? lane - 36 : 0);
    const int c = mat ? lane % 6 : 0;
    double I = (mat && r == c) ? 1.0 : (rhs ? M : 0.0);  // rhs lanes carry y in I
#pragma unroll
    for (int p = 0; p < 6; ++p) {
        // the pivot comes from a compile-time lane: v_readlane (SGPR broadcast) instead of an
        // LDS-crossbar round trip, so its reciprocal overlaps the three row/column permutes
        const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(M), 7 * p),
                                            __builtin_amdgcn_readlane(__double2loint(M), 7 * p));
        const double f = __shfl(M, r * 6 + p, 64);
        double ip = __shfl(I, rhs ? 36 + p : p * 6 + c, 64);
        double mp = __shfl(M, p * 6 + c, 64);
        if (piv == 0.0) fail = true;
        const double rp = rcp_nr(piv);
        mp = mp * rp;
        ip = ip * rp;
        if (r == p) { M = mp; I = ip; }
        else { M = fma(-f, mp, M); I = fma(-f, ip, I); }
    }
    return I;
}

// Block-banded LDLᵀ with lookahead, templated on the envelope bandwidth BW (pose blocks).
// Wave 0 carries the critical chain
//   S_k^{-1} -> L_{k+1,k} -> S_{k+1} = A_{k+1,k+1} - L_{k+1,k} A_{k+1,k}ᵀ -> S_{k+1}^{-1}
// while waves 1..15 compute the other L blocks and the trailing updates of step k
// (2 LDS-only barriers per step). Each worker's entries and LDS offsets are compile-time /
// hoisted; window slots advance incrementally (no runtime modulo in the loop).
//
// band_forward eliminates the first `nsteps` block rows of an `nrows`-row band (forward
// substitution folded in) and, when `sep` is given, stores the updated rows
// nsteps..nsteps+BW-1 — the separator a second segment meets (k_rcs_factor_twisted).
struct BandSeg {
    const double *Bd, *bs;     // [nrows][BW+1][36] block (i, i-w) row-major, [nrows][6]
    double *Lband, *Kinv, *zb; // outputs, indexed by this segment's row numbering
    int nrows, nsteps;
    double *sep;               // nullable: [BW][BW+1][36] + [BW][6]
};

// Register-resident band window. Block (i, i-w) of a live row is owned by a pair of worker
// threads (3 rows each; whole blocks on one thread for bw 25..27) for its whole life in the
// window and updated in registers; it is written to LDS once, when it becomes part of the next
// pivot column (the step's operand A_jk and the source of L), or, on the diagonal, when it becomes
// the next pivot block. Ownership follows diagonal-major rings: diagonal w has C_w = W-w+1 slots,
// row i in slot i mod C_w; at step k the slot's offset o = (slot - k - w) mod C_w says which row
// it holds (i = k+w+o): o = 0 the pivot column, 1 <= o <= BW-w a trailing block (pair wi = w+o,
// wj = o), o = C_w-1 the spare slot whose row k+W enters (staged, below). W(W+3) half blocks
// (bw 23: 648 of the 704 worker threads of a 768-thread workgroup); LDS keeps only two pivot
// columns, the pivot blocks, the staged rows and the L / S^-1 / z staging rings, so no
// read-modify-write of the trailing blocks goes through LDS.
__host__ __device__ constexpr int bd_cap(int W, int w) { return W - w + 1; }
__host__ __device__ constexpr int bd_base(int W, int w) { return w * (W + 1) - w * (w - 1) / 2; }
__host__ __device__ constexpr int bd_blocks(int W) { return W * (W + 3) / 2; }

template <int BW>
__device__ __forceinline__ void band_lds(double *lds, int R, double *&col, double *&piv, double *&bwin, double *&Lcol,
                                         double *&Kv, double *&xr, double *&part, double *&ys, double *&ringL,
                                         double *&ringK, double *&ringZ) {
    constexpr int W = BW + 1;
    col = lds;                                   // [2][W][36] pivot columns k, k+1: block (c+w, c) at [c&1][w]
    piv = col + (size_t)2 * W * 36;              // [2][36]  pivot block (c, c) at [c&1]
    bwin = piv + 72;                             // [W][6]  right-hand sides, row slot ring
    // (the entering rows are staged in band_forward's static LDS: band_static_bytes)
    Lcol = bwin + (size_t)W * 6;                 // [W][36]  (index w = 1..BW)
    Kv = Lcol + (size_t)W * 36;                  // [2][36]  S_k^{-1} double buffer
    xr = Kv + 72;                                // [W][6]  ring of solved x blocks
    part = xr + (size_t)W * 6;                   // [W][6]
    ys = part + (size_t)W * 6;                   // [2][6]  y_k snapshots
    ringL = ys + 12;                             // [R][BW][36]
    ringK = ringL + (size_t)R * BW * 36;         // [R+1][36]
    ringZ = ringK + (size_t)(R + 1) * 36;        // [R+1][6]
}
// doubles of the band layout above
__host__ __device__ constexpr size_t band_lds_doubles(int bw, int R) {
    return (size_t)(bw + 1) * 72 + 72 + (size_t)(bw + 1) * (6 + 36 + 6 + 6) + 72 + 12 + (size_t)R * bw * 36 +
           (size_t)(R + 1) * 42;
}
// static LDS of band_forward: the entering rows' staging buffers [2][W*36 + 6] (blocks, right-hand
// side) plus a few flags. A separate LDS object from the dynamic window, so that the compiler can
// tell the direct global->LDS loads into it from the window's reads (with one LDS object every
// ds_read after such a load waits for it)
// entering-row staging buffers of band_forward: a row is issued at the start of a step's second
// phase and retired before its last barrier (round 6: a third buffer with the row in flight
// across the barrier, retired one step later with vmcnt(1), measured 294 -> 303 µs at C3R)
constexpr int kBandStage = 2;
__host__ __device__ constexpr size_t band_static_bytes(int bw) { return 8 * kBandStage * ((size_t)(bw + 1) * 36 + 6) + 64; }
// The twisted kernel's merge, after both segments have exported their separator windows, reuses
// the LDS from 0: the separator's L blocks [bw(bw-1)/2][36], pivot inverses [bw][36], the
// current pivot column [2][bw][36] (step parity), the pivot blocks [bw][36], its right-hand side and
// two solution copies [3][6bw]; behind the x_p staging [nf][6] at offset 0 (twisted_lds_bytes:
// the back substitution's streamed chunks reuse the region, band_backward_stream).
__host__ __device__ constexpr size_t twisted_merge_doubles(int bw) {
    return (size_t)bw * (bw - 1) / 2 * 36 + 144 * (size_t)bw + 3 * (size_t)(6 * bw);
}

template <int BW>
__device__ __forceinline__ bool band_forward(const BandSeg &g, double *lds, int ring, unsigned long long *stamps) {
    constexpr int NT = band_nt(BW), W = BW + 1, NW = NT - 64;
    constexpr int UR = band_ur(BW), UPB = 6 / UR, UE = UR * 6;  // rows per owner, owners per block, entries
    static_assert(UPB * bd_blocks(W) <= NW, "one owned (part) block per worker thread");
    constexpr int LPT = ((BW > 1 ? BW - 1 : 0) * 36 + NW - 1) / NW;  // L entries per worker (w >= 2)
    const int nrows = g.nrows, nsteps = g.nsteps;
    double *col, *piv, *bwin, *Lcol, *Kv, *xr, *part, *ys, *ringL, *ringK, *ringZ;
    band_lds<BW>(lds, ring, col, piv, bwin, Lcol, Kv, xr, part, ys, ringL, ringK, ringZ);
    const int R = ring;
    const int RK = R + 1;                         // S^-1 / z of step k+1 are written during step k
    __shared__ int s_fail;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave index in an SGPR: the loop's wave-0 tests and the staging-row split need no per-lane
    // register (a VGPR tid carried through the step loop was spilled and reloaded every step)
    const int wv_s = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool crit = wv_s == 0;                  // wave 0
    const int wt = tid - 64;                      // worker thread index
    if (tid == 0) s_fail = 0;
    // ---- the (part) block this worker owns: slot p of diagonal w, rows oh/6 .. oh/6+UR-1
    const bool own = !crit && wt < UPB * bd_blocks(W);
    int ow = 0, op = 0;
    if (own) {
        const int b = wt / UPB;
        while (bd_base(W, ow + 1) <= b) ++ow;
        op = b - bd_base(W, ow);
    }
    const int oC = bd_cap(W, ow), oh = (max(wt, 0) % UPB) * UE;
    int oo = ((op - ow) % oC + oC) % oC;          // offset at step 0
    double t[UE];
    {   // rows 0..BW (the spare slot's row W arrives during step 0)
        const int i = ow + oo;
        const bool ld = own && oo != oC - 1 && i < nrows;
        const double *src = g.Bd + ((size_t)(ld ? i : 0) * W + ow) * 36 + oh;
#pragma unroll
        for (int j = 0; j < UE; ++j) t[j] = ld ? src[j] : 0.0;
        if (own) {
            double *dst = nullptr;
            if (ow >= 1 && oo == 0) dst = col + (size_t)ow * 36;   // column 0
            else if (ow == 0 && oo <= 1) dst = piv + oo * 36;      // pivots (0,0), (1,1)
            if (dst)
#pragma unroll
                for (int j = 0; j < UE; ++j) dst[oh + j] = t[j];
        }
    }
    for (int t2 = tid; t2 < W * 6; t2 += NT) bwin[t2] = (t2 / 6 < nrows) ? g.bs[t2] : 0.0;
    // Entering rows (W blocks + the right-hand side) come in by direct global->LDS loads
    // (global_load_lds_dwordx4, no VGPR destination): row r to staging buffer r & 1, issued by the
    // worker waves at the start of step r-W-1's second phase and retired before its last barrier;
    // the diagonal-BW block goes into the pivot column during step r-W, the rest into the owners'
    // registers at the top of step r-BW. No owner register and no spill reload waits on a global
    // load. Past the band's end the last row is loaded again (never read: readers stop at wmax).
    constexpr int RW = W * 36 + 6, NPC = RW / 2;  // doubles per staged row, 16-byte pieces
    __shared__ __attribute__((aligned(16))) double stgb[kBandStage * RW];
    // staging buffer of a row (r mod kBandStage): incremental, no runtime modulo in the loop
    auto stg = [&](int slot) { return stgb + (size_t)slot * RW; };
    auto stage_row = [&](int row, int slot, int wv, int lnv) {  // wv: worker wave index (uniform)
      for (int pb = wv * 64; pb < NPC; pb += NW) {  // (more pieces than worker lanes at bw >= 24)
        const int p = pb + lnv;
        if (p < NPC) {
            const int rr = min(row, nrows - 1);
            const double *src = p < W * 18 ? g.Bd + (size_t)rr * W * 36 + 2 * p : g.bs + (size_t)rr * 6 + 2 * (p - W * 18);
            // inline asm rather than the builtin: with the builtin the compiler waits for the load
            // before every later ds_read of the window (it cannot tell the LDS objects apart);
            // this load is retired by the explicit vmcnt(0) before the step's last barrier
            const unsigned dst = __builtin_amdgcn_readfirstlane(
                (unsigned)(size_t)(__attribute__((address_space(3))) double *)(stg(slot) + pb * 2));
            unsigned keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(src), "s"(dst)
                         : "memory");
        }
      }
    };
    if (!crit) {
        stage_row(W, W % kBandStage, wv_s - 1, lane);
        // retired here like every later row's (the compiler does not track the inline-asm load,
        // and step 0's phase 2 already copies its diagonal-BW block out of the staging buffer)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(tid) < 64) __builtin_amdgcn_s_setprio(3);
    // S_0^{-1}, y_0, z_0
    if (crit) {
        bool fail = false;
        if (lane >= 36 && lane < 42) ys[lane - 36] = bwin[lane - 36];
        const double I = ldl_inverse6(piv, bwin, lane, fail);
        if (lane < 36) { Kv[lane] = I; ringK[lane] = I; }
        else if (lane < 42) ringZ[lane - 36] = I;
        if (fail && lane == 0) s_fail = 1;
    }
    lds_barrier();
#ifdef PLBA_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
    int sk = 0, kR = 0, kRK = 1;                  // k % W (rhs row slots), k % R, (k+1) % RK
    int sB = BW % kBandStage, sW = W % kBandStage; // staging slots of rows k+BW, k+W
    int fr0 = 0;                                  // (first step of the current flush batch) % RK
    // a zero pivot sets s_fail and the sweep runs on (inf/NaN blocks are never used: the
    // caller drops the solve); no per-step LDS read of the flag on the critical chain
    for (int k = 0; k < nsteps; ++k) {
        // per-lane indices made opaque each step: everything derived from them is recomputed in
        // the step (a few integer ops) instead of being hoisted out of the loop as dozens of
        // loop-invariant registers that then spill to scratch (a scratch reload waits for every
        // outstanding global load, the spare-slot loads included)
        // (the lane index is re-derived from v_mbcnt each step: carried, it was spilled and its
        // scratch reload at the step top stalled the critical wave on vmcnt)
        int wtl = wt, owl = ow, ohl = oh, oCl = oC;
        asm volatile("" : "+v"(wtl), "+v"(owl), "+v"(ohl), "+v"(oCl));
        const int lnl = (int)__lane_id();
        const int kb = k & 1;
        const int wmax = min(BW, nrows - 1 - k);
        const double *Kk = Kv + kb * 36;
        const double *yk = ys + kb * 6;
        const double *colk = col + (size_t)kb * W * 36;
        auto slot = [&](int w) { const int x = sk + w; return x >= W ? x - W : x; };
        if (!crit && k > 0) {
            // row k+BW (last step's spare slot) from its staging buffer into the owners' registers
            // (bw 1: its block (k+1, k+1) is also this step's next pivot); its right-hand side into
            // its row slot. (Its diagonal-BW block, this step's pivot-column entry, was copied in
            // the previous step: phase 1 reads it before any barrier of this step.)
            const double *sr = stg(sB);  // row k+BW
            if (own && oo == oCl - 2) {
                const double2 *src = (const double2 *)(sr + owl * 36 + ohl);
                double2 *D = (BW == 1 && owl == 0) ? (double2 *)(piv + (kb ^ 1) * 36 + ohl) : nullptr;
#pragma unroll
                for (int v = 0; v < UE / 2; ++v) {
                    const double2 x = src[v];
                    t[2 * v] = x.x;
                    t[2 * v + 1] = x.y;
                    if (D) D[v] = x;
                }
            }
            if (wtl < 6) bwin[slot(BW) * 6 + wtl] = k + BW < nrows ? sr[W * 36 + wtl] : 0.0;
        }
        STAMP(0);
        // ---- phase 1: L_{k+w,k} = A_{k+w,k} S_k^{-1}   (w = 1 on wave 0, w >= 2 on the workers)
        if (crit) {
            if (lnl < 36 && wmax >= 1) {
                const int c = lnl % 6;
                const double *Aik = colk + 36 + (lnl / 6) * 6;
                double v = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) v = fma(Aik[m], Kk[m * 6 + c], v);
                Lcol[36 + lnl] = v;
                ringL[((size_t)kR * BW + 0) * 36 + lnl] = v;
            }
        } else {
#pragma unroll
            for (int q = 0; q < LPT; ++q) {
                const int t2 = wtl + 36 + q * NW;
                const int w = 1 + t2 / 36, e = t2 % 36;
                if (t2 < BW * 36 && w <= wmax) {
                    const double *Aik = colk + (size_t)w * 36 + (e / 6) * 6;
                    const int c = e % 6;
                    double v = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) v = fma(Aik[m], Kk[m * 6 + c], v);
                    Lcol[w * 36 + e] = v;
                    ringL[((size_t)kR * BW + (w - 1)) * 36 + e] = v;
                }
            }
        }
        STAMP(1);
        lds_barrier();
        STAMP(2);
        // ---- phase 2 (the worker waves first put row k+W+1 in flight)
        if (!crit) stage_row(k + W + 1, sB, wv_s - 1, lnl);  // (row k+BW's buffer: consumed at the top)
        if (crit) {
            if (k + 1 < nrows) {
                const int s1 = slot(1), k1b = kb ^ 1;
                // lanes 0..35: S_{k+1} = A_{k+1,k+1} - L_{k+1,k} A_{k+1,k}ᵀ
                // lanes 36..41: y_{k+1} = b_{k+1} - L_{k+1,k} y_k
                double M = 0.0;
                if (lnl < 42) {
                    const bool mat = lnl < 36;
                    const int r = mat ? lnl / 6 : lnl - 36, c = mat ? lnl % 6 : 0;
                    double sacc = 0.0;
                    if constexpr (BW >= 1) {
                        const double *L1 = Lcol + 36 + r * 6;
                        const double *A1 = mat ? colk + 36 + c * 6 : yk;
#pragma unroll
                        for (int m = 0; m < 6; ++m) sacc = fma(L1[m], A1[m], sacc);
                    }
                    double *dst = mat ? piv + k1b * 36 + lnl : bwin + s1 * 6 + r;
                    M = *dst - sacc;
                    *dst = M;
                    if (!mat) ys[k1b * 6 + r] = M;
                }
                bool fail = false;
                const double I = ldl_inverse6(piv + k1b * 36, ys + k1b * 6, lnl, fail);
                if (lnl < 36) { Kv[k1b * 36 + lnl] = I; ringK[kRK * 36 + lnl] = I; }
                else if (lnl < 42) ringZ[kRK * 6 + lnl - 36] = I;
                // the look-ahead inverse past the last eliminated row (a separator row) is not a pivot
                if (fail && lnl == 0 && k + 1 < nsteps) s_fail = 1;
            }
        } else {
            // trailing update of the owned (part) block (k+wi, k+wj), wi = w+o, wj = o:
            // A_ij -= L_ik A_jkᵀ (same fma order per entry as one entry at a time); (1,1) is wave 0's
            const int wi = owl + oo;
            if (own && oo >= 1 && oo != oCl - 1 && wi <= wmax && !(owl == 0 && oo == 1)) {
                const double2 *Li = (const double2 *)(Lcol + wi * 36 + ohl);
                const double2 *Aj = (const double2 *)(colk + (size_t)oo * 36);
                double l[UE];
#pragma unroll
                for (int v = 0; v < UE / 2; ++v) { const double2 x = Li[v]; l[2 * v] = x.x; l[2 * v + 1] = x.y; }
#pragma unroll
                for (int c = 0; c < 6; ++c) {  // column c of the target = row c of A_jk
                    double a[6];
#pragma unroll
                    for (int v = 0; v < 3; ++v) { const double2 x = Aj[c * 3 + v]; a[2 * v] = x.x; a[2 * v + 1] = x.y; }
#pragma unroll
                    for (int r = 0; r < UR; ++r) {
                        double sacc = 0.0;
#pragma unroll
                        for (int m = 0; m < 6; ++m) sacc = fma(l[r * 6 + m], a[m], sacc);
                        t[r * 6 + c] -= sacc;
                    }
                }
                // next step's pivot column (k+1+w, k+1) / the pivot block after next (k+2, k+2)
                double *dst = (owl >= 1 && oo == 1) ? col + ((size_t)(kb ^ 1) * W + owl) * 36
                            : (owl == 0 && oo == 2) ? piv + kb * 36 : nullptr;
                if (dst) {
                    double2 *D = (double2 *)(dst + ohl);
#pragma unroll
                    for (int v = 0; v < UE / 2; ++v) D[v] = make_double2(t[2 * v], t[2 * v + 1]);
                }
            }
            // the next pivot column's diagonal-BW entry (k+W, k+1), from row k+W's staging buffer
            if (wtl < 18) {
                const double *cs = stg(sW) + BW * 36;  // row k+W
                ((double2 *)(col + ((size_t)(kb ^ 1) * W + BW) * 36))[wtl] = ((const double2 *)cs)[wtl];
            }
            STAMP(5);
            // b_i -= L_ik y_k for w >= 2 (last worker wave)
            {
                const int t2 = NW - 1 - wtl;  // 0.. on the last wave
                if (t2 < (wmax - 1) * 6) {
                    const int wr = 2 + t2 / 6, r = t2 % 6;
                    double sacc = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) sacc = fma(Lcol[wr * 36 + r * 6 + m], yk[m], sacc);
                    bwin[slot(wr) * 6 + r] -= sacc;
                }
            }
            STAMP(6);
            if (kR == R - 1 || k == nsteps - 1) {  // flush the staged steps k0..k to global
                const int k0 = k - kR;
                const int cnt = kR + 1;
                if constexpr (BW >= 1)
                    for (int t2 = wtl; t2 < cnt * BW * 36; t2 += NW) {
                        const int st = t2 / (BW * 36), rem = t2 % (BW * 36), w = 1 + rem / 36, e = rem % 36;
                        const int i = k0 + st + w;
                        if (i < nrows) g.Lband[((size_t)i * W + w) * 36 + e] = ringL[(size_t)st * BW * 36 + rem];
                    }
                const int r0 = fr0;      // k0 mod RK, kept incrementally (a per-lane division by the
                fr0 = fr0 + R >= RK ? fr0 + R - RK : fr0 + R;  // runtime ring size spilled its magic number)
                for (int t2 = wtl; t2 < cnt * 36; t2 += NW) {
                    const int sl = r0 + t2 / 36;
                    g.Kinv[(size_t)k0 * 36 + t2] = ringK[(sl >= RK ? sl - RK : sl) * 36 + t2 % 36];
                }
                for (int t2 = wtl; t2 < cnt * 6; t2 += NW) {
                    const int sl = r0 + t2 / 6;
                    g.zb[(size_t)k0 * 6 + t2] = ringZ[(sl >= RK ? sl - RK : sl) * 6 + t2 % 6];
                }
            }
            STAMP(7);
            // the staged row lands before the barrier (issued at the start of this phase; read at
            // the top of step k+2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        STAMP(3);
        lds_barrier();
        STAMP(4);
        sk = (sk + 1 == W) ? 0 : sk + 1;
        sB = (sB + 1 == kBandStage) ? 0 : sB + 1;
        sW = (sW + 1 == kBandStage) ? 0 : sW + 1;
        kR = (kR + 1 == R) ? 0 : kR + 1;
        kRK = (kRK + 1 == RK) ? 0 : kRK + 1;
        oo = (oo == 0) ? oCl - 1 : oo - 1;
    }
#ifdef PLBA_STAMPS
    if (stamps && (tid & 63) == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&stamps[(tid >> 6) * 8 + q], st_acc[q]);
#endif
    __syncthreads();  // drains every wave's flush stores: the backward pass reads them
    const bool failed = s_fail != 0;
    if (g.sep && !failed) {  // rows nsteps..nsteps+BW-1, blocks w <= row (later columns) and their right-hand sides
        const int i = ow + oo;  // separator row of the owned block (k = nsteps)
        if (own && oo <= BW - ow && i < BW) {
            double *dst = g.sep + ((size_t)i * W + ow) * 36 + oh;
            const double *pv = piv + (nsteps & 1) * 36 + oh;  // (nsteps, nsteps) carries wave 0's last update
#pragma unroll
            for (int j = 0; j < UE; ++j) dst[j] = (ow == 0 && oo == 0) ? pv[j] : t[j];
        }
        for (int t2 = tid; t2 < BW * 6; t2 += NT) g.sep[(size_t)BW * W * 36 + t2] = bwin[((sk + t2 / 6) % W) * 6 + t2 % 6];
    }
    return failed;
}

// Backward substitution x_k = z_k - Σ_w L_{k+w,k}ᵀ x_{k+w} for k = nsteps-1..0, by ONE wave (no
// barriers; L prefetched one step ahead). Rows nsteps..nsteps+BW-1 take x from `xsep` (a
// separator solved elsewhere) or do not exist (xsep == nullptr, nsteps == nrows). Row k is
// written to xp[k] (or xp[nf-1-k] for a reversed segment).
// Right-looking variant for bw <= 10 (one lane per (row, component) of the BW-row window, all
// in registers): once x_i is final, its 6 values are read from the owning lanes with
// v_readlane and every window row j = i-w applies z_j -= L_{i,j}ᵀ x_i at once. The chain per
// step is one readlane batch + one 6-term dot product; no LDS round trips.
// LX: x rows go to LDS (the caller copies them out) — a global store in the loop would make
// the compiler's vmcnt waits (loads and stores share the counter) drain the L prefetches.
template <int BW, bool LX = false>
__device__ __forceinline__ void band_backward_rl(const double *Lband, const double *zb, int nsteps, int nrows,
                                                 const double *xsep, double *xp, bool reversed, int nf, int lane) {
#ifndef PLBA_BWD_PIPE
#define PLBA_BWD_PIPE 4
#endif
    constexpr int W = BW + 1, kPipe = PLBA_BWD_PIPE;
    if (nsteps <= 0) return;
    const int G = lane / 6, r = lane % 6;      // lane group G holds the window row j ≡ G (mod BW)
    const bool act = lane < BW * 6;
    const int top = xsep ? min(nrows - 1, nsteps - 1 + BW) : nsteps - 1;
    // window rows top-BW+1..top: separator x (known) or z to be completed
    double zv = 0.0;
    if (act) {
        int j = top - ((top - G) % BW + BW) % BW;  // the row of this group in [top-BW+1, top]
        if (j >= 0) zv = j >= nsteps ? (xsep ? xsep[(j - nsteps) * 6 + r] : 0.0) : zb[(size_t)j * 6 + r];
    }
    // Load cursor: row li's L block for this lane's window row li - wl, wl = ((li-G-1) mod BW)+1,
    // stepped incrementally (wl cycles BW..1 as li decreases). Loads are unconditional from
    // clamped in-range addresses and masked afterwards, so the loop carries no branches.
    int li = top, wl = ((top - G - 1) % BW + BW) % BW + 1;
    double Lr[kPipe][6], zr[kPipe];
    bool lok[kPipe], zok[kPipe];               // masks applied when the values are consumed, so
    auto load_step = [&](double (&dst)[6], double &z, bool &okL, bool &okZ) {  // no load is waited on early
        const int jl = li - wl;
        okL = act && li >= 0 && jl >= 0 && jl < nsteps;
        const int base = (max(li, 0) * W + wl) * 36 + r;
#pragma unroll
        for (int m = 0; m < 6; ++m) dst[m] = Lband[base + m * 6];
        const int iz = li - BW;
        z = zb[min(max(iz, 0), nsteps - 1) * 6 + r];
        okZ = act && iz >= 0 && iz < nsteps;
        --li;
        wl = wl == 1 ? BW : wl - 1;
    };
#pragma unroll
    for (int u = 0; u < kPipe; ++u) load_step(Lr[u], zr[u], lok[u], zok[u]);
    int gi = top % BW;                          // group holding row i (final), uniform
    // whole kPipe batches (trailing steps with i < 0 are masked no-ops): no exits inside the
    // unrolled body, so the compiler can count the prefetches in flight exactly
    for (int ib = top; ib >= 0; ib -= kPipe) {
#pragma unroll
        for (int u = 0; u < kPipe; ++u) {
            const int i = ib - u;
            double x[6];
#pragma unroll
            for (int m = 0; m < 6; ++m) {
                const int src = gi * 6 + m;
                const int lo = __builtin_amdgcn_readlane(__double2loint(zv), src);
                const int hi = __builtin_amdgcn_readlane(__double2hiint(zv), src);
                x[m] = __hiloint2double(hi, lo);
            }
            const bool mine = act && G == gi && i >= 0;  // this group holds the final row i
            if (mine && i < nsteps) {
                const int row = reversed ? nf - 1 - i : i;
                if constexpr (LX) ((__attribute__((address_space(3))) double *)xp)[row * 6 + r] = zv;
                else xp[(size_t)row * 6 + r] = zv;
            }
            // z_j -= L_{i,j}ᵀ x_i for the window rows j < nsteps (masked to zero elsewhere);
            // the group that held row i takes row i-BW
            double acc = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) acc = fma(Lr[u][m], x[m], acc);
            const double znew = zok[u] ? zr[u] : 0.0;
            zv = (mine ? znew : zv) - (lok[u] ? acc : 0.0);
            load_step(Lr[u], zr[u], lok[u], zok[u]);
            gi = gi == 0 ? BW - 1 : gi - 1;
        }
    }
}

template <int BW>
__device__ __forceinline__ void band_backward(const double *Lband, const double *zb, int nsteps, int nrows, const double *xsep,
                              double *xp, bool reversed, int nf, double *xr, double *part, int lane) {
    constexpr int W = BW + 1;
    const int last = min(nrows - 1, nsteps - 1 + BW);  // highest row coupled to the segment
    if (xsep && lane < 6)
        for (int i = 0; i < BW && nsteps + i < nrows; ++i) xr[((nsteps + i) % W) * 6 + lane] = xsep[i * 6 + lane];
    wave_lds_sync();
    // L_{k+w,k} and z_k are loaded kPipe steps ahead into a register ring (static slots: the
    // step loop is unrolled by kPipe), so their L2 latency hides behind kPipe steps of work
    constexpr int kMaxB = (BW * 6 + 63) / 64 > 0 ? (BW * 6 + 63) / 64 : 1;
    constexpr int kPipe = kMaxB == 1 ? 6 : 2;  // register budget: 12 f64 per slot per lane at bw <= 10
    double Lr[kPipe][kMaxB][6], zr[kPipe];
    auto load_step = [&](int k, double (&dst)[kMaxB][6], double &z) {
        const int wmax = (k >= 0) ? min(BW, last - k) : 0;
#pragma unroll
        for (int q = 0; q < kMaxB; ++q) {
            const int t = q * 64 + lane;
            const int w = 1 + t / 6, r = t % 6;
            const bool ok = t < wmax * 6;
            const double *L = Lband + ((size_t)(k + w) * W + w) * 36;
#pragma unroll
            for (int m = 0; m < 6; ++m) dst[q][m] = ok ? L[m * 6 + r] : 0.0;
        }
        z = (lane < 6 && k >= 0) ? zb[(size_t)k * 6 + lane] : 0.0;
    };
#pragma unroll
    for (int u = 0; u < kPipe; ++u) load_step(nsteps - 1 - u, Lr[u], zr[u]);
    for (int kb = nsteps - 1; kb >= 0; kb -= kPipe) {
#pragma unroll
        for (int u = 0; u < kPipe; ++u) {
            const int k = kb - u;
            if (k < 0) break;
            const int wmax = min(BW, last - k);
#pragma unroll
            for (int q = 0; q < kMaxB; ++q) {
                const int t = q * 64 + lane;
                if (t < wmax * 6) {
                    const int w = 1 + t / 6, r = t % 6, i = k + w;
                    const double *x = xr + (i % W) * 6;
                    double s = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) s += Lr[u][q][m] * x[m];
                    part[w * 6 + r] = s;
                }
            }
            wave_lds_sync();
            if (lane < 6) {
                double v = zr[u];
                for (int w = 1; w <= wmax; ++w) v -= part[w * 6 + lane];
                xr[(k % W) * 6 + lane] = v;
                xp[(size_t)(reversed ? nf - 1 - k : k) * 6 + lane] = v;
            }
            wave_lds_sync();
            load_step(k - kPipe, Lr[u], zr[u]);  // refill this slot kPipe steps ahead
        }
    }
}

// Streamed back substitution of the two-sided register-window band kernel (bw >= 11), both
// segments at once: wave 0 runs segment 0, wave 1 segment 1, and the other waves stream the rows
// of L they are about to need into LDS, CH rows a chunk, double-buffered with one workgroup
// barrier per chunk (the one-wave band_backward waited on its L2 prefetches, two steps ahead at
// ≈ 2.2 k cycles a step). Right-looking: the wave keeps the z values of the BW rows below the
// current row i in registers (lane entry t = q·64 + lane: ring slot t/6 = row mod BW, component
// t%6); once row i is final, x_i is broadcast by v_readlane and every lane removes
// L_{i,j}ᵀ x_i from its row j = i − w in one 6-term product, reading row i of L (contiguous in
// Lband: blocks (i, i−1) .. (i, i−BW)) from the staged chunk; row i's slot then takes row i−BW
// (z_{i−BW} staged with the row). Rows nsteps.. of a segment are the separator (x given).
struct BackSeg {
    const double *Lband, *zb, *xsep;  // segment's L rows and z, its separator x [BW][6]
    int nsteps;                       // eliminated rows (x written for rows < nsteps)
    int nrows;                        // rows of the segment's band (separator included)
    bool reversed;                    // row i is pose nf-1-i
};
__host__ __device__ constexpr int bstream_ch(int bw) { return bw <= 24 ? 4 : 3; }
__host__ __device__ constexpr size_t bstream_doubles(int bw) {
    return (size_t)4 * bstream_ch(bw) * ((size_t)bw * 36 + 6);  // [2 buffers][2 segments][CH][RS]
}
template <int BW, int NT, int CH>
__device__ __forceinline__ void band_backward_stream(const BackSeg (&sg)[2], int nf, double *xl, double *buf) {
    constexpr int RS = BW * 36 + 6, NQ = (BW * 6 + 63) / 64;  // buf: [2][2][CH][RS]
    constexpr int SEG = CH * RS;                       // doubles of one segment's chunk
    constexpr int PN = NT - 128, NP2 = SEG;            // producer threads; double2 pieces of a chunk
    constexpr int PER = (NP2 + PN - 1) / PN;           // pieces per producer thread
    static_assert(RS % 2 == 0 && PN > 0, "staged rows are double2 pieces");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int last0 = min(sg[0].nrows - 1, sg[0].nsteps - 1 + BW), last1 = min(sg[1].nrows - 1, sg[1].nsteps - 1 + BW);
    const double *L0 = sg[0].Lband, *L1 = sg[1].Lband, *z0 = sg[0].zb, *z1 = sg[1].zb;
    const int nchunk = (max(last0, last1) + CH) / CH;  // chunk c: rows last - c·CH .. last - c·CH - CH + 1
    // producers: both segments' rows of chunk c, loaded into registers one chunk period before
    // they are stored (the loads stay in flight across the LDS-only barrier)
    const int pt = tid - 128;
    double2 v[PER];
    auto load_chunk = [&](int c) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int e = pt + j * PN;                 // piece: segment e / (SEG/2), offset 2·(e % (SEG/2))
            v[j] = make_double2(0.0, 0.0);
            if (e < NP2) {
                const int s = e / (SEG / 2), o2 = 2 * (e % (SEG / 2)), u = o2 / RS, o = o2 % RS;
                const int i = (s ? last1 : last0) - (c * CH + u);
                if (i >= 0) {
                    const double *Lb = s ? L1 : L0, *zb = s ? z1 : z0;  // (no runtime index into sg: stack)
                    if (o < BW * 36) v[j] = *(const double2 *)(Lb + ((size_t)i * (BW + 1) + 1) * 36 + o);
                    else if (i - BW >= 0) v[j] = *(const double2 *)(zb + (size_t)(i - BW) * 6 + (o - BW * 36));
                }
            }
        }
    };
    auto store_chunk = [&](int c) {
        double2 *dst = (double2 *)(buf + (size_t)(c & 1) * 2 * SEG);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int e = pt + j * PN;
            if (e < NP2) dst[e] = v[j];
        }
    };
    // ---- consumer state: the ring of the segment's z (rows last-BW+1 .. last at the start)
    const bool cons = wv < 2, s1 = wv == 1;
    const double *gz = s1 ? z1 : z0, *gx = s1 ? sg[1].xsep : sg[0].xsep;
    const bool grev = s1 ? sg[1].reversed : sg[0].reversed;
    const int last = s1 ? last1 : last0, ns = s1 ? sg[1].nsteps : sg[0].nsteps;
    const int lastu = __builtin_amdgcn_readfirstlane(last);  // (per wave)
    double z[NQ];
    int ws[NQ];                                        // w = i - j of the entry's row j at step i
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int t = q * 64 + lane, sl = t / 6, r = t % 6;
        z[q] = 0.0;
        ws[q] = 0;
        if (cons && t < BW * 6) {
            const int j = last - (((last - sl) % BW) + BW) % BW;
            ws[q] = last - j;
            if (j >= ns) z[q] = gx[(j - ns) * 6 + r];
            else if (j >= 0) z[q] = gz[(size_t)j * 6 + r];
        }
    }
    if (wv >= 2) load_chunk(0);
    __syncthreads();  // (the separator x sits in the region the chunks overwrite)
    if (wv >= 2) {
        store_chunk(0);
        if (1 < nchunk) load_chunk(1);
    }
    lds_barrier();
    for (int c = 0; c < nchunk; ++c) {
        if (wv >= 2) {
            if (c + 1 < nchunk) store_chunk(c + 1);
            if (c + 2 < nchunk) load_chunk(c + 2);
        } else if (cons) {
            const double *B = buf + ((size_t)(c & 1) * 2 + wv) * SEG;
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int i = lastu - (c * CH + u);  // (uniform: scalar slot arithmetic below)
                if (i < 0) break;
                const double *Lr = B + u * RS;
                // the step's L reads first: they do not depend on x_i (a slot whose row is final
                // this step reads block BW, row i-BW's, and the staged z_{i-BW})
                double Lv[NQ][6], zr[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int r = (q * 64 + lane) % 6, w = ws[q] == 0 ? BW : ws[q];
#pragma unroll
                    for (int m = 0; m < 6; ++m) Lv[q][m] = Lr[(w - 1) * 36 + m * 6 + r];
                    zr[q] = Lr[BW * 36 + r];
                }
                const int si = i % BW;
                double x[6];
#pragma unroll
                for (int r = 0; r < 6; ++r) {  // x_i from the lanes of row i's slot
                    const int t = si * 6 + r, q = t >> 6, ln = t & 63;
                    double v = z[0];
#pragma unroll
                    for (int qq = 1; qq < NQ; ++qq) v = q == qq ? z[qq] : v;
                    x[r] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), ln),
                                            __builtin_amdgcn_readlane(__double2loint(v), ln));
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int t = q * 64 + lane, r = t % 6;
                    const bool fin = ws[q] == 0;   // row i: final; the slot takes row i - BW
                    const int w = fin ? BW : ws[q], j = i - w;
                    if (fin && t < BW * 6 && i < ns) xl[(size_t)(grev ? nf - 1 - i : i) * 6 + r] = z[q];
                    double acc = 0.0;
#pragma unroll
                    for (int m = 0; m < 6; ++m) acc = fma(Lv[q][m], x[m], acc);
                    const double zz = fin ? zr[q] : z[q];
                    z[q] = (j >= 0 && j < ns) ? zz - acc : zz;
                    ws[q] = w - 1;
                }
            }
        }
        lds_barrier();
    }
}

template <int BW>
__global__ __launch_bounds__(band_nt(BW)) void k_rcs_factor_band(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const BandSeg g{d.Bd, d.bs, d.Lband, d.Kinv, d.zb, d.nf, d.nf, nullptr};
    const bool fail = band_forward<BW>(g, lds, d.ring, d.stamps) || diag_fail(d);
    if (threadIdx.x == 0) *d.solve_okp = fail ? 0 : 1;
    if (!fail && threadIdx.x < 64) {
        double *col, *piv, *bwin, *Lcol, *Kv, *xr, *part, *ys, *ringL, *ringK, *ringZ;
        band_lds<BW>(lds, d.ring, col, piv, bwin, Lcol, Kv, xr, part, ys, ringL, ringK, ringZ);
        if constexpr (BW >= 1 && BW * 6 <= 64) band_backward_rl<BW>(d.Lband, d.zb, d.nf, d.nf, nullptr, d.xp, false, d.nf, threadIdx.x);
        else band_backward<BW>(d.Lband, d.zb, d.nf, d.nf, nullptr, d.xp, false, d.nf, xr, part, threadIdx.x);
    }
    __syncthreads();
    pose_update_wg<band_nt(BW)>(d, fail);  // applied even after a failed solve, with the previous x_p (A13)
}

// Two-sided ("twisted") banded LDLᵀ: workgroup 0 eliminates block rows 0..m-1 top-down,
// workgroup 1 eliminates rows nf-1..m+BW bottom-up (as the top-down elimination of the
// block-reversed matrix Bd2), concurrently on two CUs. The two eliminated sets do not couple
// (they are > BW blocks apart), so their Schur updates of the BW-block separator m..m+BW-1
// add: S_sep = W0 + W1 − A_sep. The workgroup that finishes second solves the separator
// (block LDLᵀ on its packed lower triangle, no pivoting: a zero pivot fails the solve as
// SimplicialLDLT does) and runs both back substitutions on two waves. Half the serial chain.
template <int BW>
__device__ __forceinline__ void k_rcs_factor_twisted_body(const Dev &d) {
    constexpr int W = BW + 1, NT = band_nt(BW), NS = 6 * BW;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int s_last, s_sfail;
    const int seg = blockIdx.x, tid = threadIdx.x;
    const size_t sep_stride = (size_t)BW * W * 36 + (size_t)BW * 6;
    const int m = d.tw_m, n1 = d.nf - BW - d.tw_m;
    const BandSeg g = seg == 0 ? BandSeg{d.Bd, d.bs, d.Lband, d.Kinv, d.zb, d.nf, m, d.tw_sep}
                               : BandSeg{d.Bd2, d.bs2, d.Lband2, d.Kinv2, d.zb2, d.nf, n1, d.tw_sep + sep_stride};
#ifdef PLBA_STAMPS
    unsigned long long tw_t0 = __builtin_readcyclecounter();
#endif
    const bool fail = band_forward<BW>(g, lds, d.ring, seg == 0 ? d.stamps : nullptr) || diag_fail(d);
#ifdef PLBA_STAMPS
    unsigned long long tw_t1 = __builtin_readcyclecounter();
#define TW_MARK(q, t)                                                     \
    do {                                                                  \
        if (tid == 0) atomicAdd(&d.stamps[16 * 8 + (q)], (t));            \
    } while (0)
    if (seg == 0) TW_MARK(0, tw_t1 - tw_t0); else TW_MARK(1, tw_t1 - tw_t0);
#else
#define TW_MARK(q, t) do {} while (0)
#endif
    // hand-off (MI355X_MICROARCH.md §Workgroup dispatch…, counter form): every wave drains its
    // L / z / separator stores, one agent release by lane 0, then the arrival counter; the
    // workgroup whose add returns 1 is last and acquires once before reading the other's data
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(&d.tw_fail[seg], fail ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(d.tw_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == 1 ? 1 : 0;
        if (old == 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(d.tw_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
            s_sfail = (__hip_atomic_load(&d.tw_fail[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                       __hip_atomic_load(&d.tw_fail[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1 : 0;
        }
    }
    __syncthreads();
    if (!s_last) return;
    if (!s_sfail) {
    // merge layout (twisted_merge_doubles) from LDS offset 0: the band windows are dead, both
    // separators having been exported to global memory before the arrival
    double *xl = lds;                                  // [nf][6] x_p staging
    double *Ls = lds + (size_t)d.nf * 6;               // [BW(BW-1)/2][36] L_IP, I > P (block I(I-1)/2 + P)
    double *Kp = Ls + (size_t)BW * (BW - 1) / 2 * 36;  // [BW][36] pivot inverses S_PP⁻¹ (after the sweep)
    double *colA = Kp + (size_t)BW * 36;               // [2][BW][36] pivot column A_IP (step parity)
    double *Sp = colA + (size_t)2 * BW * 36;           // [BW][36] pivot blocks S_PP
    double *rhs = Sp + (size_t)BW * 36, *xs0 = rhs + NS, *xsr = xs0 + NS;  // [NS] each
    // Separator system S_sep (lower block (I, J), I >= J, w = I - J < BW) by right-looking block
    // LDLᵀ with the blocks held in registers: block (I, J) is owned by UPB threads (UR rows each,
    // the band kernel's split) for the whole elimination, so a trailing update reads only its
    // L_IP rows and A_JP from LDS (54 reads for 108 FMA at UR = 3) and writes nothing back. Per
    // pivot P two barriers: the owners of column P factor S_PP LDLᵀ in their own registers and
    // solve their rows of L_IP = A_IP S_PP⁻¹; the owners of the trailing blocks apply
    // A_IJ -= L_IP A_JPᵀ and publish column P + 1 into the other parity buffer (the right-hand
    // side y_R -= L_RP y_P on the side). The pivot inverses the back substitution needs are formed
    // after the sweep, all at once (a wave-0 inverse per step was one more barrier and ≈ 1 k cycles
    // on the chain). No pivoting: a zero LDLᵀ pivot fails the solve as SimplicialLDLT does. (Round 5 held the system as a packed scalar triangle in LDS and
    // swept it with one thread per entry: runtime divisions + 12 LDS reads per FMA-6 entry;
    // ≈ 28 % of the C3R factorisation.)
    const double *W0 = d.tw_sep, *W1 = d.tw_sep + sep_stride;
    constexpr int UR = band_ur(BW), UPB = 6 / UR, UE = UR * 6, NB = BW * (BW + 1) / 2;
    static_assert(UPB * NB <= NT, "one owned separator (part) block per thread");
    const bool own = tid < UPB * NB;
    int oI = 0, oJ = 0;
    if (own) {
        const int b = tid / UPB;
        while ((oI + 1) * (oI + 2) / 2 <= b) ++oI;
        oJ = b - oI * (oI + 1) / 2;
    }
    const int oh = (tid % UPB) * UR;  // first row of the owned part
    double t[UE];
    if (own) {
        const int w = oI - oJ;
#pragma unroll
        for (int r = 0; r < UR; ++r)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const int a = oh + r;
                const double w0 = W0[((size_t)oI * W + w) * 36 + a * 6 + c];
                t[r * 6 + c] = w0 + W1[((size_t)(BW - 1 - oJ) * W + w) * 36 + c * 6 + a] -
                               d.Bd[((size_t)(m + oI) * W + w) * 36 + a * 6 + c];
            }
        // column 0: the first pivot block / pivot column
        if (oJ == 0) {
            double *dst = oI == 0 ? Sp : colA + (size_t)oI * 36;
#pragma unroll
            for (int j = 0; j < UE; ++j) dst[oh * 6 + j] = t[j];
        }
    }
    for (int q = tid; q < NS; q += NT) {
        const int i = q / 6, a = q % 6;
        rhs[q] = W0[(size_t)BW * W * 36 + i * 6 + a] + W1[(size_t)BW * W * 36 + (BW - 1 - i) * 6 + a] -
                 d.bs[(size_t)(m + i) * 6 + a];
    }
    if (tid == 0) s_sfail = 0;
    __syncthreads();
#ifdef PLBA_STAMPS
    TW_MARK(5, __builtin_readcyclecounter() - tw_t1);  // hand-off + separator assembly
#endif
    for (int P = 0; P < BW; ++P) {
        const double *colP = colA + (size_t)(P & 1) * BW * 36;
        if (own && oJ == P && oI > P) {  // rows oh..oh+UR-1 of L_IP = A_IP S_PP⁻¹ (S symmetric: S⁻¹ a_r)
            const double *S = Sp + P * 36;
            double s[21], dv[6];
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) s[ltri(i, j)] = S[i * 6 + j];
            bool zp = false;  // (a zero pivot is reported by the inverses below)
            ldl6_inplace(s, dv, zp);
            double *L = Ls + ((size_t)oI * (oI - 1) / 2 + P) * 36 + oh * 6;
#pragma unroll
            for (int r = 0; r < UR; ++r) {
                double x[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) x[c] = t[r * 6 + c];
                ldl6_solve(s, dv, x);
#pragma unroll
                for (int c = 0; c < 6; ++c) L[r * 6 + c] = x[c];
            }
        }
        __syncthreads();
        if (own && oJ > P) {  // A_IJ -= L_IP A_JPᵀ, then column P + 1 published
            const double *L = Ls + ((size_t)oI * (oI - 1) / 2 + P) * 36 + oh * 6;
            const double *Aj = colP + (size_t)oJ * 36;
            double l[UE];
#pragma unroll
            for (int j = 0; j < UE; ++j) l[j] = L[j];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double a[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) a[q] = Aj[c * 6 + q];
#pragma unroll
                for (int r = 0; r < UR; ++r) {
                    double acc = 0.0;
#pragma unroll
                    for (int q = 0; q < 6; ++q) acc = fma(l[r * 6 + q], a[q], acc);
                    t[r * 6 + c] -= acc;
                }
            }
        }
        {   // y_R -= L_RP y_P for the trailing rows (threads past the owners first)
            const int q = NT - 1 - tid, R = (P + 1) * 6 + q;
            if (q >= 0 && R < NS) {
                const double *L = Ls + ((size_t)(R / 6) * (R / 6 - 1) / 2 + P) * 36 + (R % 6) * 6;
                double acc = 0.0;
#pragma unroll
                for (int c = 0; c < 6; ++c) acc = fma(L[c], rhs[P * 6 + c], acc);
                rhs[R] -= acc;
            }
        }
        if (own && oJ == P + 1) {
            double *dst = oI == P + 1 ? Sp + (P + 1) * 36 : colA + ((size_t)((P + 1) & 1) * BW + oI) * 36;
#pragma unroll
            for (int j = 0; j < UE; ++j) dst[oh * 6 + j] = t[j];
        }
        __syncthreads();
    }
    for (int P = tid >> 6; P < BW; P += NT / 64) {  // S_PP⁻¹, one pivot block per wave
        bool f = false;
        const double I = ldl_inverse6(Sp + P * 36, rhs, tid & 63, f);
        if ((tid & 63) < 36) Kp[P * 36 + (tid & 63)] = I;
        if (f && (tid & 63) == 0) s_sfail = 1;
    }
    __syncthreads();
#ifdef PLBA_STAMPS
    unsigned long long tw_t2 = __builtin_readcyclecounter();
    TW_MARK(2, tw_t2 - tw_t1);
#endif
    if (!s_sfail) {
    // back substitution x_P = S_PP⁻¹ y_P − Σ_{I>P} L_IPᵀ x_I, right-looking: x_I is final once the
    // blocks below it are done, and its contribution is removed from every P < I in one pass.
    // x_sep in both segment orders: rows m+i for segment 0, reversed rows n1+i = original
    // m+BW-1-i for segment 1
    for (int q = tid; q < NS; q += NT) {
        const int P = q / 6, c = q % 6;
        double x = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) x = fma(Kp[P * 36 + c * 6 + r], rhs[P * 6 + r], x);
        xs0[q] = x;
    }
    __syncthreads();
    for (int I = BW - 1; I >= 1; --I) {
        if (tid < I * 6) {
            const int P = tid / 6, c = tid % 6;
            const double *L = Ls + ((size_t)I * (I - 1) / 2 + P) * 36 + c;
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < 6; ++r) acc = fma(L[r * 6], xs0[I * 6 + r], acc);
            xs0[tid] -= acc;
        }
        __syncthreads();
    }
    for (int q = tid; q < NS; q += NT) {
        xl[(size_t)m * 6 + q] = xs0[q];
        xsr[q] = xs0[(BW - 1 - q / 6) * 6 + q % 6];
    }
    __syncthreads();
    if constexpr (BW * 6 <= 64) {
        if (tid < 64) band_backward_rl<BW, true>(d.Lband, d.zb, m, d.nf, xs0, xl, false, d.nf, tid);
        else if (tid < 128) band_backward_rl<BW, true>(d.Lband2, d.zb2, n1, d.nf, xsr, xl, true, d.nf, tid - 64);
    } else {
        const BackSeg sg[2] = {{d.Lband, d.zb, xs0, m, d.nf, false}, {d.Lband2, d.zb2, xsr, n1, d.nf, true}};
        band_backward_stream<BW, NT, bstream_ch(BW)>(sg, d.nf, xl, Ls);
    }
    __syncthreads();
    for (int t = tid; t < d.nf * 6; t += NT) d.xp[t] = xl[t];
#ifdef PLBA_STAMPS
    if (tid == 0) TW_MARK(3, __builtin_readcyclecounter() - tw_t2);
    if (tid == 0) TW_MARK(4, 1);
#endif
    }  // separator solved
    }  // both segments eliminated
#undef TW_MARK
    __syncthreads();
    if (tid == 0) *d.solve_okp = s_sfail ? 0 : 1;
    pose_update_wg<NT>(d, s_sfail != 0);  // applied even after a failed solve, with the previous x_p (A13)
}

template <int BW>
__global__ __launch_bounds__(band_nt(BW)) void k_rcs_factor_twisted(Dev d0) {
    if constexpr (BW >= 1) {  // (the host never selects bw 0)
        TRIAL_SLOT(blockIdx.y)
        k_rcs_factor_twisted_body<BW>(d);
    }
}

#include "plba_band_cl.hpp"
#include "plba_bcr.hpp"
#include "plba_dense.hpp"
#include "plba_pgo.hpp"

// ---------------------------------------------------------------- update + trial evaluation
// stand-alone pose update (windows without free poses: no factorisation kernel to fuse into)
__global__ __launch_bounds__(kBlock) void k_pose_update(Dev d0) {
    TRIAL_SLOT(0)
    if (blockIdx.x == 0) pose_update_wg<kBlock>(d, false);
}

// ---------------------------------------------------------------- edge-parallel trial path
// per landmark: (Hll + λI) = L Lᵀ, g = L⁻¹ b_l (packed lower; recomputed where needed — 4x4,
// cheaper than a kernel boundary)
// Signed form (the hand-rolled LM, `sgn`): (Hll + λ·diag) = M S Mᵀ with S = diag(±1), as an
// unpivoted LDLᵀ tolerates a non-positive pivot (the reference solves the whole system with
// SimplicialLDLT, src/mapHandler.cpp:1861-1865; a rank-deficient landmark block under λ·diag ≈
// 1e-24·H meets one). Every sign is exactly 1 for a positive definite block, and the products
// are grouped so that the result is then bitwise the plain Cholesky's.
__device__ __forceinline__ void lm_chol(const Dev &d, int l, double lam, bool mul, double (&L)[10], double (&g)[4],
                                        double (&S)[4], bool sgn = false) {
    const int DIM = is_point_lm(d, l) ? 3 : 4;
    double H[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) { H[k] = d.Hll[(size_t)l * 10 + k]; L[k] = 0.0; }
#pragma unroll
    for (int k = 0; k < 4; ++k) { g[k] = 0.0; S[k] = 1.0; }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j < DIM) {
            double sj = H[pk(j, j)] + (mul ? lam * H[pk(j, j)] : lam);
#pragma unroll
            for (int p = 0; p < j; ++p) sj -= (L[pk(j, p)] * S[p]) * L[pk(j, p)];
            const double sg = (sgn && sj < 0.0) ? -1.0 : 1.0;
            S[j] = sg;
            const double djj = 1.0 / sqrt(sg * sj);  // reciprocal diagonal: every use divides by it
            L[pk(j, j)] = djj;
#pragma unroll
            for (int i = j + 1; i < 4; ++i) {
                if (i < DIM) {
                    double t = H[pk(i, j)];
#pragma unroll
                    for (int p = 0; p < j; ++p) t -= L[pk(i, p)] * (L[pk(j, p)] * S[p]);
                    L[pk(i, j)] = (t * djj) * sg;
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < DIM) {
            double t = d.bl[(size_t)l * 4 + i];
#pragma unroll
            for (int p = 0; p < i; ++p) t -= L[pk(i, p)] * g[p];
            g[i] = t * L[pk(i, i)];
        }
    }
}
// per edge: Z_e = B_e L⁻ᵀ (rows solved with L), q_e = Z_e g. The Z / q rows are staged in LDS and
// written out as contiguous pieces (per-lane 64-B / 16-B rows made every store instruction touch
// ~32 cache lines; see k_linearize)
__device__ __forceinline__ void edge_schur_body(const Dev &d, int e, double *Z, double *qe) {
    const int l = d.e_lm[e];
    if (e >= d.Ep && d.ctrl->hlm == 2) {  // GBA line: 6x6 (Hl6 + λ·diag) = L Lᵀ, Z_e = L⁻¹ b_e, q_e = Z_e·L⁻¹ b_l
        const double lam = d.lam;
        const int li = l - d.n_pt;
        double H[21], L6[21], g6[6], bb[6], z[6];
#pragma unroll
        for (int k = 0; k < 21; ++k) { H[k] = d.Hl6[(size_t)li * 21 + k]; L6[k] = 0.0; }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double sj = H[pk(j, j)] + lam * H[pk(j, j)];
#pragma unroll
            for (int p = 0; p < j; ++p) sj -= L6[pk(j, p)] * L6[pk(j, p)];
            const double djj = sqrt(sj);
            L6[pk(j, j)] = djj;
#pragma unroll
            for (int i = j + 1; i < 6; ++i) {
                double t = H[pk(i, j)];
#pragma unroll
                for (int p = 0; p < j; ++p) t -= L6[pk(i, p)] * L6[pk(j, p)];
                L6[pk(i, j)] = t / djj;
            }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) bb[k] = d.B[(size_t)e * 8 + k];
        double q0 = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double t = bb[i], tg = d.bl6[(size_t)li * 6 + i];
#pragma unroll
            for (int p = 0; p < i; ++p) {
                t -= L6[pk(i, p)] * z[p];
                tg -= L6[pk(i, p)] * g6[p];
            }
            z[i] = t / L6[pk(i, i)];
            g6[i] = tg / L6[pk(i, i)];
            q0 += z[i] * g6[i];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) Z[k] = z[k];
        Z[6] = Z[7] = 0.0;
        qe[0] = q0;
        qe[1] = 0.0;
        return;
    }
    const int DIM = e < d.Ep ? 3 : 4;
    const bool sgn = d.ctrl->hlm == 1;
    double L[10], g[4], B[8], S[4];
    lm_chol(d, l, d.lam, d.ctrl->hlm != 0, L, g, S, sgn);
#pragma unroll
    for (int k = 0; k < 8; ++k) B[k] = d.B[(size_t)e * 8 + k];
    double z[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < DIM) {
                double t = B[r * 4 + i];
#pragma unroll
                for (int p = 0; p < i; ++p) t -= L[pk(i, p)] * z[r][p];
                z[r][i] = t * L[pk(i, i)];
            }
        }
    double q0 = 0, q1 = 0;
    if (sgn) {  // hand-rolled LM (one live row): row 1 carries S·z_0, the assembly takes z_1·(S z_2)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            Z[i] = z[0][i];
            Z[4 + i] = z[0][i] * S[i];
            q0 += (z[0][i] * S[i]) * g[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            Z[i] = z[0][i];
            Z[4 + i] = z[1][i];
            q0 += z[0][i] * g[i];
            q1 += z[1][i] * g[i];
        }
    }
    qe[0] = q0;
    qe[1] = q1;
}
__global__ __launch_bounds__(kBlock) void k_edge_schur(Dev d0) {
    TRIAL_SLOT(blockIdx.y)
    const int e = blockIdx.x * kBlock + threadIdx.x;
#ifdef PLBA_SCHUR_DIRECT
    if (e < d.E) edge_schur_body(d, e, d.Z + (size_t)e * 8, d.q + (size_t)e * 2);
#else
    __shared__ __attribute__((aligned(16))) double stZ[kBlock * 8], stq[kBlock * 2];
    if (e < d.E) edge_schur_body(d, e, stZ + threadIdx.x * 8, stq + threadIdx.x * 2);
    __syncthreads();
    const int e0 = blockIdx.x * kBlock, n = min(kBlock, d.E - e0);
    {
        const double2 *s2 = reinterpret_cast<const double2 *>(stZ);
        double2 *d2 = reinterpret_cast<double2 *>(d.Z + (size_t)e0 * 8);
        for (int t = threadIdx.x; t < n * 4; t += kBlock) d2[t] = s2[t];
    }
    {
        const double2 *s2 = reinterpret_cast<const double2 *>(stq);
        double2 *d2 = reinterpret_cast<double2 *>(d.q + (size_t)e0 * 2);
        for (int t = threadIdx.x; t < n; t += kBlock) d2[t] = s2[t];
    }
#endif
}
// per landmark: x_l = L⁻ᵀ L⁻¹ (b_l - Σ u_e), oplus into the trial state, scale partial
// quad (4-lane) DPP exchanges: xor 1 = quad_perm [1,0,3,2], xor 2 = quad_perm [2,3,0,1]
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// sum over the 4 lanes of a quad, identical in all four (a+b == b+a bitwise)
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_f64<0xB1>(v);
    return v + dpp_f64<0x4E>(v);
}

// v[q] for a lane-dependent q without dynamic register indexing (which spills the array to
// scratch)
__device__ __forceinline__ double sel4(const double (&v)[4], int q) {
    // a select chain is turned back into an indexed scratch load by the compiler: blend instead
    const double m0 = q == 0 ? 1.0 : 0.0, m1 = q == 1 ? 1.0 : 0.0, m2 = q == 2 ? 1.0 : 0.0, m3 = q == 3 ? 1.0 : 0.0;
    return fma(v[3], m3, fma(v[2], m2, fma(v[1], m1, v[0] * m0)));
}

// value of quad lane Q in every lane of the quad (DPP quad_perm [Q,Q,Q,Q])
template <int Q>
__device__ __forceinline__ double quad_bcast(double v) {
    return dpp_f64<Q | (Q << 2) | (Q << 4) | (Q << 6)>(v);
}

// VertexLMLineOrth::oplusImpl (g2o_types/g2o_types.h:72-130) followed by changeOrthToPluker
// (g2o_types.h:367-387) for one line, with the transcendentals spread over the landmark's quad:
// lane q evaluates sincos of θ_q and δθ_q (θ_3 = φ), the quad exchanges them by DPP, every lane
// forms U' = R_xyz(θ)·Rx(δθ1)·Ry(δθ2)·Rz(δθ3) and W10 redundantly, lane q takes angle q of the
// result with the reference's own function (atan2 / asin / atan2 / asin) and its sincos, and the
// quad exchanges those to rebuild the Plücker vector from the new angles exactly as the
// reference does: 3 sincos + 1 inverse per lane instead of 28 calls, same formulas.
// Returns angle q of the new state. All four lanes of the quad must be active.
__device__ __forceinline__ double orth_oplus_quad(const double (&D)[4], const double (&dD)[4], int q, double (&Lp)[6]) {
    const double a = sel4(D, q), b = sel4(dD, q);
    double sa, ca, sb, cb;
    sincos(a, &sa, &ca);
    sincos(b, &sb, &cb);
    const double s1 = quad_bcast<0>(sa), c1 = quad_bcast<0>(ca), s2 = quad_bcast<1>(sa), c2 = quad_bcast<1>(ca);
    const double s3 = quad_bcast<2>(sa), c3 = quad_bcast<2>(ca), w2 = quad_bcast<3>(sa), w1 = quad_bcast<3>(ca);
    const double sx = quad_bcast<0>(sb), cx = quad_bcast<0>(cb), sy = quad_bcast<1>(sb), cy = quad_bcast<1>(cb);
    const double sz = quad_bcast<2>(sb), cz = quad_bcast<2>(cb), sp = quad_bcast<3>(sb), cp = quad_bcast<3>(cb);
    const double R[9] = {c2 * c3, s1 * s2 * c3 - c1 * s3, c1 * s2 * c3 + s1 * s3,
                         c2 * s3, s1 * s2 * s3 + c1 * c3, c1 * s2 * s3 - s1 * c3,
                         -s2,     s1 * c2,                c1 * c2};
    const double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    const double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    const double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    double T1[9], T2[9], Rn[9];
    mat3mul(R, Rx, T1);
    mat3mul(T1, Ry, T2);
    mat3mul(T2, Rz, Rn);
    const double W10 = w2 * cp + w1 * sp;
    double o;
    if (q & 1) o = asin(q == 1 ? -Rn[6] : W10);
    else o = q == 0 ? atan2(Rn[7], Rn[8]) : atan2(Rn[3], Rn[0]);
    double so, co;
    sincos(o, &so, &co);
    const double t1 = quad_bcast<0>(so), u1 = quad_bcast<0>(co), t2 = quad_bcast<1>(so), u2 = quad_bcast<1>(co);
    const double t3 = quad_bcast<2>(so), u3 = quad_bcast<2>(co), v2 = quad_bcast<3>(so), v1 = quad_bcast<3>(co);
    // rot_xyz(new angles), columns 0 and 1 (plba_math.hpp), scaled by cos φ' / sin φ'
    Lp[0] = v1 * (u2 * u3); Lp[1] = v1 * (u2 * t3); Lp[2] = v1 * (-t2);
    Lp[3] = v2 * (t1 * t2 * u3 - u1 * t3); Lp[4] = v2 * (t1 * t2 * t3 + u1 * u3); Lp[5] = v2 * (t1 * u2);
    return o;
}

// kLmLanes lanes per landmark: lane q walks edges q, q+4, ... of the landmark's CSR range for
// the back-substitution sum, the quad adds the partials (DPP, fixed order), and every lane of
// the quad then solves the 3x3/4x4 system redundantly; lane q writes component q.
constexpr int kLmLanes = 4;
constexpr int kLmsNT = 256;  // k_lm_solve workgroup: 64 landmarks
// Edge slots held in registers per lane (lane q: edges q, q+4, ... up to kLmSlots of them);
// longer tracks fall back to a loop for the remainder. Every load of the kernel that does not
// depend on another load is issued up front, so a landmark costs two dependent global round
// trips (CSR offsets -> edge records, then x_p / trial poses) instead of one per phase.
// (one slot: 2 → 1 cut the kernel's registers enough for 3 waves per SIMD; C5 94.7 → 89 µs,
// C3 unchanged; the edges of a lane are visited in the same order either way)
#ifndef PLBA_LM_SLOTS
#define PLBA_LM_SLOTS 1
#endif
constexpr int kLmSlots = PLBA_LM_SLOTS;
struct LmEdge {
    int e, h, kf;
    bool act;
    double info, obs[4], A[12], B[8];
};
__device__ __forceinline__ void lm_load_edge(const Dev &d, int e, LmEdge &s) {
    s.e = e;
    s.h = d.e_hidx[e];
    s.kf = d.e_kf[e];
    s.act = d.e_active[e] != 0;
    s.info = d.e_info[e];
#pragma unroll
    for (int k = 0; k < 4; ++k) s.obs[k] = d.e_obs[(size_t)e * 4 + k];
#pragma unroll
    for (int k = 0; k < 12; ++k) s.A[k] = d.A[(size_t)e * 12 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) s.B[k] = d.B[(size_t)e * 8 + k];
}
// u += B_eᵀ (A_e x_p) for an edge of a free pose; a GBA line's 6-entry row (flat in B, A's second
// row zero) also feeds u45 (components 4, 5)
template <bool GBA = false>
__device__ __forceinline__ void lm_hpl_x(const LmEdge &s, const double (&x)[6], double (&u)[4], double (&u45)[2]) {
    double ax0 = 0, ax1 = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        ax0 += s.A[k] * x[k];
        ax1 += s.A[6 + k] * x[k];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] += s.B[i] * ax0 + s.B[4 + i] * ax1;
    if (GBA) {
        u45[0] += s.B[4] * ax0;
        u45[1] += s.B[5] * ax0;
    }
}
// robust χ² of one active edge at the trial state (computeActiveErrors)
__device__ __forceinline__ double lm_eval(const Dev &d, const LmEdge &s, const double *T, bool pt, const double (&X)[4],
                                          const double (&Lp)[6], bool robust, double delta) {
    double err[2];
    if (pt) {
        double z;
        point_error(T, X, s.obs, d.cam, err, z);
    } else {
        line_error(T, Lp, s.obs, d.cam, err);
    }
    const double c2 = err[0] * (s.info * err[0]) + err[1] * (s.info * err[1]);
    d.chi2_last[s.e] = c2;
    double rho0 = c2, rho1;
    if (robust) huber(c2, delta, rho0, rho1);
    return rho0;
}

// OptimizationAlgorithmLevenberg trial decision + optimize() loop control.
// Runs as its own launch (sharded windows, windows without landmarks) or as the tail of the last
// k_lm_solve workgroup; the landmark partials are read with sc1 loads in both cases.
// Speculative steps: the W = Ctrl::spec_w trial slots evaluated λ_0 = λ, λ_1 = λ·ν, ... of the
// same linearisation from the same state; they are consumed in slot order exactly as g2o's loop
// would have met them (slot s is only reached when slot s-1 was rejected and the loop goes on,
// and then λ, ν here equal the λ_s, ν_s slot s used, bit for bit), and the slots after an
// accepted or iteration-ending trial are discarded. A failed solve (zero pivot) uses the last
// successful solve's x; a slot whose solve failed after an earlier slot of the same step had
// succeeded saw the wrong "last" x, so it is not consumed: the next step evaluates it again,
// alone (one slot: no concurrent writer of the buffers it reads).
constexpr int kSpecOff = 0, kSpecAlways = 1, kSpecAfterReject = 2, kSpecSticky = 3;
template <int NT>
__device__ __forceinline__ void decide_body(const Dev &d, double *sh) {
    const int W = d.ctrl->spec_w;  // trial slots this step evaluated (uniform)
    double tch[kMaxSpec], scl[kMaxSpec];
#pragma unroll
    for (int s = 0; s < kMaxSpec; ++s) {
        tch[s] = scl[s] = 0.0;
        if (s >= W) continue;
        const double *plm = d.part_lm + (size_t)s * sl_lms(d), *plms = d.part_lms + (size_t)s * sl_lms(d);
        const double *pps = d.part_ps + (size_t)s * d.n_ps;
        double a = 0.0, b = 0.0;
        if (!d.sharded) {  // 8 loads of each array in flight per thread; summed in index order
            constexpr int U = 8;
            for (int i0 = threadIdx.x; i0 < d.n_lms_blocks; i0 += NT * U) {
                double va[U], vb[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * NT;
                    const bool ok = i < d.n_lms_blocks;
                    va[u] = ok ? ld_sc1(plm + i) : 0.0;
                    vb[u] = ok ? ld_sc1(plms + i) : 0.0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    a += va[u];
                    b += vb[u];
                }
            }
        }
        for (int i = threadIdx.x; i < d.n_ps; i += NT) b += pps[i];  // poses: replicated
        tch[s] = block_sum<NT>(a, sh);
        scl[s] = block_sum<NT>(b, sh);
    }
    if (d.sharded) {  // landmark terms summed over ranks (one slot)
        tch[0] = d.red_dec[0];
        scl[0] += d.red_dec[1];
    }
    if (threadIdx.x != 0) return;
    Ctrl *c = d.ctrl;
    c->steps += 1;
    if (c->hlm) {  // src/mapHandler.cpp:1867-1895 (first step), :2121-2156 — one slot
        const double lam0 = c->lambda;
        const bool first = c->iter == 0;
        int result = 0;
        c->hlm_solves += 1;
        // sharded: the landmark pivots are checked on the rank that owns the landmark, so the
        // decision uses the failures summed over the ranks (k_decide_pack), the same on every rank
        const bool ok = d.sharded ? d.red_dec[2] == 0.0
                                  : __hip_atomic_load(&c->solve_ok[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        const double dx2 = ok ? scl[0] : 0.0;  // a failed solve leaves DX = 0 (|DX| < minchg stops)
        c->dx2 = dx2;
        bool apply;
        if (first) {
            apply = true;
        } else if (c->currentChi > c->err_prev) {
            c->lambda /= c->hlm_k;
            apply = false;
            result = 1;
        } else {
            c->lambda *= c->hlm_k;
            apply = true;
        }
        if (ok) c->last_ok = (c->last_ok + 1) % d.nbx;
        apply = apply && ok;  // (an LDLᵀ breakdown leaves X unchanged)
        if (apply) {
            c->cur = (c->cur + 1) % d.nbs;
            c->hlm_acc += 1;
        }
        if (c->ntrace < kTraceCap)
            d.trace[c->ntrace++] = plba_iter_trace{c->stage, c->iter, 1, result, c->currentChi, c->currentChi, lam0,
                                                   c->lambda};
        c->iters_done[c->stage] += 1;
        c->iter += 1;
        const bool small = !first && sqrt(dx2) < c->hlm_minchg;
        c->err_prev = c->currentChi;
        if (small || c->iter >= c->max_iters[c->stage]) {
            c->chi2_final[c->stage] = c->currentChi;
            c->all_done = 1;
        } else {
            c->need_iter = 1;
        }
        c->spec_w = 1;
        return;
    }
    const int cur0 = c->cur, lo0 = c->last_ok, ch0 = c->chi_src;
    bool any_ok = false, hold = false, trials_go_on = false, done = false;
    c->need_iter = 0;  // (iter_init_ctrl's reset when k_iter_reduce took the fast path)
#pragma unroll
    for (int s = 0; s < kMaxSpec; ++s) {
        if (done || s >= W) continue;
        const bool ok = c->solve_ok[s] != 0;
        if (!ok && any_ok) {  // evaluated with the wrong "last successful" x: evaluate again alone
            hold = true;
            done = true;
            continue;
        }
        c->chi_src = (ch0 + 1 + s) % d.nbx;  // the edges now hold this trial's χ² (stale if rejected)
        if (ok) {
            c->last_ok = (lo0 + 1 + s) % d.nbx;
            any_ok = true;
        }
        double tempChi = tch[s];
        if (!ok) tempChi = 1.7976931348623157e308;
        const double scale = scl[s] + 1e-3;
        const double rho = (c->currentChi - tempChi) / scale;
        c->tempChi = tempChi;
        c->scale = scale;
        c->rho = rho;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            const double sf = fmax(1. / 3., alpha);
            c->lambda *= sf;
            c->ni = 2;
            c->currentChi = tempChi;
            c->accept = 1;
            c->qmax += 1;
            c->cur = (cur0 + 1 + s) % d.nbs;  // the trial becomes the current estimate
        } else {
            c->lambda *= c->ni;
            c->ni *= 2;
            c->accept = 0;
            c->spec_sticky = 1;
            if (!isfinite(c->lambda)) c->broke = 1;
            else c->qmax += 1;
        }
        const bool again = !c->broke && rho < 0 && c->qmax < c->max_trials;
        if (again) {  // another damped trial of this iteration: the next slot, or the next step
            trials_go_on = true;
            continue;
        }
        trials_go_on = false;
        done = true;
        // end of OptimizationAlgorithmLevenberg::solve(iter)
        const int terminate = (c->qmax == c->max_trials || rho == 0 || !isfinite(c->lambda)) ? 1 : 0;
        if (c->ntrace < kTraceCap)
            d.trace[c->ntrace++] = plba_iter_trace{c->stage, c->iter, c->qmax, terminate, c->chi2_start, c->currentChi,
                                                   c->lambda_start, c->lambda};
        c->iters_done[c->stage] += 1;
        c->iter += 1;
        if (terminate || c->iter >= c->max_iters[c->stage]) {  // optimize() returns
            c->chi2_final[c->stage] = c->currentChi;
            c->spec_sticky = 0;
            if (c->stage + 1 < c->n_stages) c->switch_pending = 1;
            else c->all_done = 1;
        } else {
            // the next iteration's init (iter_init_ctrl with iter > 0), done here so that
            // k_iter_reduce can skip its global reduction (iter_init_fast)
            c->need_iter = 1;
            c->chi2_start = c->currentChi;
            c->lambda_start = c->lambda;
            c->qmax = 0;
            c->accept = 0;
            c->rho = 0.0;
            c->broke = 0;
        }
    }
    // the next step's trial slots (Dev::spec_policy)
    int w = 1;
    if (d.spec_max > 1 && !hold) {
        const int pol = d.spec_policy;
        if (pol == kSpecAlways) w = d.spec_max;
        else if (pol == kSpecAfterReject) w = trials_go_on ? d.spec_max : 1;
        else if (pol == kSpecSticky) w = c->spec_sticky ? d.spec_max : 1;
    }
    c->spec_w = w;
}
__global__ __launch_bounds__(kBlock) void k_decide(Dev d) {
    TRIAL_GUARD
    __shared__ double sh[kBlock / 64];
    decide_body<kBlock>(d, sh);
}

#ifdef PLBA_LM_WPE
__global__ __launch_bounds__(kLmsNT, PLBA_LM_WPE) void k_lm_solve(Dev d0) {
#else
__global__ __launch_bounds__(kLmsNT) void k_lm_solve(Dev d0) {
#endif
    // Not TRIAL_SLOT: the folded decision (last arriver) rewrites Ctrl::spec_w inside this launch,
    // so a workgroup dispatched after it would read the NEXT step's width. Every workgroup of the
    // grid (gridDim.y = spec_max) therefore arrives, idle slots included, and all of them read
    // spec_w before arriving: the arrival total does not depend on spec_w and no workgroup can
    // observe the decision's writes.
    TRIAL_GUARD_OF(d0)
    __shared__ double sh[kLmsNT / 64];
    const int nslots = d0.ctrl->spec_w;
    if ((int)blockIdx.y >= nslots) {
        if (d0.fold && arrive_last(d0.cnt, (int32_t)(gridDim.x * gridDim.y))) decide_body<kLmsNT>(d0, sh);
        return;
    }
    const Dev d = slot_view(d0, (int)blockIdx.y);
#ifdef PLBA_LMS_STAMPS  // diagnostic build only: per-workgroup phase times (d.stamps row 15)
#define LMS_T(v) const unsigned long long v = __builtin_readcyclecounter()
#else
#define LMS_T(v)
#endif
    LMS_T(lt0);
    const int gt = blockIdx.x * kLmsNT + threadIdx.x;
    const int l = gt / kLmLanes, q = gt % kLmLanes;   // a quad never straddles a wave
    const bool live = l < d.n_lm;
    const int lc = live ? l : 0;
    const Ctrl *cg = d.ctrl;
    const bool solve = *d.solve_okp != 0;
    const bool robust = cg->robust != 0;
    const double lam = d.lam;
    const bool hlm = cg->hlm != 0;
    // ---- round 1: landmark record + this lane's edge slots
    const bool act = live && d.lm_active[lc] != 0;
    const int off0 = d.lm_off[lc], off1 = d.lm_off[lc + 1];
    double Xc[4], bl[4], H[10];
#pragma unroll
    for (int k = 0; k < 4; ++k) Xc[k] = d.Xc[(size_t)lc * 4 + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) bl[k] = d.bl[(size_t)lc * 4 + k];
#pragma unroll
    for (int k = 0; k < 10; ++k) H[k] = d.Hll[(size_t)lc * 10 + k];
    LmEdge sl[kLmSlots];
    bool sv[kLmSlots];
#pragma unroll
    for (int j = 0; j < kLmSlots; ++j) {
        const int e = off0 + q + kLmLanes * j;
        sv[j] = act && e < off1;
        lm_load_edge(d, sv[j] ? e : 0, sl[j]);
    }
    // ---- round 2: x_p of each slot's free pose, the slot's trial pose
    const double *Tt0 = d.Tt;
    double xs[kLmSlots][6], Ts[kLmSlots][12];
#pragma unroll
    for (int j = 0; j < kLmSlots; ++j) {
        const int h = max(sl[j].h, 0);
#pragma unroll
        for (int k = 0; k < 6; ++k) xs[j][k] = d.xp[6 * h + k];
#pragma unroll
        for (int k = 0; k < 12; ++k) Ts[j][k] = Tt0[(size_t)sl[j].kf * 12 + k];
    }
    double chi = 0.0, sc = 0.0;
    // r = b_l − Σ_e Hpl_eᵀ x_p,  Hpl_eᵀ x_p = B_eᵀ (A_e x_p)  (edges of a fixed pose: 0)
    double u[4] = {0, 0, 0, 0}, u45[2] = {0, 0};
    const bool gba_ln = cg->hlm == 2 && live && !is_point_lm(d, l);  // uniform across the quad
    if (act && solve && !(d.diag & 4)) {
        if (gba_ln) {
#pragma unroll
            for (int j = 0; j < kLmSlots; ++j)
                if (sv[j] && sl[j].h >= 0) lm_hpl_x<true>(sl[j], xs[j], u, u45);
        } else {
#pragma unroll
            for (int j = 0; j < kLmSlots; ++j)
                if (sv[j] && sl[j].h >= 0) lm_hpl_x(sl[j], xs[j], u, u45);
        }
        for (int e = off0 + q + kLmLanes * kLmSlots; e < off1; e += kLmLanes) {  // long tracks
            LmEdge s;
            lm_load_edge(d, e, s);
            if (s.h < 0) continue;
            double x[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) x[k] = d.xp[6 * s.h + k];
            if (gba_ln) lm_hpl_x<true>(s, x, u, u45);
            else lm_hpl_x(s, x, u, u45);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = quad_sum(u[i]);  // all lanes: DPP reads the whole quad
    LMS_T(lt1);
    if (cg->hlm == 2) {
        u45[0] = quad_sum(u45[0]);
        u45[1] = quad_sum(u45[1]);
    }
    if (live && gba_ln) {
        // GBA line (src/mapHandler.cpp:3673-3691): x = (Hl6 + λ·diag)⁻¹ (b_l − Σ_e b_e a_e·x_p),
        // X += DX on the 6 endpoint coordinates, ‖DX‖² partial; lane q == 0 writes
        const int li = l - d.n_pt, j = d.ln_gidx[li];
        const double *XLc = d.XLc + (size_t)j * 6;
        double *XLt = d.XLt + (size_t)j * 6;
        double *Xt = d.Xt + (size_t)l * 4;
        if (act && solve) {
            double H[21], L6[21], y[6], x[6];
#pragma unroll
            for (int k = 0; k < 21; ++k) { H[k] = d.Hl6[(size_t)li * 21 + k]; L6[k] = 0.0; }
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) {
                double sj = H[pk(jj, jj)] + lam * H[pk(jj, jj)];
#pragma unroll
                for (int p = 0; p < jj; ++p) sj -= L6[pk(jj, p)] * L6[pk(jj, p)];
                if (!(sj > 0.0))  // a non-positive pivot fails the solve (X unchanged, DX = 0)
                    __hip_atomic_store(d.solve_okp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const double djj = sqrt(sj);
                L6[pk(jj, jj)] = djj;
#pragma unroll
                for (int i = jj + 1; i < 6; ++i) {
                    double t = H[pk(i, jj)];
#pragma unroll
                    for (int p = 0; p < jj; ++p) t -= L6[pk(i, p)] * L6[pk(jj, p)];
                    L6[pk(i, jj)] = t / djj;
                }
            }
            const double uu[6] = {u[0], u[1], u[2], u[3], u45[0], u45[1]};
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double t = d.bl6[(size_t)li * 6 + i] - uu[i];
#pragma unroll
                for (int p = 0; p < i; ++p) t -= L6[pk(i, p)] * y[p];
                y[i] = t / L6[pk(i, i)];
            }
#pragma unroll
            for (int i = 5; i >= 0; --i) {
                double t = y[i];
#pragma unroll
                for (int p = i + 1; p < 6; ++p) t -= L6[pk(p, i)] * x[p];
                x[i] = t / L6[pk(i, i)];
            }
            if (q == 0) {
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    sc += x[i] * x[i];
                    XLt[i] = XLc[i] + x[i];
                }
            }
        } else if (q == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) XLt[i] = XLc[i];
        }
        if (q == 0)
#pragma unroll
            for (int i = 0; i < 4; ++i) Xt[i] = Xc[i];
    } else if (live) {
        double *Xt = d.Xt + (size_t)l * 4;
        if (act) {
            const bool pt = is_point_lm(d, l);
            const int DIM = pt ? 3 : 4;
            double x[4] = {0, 0, 0, 0};
            if (solve) {
                // (Hll + λI) = L Lᵀ (packed lower), x = L⁻ᵀ L⁻¹ (b_l − u); the hand-rolled LM in
                // the signed form of lm_chol, x = L⁻ᵀ S L⁻¹ (b_l − u)
                const bool sgn = cg->hlm == 1;
                double L[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, S[4] = {1.0, 1.0, 1.0, 1.0};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (j < DIM) {
                        double sj = H[pk(j, j)] + (hlm ? lam * H[pk(j, j)] : lam);
#pragma unroll
                        for (int p = 0; p < j; ++p) sj -= (L[pk(j, p)] * S[p]) * L[pk(j, p)];
                        const double sg = (sgn && sj < 0.0) ? -1.0 : 1.0;
                        S[j] = sg;
                        // a zero pivot fails the hand-rolled LM's solve (the oracle's unpivoted
                        // LDLᵀ; the step is then not applied, k_decide's hlm branch); GBA keeps
                        // the Cholesky form and fails on any non-positive pivot
                        if (hlm && (sgn ? sj == 0.0 : !(sj > 0.0)))
                            __hip_atomic_store(d.solve_okp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const double djj = 1.0 / sqrt(sg * sj);  // reciprocal diagonal (as lm_chol)
                        L[pk(j, j)] = djj;
#pragma unroll
                        for (int i = j + 1; i < 4; ++i) {
                            if (i < DIM) {
                                double t = H[pk(i, j)];
#pragma unroll
                                for (int p = 0; p < j; ++p) t -= L[pk(i, p)] * (L[pk(j, p)] * S[p]);
                                L[pk(i, j)] = (t * djj) * sg;
                            }
                        }
                    }
                }
                double y[4] = {0, 0, 0, 0};
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i < DIM) {
                        double t = bl[i] - u[i];
#pragma unroll
                        for (int p = 0; p < i; ++p) t -= L[pk(i, p)] * y[p];
                        y[i] = t * L[pk(i, i)];
                    }
#pragma unroll
                for (int i = 0; i < 4; ++i) y[i] *= S[i];
#pragma unroll
                for (int i = 3; i >= 0; --i)
                    if (i < DIM) {
                        double t = y[i];
#pragma unroll
                        for (int p = i + 1; p < 4; ++p)
                            if (p < DIM) t -= L[pk(p, i)] * x[p];
                        x[i] = t * L[pk(i, i)];
                    }
                if (q == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) d.xl[(size_t)l * 4 + i] = x[i];
                }
            } else {  // failed solve: the last successful solve's x (A13)
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = d.xl_prev[(size_t)l * 4 + i];
            }
            if (q == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i < DIM) sc += hlm ? x[i] * x[i] : x[i] * (lam * x[i] + bl[i]);
            }
            double X[4] = {0, 0, 0, 0}, Lp[6] = {0, 0, 0, 0, 0, 0};
            if (pt) {
                X[0] = Xc[0] + x[0]; X[1] = Xc[1] + x[1]; X[2] = Xc[2] + x[2]; X[3] = 0.0;
                if (q == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Xt[i] = X[i];
                }
            } else if (!(d.diag & 1)) {
                Xt[q] = orth_oplus_quad(Xc, x, q, Lp);
                if (q == 0) {
                    double *Lt = d.Lpt + (size_t)(l - d.n_pt) * 8;
#pragma unroll
                    for (int k = 0; k < 6; ++k) Lt[k] = Lp[k];
                }
            }
            // the landmark's edges at the trial state (computeActiveErrors of the trial); the
            // trial poses were written by the factorisation kernel
            const double delta = pt ? d.huber_pt : d.huber_ln;
            if (!(d.diag & 2) && !hlm)  // (the hand-rolled LM scores a step at the next linearisation)
#pragma unroll
            for (int j = 0; j < kLmSlots; ++j)
                if (sv[j] && sl[j].act) chi += lm_eval(d, sl[j], Ts[j], pt, X, Lp, robust, delta);
            for (int e = off0 + q + kLmLanes * kLmSlots; e < off1 && !hlm; e += kLmLanes) {  // long tracks
                if (!d.e_active[e]) continue;
                LmEdge s;
                lm_load_edge(d, e, s);
                chi += lm_eval(d, s, Tt0 + (size_t)s.kf * 12, pt, X, Lp, robust, delta);
            }
        } else {
            if (q == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) Xt[i] = Xc[i];
                if (!is_point_lm(d, l)) {  // an inactive line keeps its Plücker vector too
                    const double *Lc = d.Lpc + (size_t)(l - d.n_pt) * 8;
                    double *Lt = d.Lpt + (size_t)(l - d.n_pt) * 8;
#pragma unroll
                    for (int k = 0; k < 6; ++k) Lt[k] = Lc[k];
                }
            }
        }
    }
    LMS_T(lt2);
    const double s2 = block_sum<kLmsNT>(sc, sh);
    const double s1 = block_sum<kLmsNT>(chi, sh);
    if (threadIdx.x == 0) {
        st_sc1(d.part_lms + blockIdx.x, s2);
        st_sc1(d.part_lm + blockIdx.x, s1);
    }
    LMS_T(lt3);
    // the last workgroup to finish takes the trial decision (k_decide's work)
#ifdef PLBA_LMS_STAMPS
    const bool lms_last = d.fold && arrive_last(d.cnt, (int32_t)(gridDim.x * gridDim.y));
    LMS_T(lt4);
    if (lms_last) decide_body<kLmsNT>(d0, sh);
    LMS_T(lt5);
    if (threadIdx.x == 0 && d.stamps) {
        unsigned long long *st = d.stamps + 15 * 8;
        atomicAdd(st + 0, lt1 - lt0);
        atomicAdd(st + 1, lt2 - lt1);
        atomicAdd(st + 2, lt3 - lt2);
        atomicAdd(st + 3, lt4 - lt3);
        if (lms_last) atomicAdd(st + 4, lt5 - lt4);
        atomicAdd(st + 5, 1ull);
        atomicAdd(st + 6, lt4 - lt0);
        if (lms_last) atomicAdd(st + 7, 1ull);
    }
#else
    if (d.fold && arrive_last(d.cnt, (int32_t)(gridDim.x * gridDim.y))) decide_body<kLmsNT>(d0, sh);
#endif
}
// sharded: this rank's trial χ² and landmark scale terms into the all-reduced decision array
__global__ __launch_bounds__(kBlock) void k_decide_pack(Dev d) {
    TRIAL_GUARD
    __shared__ double sh[kBlock / 64];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < d.n_lms_blocks; i += kBlock) a += d.part_lm[i];
    for (int i = threadIdx.x; i < d.n_lms_blocks; i += kBlock) b += d.part_lms[i];
    const double ta = block_sum<kBlock>(a, sh);
    const double tb = block_sum<kBlock>(b, sh);
    if (threadIdx.x == 0) {
        d.red_dec_loc[0] = ta;
        d.red_dec_loc[1] = tb;
        // a failed solve on this rank (the hand-rolled LM's landmark pivots are rank-local): the
        // ranks sum the failures so that every rank takes the same decision (decide_body)
        d.red_dec_loc[2] = d.ctrl->solve_ok[0] != 0 ? 0.0 : 1.0;
    }
}

// changeOrthToPluker (g2o_types.h:367-387) of every line at the current state into Lpb[cur];
// launched once per schedule (estimates may have been reset or uploaded in between)
__global__ void k_line_pluker(Dev d) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= d.n_ln) return;
    const int cur = d.ctrl->cur;
    double L[6];
    orth_to_pluker(d.Xb[cur] + (size_t)(d.n_pt + l) * 4, L);
    double *o = d.Lpb[cur] + (size_t)l * 8;
#pragma unroll
    for (int k = 0; k < 6; ++k) o[k] = L[k];
}

// ---------------------------------------------------------------- outlier pass helpers
// computeError() at the current state for edges of `level`
__global__ void k_refresh(Dev d, int level) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= d.E || d.e_level[e] != level) return;
    const double *T = Tcur(d) + (size_t)d.e_kf[e] * 12;
    const double *X = Xcur(d) + (size_t)d.e_lm[e] * 4;
    const double *obs = d.e_obs + (size_t)e * 4;
    double err[2];
    if (e < d.Ep) {
        double z;
        point_error(T, X, obs, d.cam, err, z);
    } else {
        double L[6];
        orth_to_pluker(X, L);
        line_error(T, L, obs, d.cam, err);
    }
    const double info = d.e_info[e];
    chi2cur(d)[e] = err[0] * (info * err[0]) + err[1] * (info * err[1]);
}
// isDepthPositive() at the current state
__global__ void k_depth(Dev d, uint8_t *out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= d.Ep) return;
    double Pc[3];
    point_pc(Tcur(d) + (size_t)d.e_kf[e] * 12, Xcur(d) + (size_t)d.e_lm[e] * 4, Pc);
    out[e] = Pc[2] > 0.0 ? 1 : 0;
}

// unsharded download: poses, landmark states and per-edge outputs in the caller's order, one
// staging block (Tcw | pt_xyz | ln_orth | χ² by e_gpos, points then lines | bytes:
// isDepthPositive [Ep] | levels by e_gpos)
__global__ void k_out_scatter(Dev d, double *od, int want_depth, int cur, int chi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double *T = d.Tb[cur], *X = d.Xb[cur];  // the host's current state / χ² buffer index
    const size_t nk = d.n_kf, np = d.n_pt, nl = d.n_ln, E = d.E;
    if (i < d.n_kf)
#pragma unroll
        for (int k = 0; k < 12; ++k) od[(size_t)i * 12 + k] = T[(size_t)i * 12 + k];
    double *opt = od + nk * 12;
    if (i < d.n_lm) {
        const int gp = d.lm_gpos[i];
        const double *x = X + (size_t)i * 4;
        if (gp < d.n_pt) {
#pragma unroll
            for (int k = 0; k < 3; ++k) opt[(size_t)gp * 3 + k] = x[k];
        } else {
            double *o = opt + np * 3 + (size_t)(gp - d.n_pt) * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = x[k];
        }
    }
    if (i < d.E) {
        const int g = d.e_gpos[i];
        opt[np * 3 + nl * 4 + g] = d.chi2b[chi][i];
        uint8_t *ob = reinterpret_cast<uint8_t *>(opt + np * 3 + nl * 4 + E);
        ob[(size_t)d.Ep + g] = d.e_level[i];
        if (want_depth && i < d.Ep) {
            double Pc[3];
            point_pc(T + (size_t)d.e_kf[i] * 12, X + (size_t)d.e_lm[i] * 4, Pc);
            ob[g] = Pc[2] > 0.0 ? 1 : 0;
        }
    }
}

// sharded: scatter this rank's landmark states and per-edge outputs to their whole-window
// positions (the buffer is zeroed first and summed over ranks afterwards)
__global__ void k_gather(Dev d, const uint8_t *depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < d.n_lm)
#pragma unroll
        for (int k = 0; k < 4; ++k) d.gat[(size_t)d.lm_gpos[i] * 4 + k] = Xcur(d)[(size_t)i * 4 + k];
    if (i < d.E) {
        double *o = d.gat + (size_t)d.n_lm_g * 4;
        const int g = d.e_gpos[i];
        o[g] = chi2cur(d)[i];
        o[(size_t)d.E_g + g] = i < d.Ep ? (double)depth[i] : 0.0;
        o[2 * (size_t)d.E_g + g] = (double)d.e_level[i];
    }
}

}  // namespace plba
