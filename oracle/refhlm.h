/*
 * refhlm.h — TEST INFRASTRUCTURE ONLY. CPU oracle for the hand-rolled Levenberg–Marquardt
 * local bundle adjustment of the Plücker map:
 *   int MapHandler::levMarquardtOptimizationLBAForPluker(...)   src/mapHandler.cpp:1618-2332
 * with the window lists of MapHandler::localBundleAdjustmentForPluker() (:1505-1615).
 *
 * Only tests/ and bench.py's cpu_baseline leg may link or call it — as the checker, never as
 * the product.
 *
 * PARITY UNPINNED against the reference: the reference ships no tests or fixtures and cannot
 * be built here (Eigen / OpenCV / g2o absent). The restatement is pinned by
 * known-answer tests instead (tests/test_hlm_oracle.py): central-difference checks of the
 * scalar-residual gradients, se(3) exp/log round trips, and the block (Schur) solve against a
 * literal dense N×N LDLᵀ of the reference's H on small windows.
 */
#ifndef PLBA_REFHLM_H
#define PLBA_REFHLM_H

#include "../include/plba.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct refhlm_opts {
    int32_t dense;    /* 1: assemble the reference's dense N×N H and LDLᵀ it (small windows only) */
    int32_t verbose;
} refhlm_opts;

/* The whole levMarquardtOptimizationLBAForPluker loop on a window (inputs as plba_hlm_lba). */
int refhlm_lba(const plba_graph *g, const plba_hlm_state *st, const plba_hlm_params *p, const refhlm_opts *o,
               plba_hlm_result *res, plba_iter_trace *trace, int32_t trace_cap, int32_t *n_trace);

/* Single-observation kernels for known-answer tests (Tcw = Tiw row-major 3x4):
 * r = ‖e‖, w = Cauchy weight, Jp[6] (pose), Jl[3|4] (landmark), as the reference forms them. */
void refhlm_point_obs(const double *Tcw, const double *xyz, const double *obs, double fx, double fy, double cx,
                      double cy, double homog_th, double *r, double *w, double *Jp, double *Jl);
void refhlm_line_obs(const double *Tcw, const double *pluker, const double *obs, double fx, double fy, double cx,
                     double cy, double homog_th, double *r, double *w, double *Jp, double *Jl);
/* src2/auxiliar.cpp:113-173 (T row-major 4x4, x = [t; ω]) */
void refhlm_expmap(const double *x, double *T);
void refhlm_logmap(const double *T, double *x);
void refhlm_inverse_se3(const double *T, double *Tinv);

#ifdef __cplusplus
}
#endif
#endif
