/*
 * refcpu.h — TEST INFRASTRUCTURE ONLY. CPU oracle for the Plücker LBA path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may link or call
 * anything under oracle/ — as the checker / the timed CPU baseline, never as the product.
 *
 * PARITY UNPINNED against the reference: the reference ships no tests or golden vectors
 *  and cannot be built here (needs g2o, Eigen, OpenCV, SuiteSparse — none
 * present). The restatement is instead pinned by known-answer tests
 * (tests/test_oracle_kat.py): central-difference Jacobians, zero-noise fixed points, an
 * independent scipy least-squares minimiser on stage 2, and Plücker↔orth round trips.
 */
#ifndef PLBA_REFCPU_H
#define PLBA_REFCPU_H

#include "../include/plba.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct refcpu_opts {
    int32_t corrected_line_jacobian; /* 0 = bug-compatible g2o_types.h:429-430          */
    int32_t verbose;
    int32_t max_trials;              /* 10 */
    double  tau;                     /* 1e-5 */
    int32_t stage_iters[2];          /* 5, 10 */
} refcpu_opts;

void refcpu_default_opts(refcpu_opts *o);

/* Full two-stage schedule of src/mapHandler.cpp:6119-6160 on a window. */
int refcpu_lba_plucker(const plba_graph *g, const refcpu_opts *o, plba_result *res,
                       plba_iter_trace *trace, int32_t trace_cap, int32_t *n_trace);

/* Single-edge kernels for known-answer tests.
 * Tcw: row-major 3x4. err out [2]/[4]; Ji: point 2x3 / line 4x4 (row-major); Jj: 2x6 / 4x6. */
void refcpu_point_edge(const double *Tcw, const double *xyz, const double *obs, double fx, double fy,
                       double cx, double cy, double *err, double *Ji, double *Jj);
void refcpu_line_edge(const double *Tcw, const double *orth, const double *obs, double fx, double fy,
                      double cx, double cy, int corrected, double *err, double *Ji, double *Jj);
void refcpu_pose_oplus(double *Tcw, const double *delta6);
void refcpu_line_oplus(double *orth, const double *delta4);
void refcpu_orth_to_pluker(const double *orth, double *plk);
void refcpu_pluker_to_orth(const double *plk, double *orth);

#ifdef __cplusplus
}
#endif
#endif
