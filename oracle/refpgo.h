/*
 * refpgo.h — TEST INFRASTRUCTURE ONLY. CPU oracle for the loop-closure pose graph
 * (SURVEY.md §8f row 4):
 *   bool MapHandler::loopClosureOptimizationEssGraphG2O()  src/mapHandler.cpp:5070-5299
 *   bool MapHandler::loopClosureOptimizationCovGraphG2O()  src/mapHandler.cpp:5301-5531
 * i.e. the g2o calls they make (g2o is un-vendored and unpinned; restated from
 * its published source): VertexSE3 / EdgeSE3 (types_slam3d, isometry3d_mappings),
 * SparseOptimizer::initializeOptimization / computeInitialGuess (EstimatePropagator) /
 * computeActiveErrors, OptimizationAlgorithmLevenberg::solve with setUserLambdaInit, and a dense
 * Cholesky standing in for LinearSolverCholmod (same solution; fails on a non-positive pivot).
 *
 * Only tests/ may link or call it — as the checker, never as the product.
 *
 * PARITY UNPINNED against the reference: no tests or fixtures exist and g2o/Eigen/Cholmod are
 * absent. Pinned by known-answer tests (tests/test_pgo_oracle.py): Eigen's
 * matrix -> quaternion against scipy, MQT round trips, central-difference Jacobians, the
 * initial guess on graphs with a known answer, zero-noise loops that must converge to χ² ≈ 0.
 */
#ifndef PLBA_REFPGO_H
#define PLBA_REFPGO_H

#include "../include/plba.h"

#ifdef __cplusplus
extern "C" {
#endif

/* computeInitialGuess + computeActiveErrors + optimize(max_iters), as plba_pgo_optimize. */
int refpgo_optimize(const plba_pgo_graph *g, const plba_pgo_params *p, plba_pgo_result *r);
/* computeInitialGuess only: v_T_out[n_v][12] */
int refpgo_initial_guess(const plba_pgo_graph *g, double *v_T_out);

/* Single pieces for known-answer tests (Isometry3 = row-major 3x4). */
void refpgo_quat_from_R(const double *R9, double *q_xyzw);          /* Eigen Quaternion(Matrix3)  */
void refpgo_to_mqt(const double *T12, double *v6);                    /* internal::toVectorMQT      */
void refpgo_from_mqt(const double *v6, double *T12);                  /* internal::fromVectorMQT    */
void refpgo_edge_error(const double *Z12, const double *Xi12, const double *Xj12, double *e6);
void refpgo_edge_jacobians(const double *Z12, const double *Xi12, const double *Xj12, double *Ji36,
                           double *Jj36);                             /* row-major 6x6 de/dδ        */
void refpgo_oplus(const double *X12, const double *d6, double *out12); /* VertexSE3::oplusImpl      */

#ifdef __cplusplus
}
#endif
#endif
