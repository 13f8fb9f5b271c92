/*
 * plba.h — C ABI of the MI355X local-bundle-adjustment backend.
 *
 * Drop-in boundary for the g2o solve inside
 *   void PLSLAM::MapHandler::localBundleAdjustmentForPlukerWithG2O()
 *   (reference: include/mapHandler.h:134, src/mapHandler.cpp:5851-6323)
 *
 * The reference builds a g2o::SparseOptimizer on the stack (src/mapHandler.cpp:5923-5929),
 * adds VertexLMPose / VertexLMPointXYZ / VertexLMLineOrth vertices and EdgePosePoint /
 * EdgePoseLine edges (g2o_types/g2o_types.h:28-502), then runs
 *   initializeOptimization(); optimize(5);  ... classify ...;
 *   initializeOptimization(0); optimize(10);                     (src/mapHandler.cpp:6119-6152)
 * Each entry point below replaces one of those g2o calls:
 *
 *   plba_create / plba_destroy        ~ g2o::SparseOptimizer ctor + setAlgorithm(Levenberg(BlockSolverX(
 *                                       LinearSolverEigen)))  / dtor          (src/mapHandler.cpp:5923-5929)
 *   plba_upload                       ~ addVertex / addEdge / setRobustKernel / SetParams loop
 *                                                                              (src/mapHandler.cpp:5931-6117)
 *   plba_set_edge_levels              ~ Edge::setLevel                        (src/mapHandler.cpp:6130,6143)
 *   plba_set_robust                   ~ Edge::setRobustKernel(0 | Huber)      (src/mapHandler.cpp:6133,6146)
 *   plba_initialize_optimization      ~ SparseOptimizer::initializeOptimization(int level)
 *                                                                              (src/mapHandler.cpp:6121,6151)
 *   plba_optimize                     ~ SparseOptimizer::optimize(int iterations)
 *                                                                              (src/mapHandler.cpp:6122,6152)
 *   plba_refresh_edge_errors          ~ Edge::computeError() on level-1 edges (src/mapHandler.cpp:6158-6160,6226-6228)
 *   plba_get_edge_chi2                ~ Edge::chi2() / EdgePosePoint::isDepthPositive()
 *                                                                              (src/mapHandler.cpp:6129,6142,6161,6230)
 *   plba_download                     ~ Vertex::estimate()                    (src/mapHandler.cpp:6297-6319)
 *   plba_lba_plucker                  the whole two-stage schedule of src/mapHandler.cpp:6119-6160 on device,
 *                                     with no host round trip between the stages.
 *
 * Conventions: all arrays are host pointers owned by the caller and copied by the call;
 * FP64 everywhere; indices are int32; every function returns PLBA_OK (0) or a negative
 * PLBA_E* status and never throws or exits (the reference exit(0)s on index errors,
 * src/mapHandler.cpp:5894,5910,5998,6062). A context is single-threaded (one LBA at a time,
 * as handlerThread guarantees, src/mapHandler.cpp:1186-1188).
 */
#ifndef PLBA_H
#define PLBA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLBA_OK              0
#define PLBA_E_INVALID     (-1)   /* bad argument / index out of range                 */
#define PLBA_E_DEVICE      (-2)   /* HIP runtime error                                 */
#define PLBA_E_STATE       (-3)   /* call out of order (e.g. optimize before upload)   */
#define PLBA_E_NOMEM       (-4)
#define PLBA_E_COMM        (-5)   /* RCCL error (sharded windows)                      */

/* One LBA window in g2o vertex/edge form (structure-of-arrays).
 * Vertex ids follow src/mapHandler.cpp:5941 (pose id = kf_idx), :5983 (point id =
 * idx+max_kf_id+1), :6047 (line id = idx+maxPointId+1). Ids order the Hessian exactly as
 * g2o's buildIndexMapping does (free poses by id, then landmarks by id). Edge arrays are in
 * g2o insertion order (all point edges, then all line edges). */
typedef struct plba_graph {
    int32_t n_kf, n_pt, n_ln, n_ept, n_eln;
    double fx, fy, cx, cy;            /* EdgePosePoint/EdgePoseLine::SetParams (g2o_types.h:217,313) */
    const double  *kf_Tcw;            /* [n_kf][12]  row-major 3x4 [R | t] of Tcw = T_kf_w^-1     */
    const uint8_t *kf_fixed;          /* [n_kf]      VertexLMPose::setFixed                        */
    const int32_t *kf_id;             /* [n_kf]      vertex id                                     */
    const double  *pt_xyz;            /* [n_pt][3]   VertexLMPointXYZ estimate                     */
    const int32_t *pt_id;             /* [n_pt]                                                    */
    const double  *ln_orth;           /* [n_ln][4]   VertexLMLineOrth estimate (θ1,θ2,θ3,φ)        */
    const int32_t *ln_id;             /* [n_ln]                                                    */
    const int32_t *ept_lm, *ept_kf;   /* [n_ept]     vertex 0 (point index) / vertex 1 (kf index)  */
    const double  *ept_obs;           /* [n_ept][2]  pixel measurement                             */
    const double  *ept_info;          /* [n_ept]     Ω = info·I2 (info already float-rounded)      */
    const int32_t *eln_lm, *eln_kf;   /* [n_eln]                                                   */
    const double  *eln_obs;           /* [n_eln][4]  (spl.x, spl.y, epl.x, epl.y)                  */
    const double  *eln_info;          /* [n_eln]     Ω = info·I4                                   */
    double huber_pt, huber_ln;        /* RobustKernelHuber::setDelta ((float)sqrt(5.991))          */
} plba_graph;

/* Per outer-LM-iteration trace (OptimizationAlgorithmLevenberg::solve). */
typedef struct plba_iter_trace {
    int32_t stage;        /* 0 or 1 (optimize(5) / optimize(10))                    */
    int32_t iter;         /* iteration index inside optimize()                      */
    int32_t trials;       /* damped trials run (1..10)                              */
    int32_t result;       /* 0 OK, 1 Terminate, 2 Fail                              */
    double  chi2_start;   /* activeRobustChi2 at linearisation                     */
    double  chi2_end;     /* currentChi after the trial loop                        */
    double  lambda_start; /* λ used by the first trial                              */
    double  lambda_end;   /* λ after the trial loop                                 */
} plba_iter_trace;

/* Output of plba_lba_plucker (all optional; NULL = not wanted). */
typedef struct plba_result {
    double  *kf_Tcw;        /* [n_kf][12] final Tcw (fixed poses unchanged)                   */
    double  *pt_xyz;        /* [n_pt][3]                                                       */
    double  *ln_orth;       /* [n_ln][4]                                                       */
    double  *ept_chi2;      /* [n_ept] chi2 as the post-solve outlier pass sees it (A13 rules) */
    uint8_t *ept_depth_ok;  /* [n_ept] isDepthPositive() at the final state                    */
    uint8_t *ept_level;     /* [n_ept] level after the stage-1 classification                  */
    double  *eln_chi2;      /* [n_eln]                                                         */
    uint8_t *eln_level;     /* [n_eln]                                                         */
    int32_t  iters[2];      /* outer iterations executed by optimize(5) and optimize(10)      */
    double   chi2[2];       /* final activeRobustChi2 of each stage                            */
    double   solve_ms;      /* wall time inside the two optimize() calls                       */
} plba_result;

typedef struct plba_opts {
    int32_t device;                  /* HIP device ordinal                                         */
    int32_t corrected_line_jacobian; /* 0 = reproduce g2o_types.h:429-430 (orth used as Plücker)   */
    int32_t verbose;                 /* print a per-iteration log to stderr                        */
    int32_t max_trials;              /* g2o maxTrialsAfterFailure (10)                             */
    double  tau;                     /* g2o Levenberg τ (1e-5)                                     */
} plba_opts;

typedef struct plba_ctx plba_ctx;

void        plba_default_opts(plba_opts *o);
int         plba_create(plba_ctx **ctx, const plba_opts *opts);
int         plba_destroy(plba_ctx *ctx);
const char *plba_last_error(const plba_ctx *ctx);

int plba_upload(plba_ctx *ctx, const plba_graph *g);
int plba_reset_estimates(plba_ctx *ctx);                       /* back to the uploaded estimates */
int plba_set_edge_levels(plba_ctx *ctx, const uint8_t *ept_level, const uint8_t *eln_level);
int plba_set_robust(plba_ctx *ctx, int32_t robust);            /* 1 = Huber on every edge, 0 = none */
int plba_initialize_optimization(plba_ctx *ctx, int32_t level);
int plba_optimize(plba_ctx *ctx, int32_t iterations, int32_t *iters_done, double *final_chi2);
int plba_refresh_edge_errors(plba_ctx *ctx, int32_t level);    /* computeError() on edges of `level` */
int plba_get_edge_chi2(plba_ctx *ctx, double *ept_chi2, uint8_t *ept_depth_ok, double *eln_chi2);
int plba_download(plba_ctx *ctx, double *kf_Tcw, double *pt_xyz, double *ln_orth);
int plba_lba_plucker(plba_ctx *ctx, plba_result *res);         /* full two-stage schedule          */
int plba_get_trace(plba_ctx *ctx, plba_iter_trace *out, int32_t cap, int32_t *n);
int plba_synchronize(plba_ctx *ctx);

/* Per-kernel timing of the last plba_lba_plucker call (HIP events on the solver stream).
 * names[i] points to a static string; ms[i] is the summed time of that kernel. */
int plba_enable_kernel_timing(plba_ctx *ctx, int32_t on);   /* HIP-event timing of each launch */
/* Structure of the uploaded window: out[0]=free poses, [1]=envelope bandwidth (pose blocks),
 * [2]=reduced-camera blocks, [3]=Schur triples, [4]=edges, [5]=landmarks, [6]=banded (1/0),
 * [7]=assembly chunks, [8]=edges with a free pose, [9]=point edges, [10]=step hipGraph in use,
 * [11]=sharded code path, [12]=two-sided (twisted) band factorisation, [13]=column-lane
 * band factorisation (bandwidth <= 9), [14]=super-rows of the block-cyclic-reduction
 * factorisation (0 = not used), [15]=dense RCS on the multi-workgroup MFMA path,
 * [16]=times a block-cyclic-reduction hand-off timed out and the schedule was re-solved with
 * the column-lane factorisation (the context then keeps that factorisation), [17]=trial slots
 * a step evaluates at most (speculative damped trials, 1 = off), [18]=their policy
 * (0 off, 1 always, 2 after a rejection in the iteration, 3 after the first rejection of the
 * optimize() call), [19]=device steps the last schedule took, [20]=unused (always 0; it was the
 * four-segment column-lane factorisation, removed in round 5), [21]=window structure built on the
 * device (1) or on the host (0).
 * Counts are this rank's when the window is sharded. */
int plba_structure_stats(plba_ctx *ctx, int64_t *out, int32_t cap);
int plba_kernel_times(plba_ctx *ctx, const char **names, double *ms, int32_t *launches,
                      int32_t cap, int32_t *n);

/* ---- Hand-rolled Levenberg–Marquardt local BA:
 *   int MapHandler::levMarquardtOptimizationLBAForPluker(X_aux, kf_list, pt_list, ls_list,
 *                                                         pt_obs_list, ls_obs_list)
 *   (src/mapHandler.cpp:1618-2332; window lists built by localBundleAdjustmentForPluker, :1505-1615)
 * One scalar residual r = ‖e‖ per observation with a Cauchy weight w = 1/(1+r²)
 * (src2/auxiliar.cpp:556-559), H += w·JᵀJ, g += w·J·r, Marquardt damping H(i,i) += λ·H(i,i),
 * DX = H⁻¹g, poses X_i ← log(exp(X_i)·exp(DX_i)⁻¹), points X += DX, lines updateOrthCoord.
 * The window is the plba_graph of plba_upload, read as the reference's lists:
 *   kf_fixed[k] == 0  <=>  KF k is in kf_list (local && kf_idx != 0, :1516)
 *   kf_Tcw  = inverse_se3(T_kf_w), the MAP pose (:1657-1659): fixed KFs and every line
 *             observation use it on every iteration (:2010-2012), free KFs on the first one
 *   pt_xyz  = point3D (:1536), ln_orth = orthNDw = changePlukerToOrth(NDw) (:1577)
 *   edges   = pt_obs_list / ls_obs_list (obs_list[i] / NDw_obs_list[i]); the info, Huber and
 *             level fields are not used by this solver. */
typedef struct plba_hlm_state {
    const double *kf_x;        /* [n_kf][6] KeyFrame::x_kf_w = X_aux pose blocks [t; ω] (:1518)   */
    const double *ln_pluker;   /* [n_ln][6] MapLine::NDw of the map (first linearisation, :1744)  */
    const double *ln_line3d;   /* GBA only: [n_ln][6] MapLine::line3D endpoints [P; Q] (:3089)    */
} plba_hlm_state;

typedef struct plba_hlm_params {
    double  lambda0;           /* SlamConfig::lambdaLbaLM()  1e-5 (src/slamConfig.cpp:65)         */
    double  lambda_k;          /* SlamConfig::lambdaLbaK()   10   (src/slamConfig.cpp:66)         */
    double  homog_th;          /* Config::homogTh()          1e-7 (src2/config.cpp:80)            */
    double  min_error;         /* Config::minError()         1e-7 (src2/config.cpp:84)            */
    double  min_error_change;  /* Config::minErrorChange()   1e-7 (src2/config.cpp:85)            */
    int32_t max_iters;         /* SlamConfig::maxItersLba()  15   (src/slamConfig.cpp:67)         */
    int32_t err_per_obs;       /* 0 = the reference: err /= (Npt_obs + Nls_obs), both counters stay
                                  0 (:1642,1731,1849) so err becomes +inf and every step after the
                                  first is accepted; 1 = divide by the observation count instead */
    int32_t variant;           /* PLBA_HLM_LBA_PLUCKER or PLBA_HLM_GBA                            */
    int32_t pad;
} plba_hlm_params;

/* plba_hlm_params.variant
 * PLBA_HLM_GBA = MapHandler::levMarquardtOptimizationGBA (src/mapHandler.cpp:3128-3726, window of
 * globalBundleAdjustment :3022-3126): every KF but kf_idx 0 free; lines are 6-dim landmarks, the
 * endpoints line3D = [P; Q] (state_ln_line3d), observed as image line equations (a, b, c) in
 * eln_obs[.][0..2]; residual e = (l·π(P), l·π(Q)); from the second linearisation on both
 * endpoints are read from X at the aliased offset 6Nkf+3Npt+3·j (:3547-3548); Hmax is an int
 * (:3386, truncation); the stop tests use numeric_limits<double>::epsilon() (pass it as
 * min_error / min_error_change). */
#define PLBA_HLM_LBA_PLUCKER 0
#define PLBA_HLM_GBA         1

typedef struct plba_hlm_result {
    double  *kf_x;             /* [n_kf][6] X pose blocks at exit (KFs not in kf_list: input x)   */
    double  *kf_Tcw;           /* [n_kf][12] inverse_se3(expmap_se3(x)) of each free KF, map pose
                                  of the others                                                   */
    double  *pt_xyz;           /* [n_pt][3]                                                       */
    double  *ln_orth;          /* [n_ln][4]                                                       */
    int32_t  linearizations;   /* H/g builds executed (1 .. max_iters)                            */
    int32_t  solves;           /* SimplicialLDLT solves executed                                  */
    int32_t  accepted;         /* solves whose DX was applied                                     */
    int32_t  pad;
    double   err;              /* last err (after the division)                                   */
    double   lambda;           /* λ at exit                                                       */
    double   dx_norm;          /* ‖DX‖ of the last solve                                          */
    double   solve_ms;         /* wall time of the loop                                           */
    double  *ln_line3d;        /* GBA: [n_ln][6] line3D at exit                                   */
} plba_hlm_result;

void plba_hlm_default_params(plba_hlm_params *p);
/* The whole loop on the uploaded window, on the device (one captured step per iteration).
 * Per-iteration records (plba_get_trace): stage 0, iter, trials 1, result 0 = DX applied,
 * 1 = DX rejected (err > err_prev), 3 = stopped before the solve; chi2_start = chi2_end = err,
 * lambda_start / lambda_end around the iteration.
 * Deliberate divergence (INTEGRATION.md B'): a free keyframe with no active observation gets 1.0
 * on its diagonal (DX = 0) and a zero pivot elsewhere keeps X unchanged, where the reference's
 * Eigen SimplicialLDLT would solve on a partial factor and produce inf / NaN. */
int plba_hlm_lba(plba_ctx *ctx, const plba_hlm_state *st, const plba_hlm_params *p, plba_hlm_result *res);

/* ---- Loop-closure pose graph:
 *   bool MapHandler::loopClosureOptimizationEssGraphG2O()  (src/mapHandler.cpp:5070-5299)
 *   bool MapHandler::loopClosureOptimizationCovGraphG2O()  (src/mapHandler.cpp:5301-5531)
 * g2o::SparseOptimizer with g2o::VertexSE3 vertices and g2o::EdgeSE3 edges,
 * OptimizationAlgorithmLevenberg over BlockSolver_6_3 + LinearSolverCholmod,
 * setUserLambdaInit(1e-10) (:5085), then initializeOptimization(); computeInitialGuess();
 * computeActiveErrors(); optimize(maxItersPGO) (:5182-5185).
 *   VertexSE3::oplusImpl:  X <- X · fromVectorMQT(δ),  δ = [Δt; qx qy qz]
 *   EdgeSE3::computeError: e = toVectorMQT(Z⁻¹ · X_from⁻¹ · X_to), χ² = eᵀΩe
 * Poses are Isometry3 (row-major 3x4 [R | t]). The reference replaces Cholmod's supernodal
 * Cholesky here by a dense LDLᵀ on the device: same solution; the solve fails when a pivot is
 * not positive (CHOLMOD_NOT_POSDEF), which g2o treats as a rejected trial. */
typedef struct plba_pgo_graph {
    int32_t        n_v;     /* vertices                                                         */
    int32_t        n_e;     /* edges                                                            */
    const int32_t *v_id;    /* [n_v] g2o vertex ids (the reference: KF indices), unique         */
    const double  *v_T;     /* [n_v][12] VertexSE3 estimates                                    */
    const uint8_t *v_fixed; /* [n_v] setFixed                                                   */
    const int32_t *e_v;     /* [n_e][2] vertex positions (0..n_v-1) of vertex(0), vertex(1)     */
    const double  *e_Z;     /* [n_e][12] setMeasurement                                         */
    const double  *e_info;  /* [n_e][36] information, row-major; NULL = identity (the reference) */
} plba_pgo_graph;

typedef struct plba_pgo_params {
    double  user_lambda_init; /* setUserLambdaInit: 1e-10 (:5085); <= 0: τ·max|H_ii|, τ = 1e-5   */
    int32_t max_iters;        /* optimize(SlamConfig::maxItersPGO()) — 100 (src/slamConfig.cpp:79) */
    int32_t initial_guess;    /* 1: computeInitialGuess() (the reference calls it)              */
    int32_t max_trials;       /* OptimizationAlgorithmLevenberg maxTrialsAfterFailure: 10        */
    int32_t pad;
} plba_pgo_params;

typedef struct plba_pgo_result {
    double          *v_T;        /* [n_v][12] final estimates (NULL = not wanted)                */
    plba_iter_trace *trace;      /* [trace_cap] per-iteration records (stage 0), may be NULL     */
    int32_t          trace_cap;
    int32_t          n_trace;
    int32_t          iterations; /* outer iterations run by optimize()                          */
    int32_t          trials;     /* damped trials run                                           */
    int32_t          solve_fails;/* trials whose factorisation met a non-positive pivot         */
    int32_t          n_free;     /* vertices in the Hessian (active, not fixed)                 */
    double           chi2_initial; /* activeChi2 after computeInitialGuess                      */
    double           chi2_final;
    double           lambda_final;
    double           solve_ms;   /* wall time of optimize()                                     */
} plba_pgo_result;

void plba_pgo_default_params(plba_pgo_params *p);
/* computeInitialGuess (host: g2o's EstimatePropagator, Dijkstra from the fixed vertices over the
 * active edges, unit edge cost) and optimize() on the device (per-edge linearisation, dense
 * assembly, multi-workgroup LDLᵀ with MFMA trailing updates, one host decision per trial). */
int plba_pgo_optimize(plba_ctx *ctx, const plba_pgo_graph *g, const plba_pgo_params *p, plba_pgo_result *res);

/* ---- Sharded windows: one context per GPU, one window split over nranks.
 * Landmarks (with all their edges) are partitioned by the keyframe range of their first
 * observation (kf_obs_list[0], the base KF of map_points_kf_idx); poses are replicated.
 * Per LM trial each rank assembles its partial reduced camera system and the ranks exchange it
 * with one all-gather of each rank's block-row runs, summed in rank order (PLBA_SHARD_XCHG=allreduce:
 * one all-reduce of the whole system), plus a 13·nf-double all-reduce per outer iteration and a
 * 3-double one per trial (trial χ², scale, failed solves); every rank then factorises the identical
 * system redundantly, so accept/reject
 * decisions agree bit for bit across ranks. plba_download / plba_get_edge_chi2 /
 * plba_lba_plucker return the FULL window on every rank (one final gather all-reduce).
 * Call exactly one plba_comm_init_* before plba_upload; every rank uploads the same full
 * graph and then makes the same sequence of calls. */

/* In-place sum over ranks of n doubles in host memory (caller's transport, e.g. gloo). */
typedef int (*plba_host_allreduce_fn)(void *user, double *buf, int64_t n);

/* Landmark -> rank assignment used by sharded uploads (pure host code, no device needed). */
int plba_shard_plan(const plba_graph *g, int32_t nranks, int32_t *pt_owner, int32_t *ln_owner);
/* RCCL transport over xGMI: rank 0 creates the id, the caller broadcasts its 128 bytes. */
int plba_comm_unique_id(uint8_t id[128]);
int plba_comm_init_rccl(plba_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
/* Host transport (tests / hosts without RCCL): device buffers are staged through pinned memory. */
int plba_comm_init_host(plba_ctx *ctx, int32_t nranks, int32_t rank, plba_host_allreduce_fn fn, void *user);
/* What the transport itself reports, so that a multi-GPU record proves N ranks on N distinct GPUs:
 * out[0] transport (0 none, 1 RCCL, 2 host), [1] ranks (RCCL: ncclCommCount), [2] this rank
 * (RCCL: ncclCommUserRank), [3] the communicator's device (RCCL: ncclCommCuDevice; else the
 * context's), [4] the HIP device ordinal the context runs on (hipGetDevice), [5] its PCI domain,
 * [6] PCI bus, [7] PCI device. Entries past cap are not written. */
int plba_comm_info(plba_ctx *ctx, int32_t *out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PLBA_H */
