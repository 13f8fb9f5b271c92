// plba_build.hpp — device-side window build: the structure plba_upload
// needs — landmark order, landmark-major edge CSR, free-pose edge lists, the reduced-camera
// envelope and the Schur triples grouped by block — built from the caller's raw graph arrays by
// sort / scan / scatter kernels on the solver stream (csrc/plba_build.hip, rocPRIM radix sorts),
// instead of O(E) and O(Σ track²) host loops.
//
// The outputs are bit-for-bit the arrays the host build (plba.hip do_upload) produces: the same
// orders (stable sorts by the same keys), so the solve is unchanged.
//
// Reference: MapHandler::localBundleAdjustmentForPlukerWithG2O graph build
// (src/mapHandler.cpp:5868-6117) + formLocalMap (:1073-1137) hand the solver a fresh window per
// call; consecutive windows share most of their structure, but every call rebuilds it here too,
// just on the device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/plba.h"

namespace plba {

// grow-only device memory owned by the context, carved per build
struct BuildMem {
    char *base = nullptr;
    size_t cap = 0;
    void release(hipStream_t s);
    int reserve(size_t bytes, hipStream_t s);
};

struct WindowBuild {
    // ---- inputs (host)
    const plba_graph *g = nullptr;
    int nranks = 1, rank = 0;
    int nf = 0;                       // free poses (kf_hidx >= 0)
    const int32_t *kf_hidx = nullptr; // [n_kf] Hessian index of each free pose, -1 fixed
    const int32_t *kpos = nullptr;    // [n_kf] rank of each keyframe by vertex id
    hipStream_t stream = nullptr;
    // ---- outputs of stage 1 (device pointers into BuildMem A unless noted)
    int n_pt = 0, n_ln = 0, n_lm = 0, Ep = 0, El = 0, E = 0;
    int64_t n_free_edges = 0;
    int32_t *e_lm = nullptr, *e_kf = nullptr, *e_hidx = nullptr, *e_orig = nullptr, *e_gpos = nullptr;
    double *e_obs = nullptr, *e_info = nullptr, *X = nullptr;
    int32_t *lm_off = nullptr, *lm_gpos = nullptr, *pe_off = nullptr, *pe_list = nullptr;
    std::vector<int32_t> first_blk;   // host: [nf] envelope (lowest coupled free pose)
    // ---- stage 2 (after the host fixed the block layout): triples
    int64_t n_triples = 0;
    int32_t *trip = nullptr, *blk_off = nullptr;   // device ([T][2] in BuildMem B, [nblk+1] in A)
    std::vector<int32_t> h_blk_off;   // host copy of blk_off
    bool invalid = false;             // an edge references a missing vertex (stage 1)
    alignas(16) unsigned char s1[1024];  // stage-1 device layout, read by stage 2 (plba_build.hip)
};

// stage 1: everything up to the envelope. Returns PLBA_OK / error code; on an invalid edge sets
// wb.invalid and returns PLBA_E_INVALID (the caller reports which edge).
int build_stage1(BuildMem &A, WindowBuild &wb, char *err, size_t errlen);
// stage 2: Schur triples (e1 at pose i1 <= e2 at pose i2, same landmark) counting-sorted by block
// blk_base[i2] + (i1 - first_blk[i2]), landmark order inside a block; blk_off[nblk+1].
int build_stage2(BuildMem &A, BuildMem &B, WindowBuild &wb, const std::vector<int64_t> &blk_base, int nblk,
                 char *err, size_t errlen);

}  // namespace plba
