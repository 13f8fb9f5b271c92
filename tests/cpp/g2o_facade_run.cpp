// TEST PROGRAM: the graph-build / two-stage solve / read-back sequence of
// PLSLAM::MapHandler::localBundleAdjustmentForPlukerWithG2O() (src/mapHandler.cpp:5923-6160),
// written against the g2o facade (include/plba_g2o.hpp) with the reference's class and method
// names, solved on the GPU through libplba.so. Eigen is not in this image, so Mat4/Vec/IsoInfo below
// stand in for Eigen::Matrix4d / Vector2d,3d,4d / Matrix2d::Identity()*s (same element access).
//
// usage: g2o_facade_run <graph.bin> <out.bin> [mutate]   (formats: tests/test_g2o_facade.py)
//   mutate: between the two optimize() calls, fix the first free keyframe, move the measurement of
//           point edge 0 and scale the information of point edge 1 (g2o applies such changes at the
//           next optimize(); the facade must re-marshal the window)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "plba_g2o.hpp"

struct Mat4 {
    double a[16] = {};
    double &operator()(int r, int c) { return a[r * 4 + c]; }
    double operator()(int r, int c) const { return a[r * 4 + c]; }
};
struct Vec {
    double a[4] = {};
    double &operator()(int i) { return a[i]; }
    double operator()(int i) const { return a[i]; }
};
// stand-ins for the map objects the read-back writes (KeyFrame::T_kf_w Matrix4d, MapPoint::point3D
// Vector3d, MapLine NDw from Vector4d orth): the same member calls as src/mapHandler.cpp:6296-6319
struct KeyFrame {
    int kf_idx;
    Mat4 T_kf_w;
};
struct MapPoint {
    int idx;
    Vec point3D;
};
struct MapLine {
    int idx;
    Vec orth_written;
};
struct IsoInfo {  // Eigen::Matrix<N,N>::Identity() * s
    double s;
    double operator()(int r, int c) const { return r == c ? s : 0.0; }
};

template <class T>
static bool rd(FILE *f, std::vector<T> &v, size_t n) {
    v.resize(n);
    return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s graph.bin out.bin\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<int> hdr;
    std::vector<double> cam, kfT, pts, lns, eobs, einfo, lobs, linfo;
    std::vector<int> kfid, kffix, ptid, lnid, elm, ekf, llm, lkf;
    bool ok = rd(f, hdr, 5);
    const int nk = hdr[0], np = hdr[1], nl = hdr[2], ne = hdr[3], nle = hdr[4];
    ok = ok && rd(f, cam, 6) && rd(f, kfT, (size_t)nk * 12) && rd(f, kfid, nk) && rd(f, kffix, nk) &&
         rd(f, pts, (size_t)np * 3) && rd(f, ptid, np) && rd(f, lns, (size_t)nl * 4) && rd(f, lnid, nl) &&
         rd(f, elm, ne) && rd(f, ekf, ne) && rd(f, eobs, (size_t)ne * 2) && rd(f, einfo, ne) && rd(f, llm, nle) &&
         rd(f, lkf, nle) && rd(f, lobs, (size_t)nle * 4) && rd(f, linfo, nle);
    fclose(f);
    if (!ok) {
        fprintf(stderr, "short graph file\n");
        return 2;
    }
    const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3];
    const float thHuberMono = (float)cam[4], thHuberLine = (float)cam[5];

    g2o::SparseOptimizer optimizer;
    auto linearSolver = g2o::make_unique<SlamLinearSolver>();
    auto blockSolver = g2o::make_unique<g2o::BlockSolverX>(std::move(linearSolver));
    g2o::OptimizationAlgorithm *algorithm = new g2o::OptimizationAlgorithmLevenberg(std::move(blockSolver));
    optimizer.setAlgorithm(algorithm);

    for (int k = 0; k < nk; ++k) {  // pose vertices: estimate Tcw, id = kf_idx
        VertexLMPose *vPose = new VertexLMPose();
        Mat4 T;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) T(r, c) = kfT[k * 12 + r * 4 + c];
        T(3, 3) = 1.0;
        vPose->setEstimate(T);
        vPose->setId(kfid[k]);
        vPose->setFixed(kffix[k] != 0);
        optimizer.addVertex(vPose);
    }
    for (int p = 0; p < np; ++p) {
        VertexLMPointXYZ *vPoint = new VertexLMPointXYZ();
        Vec x;
        for (int i = 0; i < 3; ++i) x(i) = pts[p * 3 + i];
        vPoint->setEstimate(x);
        vPoint->setId(ptid[p]);
        vPoint->setFixed(false);
        vPoint->setMarginalized(true);
        optimizer.addVertex(vPoint);
    }
    for (int l = 0; l < nl; ++l) {
        VertexLMLineOrth *vLine = new VertexLMLineOrth();
        Vec o;
        for (int i = 0; i < 4; ++i) o(i) = lns[l * 4 + i];
        vLine->setEstimate(o);
        vLine->setId(lnid[l]);
        vLine->setMarginalized(true);
        vLine->setFixed(false);
        optimizer.addVertex(vLine);
    }
    std::vector<EdgePosePoint *> vpEdgesMono;
    for (int e = 0; e < ne; ++e) {
        EdgePosePoint *ed = new EdgePosePoint();
        ed->setVertex(0, dynamic_cast<g2o::OptimizableGraph::Vertex *>(optimizer.vertex(ptid[elm[e]])));
        ed->setVertex(1, dynamic_cast<g2o::OptimizableGraph::Vertex *>(optimizer.vertex(kfid[ekf[e]])));
        Vec obs;
        obs(0) = eobs[e * 2];
        obs(1) = eobs[e * 2 + 1];
        ed->setMeasurement(obs);
        ed->setInformation(IsoInfo{einfo[e]});
        g2o::RobustKernelHuber *rk = new g2o::RobustKernelHuber;
        ed->setRobustKernel(rk);
        rk->setDelta(thHuberMono);
        ed->SetParams(fx, fy, cx, cy);
        optimizer.addEdge(ed);
        vpEdgesMono.push_back(ed);
    }
    std::vector<EdgePoseLine *> vlEdgesMono;
    for (int e = 0; e < nle; ++e) {
        EdgePoseLine *ed = new EdgePoseLine();
        ed->setVertex(0, dynamic_cast<g2o::OptimizableGraph::Vertex *>(optimizer.vertex(lnid[llm[e]])));
        ed->setVertex(1, dynamic_cast<g2o::OptimizableGraph::Vertex *>(optimizer.vertex(kfid[lkf[e]])));
        Vec obs;
        for (int i = 0; i < 4; ++i) obs(i) = lobs[e * 4 + i];
        ed->setMeasurement(obs);
        ed->setInformation(IsoInfo{linfo[e]});
        g2o::RobustKernelHuber *rk = new g2o::RobustKernelHuber;
        ed->setRobustKernel(rk);
        rk->setDelta(thHuberLine);
        ed->SetParams(fx, fy, cx, cy);
        optimizer.addEdge(ed);
        vlEdgesMono.push_back(ed);
    }

    const bool mutate = argc > 3 && std::string(argv[3]) == "mutate";
    optimizer.initializeOptimization();
    const int it1 = optimizer.optimize(5);
    if (mutate) {
        for (int k = 0; k < nk; ++k)
            if (!kffix[k]) {
                optimizer.vertex(kfid[k])->setFixed(true);
                break;
            }
        if (ne > 0) {
            Vec obs;
            obs(0) = eobs[0] + 3.0;
            obs(1) = eobs[1] - 2.0;
            vpEdgesMono[0]->setMeasurement(obs);
        }
        if (ne > 1) vpEdgesMono[1]->setInformation(IsoInfo{4.0 * einfo[1]});
    }
    for (auto *e : vpEdgesMono) {
        if (e->chi2() > 5.991 || !e->isDepthPositive()) e->setLevel(1);
        e->setRobustKernel(0);
    }
    for (auto *e : vlEdgesMono) {
        if (e->chi2() > 5.991) e->setLevel(1);
        e->setRobustKernel(0);
    }
    optimizer.initializeOptimization(0);
    const int it2 = optimizer.optimize(10);
    if (it1 < -1 || it2 < -1 || !optimizer.lastError().empty()) {
        fprintf(stderr, "facade: %s\n", optimizer.lastError().c_str());
        return 1;
    }
    // post-solve outlier pass inputs (src/mapHandler.cpp:6154-6293): level-1 edges recomputed
    std::vector<double> pchi(ne), lchi(nle);
    std::vector<unsigned char> pdep(ne), plev(ne), llev(nle);
    for (int i = ne - 1; i >= 0; --i) {
        EdgePosePoint *e = vpEdgesMono[i];
        if (e->level() == 1) e->computeError();
        pchi[i] = e->chi2();
        pdep[i] = e->isDepthPositive() ? 1 : 0;
        plev[i] = (unsigned char)e->level();
    }
    for (int i = nle - 1; i >= 0; --i) {
        EdgePoseLine *e = vlEdgesMono[i];
        if (e->level() == 1) e->computeError();
        lchi[i] = e->chi2();
        llev[i] = (unsigned char)e->level();
    }
    // write-back values (src/mapHandler.cpp:6296-6319): Tcw, points, orth lines
    FILE *o = fopen(argv[2], "wb");
    if (!o) return 2;
    const int its[2] = {it1, it2};
    fwrite(its, sizeof(int), 2, o);
    for (int k = 0; k < nk; ++k) {
        const Mat4 T = static_cast<VertexLMPose *>(optimizer.vertex(kfid[k]))->estimate();
        for (int r = 0; r < 3; ++r) fwrite(&T.a[r * 4], sizeof(double), 4, o);
    }
    // the reference's read-back statements, verbatim apart from the stand-in containers
    // (src/mapHandler.cpp:6297-6319)
    std::vector<KeyFrame> kfs(nk);
    std::vector<MapPoint> local_pt(np);
    std::vector<MapLine> local_ls(nl);
    for (int k = 0; k < nk; ++k) kfs[k].kf_idx = kfid[k];
    for (int p = 0; p < np; ++p) local_pt[p].idx = p;
    for (int l = 0; l < nl; ++l) local_ls[l].idx = l;
    for (int k = 0; k < nk; ++k) {
        if (kffix[k]) continue;  // idx_nofix_kfs
        KeyFrame *pKFi = &kfs[k];
        VertexLMPose *vPose = dynamic_cast<VertexLMPose *>(optimizer.vertex(pKFi->kf_idx));
        pKFi->T_kf_w = vPose->estimate().inverse();
    }
    for (MapPoint &mp : local_pt) {
        MapPoint *pMP = &mp;
        VertexLMPointXYZ *vPoint = dynamic_cast<VertexLMPointXYZ *>(optimizer.vertex(ptid[pMP->idx]));
        pMP->point3D = vPoint->estimate();
    }
    for (MapLine &ml : local_ls) {
        MapLine *lML = &ml;
        VertexLMLineOrth *vLine = dynamic_cast<VertexLMLineOrth *>(optimizer.vertex(lnid[lML->idx]));
        Vec orth = vLine->estimate();
        lML->orth_written = orth;
    }
    for (int p = 0; p < np; ++p) {
        const Vec x = static_cast<VertexLMPointXYZ *>(optimizer.vertex(ptid[p]))->estimate();
        fwrite(x.a, sizeof(double), 3, o);
    }
    for (int l = 0; l < nl; ++l) {
        const Vec x = static_cast<VertexLMLineOrth *>(optimizer.vertex(lnid[l]))->estimate();
        fwrite(x.a, sizeof(double), 4, o);
    }
    fwrite(pchi.data(), sizeof(double), ne, o);
    fwrite(pdep.data(), 1, ne, o);
    fwrite(plev.data(), 1, ne, o);
    fwrite(lchi.data(), sizeof(double), nle, o);
    fwrite(llev.data(), 1, nle, o);
    for (int k = 0; k < nk; ++k) fwrite(kfs[k].T_kf_w.a, sizeof(double), 16, o);  // zero for fixed KFs
    for (int p = 0; p < np; ++p) fwrite(local_pt[p].point3D.a, sizeof(double), 3, o);
    for (int l = 0; l < nl; ++l) fwrite(local_ls[l].orth_written.a, sizeof(double), 4, o);
    fclose(o);
    return 0;
}
