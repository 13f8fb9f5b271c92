"""Worker functions for multi-process tests (imported by spawned ranks)."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pl-slam-plucker_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_gloo(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def dense_schur_part(g, owned_pt, owned_ln, lam=1e-3):
    """Reduced camera system contribution of the given landmarks (numpy, oracle Jacobians):
    Σ_edges JpᵀΩJp − Σ_l Hpl_l (Hll_l+λI)⁻¹ Hpl_lᵀ, and the matching right-hand side."""
    import oracle_api as oa
    cam = (g.fx, g.fy, g.cx, g.cy)
    free = np.nonzero(g.kf_fixed == 0)[0]
    hid = -np.ones(g.n_kf, int)
    hid[free[np.argsort(g.kf_id[free], kind="stable")]] = np.arange(len(free))
    n = 6 * len(free)
    S, bs = np.zeros((n, n)), np.zeros(n)
    for kind, owned in (("pt", owned_pt), ("ln", owned_ln)):
        lm_arr = g.ept_lm if kind == "pt" else g.eln_lm
        for l in np.nonzero(owned)[0]:
            D = 3 if kind == "pt" else 4
            Hll, bl = lam * np.eye(D), np.zeros(D)
            rows = []
            for e in np.nonzero(lm_arr == l)[0]:
                k = (g.ept_kf if kind == "pt" else g.eln_kf)[e]
                if kind == "pt":
                    err, Ji, Jj = oa.point_edge(g.kf_Tcw[k], g.pt_xyz[l], g.ept_obs[e], cam)
                    w = g.ept_info[e]
                else:
                    err, Ji, Jj = oa.line_edge(g.kf_Tcw[k], g.ln_orth[l], g.eln_obs[e], cam)
                    err, Ji, Jj, w = err[:2], Ji[:2], Jj[:2], g.eln_info[e]
                Hll += w * Ji.T @ Ji
                bl -= w * Ji.T @ err
                h = hid[k]
                if h >= 0:
                    S[6 * h:6 * h + 6, 6 * h:6 * h + 6] += w * Jj.T @ Jj
                    bs[6 * h:6 * h + 6] -= w * Jj.T @ err
                    rows.append((h, w * Jj.T @ Ji))
            Hinv = np.linalg.inv(Hll)
            for h1, P1 in rows:
                bs[6 * h1:6 * h1 + 6] -= P1 @ Hinv @ bl
                for h2, P2 in rows:
                    S[6 * h1:6 * h1 + 6, 6 * h2:6 * h2 + 6] -= P1 @ Hinv @ P2.T
    return S, bs


def plan_and_schur_worker(rank, world, port, outdir):
    """CPU rank: shard plan, partial RCS of the own landmarks, summed over gloo with the
    product's host all-reduce hook; writes what it saw for the parent to check."""
    dist = init_gloo(rank, world, port)
    from plba import synth
    from plba.dist import host_allreduce
    from plba.lib import shard_plan
    g = synth.generate("C1L", fixed_frac=0.2)
    po, lo = shard_plan(g, world)
    S, bs = dense_schur_part(g, po == rank, lo == rank)
    buf = np.concatenate([S.ravel(), bs])
    host_allreduce()(buf)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), po=po, lo=lo, sum=buf)
    dist.barrier()
    dist.destroy_process_group()


def comm_info_worker(rank, world, port, outdir):
    """CPU rank: what bench.py's sharded line records about the transport, gathered over gloo
    (plba.dist.gather_comm_info) from a per-rank comm_info() as an RCCL rank on GPU `rank` would
    report it."""
    import json
    dist = init_gloo(rank, world, port)
    from plba.dist import gather_comm_info
    info = dict(transport="rccl", ranks=world, rank=rank, comm_device=rank, hip_device=rank,
                pci=f"0000:{0x11 + 0x20 * rank:02x}:00")
    summ = gather_comm_info(info)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(summ, f)
    dist.barrier()
    dist.destroy_process_group()


def sharded_hlm_worker(rank, world, port, outdir, cfg, params):
    """GPU rank: the hand-rolled LM on a sharded window over the host transport (a
    landmark pivot that fails on one rank must fail the solve on every rank)."""
    dist = init_gloo(rank, world, port)
    from plba import capi, synth
    from plba.dist import sharded_solver
    from plba.hlm import hlm_window
    win = hlm_window(synth.generate(cfg))
    s = sharded_solver(device=0, transport="host")
    info = s.comm_info()
    s.upload(win.graph)
    out = s.hlm_lba(win, capi.hlm_params(**params))
    np.savez(os.path.join(outdir, f"rank{rank}.npz"),
             **out, info=np.array([info["ranks"], info["rank"], info["hip_device"]]))
    s.close()
    dist.barrier()
    dist.destroy_process_group()


def sharded_gpu_worker(rank, world, port, outdir, cfg, transport, host_build=False, own_device=False):
    """GPU rank (all ranks may share one GPU with the host transport): full sharded LBA.
    host_build: PLBA_HOST_BUILD=1 (the host window build and its shard_plan) instead of the device
    build's own ownership kernel (k_b_owner). own_device: rank r on GPU r (one process per GPU,
    the RCCL transport's deployment)."""
    if host_build:
        os.environ["PLBA_HOST_BUILD"] = "1"
    dist = init_gloo(rank, world, port)
    from plba import synth
    from plba.dist import sharded_solver
    from plba.lib import shard_plan
    g = synth.generate(cfg)
    po, lo = shard_plan(g, world)  # the documented plan (plba_shard_plan)
    plan_lm = int((po == rank).sum() + (lo == rank).sum())
    plan_e = int((po[g.ept_lm] == rank).sum() + (lo[g.eln_lm] == rank).sum())
    s = sharded_solver(device=rank if own_device else 0, transport=transport)
    s.upload(g)
    out = s.lba_plucker()
    s.reset()
    out2 = s.lba_plucker()
    st = s.structure_stats()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"),
             **{k: v for k, v in out.items() if k not in ("trace", "solve_ms")},
             trace_chi2=np.array([t["chi2_end"] for t in out["trace"]]),
             rerun_equal=np.array(all(np.array_equal(out[k], out2[k]) for k in ("kf_Tcw", "pt_xyz", "ln_orth"))),
             local_landmarks=np.array(st["landmarks"]), local_edges=np.array(st["edges"]),
             plan_landmarks=np.array(plan_lm), plan_edges=np.array(plan_e),
             bcr_fallbacks=np.array(st["bcr_fallbacks"]))
    s.close()
    dist.barrier()
    dist.destroy_process_group()
