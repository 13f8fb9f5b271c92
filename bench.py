#!/usr/bin/env python3
"""Benchmark: LM iterations/sec of the Plücker local BA (BASELINE.json metric) on MI355X.

One *step* = one full `localBundleAdjustmentForPlukerWithG2O` solve on a device-resident
window: reset estimates -> optimize(5) with Huber -> outlier classification -> optimize(10)
-> level-1 χ² refresh (src/mapHandler.cpp:6119-6160), all on the GPU.
`value` = Σ over ranks of outer LM iterations executed in the timed steps ÷ max-over-ranks
wall time. Workload (N=1): config C3 = 100 KF / 20k points / 4k lines (BASELINE.json
configs[2], the window north_star quotes its ≥50x target on).

Multi-GPU (`--gpus N`, launched by torch.distributed.run), two modes:
  --mode replicas (default)  every rank solves its own independent C3 window (different seed):
                             a C3 window fits one GPU, and north_star shards a window only "when
                             the window exceeds one GPU", so more GPUs = more windows, with no
                             data-path collective (weak scaling; the same workload and unit as the
                             N = 1 line). For N > 1 rank 0 then runs the sharded C5 job below as a
                             child process group (bounded by a timeout, killed by its process
                             group id if it overruns) and embeds its line as "shard_run".
  --mode shard               ONE window split over the ranks by landmark:
                             BASELINE.json configs[4] (C5, 1000 KF, "report 1/2/4/8 scaling")
                             for every N > 1 (`--config C4` gives configs[3]); partial reduced
                             camera systems summed with RCCL all-reduces inside the captured step
                             graph (strong scaling); rank 0 also times the same window unsharded on
                             its GPU ("scaling_reference", the curve's 1-GPU point);
                             `--transport host` rehearses it with gloo.
The barrier and max-over-ranks timing use torch.distributed in both.

Extra JSON objects:
  roofline      dominant kernel (by device time), algorithmic bytes per launch / avg launch
                time measured with HIP events on the solver stream; traffic from the committed
                rocprofv3 PMC summary (profiles/pmc_<cfg>.json) when present.
  cpu_baseline  the CPU oracle (single-threaded g2o-structured restatement, oracle/) timed on
                this host on a bounded sample (rank 0, N=1 only).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pl-slam-plucker_amd"))

import numpy as np  # noqa: E402

from plba import synth  # noqa: E402
from plba.roofline import kernel_bytes  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="C3")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-runs", type=int, default=5)
    p.add_argument("--device", type=int, default=None, help="override LOCAL_RANK (multi-rank rehearsal on 1 GPU)")
    p.add_argument("--mode", choices=["replicas", "shard"], default=None,
                   help="default: replicas (one C3 window per GPU); shard: one C5 window over all ranks")
    p.add_argument("--transport", choices=["rccl", "host"], default="rccl", help="--mode shard all-reduce transport")
    p.add_argument("--no-shard-run", action="store_true", help="replicas, N > 1: skip the embedded sharded C5 run")
    p.add_argument("--shard-timeout", type=float, default=90.0, help="seconds allowed to the embedded sharded run")
    p.add_argument("--no-host-mirror", action="store_true", help="N = 1: skip the host-mirror per-call timing")
    p.add_argument("--windows", type=int, default=4,
                   help="N = 1: also time this many independent windows solved concurrently on the one GPU "
                        "(one context + stream each, one host thread each), reported as 'concurrent_windows' "
                        "beside the single-window value (0 disables)")
    return p.parse_args()


def cpu_model() -> str:
    """`lscpu` model name of this host (reported next to every CPU number)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg: str, runs: int):
    """Time the CPU oracle (refcpu, -O3 -march=native, 1 thread) on the same window, pinned to one
    core (the `taskset -c <cpu>` of BASELINE.md §2, via sched_setaffinity on this process)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_api as oa
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "native"], check=True)
    oa.ORACLE_SO = os.path.join(ROOT, "oracle", "librefcpu_native.so")
    g = synth.generate(cfg)
    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    try:
        oa.lba_plucker(g)  # warm
        ms, iters = [], []
        for _ in range(runs):
            r = oa.lba_plucker(g)
            ms.append(r["solve_ms"])
            iters.append(int(r["iters"][0] + r["iters"][1]))
    finally:
        os.sched_setaffinity(0, prev)
    med = statistics.median(ms)
    it = iters[0]
    # refcpu-fast: the same restatement with fixed-size blocks — a sanity lower
    # bound reported beside the baseline, not the speedup basis
    fast = None
    try:
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "fast"], check=True)
        oa._lib = None
        oa.ORACLE_SO = os.path.join(ROOT, "oracle", "librefcpu_fast_native.so")
        os.sched_setaffinity(0, {core})
        try:
            oa.lba_plucker(g)
            fms = [oa.lba_plucker(g)["solve_ms"] for _ in range(runs)]
        finally:
            os.sched_setaffinity(0, prev)
        fmed = statistics.median(fms)
        fast = dict(value=it / (fmed / 1e3), ms_per_lba=fmed, kind="port-fast",
                    note="oracle/refcpu.cpp -DREFCPU_FAST: inline fixed-capacity blocks, compile-time "
                         "Schur / quadratic-form block sizes, pair->block lookups resolved once; same results")
    except Exception as e:  # the lower bound is informational
        fast = {"error": repr(e)}
    return dict(value=it / (med / 1e3), unit="LM iterations/s", cores=1, kind="port", refcpu_fast=fast,
                cpu_model=cpu_model(), pinned_core=core, host_cpus=os.cpu_count(),
                final_chi2=[float(r["chi2"][0]), float(r["chi2"][1])],
                sample=f"{cfg} window ({g.n_kf} KF, {g.n_pt} pts, {g.n_ln} lines, {g.n_ept + g.n_eln} edges), "
                       f"full 2-stage LBA ({it} outer iterations), 1 warm + {runs} timed runs, median "
                       f"{med:.1f} ms/LBA; oracle/refcpu.cpp (g2o-structured restatement) -O3 -march=native, "
                       f"1 thread pinned to core {core}",
                ms_per_lba=med)


def concurrent_windows(a, dev: int, k: int):
    """k independent windows of the same config solved at the same time on one GPU (one context,
    stream and host thread each; ctypes releases the GIL inside the C calls): aggregate LM it/s.
    A serving view — several SLAM sessions sharing a GPU — reported beside `value`, never as it."""
    import threading
    from plba.lib import Solver
    base = synth.CONFIGS[a.config][3]
    solvers = [Solver(device=dev) for _ in range(k)]
    for i, sv in enumerate(solvers):
        sv.upload(synth.generate(a.config, seed=base + 97 * (i + 1)))
        sv.reset()
        sv.lba_plucker(want_outputs=False, with_trace=False)  # warm: graphs, code objects
        sv.synchronize()
    steps = max(1, a.steps)
    iters = [0] * k
    go = threading.Barrier(k + 1)

    def run(i):
        sv = solvers[i]
        go.wait()
        for _ in range(steps):
            sv.reset()
            r = sv.lba_plucker(want_outputs=False, with_trace=False)
            iters[i] += int(r["iters"][0] + r["iters"][1])
        sv.synchronize()

    th = [threading.Thread(target=run, args=(i,)) for i in range(k)]
    for t in th:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    for sv in solvers:
        sv.close()
    return {"windows": k, "value": sum(iters) / dt, "unit": "LM iterations/s", "steps_per_window": steps,
            "ms_per_lba": dt / steps * 1e3,
            "note": "independent windows of the same config, one context + stream + host thread each, "
                    "solved concurrently on one GPU (serving view; not the headline)"}


def host_mirror(cfg: str, dev: int, calls: int = 3, background=None, scan_calls: int = 0):
    """The drop-in's whole per-call cost on the host mirror: the C++
    MapHandler::localBundleAdjustmentForPlukerWithG2O (src/mapHandler.cpp:5851-6323) on a synthetic
    map holding the config's window — gather + graph marshalling (:5868-6117), the device solve
    (upload + two-stage LM + download), the outlier pass (:6154-6293) and the write-back
    (:6296-6319). Successive calls run on the same map, which each call mutates as the reference's
    does (outliers removed, fixed observers left local); the first call also creates the context."""
    from plba.slam_map import HostMap, make_map
    g = synth.generate(cfg)
    t0 = time.perf_counter()
    hm = HostMap(make_map(g), device=dev)
    if background:   # (n_kf, n_pt, n_ln) of non-local map around the window
        hm.add_background(*background, seed=11)
    build_s = time.perf_counter() - t0

    def summary(rows, mode):
        warm = rows[1:]
        med = {k: statistics.median(r[k] for r in warm)
               for k in ("gather_ms", "upload_ms", "solve_ms", "bookkeeping_ms", "dirty_landmarks")}
        return {"mode": mode, "gather_ms": med["gather_ms"], "upload_ms": med["upload_ms"],
                "gather_plus_upload_ms": med["gather_ms"] + med["upload_ms"], "solve_ms": med["solve_ms"],
                "outlier_and_writeback_ms": med["bookkeeping_ms"],
                "total_ms": med["gather_ms"] + med["solve_ms"] + med["bookkeeping_ms"],
                "dirty_landmarks": med["dirty_landmarks"],
                "first_call_ms": rows[0]["gather_ms"] + rows[0]["solve_ms"] + rows[0]["bookkeeping_ms"], "calls": calls}
    try:
        rows = [hm.local_ba() for _ in range(calls + 1)]
        out = summary(rows, "incremental")
        if scan_calls:   # the same map, the reference's map-scanning gather (A/B)
            hm.set_incremental(False)
            out["scan"] = summary([hm.local_ba() for _ in range(scan_calls + 1)], "scan")
    finally:
        hm.close()
    out["map"] = {"keyframes": hm.n_kf, "points": hm.n_pt, "lines": hm.n_ln, "build_s": build_s}
    out["window"] = {k: rows[-1][k] for k in ("n_free_kf", "n_fixed_kf", "n_pt", "n_ln", "n_ept", "n_eln")}
    out["note"] = ("median of calls 2..%d of MapHandler::localBundleAdjustmentForPlukerWithG2O (host/map_handler.cpp) "
                   "on one synthetic map: gather = window gather + g2o-graph marshalling (incremental: the local "
                   "registry and cached observation runs; scan: the reference's scan of every map landmark), "
                   "upload = plba_upload (part of solve), solve = plba_upload + plba_lba_plucker incl. outputs "
                   "(PCIe-inclusive), outlier_and_writeback = the outlier pass + pose/landmark write-back" % (calls + 1))
    return out


def relaunch_distributed(a) -> int:
    """`--gpus N` (N > 1) without a torch.distributed launcher: start N ranks of this same command
    under torch.distributed.run (127.0.0.1) as a child process, before anything touches the GPU,
    and return its exit code."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


# Per-step phase split of a (sharded) window from one kernel-timed LBA (DESIGN §7's model):
# work every rank does on its own landmark share, work every rank repeats on the whole reduced
# camera system, and the collectives between them.
SHARDED_KERNELS = ("k_linearize", "k_iter_reduce", "k_edge_schur", "k_rcs_chunk", "k_lm_solve", "k_shard_pack")


def phases(ktimes: dict, steps: int) -> dict:
    st = max(int(steps or 0), 1)
    sh = sum(ms for k, (ms, n) in ktimes.items() if k in SHARDED_KERNELS)
    co = sum(ms for k, (ms, n) in ktimes.items() if k == "collectives")
    rep = sum(ms for k, (ms, n) in ktimes.items() if k not in SHARDED_KERNELS and k != "collectives")
    return {"device_steps_per_lba": st, "sharded_us_per_step": sh * 1e3 / st,
            "replicated_us_per_step": rep * 1e3 / st, "collective_us_per_step": co * 1e3 / st,
            "note": "event-timed kernels of one instrumented LBA: sharded = per-rank edge/landmark work "
                    "(divides by N), replicated = factorisation + init/finalize/decide (every rank), "
                    "collective = the exchanges (host transport: incl. the host round trip)"}


def shard_child(a, world: int):
    """Rank 0 of a replicas job with N > 1: the sharded C5 strong-scaling job on the same N GPUs,
    as a child process group (its own torch.distributed.run), after the replicas measurement. A
    run that overruns --shard-timeout is killed by its process group id and reported as such; the
    replicas line is printed either way."""
    import signal
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                        "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--mode", "shard",
           "--steps", str(max(1, min(a.steps, 10))), "--warmup", "1", "--no-cpu-baseline",
           "--transport", a.transport] + (["--device", str(a.device)] if a.device is not None else [])
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=a.shard_timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"error": f"timeout after {a.shard_timeout:.0f} s (process group killed)"}
    wall = time.perf_counter() - t0
    for line in reversed(out.splitlines()):
        if line.startswith("{"):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            keep = ("value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "scaling_reference",
                    "final_chi2_gpu", "comm")
            d = {k: r[k] for k in keep if k in r}
            d["workload"] = r.get("config", {}).get("workload")
            d["end_to_end"] = r.get("config", {}).get("end_to_end")
            d["child_wall_s"] = wall
            return d
    return {"error": f"exit {p.returncode}, no JSON line", "stderr_tail": err[-2000:]}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(a))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s); refusing to report "
              f"a {world}-rank measurement as {a.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # gloo prints "[Gloo] Rank r is connected to ..." on the process's stdout (fd 1) while
        # the group forms: send fd 1 to stderr for the init, so stdout carries only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    from plba.lib import Solver

    if a.mode is None:
        a.mode = "replicas"
    shard = a.mode == "shard"
    if shard and "--config" not in sys.argv:
        # BASELINE.json configs[4]: the 1000-KF window, "report 1/2/4/8 scaling" — every N > 1
        # shards the same C5 window, so the N = 2, 4, 8 points form one strong-scaling curve
        # (its one-GPU point is measured in the same job: "scaling_reference")
        a.config = "C5"
    base_seed = synth.CONFIGS[a.config][3]
    dev = local if a.device is None else a.device
    create_ms = None
    if shard:  # one window for all ranks
        g = synth.generate(a.config, seed=base_seed)
        # (RCCL prints a version banner on stdout at communicator init: fd 1 -> stderr meanwhile,
        # so stdout carries only the JSON line)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if dist is None:
                from plba.lib import comm_unique_id
                s = Solver(device=dev)
                if a.transport == "rccl":
                    s.comm_init_rccl(1, 0, comm_unique_id())
                else:
                    s.comm_init_host(1, 0, lambda buf: None)
            else:
                from plba.dist import sharded_solver
                s = sharded_solver(device=dev, transport=a.transport)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        # what the transport itself reports on every rank (RCCL's rank count / rank / device, the
        # HIP device and its PCI location): the record proves N ranks ran on N distinct GPUs
        from plba.dist import comm_summary, gather_comm_info
        comm = gather_comm_info(s.comm_info()) if dist is not None else comm_summary([s.comm_info()])
    else:
        g = synth.generate(a.config, seed=base_seed + 97 * rank)
        t0 = time.perf_counter()
        s = Solver(device=dev)
        create_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    s.upload(g)
    s.synchronize()
    upload_ms = (time.perf_counter() - t0) * 1e3
    setup_s = time.perf_counter() - T_START  # process start -> window resident (shard-timeout budget)

    def step(with_trace=True):
        s.reset()
        return s.lba_plucker(want_outputs=False, with_trace=with_trace)

    for _ in range(a.warmup):
        step()
    # one instrumented (kernel-timed) step outside the timed region, for the roofline
    s.L.plba_enable_kernel_timing(s.ctx, 1)
    r = step()
    ktimes = s.kernel_times()
    info = s.structure_stats()
    s.L.plba_enable_kernel_timing(s.ctx, 0)
    ph = phases(ktimes, info.get("device_steps")) if shard else None

    s.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    iters = 0
    trials = 0
    trials_per_lba = int(sum(t["trials"] for t in r["trace"]))  # the instrumented step's (same window)
    for _ in range(a.steps):
        r = step(with_trace=False)
        iters += int(r["iters"][0] + r["iters"][1])
        trials += trials_per_lba
    s.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    tot_iters = iters
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        if not shard:  # replicas: every rank's iterations count; shard: one window's
            ti = torch.tensor([iters], dtype=torch.float64)
            dist.all_reduce(ti, op=dist.ReduceOp.SUM)
            tot_iters = int(ti.item())

    # End-to-end LBA call on a NEW window of the same config: upload (host
    # marshalling + one pinned copy) + step-graph capture + the two-stage solve + download of every
    # output, as the drop-in use pays it per call; the second of two windows is reported (the
    # first pays one-time arena / code-object costs). Outside the timed region.
    e2e = []
    for k in range(2):
        # (sharded: every rank uploads the same window — each keeps its landmark share)
        g2 = synth.generate(a.config, seed=base_seed + 7919 * (k + 1) + (0 if shard else 97 * rank))
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        s.upload(g2)
        t1 = time.perf_counter()
        r2 = s.lba_plucker(want_outputs=True, with_trace=False)
        t2 = time.perf_counter()
        e2e.append(dict(end_to_end_ms=(t2 - t0) * 1e3, upload_ms=(t1 - t0) * 1e3,
                        solve_and_download_ms=(t2 - t1) * 1e3, solve_ms=float(r2["solve_ms"])))

    # the same window unsharded on one GPU (rank 0, outside the timed region): the N = 1 point of
    # the sharded strong-scaling curve
    scaling_ref = None
    if shard and world > 1:
        if rank == 0:
            ref = Solver(device=dev)
            ref.upload(g)
            for _ in range(max(a.warmup, 1)):
                ref.reset()
                ref.lba_plucker(want_outputs=False, with_trace=False)
            ref.synchronize()
            t0 = time.perf_counter()
            ri = 0
            for _ in range(a.steps):
                ref.reset()
                rr = ref.lba_plucker(want_outputs=False, with_trace=False)
                ri += int(rr["iters"][0] + rr["iters"][1])
            ref.synchronize()
            rdt = time.perf_counter() - t0
            ref.L.plba_enable_kernel_timing(ref.ctx, 1)
            ref.reset()
            ref.lba_plucker(want_outputs=False, with_trace=False)
            ref_ph = phases(ref.kernel_times(), ref.structure_stats().get("device_steps"))
            ref.close()
            scaling_ref = {"config": a.config, "n_gpus": 1, "mode": "the same window, unsharded, one GPU",
                           "value": ri / rdt, "unit": "LM iterations/s", "steps": a.steps,
                           "speedup_of_this_run": (tot_iters / dt) / (ri / rdt), "phases": ref_ph}
        dist.barrier()

    hmirror = hmirror_map = None
    if world == 1 and not shard and not a.no_host_mirror:
        try:
            hmirror = host_mirror(a.config, dev)
        except Exception as e:  # informational: must never hide the single-window number
            hmirror = {"error": repr(e)}
        if a.config == "C3":
            # the same window inside a map of C5's size (BASELINE.json configs[4]: 1000 KF / 200k
            # points / 40k lines), incremental gather and the reference's map scan on the same map
            try:
                hmirror_map = host_mirror(a.config, dev, background=(900, 180000, 36000), scan_calls=3)
            except Exception as e:
                hmirror_map = {"error": repr(e)}

    conc = None
    if world == 1 and not shard and a.windows > 1:
        try:
            conc = concurrent_windows(a, dev, a.windows)
        except Exception as e:  # informational: must never hide the single-window number
            conc = {"error": repr(e)}

    # replicas, N > 1: the sharded C5 window on the same GPUs (child job; the other ranks wait)
    shard_run = None
    if not shard and world > 1 and not a.no_shard_run:
        if rank == 0:
            shard_run = shard_child(a, world)
        dist.barrier()

    if rank == 0:
        # dominant kernel by device time in the instrumented step
        name, (kms, nl) = max(((k, v) for k, v in ktimes.items() if v[1] > 0), key=lambda kv: kv[1][0])
        avg_ms = kms / max(nl, 1)
        # rocprofv3 names the banded factorisation by its template (k_rcs_factor_band<BW>)
        prof_name = name
        if name == "k_rcs_factor" and info.get("banded"):
            if info.get("bcr_rows"):
                prof_name = "k_rcs_factor_bcr"
            else:
                prof_name = "k_rcs_factor_twisted" if info.get("twisted") else "k_rcs_factor_band"
                if info.get("column_lane"):
                    prof_name += "_cl"
        alg = kernel_bytes(g, prof_name if prof_name == "k_rcs_factor_bcr" else name, info)
        # block pivot steps on the factorisation's critical path (forward chain + backward chain)
        chain = None
        if name == "k_rcs_factor" and info.get("banded") and not info.get("bcr_rows"):
            nf_, bw_ = int(info["nf"]), int(info["bw"])
            if info.get("twisted"):
                chain = 2 * ((nf_ - bw_ + 1) // 2 + bw_)
            else:
                chain = 2 * nf_
        achieved = alg / (avg_ms * 1e-3) / 1e9
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{a.config}.json")
        traffic = None
        if os.path.exists(pmc_path):
            try:
                traffic = json.load(open(pmc_path)).get(prof_name, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        per_kernel = {}
        # the iteration kernels exit at once on steps without a new linearisation (ITER_GUARD): their
        # bandwidth is over the launches that worked — one per outer iteration of the LBA
        lin_per_lba = int(sum(max(int(x), 0) for x in r["iters"]))
        for k, (ms_k, n_k) in ktimes.items():
            if n_k <= 0:
                continue
            b = kernel_bytes(g, "k_rcs_factor_bcr" if (k == "k_rcs_factor" and info.get("bcr_rows")) else k, info)
            us = ms_k / n_k * 1e3
            work = min(n_k, lin_per_lba) if k in ("k_linearize", "k_iter_reduce") else n_k
            us_w = ms_k / max(work, 1) * 1e3
            per_kernel[k] = {"us_per_launch": round(us, 2), "launches_per_lba": n_k, "working_launches": work,
                             "us_per_working_launch": round(us_w, 2),
                             "alg_bytes": int(b), "GBs": round(b / (us_w * 1e-6) / 1e9, 1) if b else None}
        it_per_lba = tot_iters / max(a.steps * (1 if shard else world), 1)
        iter_bytes = synth.algorithmic_bytes_per_iter(g)
        out = {
            "metric": "LM iterations/sec (and ms/iter) on local-BA window; final \u03c7\u00b2 vs g2o",
            "value": tot_iters / dt,
            "unit": "LM iterations/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded EuRoC-shaped window, SURVEY.md §8d)",
            "config": {
                "workload": f"{a.config}: {g.n_kf} KF ({int(g.kf_fixed.sum())} fixed) / {g.n_pt} points / "
                            f"{g.n_ln} Plücker lines, {g.n_ept}+{g.n_eln} edges; "
                            + (f"one window sharded over {world} GPU(s) by landmark ({a.transport} all-reduce)"
                               if shard else "one independent window per GPU"),
                "edges": int(g.n_ept + g.n_eln),
                # SURVEY.md §8d sizes the configs at 5 observations per landmark; the generator's
                # visibility rejection leaves ~4.7 (C3: 112,416 of the nominal 120,000 edges)
                "survey_nominal_edges": int(5 * (g.n_pt + g.n_ln)),
                "lm_iterations_per_lba": it_per_lba,
                "trials_per_lba": trials / a.steps,
                "ms_per_lm_iteration": dt / max(iters, 1) * 1e3,
                # plba_create pre-warms the context (code objects, first device build, pinned
                # staging): create_ms is that one-time cost, upload_ms the process's first window
                "create_ms": create_ms,
                "upload_ms": upload_ms,
                "end_to_end": e2e[-1],
                "factorisation": ("block cyclic reduction over %d super-rows" % info["bcr_rows"] if info.get("bcr_rows")
                                  else "dense blocked LDLT (MFMA)" if not info.get("banded")
                                  else "%s%s band LDLT (bw %d)" % ("two-sided " if info.get("twisted") else "",
                                                                   "column-lane" if info.get("column_lane") else "register-window",
                                                                   info.get("bw", 0))),
                "speculative_trials": {"slots": info.get("spec_slots", 1), "policy": info.get("spec_policy", 0),
                                       "device_steps_per_lba": info.get("device_steps")},
                "parallelism": (f"landmark-sharded window over {world} GPU(s)" if shard
                                else f"{world} independent windows (1 per GPU)"),
            },
            "roofline": {
                "kernel": prof_name,
                # the factorisation is a serial chain of block pivots: its limiter is latency, the HBM
                # fraction is reported per the contract (peak = HBM) but is not its bound
                "bound": "latency" if name == "k_rcs_factor" else "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "alg_bytes_per_launch": alg,
                "avg_launch_us": avg_ms * 1e3,
                "launches_per_lba": nl,
                "critical_path_block_steps": chain,
                "us_per_block_step": avg_ms * 1e3 / chain if chain else None,
                "note": ("latency-bound factorisation of the reduced camera system (a serial chain of 6x6 "
                         "pivot blocks or of dense super-row eliminations) + back substitution + pose update; "
                         "bytes/launch are tiny by nature — see DESIGN.md §4"),
            },
            "iteration_roofline": {
                "alg_bytes_per_iter": iter_bytes,
                "achieved_GBs": iter_bytes * (tot_iters / dt) / 1e9,
                "frac": iter_bytes * (tot_iters / dt) / 1e9 / HBM_PEAK_GBS,
            },
            "kernels": per_kernel,
        }
        out["final_chi2_gpu"] = [float(r["chi2"][0]), float(r["chi2"][1])]
        if ph is not None:
            out["phases"] = ph
        if shard:
            out["comm"] = {
                **comm,
                "setup_s_rank0": setup_s,
                "note": "plba_comm_info on every rank (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice; "
                        "hipGetDevice and the PCI location of the context's device); setup_s = process start "
                        "to the window resident on the device, incl. torch / RCCL init",
            }
        if scaling_ref is not None:
            out["scaling_reference"] = scaling_ref
        if shard_run is not None:
            out["shard_run"] = shard_run
            # first-class: the one-window sharded rate (configs[4]) and its speed-up over the same
            # window unsharded on one GPU, beside the replicas value
            out["shard_value"] = shard_run.get("value")
            out["shard_speedup"] = (shard_run.get("scaling_reference") or {}).get("speedup_of_this_run")
        if conc is not None:
            out["concurrent_windows"] = conc
        if hmirror is not None:
            out["host_mirror"] = hmirror
        if hmirror_map is not None:
            out["host_mirror_c5_map"] = hmirror_map
        if world == 1 and not a.no_cpu_baseline:
            try:
                cb = cpu_baseline(a.config, a.cpu_runs if a.config in ("C1", "C1L", "C2", "C3") else 1)
                out["final_chi2_cpu"] = cb.pop("final_chi2")
                out["final_chi2_rel_diff"] = max(abs(x - y) / abs(y) for x, y in
                                                 zip(out["final_chi2_gpu"], out["final_chi2_cpu"]))
                out["cpu_baseline"] = cb
                out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            except Exception as e:  # the baseline must never hide the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    s.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
