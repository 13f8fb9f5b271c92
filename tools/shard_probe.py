"""Probe: N ranks of a sharded window on the visible GPUs (rank r -> device r % ndev).
usage: python tools/shard_probe.py N cfg transport"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dist_workers as dw  # noqa: E402


def worker(rank, world, port, cfg, transport):
    dist = dw.init_gloo(rank, world, port)
    import torch
    from plba import synth
    from plba.dist import sharded_solver
    ndev = torch.cuda.device_count()
    g = synth.generate(cfg)
    s = sharded_solver(device=rank % ndev, transport=transport)
    s.upload(g)
    out = s.lba_plucker()
    t0 = time.time()
    for _ in range(3):
        s.reset()
        out = s.lba_plucker(want_outputs=False)
    dt = (time.time() - t0) / 3
    print(f"rank {rank}: iters {out['iters']} chi2 {out['chi2']} {dt*1e3:.2f} ms/LBA stats {s.structure_stats()}",
          flush=True)
    s.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    n, cfg, tr = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    mp.spawn(worker, args=(n, dw.free_port(), cfg, tr), nprocs=n, join=True)
