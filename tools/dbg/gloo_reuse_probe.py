"""Debug probe (round 6): the overlapped exchange's pattern of gloo collectives on device tensors, without the
rasterizer — per trial, per Gaussian range, one all-reduce per gradient slice (posted while the next range's
"kernel" is queued behind a short spin), every work waited, the works dropped, and at once the next trial's
posts (whose pinned staging buffers may reuse the dropped ones).  Every slice's expected sum is known
exactly (integers), so any wrong element is a lost or cross-wired copy.
Modes: device (the device slices posted, as gsr_dist does), sync (the same after a device synchronisation per
post: the slice's fill has certainly run), host (each slice copied to host memory by a blocking copy, the host
tensor reduced, copied back), gsr (gsr_dist's collective, which stages gloo's device tensors that way).
python tools/dbg/gloo_reuse_probe.py WORLD TRIALS [P] [RANGES] [MODE]"""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]


def worker(rank, world, port, trials, P, ranges, outdir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cs = (P + ranges - 1) // ranges
    widths = {"means3D": 3, "opacity": 1, "scales": 3, "rotations": 4}
    bad, first = 0, None
    for t in range(trials):
        # this trial's rows: rank- and trial-dependent integers, so the sum over ranks is known
        g = {k: torch.empty(P, w, device=dev) for k, w in widths.items()}
        works = []
        for r in range(ranges):
            b, e = r * cs, min(P, (r + 1) * cs)
            for i, (k, w) in enumerate(widths.items()):
                g[k][b:e].fill_(float((rank + 1) * (t % 7 + 1) + 10 * i + 100 * r))
            if mode == "sync":
                torch.cuda.synchronize()
            if mode == "gsr":  # gsr_dist's staged collective (what the exchange now posts on gloo)
                from gsr_dist import _all_reduce
                works += [(_all_reduce(g[k][b:e], dist.ReduceOp.SUM, None, async_op=True), None, None)
                          for k in widths]
            elif mode == "host":
                hs = [(g[k][b:e], g[k][b:e].cpu()) for k in widths]
                works += [(dist.all_reduce(h, op=dist.ReduceOp.SUM, async_op=True), d, h) for d, h in hs]
            else:
                works += [(dist.all_reduce(g[k][b:e], op=dist.ReduceOp.SUM, async_op=True), None, None)
                          for k in widths]
            torch.cuda._sleep(20000)  # (the next range's kernel, queued behind the post)
        for w_, d, h in works:
            w_.wait()
            if d is not None:
                d.copy_(h)
        works = []
        s = world * (world + 1) // 2
        ok = True
        for r in range(ranges):
            b, e = r * cs, min(P, (r + 1) * cs)
            for i, k in enumerate(widths):
                want = float(s * (t % 7 + 1) + world * (10 * i + 100 * r))
                got = g[k][b:e]
                nbad = int((got != want).sum())
                if nbad:
                    ok = False
                    if first is None:
                        vals = torch.unique(got).tolist()[:6]
                        first = {"trial": t, "range": r, "tensor": k, "wrong": nbad, "want": want, "values": vals}
        bad += 0 if ok else 1
        del g
        if rank == 0 and (t + 1) % 100 == 0:
            print(f"[rank 0] {mode}: {t + 1} trials, {bad} wrong", flush=True)
    print(f"[rank {rank}] {mode}: {bad} of {trials} trials wrong {first or ''}", flush=True)
    with open(os.path.join(outdir, f"reuse{rank}.json"), "w") as f:
        json.dump({"bad": bad, "trials": trials, "first": first}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, trials = int(sys.argv[1]), int(sys.argv[2])
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    ranges = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    mode = sys.argv[5] if len(sys.argv) > 5 else "device"
    outdir = os.path.join(ROOT, "gpurun_out", "gloo_reuse")
    os.makedirs(outdir, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    t0 = time.time()
    mp.start_processes(worker, args=(world, port, trials, P, ranges, outdir, mode), nprocs=world, join=True,
                       start_method="spawn")
    print(f"done in {time.time() - t0:.0f} s")
