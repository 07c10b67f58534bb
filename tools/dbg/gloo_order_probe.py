"""Debug probe (round 6): does gloo's device-to-host staging of a device tensor
wait for the work queued before the collective was posted?

Each trial, on torch's current stream: x := -1, a ~`SLEEP` cycle spin kernel,
x := rank + 1, then dist.all_reduce(x, async_op=True) is posted and waited.
If the staging copy does not wait for the stream, the sum is not
world (world + 1) / 2.  Modes (posted from where the overlapped exchange posts):
  main      the main thread
  ctypes    a ctypes callback called from inside a foreign call (libc qsort)
  autograd  a custom autograd Function's backward (the autograd device thread),
            via a ctypes callback as the rasterizer backward does
  slice     a row slice of a larger tensor, as the exchange posts dmeans3D[b:e]
python tools/dbg/gloo_order_probe.py WORLD TRIALS [modes]"""
import ctypes
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SLEEP = int(os.environ.get("PROBE_SLEEP", "2000000"))


def worker(rank, world, port, trials, modes, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    want = world * (world + 1) / 2
    n = 250_000 * 3
    big = torch.zeros(4 * n, device=dev)
    libc = ctypes.CDLL(None)
    CMP = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
    res = {}

    def prepare(x):
        x.fill_(-1.0)
        torch.cuda._sleep(SLEEP)
        x.fill_(float(rank + 1))

    def post(x, works):
        works.append(dist.all_reduce(x, op=dist.ReduceOp.SUM, async_op=True))

    def via_qsort(fn):
        arr = (ctypes.c_int * 2)(2, 1)
        done = []

        def cmp(a, b):
            if not done:
                done.append(1)
                fn()
            return 0
        cb = CMP(cmp)
        libc.qsort(arr, 2, ctypes.sizeof(ctypes.c_int), cb)

    class Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, inp):
            return inp * 1.0

        @staticmethod
        def backward(ctx, g):
            x = ctx.x
            works = ctx.works
            prepare(x)
            via_qsort(lambda: post(x, works))
            for w in works:
                w.wait()
            return g

    for mode in modes:
        bad, worst = 0, None
        for t in range(trials):
            works = []
            if mode == "main":
                x = torch.empty(n, device=dev)
                prepare(x)
                post(x, works)
            elif mode == "slice":
                x = big[n:2 * n]
                prepare(x)
                post(x, works)
            elif mode == "ctypes":
                x = torch.empty(n, device=dev)
                prepare(x)
                via_qsort(lambda: post(x, works))
            elif mode == "autograd":
                x = torch.empty(n, device=dev)
                a = torch.ones(4, device=dev, requires_grad=True)
                y = Fn.apply(a)
                gf = y.grad_fn
                gf.x, gf.works = x, works  # (the backward reads them from ctx)
                y.sum().backward()
                works = []
            for w in works:
                w.wait()
            torch.cuda.synchronize()
            got = x.float()
            ok = bool((got == want).all())
            if not ok:
                bad += 1
                vals = torch.unique(got).tolist()[:8]
                worst = {"trial": t, "values": vals, "n_wrong": int((got != want).sum())}
        res[mode] = {"bad": bad, "trials": trials, "example": worst}
        print(f"[rank {rank}] {mode}: {bad} of {trials} wrong {worst or ''}", flush=True)
    with open(os.path.join(outdir, f"probe{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, trials = int(sys.argv[1]), int(sys.argv[2])
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["main", "slice", "ctypes", "autograd"]
    outdir = os.path.join(ROOT, "gpurun_out", "gloo_probe")
    os.makedirs(outdir, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    t0 = time.time()
    mp.start_processes(worker, args=(world, port, trials, modes, outdir), nprocs=world, join=True,
                       start_method="spawn")
    print(f"done in {time.time() - t0:.0f} s")
