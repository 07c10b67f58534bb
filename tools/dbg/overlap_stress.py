"""Debug (round 6): the C4 multi-rank test's exact sequence repeated REPS times
inside each rank — plain step, float64 yardstick all-reduce, `del plain`, then
the overlapped (a NEW exchange object each time, as the test's `with`), factored
and all-reduce forms on fresh parameters — so the caching allocator's block
history matches the test's (tools/dbg/overlap_repro.py kept `plain` and one
exchange object, which it does not).  Per repetition: max rel L2 per form and,
for the overlapped form, per-range errors and this rank's posted-vs-plain range
sums (tests/test_gpu_dist.py's diagnosis).
python tools/dbg/overlap_stress.py WORLD REPS"""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def worker(rank, world, ports, reps, outdir):
    import test_gpu_dist as T
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1")
    res = []
    # one process group for every repetition; T._full_rank_worker initialises and destroys its own, so the
    # repetitions run it whole (fresh group, same process and allocator)
    for r in range(reps):
        # a port free right now, chosen by rank 0 per repetition and handed over in a file (ports chosen up
        # front were taken by gloo's own connections within ~50 repetitions)
        pf = os.path.join(outdir, f"port_{r}")
        if rank == 0:
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            with open(pf + ".tmp", "w") as f:
                f.write(str(port))
            os.replace(pf + ".tmp", pf)
        else:
            while not os.path.exists(pf):
                time.sleep(0.01)
            port = int(open(pf).read())
        os.environ["MASTER_PORT"] = str(port)
        T._full_rank_worker(rank, world, port, outdir, 1_000_000, 0, 8, ["overlap", "factored", "allreduce"], 4)
        d = json.load(open(os.path.join(outdir, f"full{rank}.json")))
        worst = {f: max(v["rel_l2"] for k, v in fd.items() if not k.startswith("_")) for f, fd in d["forms"].items()}
        res.append({"rep": r, "worst": worst, "overlap": d["forms"]["overlap"]})
        if max(worst.values()) > 1e-5:  # keep the failing repetition's whole diagnosis at once
            json.dump(d, open(os.path.join(outdir, f"fail_rep{r}_rank{rank}.json"), "w"))
        json.dump(res, open(os.path.join(outdir, f"stress{rank}.json"), "w"))
        print(f"[rank {rank}] rep {r}: " + ", ".join(f"{f} {x:.2e}" for f, x in worst.items()), flush=True)
    json.dump(res, open(os.path.join(outdir, f"stress{rank}.json"), "w"))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, reps = int(sys.argv[1]), int(sys.argv[2])
    outdir = os.path.join(ROOT, "gpurun_out", "ovl_stress")
    os.makedirs(outdir, exist_ok=True)
    for f in os.listdir(outdir):
        if f.startswith("port_"):
            os.remove(os.path.join(outdir, f))
    ports = [0]
    t0 = time.time()
    mp.start_processes(worker, args=(world, ports, reps, outdir), nprocs=world, join=True, start_method="spawn")
    rs = [json.load(open(os.path.join(outdir, f"stress{k}.json"))) for k in range(world)]
    bad = [x for x in rs[0] if max(x["worst"].values()) > 1e-5]
    print(f"{len(bad)} of {reps} repetitions wrong; {time.time() - t0:.0f} s")
    if bad:
        import test_gpu_dist as T
        for x in bad:
            rep = x["rep"]
            T._print_overlap_diagnosis([{"forms": {"overlap": r[rep]["overlap"]}} for r in rs])
