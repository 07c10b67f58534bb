"""Debug: repeat the C4 overlapped exchange at full workload and report each
repetition's max relative L2 against the float64 sum of the plain per-view
gradients (development; tests/test_gpu_dist.py has the test).
python tools/dbg/overlap_repro.py WORLD REPS [chunks]   env OVL_SYNC=1: synchronize in the hook"""
import json, math, os, socket, sys, time
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, reps, chunks, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_scene as S
    import gsr_dist
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    torch.set_num_threads(max(1, 16 // world))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, H, P = 1920, 1080, 1_000_000
    raw = S.make_gaussians(P, sh_degree=3, sg_degree=0, aspect=H / W)
    inp = {k: v.detach().contiguous().to(dev) for k, v in S.activated_inputs(raw).items()}
    cam = S.orbit_cameras(8, W, H)[rank].to(dev)
    st = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
        kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=3, sg_degree=0, campos=cam.camera_center,
        prefiltered=False, require_depth=True, debug=False)
    g = {k: v.to(dev) for k, v in S.upstream_grads(H, W, seed=11 + rank).items()}
    keys = ["means3D", "opacities", "scales", "rotations", "shs"]

    def step():
        ps = {k: inp[k].clone().requires_grad_(True) for k in keys}
        color, radii, md, alpha, normal = GaussianRasterizer(st)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=inp["sg_axis"], sg_sharpness=inp["sg_sharpness"],
            sg_color=inp["sg_color"], scales=ps["scales"], rotations=ps["rotations"])
        torch.autograd.backward([color, md, normal], [g["color"], g["mdepth"], g["normal"]])
        torch.cuda.synchronize()
        return {k: ps[k].grad for k in keys}

    plain = step()
    want = {}
    for k in keys:
        w = plain[k].double()
        dist.all_reduce(w)
        want[k] = w
    ex = gsr_dist.OverlappedViewGrads(chunks=chunks)
    if os.environ.get("OVL_SYNC"):
        orig = ex.on_chunk
        def on_chunk(b, e, grads):
            torch.cuda.synchronize()
            orig(b, e, grads)
        ex.on_chunk = on_chunk
    res = []
    for r in range(reps):
        with ex:
            got = step()
        errs = {k: float((got[k].double() - want[k]).norm() / want[k].norm()) for k in keys}
        # which range is off (means3D rows)
        d = (got["means3D"].double() - want["means3D"]).norm(dim=1)
        cs = ex._cs
        per_range = [float(d[b:b + cs].norm() / want["means3D"][b:b + cs].norm().clamp_min(1e-30))
                     for b in range(0, P, cs)]
        res.append({"rep": r, "max": max(errs.values()), "errs": errs, "ranges": per_range})
    json.dump(res, open(os.path.join(outdir, f"ovl{rank}.json"), "w"))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, reps = int(sys.argv[1]), int(sys.argv[2])
    chunks = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    outdir = os.path.join(ROOT, "gpurun_out", "ovl")
    os.makedirs(outdir, exist_ok=True)
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    t0 = time.time()
    mp.start_processes(worker, args=(world, port, reps, chunks, outdir), nprocs=world, join=True, start_method="spawn")
    r0 = json.load(open(os.path.join(outdir, "ovl0.json")))
    bad = 0
    for r in r0:
        flag = r["max"] > 1e-5
        bad += flag
        print(r["rep"], f"{r['max']:.2e}", "BAD" if flag else "", {k: f"{v:.1e}" for k, v in r["errs"].items()} if flag else "",
              [f"{x:.1e}" for x in r["ranges"]] if flag else "")
    print(f"{bad} of {len(r0)} repetitions wrong; {time.time() - t0:.0f} s")
