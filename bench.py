#!/usr/bin/env python3
"""Benchmark: differentiable Gaussian-splatting raster, forward + backward.

BASELINE.json metric: "train iters/sec (fwd+bwd raster) at 1080p, 1M Gaussians;
HBM GB/s vs peak".  One step = one GaussianRasterizer forward + autograd
backward (the reference's render() call pattern) over one 1920x1080
view of 1M synthetic Gaussians (SH degree 3, require_depth=True, the state
after iteration 7000).  Inputs are activated tensors already resident in HBM;
losses, optimiser and the Python getters are outside the step.

  python bench.py [--gpus N --steps K --warmup W] [--config C2|C3|C5] [--no-depth] [--forward-only]

--config C2 is BASELINE.json configs[1] (100k Gaussians, one 800x800 view,
forward only); --no-depth is require_depth=False (training iterations <
7000); --forward-only times the forward alone (no autograd graph).

With N > 1 (launched by torch.distributed.run, one rank per GPU) every rank
renders its own view (C4: cameras orbiting the scene) of the same Gaussians
and the per-Gaussian gradients are summed over the ranks every step (the only
exchange of view-parallel training): by default gsr_dist.OverlappedViewGrads —
inside the rasterizer backward, range by range as the per-Gaussian backward
produces them, the geometry rows all-reduced and the DC rows all-gathered over
RCCL while the next range computes, then the SH / SG rows rebuilt on every rank
from the per-view DC rows and camera centres (2.6x fewer xGMI bytes at SH 3);
`--exchange factored` runs that exchange after the backward, `--exchange
allreduce` all-reduces every row.  `value` =
views/s over all ranks, time = max over ranks.

Rank 0 prints one JSON line: the contract fields, a `roofline` object for the
dominant kernel (algorithmic bytes per launch / its HIP-event-timed average
duration in the timed region, vs 8 TB/s HBM peak; `traffic` from the
committed rocprofv3 PMC summary when present).  Inside the timed region only
the dominant stage is bracketed by hipEvents (each recorded event idles the
stream ~10 us); the other stages' times come from --stage-steps untimed steps
with every stage bracketed and a `cpu_baseline` object (the C oracle on the host
cores, bounded sample, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
CLOCK_HZ = 2.4e9  # max clock (MI355X_MICROARCH.md chip table)
SIMDS = 256 * 4  # 256 CUs x 4 SIMD-32
# VALU issue peak (MI355X_MICROARCH.md, per-instruction cycle constants): a wave64 VALU instruction
# occupies its SIMD-32 for 2 cycles when waves interleave (one wave alone: 4); a transcendental
# (v_exp / v_rsq / v_rcp / v_sqrt / v_log) twice that (one wave alone: 8).  The box's plain-fp32 code
# does not reach it (tools/probe/valu_rate.hip, profiles/r4_valu_rate_probe.txt: 4.41 cycles per
# instruction at best), so `roofline.bound` is decided by the measured VALU pipe occupancy
# (SQ_ACTIVE_INST_VALU, in 4-cycle units, over the launch's SIMD-cycles), not by this peak.
VALU_PEAK_CYCLES = 2
TRANS_PEAK_CYCLES = 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launcher_cmd(argv, nproc: int, port: int):
    """The torch.distributed.run command that runs this bench with one rank
    per GPU (the driver's own launch line), for `bench.py
    --gpus N` started without a launcher."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def free_port() -> int:
    """A free port for the launcher's rendezvous, outside the kernel's ephemeral range (a port picked by
    binding to 0 is ephemeral, and outgoing connections can take it again before the launcher binds it)."""
    import random
    import socket

    lo = 32768
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        pass
    rng = random.Random()
    for _ in range(256):
        p = rng.randrange(10000, max(10001, lo))
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_launch(args, env=None):
    """-> None when this process is the bench itself (WORLD_SIZE matches
    --gpus, or N = 1), else the child command that launches N ranks.
    Raises SystemExit on a WORLD_SIZE / --gpus mismatch (a launcher that
    started another number of ranks than asked for)."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; launch one rank per GPU "
                             f"(torch.distributed.run --nproc-per-node {args.gpus}) or pass --gpus {ws}")
        return None
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if args.gpus == 1:
        return None
    return launcher_cmd(sys.argv[1:], args.gpus, free_port())


def launch_ranks(cmd, args) -> int:
    """Run the N-rank bench as a child process (never exec: nothing here has
    touched the GPU yet, and the child initialises it per rank) and relay its
    output; rank 0 prints the JSON line."""
    import subprocess

    # (no GPU API here: the device check runs in the ranks, check_devices)
    log("[bench] launching", " ".join(cmd))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def check_devices(args, world: int) -> None:
    """In each rank, before it touches the GPU: RCCL refuses two ranks on one
    device, so an N-rank RCCL bench needs N visible devices (device_count()
    does not initialise the GPU on this image)."""
    if world > 1 and args.dist_backend == "nccl":
        ndev = torch.cuda.device_count()
        if ndev < world:
            raise SystemExit(f"bench.py: --gpus {world} with RCCL needs {world} devices, {ndev} visible "
                             "(RCCL refuses two ranks on one device; --dist-backend gloo rehearses N ranks on one GPU)")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["C2", "C3", "C5"], default="C3",
                    help="C3: 1M Gaussians, SH 3 (the metric's config); C5: 5M Gaussians, SH 3 + SG 7; "
                         "C2: 100k Gaussians, 800x800, forward only")
    ap.add_argument("--P", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--forward-only", action="store_true", help="time the forward alone (C2's workload)")
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--sg-degree", type=int, default=None)
    ap.add_argument("--no-depth", action="store_true", help="require_depth=False (iterations < 7000)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", choices=["overlap", "factored", "allreduce"], default="overlap",
                    help="N > 1: gradient exchange: gsr_dist.OverlappedViewGrads (inside the backward, range by "
                         "range), FactoredViewGrads (after it), or an all-reduce of every row")
    ap.add_argument("--chunks", type=int, default=4, help="--exchange overlap: Gaussian ranges per backward")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: nccl (= RCCL over xGMI, the measured path); gloo only to rehearse the N > 1 "
                         "protocol with several ranks on one GPU (RCCL refuses two ranks on one device)")
    ap.add_argument("--cpu-tile-stride", type=int, default=0, help="0 = auto")
    ap.add_argument("--stage-steps", type=int, default=5,
                    help="untimed steps with every stage bracketed by hipEvents (the per-stage table)")
    ap.add_argument("--e2e", action="store_true",
                    help="time the whole training iteration after iteration 7000 (train.py:142-262: render, "
                         "depth-normal, PatchMatch with sample_depth + NCC, SSIM, backward, densification "
                         "statistics, Adam) instead of the raster alone; one line with a per-component breakdown")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)  # tests: ranks report and exit
    ap.add_argument("--all-stage-events", action="store_true",
                    help="bracket every stage with hipEvents inside the timed region too (each event pair "
                         "idles the stream ~10 us; default: only the dominant stage)")
    a = ap.parse_args()
    preset = {"C2": (100_000, 0, 800, 800), "C3": (1_000_000, 0, 1920, 1080), "C5": (5_000_000, 7, 1920, 1080)}[a.config]
    a.P = preset[0] if a.P is None else a.P
    a.sg_degree = preset[1] if a.sg_degree is None else a.sg_degree
    a.width = preset[2] if a.width is None else a.width
    a.height = preset[3] if a.height is None else a.height
    a.forward_only = a.forward_only or a.config == "C2"
    # PMC counters in profiles/ are per workload: pmc_<key>.json written by tools/pmc_summary.py
    a.preset_workload = (a.P, a.sg_degree, a.width, a.height) == preset and a.sh_degree == 3
    a.workload_key = a.config + ("-nodepth" if a.no_depth else "") + (
        "-fwd" if a.forward_only and a.config != "C2" else "")
    return a


def row_entries(plist, ranges, grid_x):
    """The tile lists' row entries (one (Gaussian, column span) entry per Gaussian and tile
    row it has a live tile in), counted from the final lists: the distinct (Gaussian, tile row) pairs."""
    import numpy as np

    n = ranges[:, 1].astype(np.int64) - ranges[:, 0].astype(np.int64)
    rows = np.repeat(np.arange(len(ranges), dtype=np.int64) // grid_x, n)
    live = np.concatenate([plist[a:b] for a, b in ranges.astype(np.int64) if b > a]) if n.sum() else np.zeros(0, np.uint32)
    key = live.astype(np.int64) * (int(rows.max()) + 1 if len(rows) else 1) + rows
    return int(np.unique(key).size)


def stage_bytes(P, K, K_live, HW, shm, sgm, geom, K_contrib=None, E_rows=None):
    """Algorithmic (compulsory) HBM bytes per launch of each stage, from the
    per-unit figures of SURVEY.md §8(d).  K is the reference's instance count
    (rect tiles); the binning stages produce the K_live instances that survive
    tile culling.  The raster kernels read each tile's list
    only up to its max contributor (the last position any pixel blended: the
    backward's loop bound, the forward's saturation point), so their gather
    unit count is K_contrib = sum over tiles of max_contrib (None: K_live,
    the upper bound of SURVEY §8(d)'s formula).  tile_lists counts the two
    counting passes' own traffic: per Gaussian the q-order index
    (4 B), the 32-B footprint gathered by the rows pass and its 32-B row
    record written and read back; per row entry (E_rows: Gaussian, column
    span, 8 B) one write and two reads (tiles count, tiles emit); per live
    instance the 4-B point-list write."""
    K_r = K_live if K_contrib is None else K_contrib
    Bp = 44 + 12 * shm + 28 * sgm
    G = 64 if geom else 36
    Opx = 36 if geom else 20
    Ipx = 56 if geom else 24
    A = 68 if geom else 40
    return {
        "preprocess": P * (Bp + 80),
        "depth_order": P * 36,  # splat rect/conic read, depth sort (key, index) in and out, counts gathered
        "scan": P * 16,
        "emit_keys": P * 36 + K_live * 6,
        "sort": K_live * 12,
        "tile_ranges": K_live * 2,
        # q-ordered Gaussians (index + splat rect/conic + radius) in, per-tile lists out
        "tile_lists": P * (4 + 32 + 32 + 32) + (E_rows or 0) * 24 + K_live * 4,
        "render_fwd": K_r * (4 + G) + HW * Opx,
        "bwd_clear": P * A,
        "render_bwd": HW * Ipx + K_r * (4 + G),
        # accumulators, geometry rows (44 B), the forward-saved colour -> direction Jacobian (36 B, in place
        # of the SH row) and the SG lobe rows, radii + clamped; every gradient row written
        "preprocess_bwd": P * (A + 44 + 36 + 28 * sgm + 8 + Bp),
    }


def load_pmc(workload_key, kernel_stage):
    """(HBM bytes per launch, VALU and transcendental VALU instructions per launch, file) of
    `kernel_stage` from profiles/pmc_<workload_key>.json (written by
    tools/profile.sh + tools/pmc_summary.py from separate rocprofv3 --pmc
    passes of this same workload, gfx950 FETCH_SIZE x2 correction applied)."""
    name = f"pmc_{workload_key}.json"
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            st = json.load(f)["stages"][kernel_stage]
        sq = st.get("sq_per_call", {})
        return (st["hbm_bytes_per_launch"], sq.get("SQ_INSTS_VALU"), sq.get("SQ_INSTS_VALU_TRANS_F32"),
                sq.get("SQ_ACTIVE_INST_VALU"), name)
    except Exception:  # noqa: BLE001 - absent summary -> null
        return None, None, None, None, None


def host_cores():
    """The CPU cores this process may use: its affinity set, capped by the
    cgroup CPU quota (a GPU box shares a larger machine; os.cpu_count() shows
    every CPU of the machine)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except Exception:  # noqa: BLE001 - no cgroup v2 quota
        pass
    return (min(n, quota) if quota else n), {"nproc": os.cpu_count(), "affinity": n, "cgroup_quota_cores": quota}


def getter_baseline(raw, cores):
    """The reference's Python preprocess path on the host cores: the
    GaussianModel getters (scene/gaussian_model.py:146-212, restated in
    gsr_scene.activated_inputs) over the workload's Gaussians in torch on
    the CPU, median of 5 calls."""
    import gsr_scene as S

    torch.set_num_threads(cores)
    times = []
    with torch.no_grad():
        for _ in range(6):
            t0 = time.perf_counter()
            S.activated_inputs(raw)
            times.append(time.perf_counter() - t0)
    ms = sorted(times[1:])[2] * 1e3
    return {"ms_per_call": round(ms, 3), "calls_per_s": round(1e3 / ms, 3), "threads": cores,
            "what": "torch-CPU GaussianModel getters (gaussian_model.py:146-212) over all P Gaussians"}


def cpu_baseline(args, inputs_cpu, cam, tanx, tany, grads_cpu, raw):
    """Time the C oracle (tests' checker) on this host's cores: full
    per-Gaussian work and binning, every s-th tile rendered forward and
    backward, tile time extrapolated x s; plus the torch-CPU getter leg."""
    sys.path.insert(0, ROOT)
    from oracle import gsr_oracle as O

    cores, host = host_cores()
    O.set_threads(cores)
    tiles = ((args.width + 15) // 16) * ((args.height + 15) // 16)
    stride = args.cpu_tile_stride or 1  # default: the whole iteration, no extrapolation
    O.set_tile_stride(stride)
    geom = not args.no_depth
    a = (torch.zeros(3), inputs_cpu["means3D"], None, inputs_cpu["opacities"], inputs_cpu["scales"],
         inputs_cpu["rotations"], None, inputs_cpu["shs"], inputs_cpu["sg_axis"], inputs_cpu["sg_sharpness"],
         inputs_cpu["sg_color"], args.sh_degree, args.sg_degree, 1.0, cam.world_view_transform,
         cam.full_proj_transform, tanx, tany, 0.0)
    t0 = time.time()
    o = O.forward(*a, args.height, args.width, cam.camera_center, False, geom)
    tf = O.last_times()
    tb = dict(render_bwd=0.0, preprocess_bwd=0.0)
    if not args.forward_only:
        O.backward(o["state"], *a, grads_cpu["color"], grads_cpu["mdepth"], grads_cpu["alpha"], grads_cpu["normal"],
                   o["alpha"], o["normal"], o["mdepth"], cam.camera_center, o["radii"])
        tb = O.last_times()
    wall = time.time() - t0
    O.set_tile_stride(1)
    per_iter = tf["preprocess_binning"] + stride * tf["render"] + stride * tb["render_bwd"] + tb["preprocess_bwd"]
    what = "forward" if args.forward_only else "forward+backward"
    return {"value": round(1.0 / per_iter, 6), "unit": "iters/s", "cores": cores, "kind": "port", "host": host,
            "sample": (f"C oracle (oracle/gsr_oracle.c, OpenMP, {cores} threads), full {args.config} scene, {what}: "
                       f"per-Gaussian preprocess, binning/sort and per-Gaussian backward measured in full; tile "
                       f"rendering on every {stride}th of {tiles} tiles, extrapolated x{stride}; {wall:.1f} s wall; "
                       f"split s: {tf['preprocess_binning']:.2f} pre+bin, {tf['render'] * stride:.2f} render, "
                       f"{tb['render_bwd'] * stride:.2f} render_bwd, {tb['preprocess_bwd']:.2f} pre_bwd"),
            "getters": getter_baseline(raw, cores)}


def exchange_pattern(mode, P, shm, sgm, world, chunks, dev):
    """The collectives one step of the view-parallel exchange posts (gsr_dist),
    on buffers of the same sizes, for timing the exchange alone.  Returns
    (post() -> works, bus bytes per rank per step): ring all-reduce moves
    2 (N-1)/N of its payload per rank, all-gather (N-1)/N of its output."""
    f = dict(dtype=torch.float32, device=dev)
    geo = torch.zeros(P * 11, **f)  # means3D 3 + opacity 1 + scales 3 + rotations 4
    dc = torch.zeros(P * 3, **f)
    gathered = torch.empty(P * 3 * world, **f)
    full = torch.zeros(P * (11 + 3 * shm + 7 * sgm), **f)
    ring = (world - 1) / world
    if mode == "allreduce":
        def post():
            return [dist.all_reduce(full, async_op=True)]
        return post, 2 * ring * full.numel() * 4
    cs = ((P + chunks - 1) // chunks + 255) // 256 * 256 if mode == "overlap" else P
    # one all-reduce of the geometry rows and one all-gather of the DC rows per Gaussian range
    def post():
        ws = []
        for b in range(0, P, cs):
            e = min(P, b + cs)
            ws.append(dist.all_reduce(geo[11 * b:11 * e], async_op=True))
            ws.append(dist.all_gather_into_tensor(gathered[3 * world * b:3 * world * e], dc[3 * b:3 * e],
                                                  async_op=True))
        return ws
    return post, (2 * ring * geo.numel() + ring * gathered.numel()) * 4


def _max_over_ranks(t):
    """MAX over the ranks in place (gsr_dist's collective: RCCL on the device; the gloo rehearsal staged
    through host memory, as gsr_dist does for every gloo collective on device tensors)."""
    from gsr_dist import _all_reduce
    _all_reduce(t, dist.ReduceOp.MAX, None)


def time_exchange(mode, P, shm, sgm, world, chunks, dev, reps=10):
    post, bus_bytes = exchange_pattern(mode, P, shm, sgm, world, chunks, dev)
    for _ in range(2):
        for w in post():
            w.wait()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        for w in post():
            w.wait()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / reps * 1e3
    t = torch.tensor([ms], device=dev, dtype=torch.float64)
    _max_over_ranks(t)
    ms = float(t.item())
    return {"isolated_ms": round(ms, 4), "bus_bytes_per_rank": int(bus_bytes),
            "bus_GBps": round(bus_bytes / (ms * 1e-3) / 1e9, 2)}


# the e2e step's SAMPLE raster (render_fwd_kernel<SAMPLE>) as its rocprofv3 kernel name (tools/pmc_summary.py)
SAMPLE_KERNEL = "render_fwd_kernel<true, false, true>"


def sample_fwd_bytes(cap):
    """Algorithmic bytes of one SAMPLE-raster launch (stage sample_fwd) from a captured
    sample_rasterized_depth call (_C.CAPTURE_SAMPLE): per tile, its list read once up to the
    largest last contributor of its points (4-B id + the 48-B record words the raster stages),
    and per point in view 12 B in (projected xy, |p_view|) + 26 B out (the point, inside, median
    depth, last contributor, dT/dt_m and its flag).  Returns (bytes, list entries, points)."""
    from diff_gaussian_rasterization import _C

    pts = cap["points3D"].detach().reshape(-1, 3).float()
    out = cap["out"]
    PN = pts.shape[0]
    _, last = _C.debug_sample_points(out[7], PN)
    W, H = cap["W"], cap["H"]
    ph = torch.cat([pts, torch.ones(PN, 1, device=pts.device)], 1) @ cap["projmatrix"].float()
    ndc = (ph[:, :2] / (ph[:, 3:4] + 1e-7)).double()
    tx = torch.floor((((ndc[:, 0] + 1.0) * W - 1.0) * 0.5 + 0.5) / 16.0).long()  # rasterizer_impl.cu:127-131
    ty = torch.floor((((ndc[:, 1] + 1.0) * H - 1.0) * 0.5 + 0.5) / 16.0).long()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    m = out[4].reshape(-1) & (tx >= 0) & (tx < gx) & (ty >= 0) & (ty < gy)
    lt = torch.from_numpy(last.astype("int64")).to(pts.device)
    maxl = torch.zeros(gx * gy, dtype=torch.int64, device=pts.device).scatter_reduce(
        0, (ty * gx + tx)[m], lt[m], reduce="amax")
    entries, n_in = int(maxl.sum()), int(m.sum())
    return entries * (4 + 48) + n_in * 38, entries, n_in


def e2e_cpu_baseline(args, ts, view, nearest, cap):
    """The training iteration's work on the host cores, component by component, on the same
    state: the torch-CPU getters (gaussian_model.py:146-212), the C oracle's raster forward +
    backward of the view (tile stride as bench.py's cpu_baseline) and sample_depth forward +
    backward of the PatchMatch points from the nearest view, the oracle's warp_patch_ncc over
    every pixel, the SSIM and depth-to-normal losses forward + backward in torch-CPU
    (oracle/ssim_ref.py, fp32), and one torch-CPU Adam step over the parameters.  The value is
    1 / (sum of the component times): a sum of measured components, not one chained run."""
    sys.path.insert(0, ROOT)
    import gsr_scene as S
    from oracle import gsr_oracle as O
    from oracle import ssim_ref as SR

    cores, host = host_cores()
    torch.set_num_threads(cores)
    O.set_threads(cores)
    g = ts.g
    raw = S.RawGaussians(*[getattr(g, "_" + f).detach().cpu() if f != "filter_3D" else g.filter_3D.detach().cpu()
                           for f in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity",
                                     "sg_axis", "sg_sharpness", "sg_color", "filter_3D")])
    sec = {}
    gb = getter_baseline(raw, cores)
    sec["getters"] = gb["ms_per_call"] * 1e-3
    inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    W, H = args.width, args.height
    cam = lambda v: (v.world_view_transform.cpu(), v.full_proj_transform.cpu(), v.camera_center.cpu(),  # noqa: E731
                     math.tan(v.FoVx / 2), math.tan(v.FoVy / 2))
    wv, fp, cc, tx_, ty_ = cam(view)
    stride = args.cpu_tile_stride or 1
    O.set_tile_stride(stride)
    a = (torch.zeros(3), inp["means3D"], None, inp["opacities"], inp["scales"], inp["rotations"], None, inp["shs"],
         inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], args.sh_degree, args.sg_degree, 1.0, wv, fp, tx_, ty_,
         0.0)
    gr = S.upstream_grads(H, W)
    o = O.forward(*a, H, W, cc, False, True)
    tf = O.last_times()
    O.backward(o["state"], *a, gr["color"], gr["mdepth"], gr["alpha"], gr["normal"], o["alpha"], o["normal"],
               o["mdepth"], cc, o["radii"])
    tb = O.last_times()
    O.set_tile_stride(1)
    sec["render"] = tf["preprocess_binning"] + stride * tf["render"] + stride * tb["render_bwd"] + tb["preprocess_bwd"]
    del o
    nwv, nfp, ncc_, ntx, nty = cam(nearest)
    pts = cap["points3D"].detach().cpu().float()
    t0 = time.perf_counter()
    so = O.sample_forward(pts, inp["means3D"], inp["opacities"], inp["scales"], inp["rotations"], 1.0, None, nwv, nfp,
                          ntx, nty, 0.0, H, W, ncc_, False)
    O.sample_backward(so["state"], pts, inp["means3D"], inp["opacities"], inp["scales"], inp["rotations"], 1.0, None,
                      nwv, nfp, so["inside"], torch.randn(pts.shape) * 1e-2, ntx, nty, 0.0)
    sec["sample_depth"] = time.perf_counter() - t0
    del so
    # warp_patch_ncc at every pixel (the step computes it at the geometrically consistent ones)
    ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    uvs = torch.stack([xs.reshape(-1), ys.reshape(-1)], 1).int()
    dep = torch.full((H * W,), 5.0)
    nrm = torch.tensor([0.0, 0.0, -1.0]).expand(H * W, 3).contiguous()
    wr, wn = view.world_view_transform.cpu(), nearest.world_view_transform.cpu()
    r_rel = wn[:3, :3].T @ wr[:3, :3]
    t_rel = -r_rel @ wr[3, :3] + wn[3, :3]
    gray = lambda v: (0.299 * v.original_image[0] + 0.587 * v.original_image[1] + 0.114 * v.original_image[2]).cpu()  # noqa: E731
    t0 = time.perf_counter()
    O.warp_patch_ncc(dep, nrm, uvs, r_rel.T.contiguous(), t_rel, gray(view), gray(nearest), view.Fx, view.Fy, view.Cx,
                     view.Cy, nearest.Fx, nearest.Fy, nearest.Cx, nearest.Cy)
    sec["ncc"] = time.perf_counter() - t0
    img = view.original_image.cpu()[None].clone().requires_grad_(True)
    gt = (img.detach() * 0.9 + 0.05)
    t0 = time.perf_counter()
    loss = 0.8 * (img - gt).abs().mean() + 0.2 * (1.0 - SR.ssim(img, gt, padding="valid"))
    loss.backward()
    sec["l1_ssim"] = time.perf_counter() - t0
    d = torch.full((1, H, W), 5.0, requires_grad=True)
    t0 = time.perf_counter()
    n_, _ = SR.depth_to_normal(d, view.Fx, view.Fy, view.Cx, view.Cy)
    n_.sum().backward()
    sec["depth_normal"] = time.perf_counter() - t0
    ps = [torch.zeros(p.shape, requires_grad=True) for p in g.parameters() if p.numel()]
    for q in ps:
        q.grad = torch.ones_like(q)
    opt = torch.optim.Adam(ps, lr=1e-3, eps=1e-15)
    opt.step()
    t0 = time.perf_counter()
    opt.step()
    sec["adam"] = time.perf_counter() - t0
    total = sum(sec.values())
    return {"value": round(1.0 / total, 6), "unit": "iters/s", "cores": cores, "kind": "port", "host": host,
            "sample": ("one training iteration's components on the host cores, summed: "
                       + ", ".join(f"{k} {v:.2f} s" for k, v in sec.items())
                       + f" (raster tiles every {stride}th, extrapolated; C oracle and torch-CPU)"),
            "component_s": {k: round(v, 4) for k, v in sec.items()}}


def run_e2e(args, dev):
    """bench.py --e2e: one training iteration (gsr_train.TrainStep) per step."""
    import gsr_train
    from diff_gaussian_rasterization import _C

    W, H, P = args.width, args.height, args.P
    ts, view, nearest = gsr_train.synthetic_training_setup(P, W, H, args.sh_degree, args.sg_degree, device=dev)
    for _ in range(args.warmup):
        ts.step(view, nearest)
    torch.cuda.synchronize(dev)
    comps = {k: [] for k in ts.COMPONENTS}
    ts.timing = True
    for _ in range(max(1, args.stage_steps)):
        ts.step(view, nearest)
        for k, v in ts.component_ms().items():
            comps[k].append(v)
    ts.timing = False
    # the library's stages per step (untimed steps, every stage bracketed); the dominant one is the roofline's
    _C.timing_collect()
    _C.timing_stages(None)
    _C.timing_enable(True)
    for _ in range(max(1, args.stage_steps)):
        ts.step(view, nearest)
    torch.cuda.synchronize(dev)
    _C.timing_enable(False)
    table = {k: ms / max(1, args.stage_steps) for k, (ms, n) in _C.timing_collect().items() if n}
    dom = max(table, key=table.get)
    _C.timing_stages([dom])
    _C.timing_enable(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = ts.step(view, nearest)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    _C.timing_enable(False)
    _C.timing_stages(None)
    dom_ms, dom_n = _C.timing_collect()[dom]
    ms = elapsed / args.steps * 1e3
    # one more step with the sample_depth call captured (its points and per-point last contributors)
    _C.CAPTURE_SAMPLE = True
    try:
        ts.step(view, nearest)
        torch.cuda.synchronize(dev)
        cap = _C.last_sample
    finally:
        _C.CAPTURE_SAMPLE = False
        _C.last_sample = None
    roofline = None
    if dom == "sample_fwd" and cap is not None:
        nbytes, entries, n_in = sample_fwd_bytes(cap)
        launch_ms = dom_ms / max(1, dom_n)
        achieved = nbytes / (launch_ms * 1e-3) / 1e9
        traffic = pipe_busy = valu_insts = None
        pmc_file = None
        if args.preset_workload:
            try:
                with open(os.path.join(ROOT, "profiles", "pmc_e2e.json")) as f:
                    kt = json.load(f)["kernels"][SAMPLE_KERNEL]
                traffic, valu_insts = kt.get("hbm_bytes"), kt.get("valu_insts")
                if kt.get("valu_active"):
                    pipe_busy = kt["valu_active"] * 4 / (launch_ms * 1e-3 * CLOCK_HZ * SIMDS)
                pmc_file = "profiles/pmc_e2e.json"
            except Exception:  # noqa: BLE001 - no e2e PMC summary yet -> null
                pass
        hbm_frac = achieved / HBM_PEAK_GBPS
        roofline = {"bound": "valu" if pipe_busy is not None and pipe_busy > hbm_frac else "hbm", "kernel": dom,
                    "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(hbm_frac, 5), "traffic": traffic, "algorithmic_bytes_per_launch": int(nbytes),
                    "algorithmic_units": (f"per tile its list read once up to the largest last contributor of its "
                                          f"points ({entries} entries) x (4 + 48) B + {n_in} points in view x 38 B"),
                    "avg_launch_ms": round(launch_ms, 4),
                    "valu": None if pipe_busy is None else {"pipe_busy": round(pipe_busy, 4),
                                                           "insts_per_launch": valu_insts,
                                                           "pipe_busy_source": "SQ_ACTIVE_INST_VALU x 4 / SIMD-cycles "
                                                                               "of the live launch time"},
                    "pmc_source": pmc_file, "pmc_kernel": SAMPLE_KERNEL,
                    "stage_ms_per_step": {k: round(v, 4) for k, v in table.items()}}
    elif table:
        roofline = {"kernel": dom, "achieved": None, "note": f"dominant stage {dom}: no e2e byte model for it",
                    "stage_ms_per_step": {k: round(v, 4) for k, v in table.items()}}
    cpu = None
    if not args.no_cpu_baseline and cap is not None:
        try:
            cpu = e2e_cpu_baseline(args, ts, view, nearest, cap)
        except Exception as e:  # noqa: BLE001 - report, never hide
            cpu = {"value": None, "error": repr(e)}
    line = {
        "metric": "train iters/sec (full training iteration after iteration 7000) at 1080p, 1M Gaussians",
        "value": round(args.steps / elapsed, 3), "unit": "iters/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (ground truth: renders of perturbed Gaussians)",
        "config": {"workload": (f"e2e {args.config}: {P} Gaussians (SH {args.sh_degree}, SG {args.sg_degree}), "
                                f"{W}x{H}, train.py:142-262 after iteration 7000: getters, render(require_depth), "
                                "L1 + fused SSIM, depth_to_normal loss, PatchMatch (sample_depth from the nearest "
                                "view + geometric loss + warp_patch_ncc), backward, densification statistics, "
                                "FusedAdam step"),
                   "P": P, "width": W, "height": H, "loss": float(loss)},
        "components_ms": {k: round(sorted(v)[len(v) // 2], 4) for k, v in comps.items()},
        "roofline": roofline, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    cmd = check_launch(args)
    if cmd is not None:
        sys.exit(launch_ranks(cmd, args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_probe:  # (tests/test_bench_launch.py: the launch wiring on CPU, no GPU touched)
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.tensor([rank + 1])
            dist.all_reduce(t)
            ranks = int(t.item())
            dist.destroy_process_group()
        else:
            ranks = 1
        if rank == 0:
            print(json.dumps({"n_gpus": world, "rank_sum": ranks}), flush=True)
        return
    check_devices(args, world)
    # (a rehearsal with more ranks than GPUs shares the devices; device_count() does not initialise the GPU)
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    if args.e2e:
        if world > 1:
            raise SystemExit("bench.py --e2e runs on one GPU")
        return run_e2e(args, dev)
    if world > 1:
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from diff_gaussian_rasterization import _C

    W, H, P = args.width, args.height, args.P
    geom = not args.no_depth
    if world > 1:
        cam_cpu = S.orbit_cameras(8, W, H)[rank % 8]
        tag = "C4" if args.config == "C3" else "C5"
        workload = f"{tag}: {P} Gaussians (SH {args.sh_degree}, SG {args.sg_degree}), one {W}x{H} view per GPU (orbit), fwd+bwd + RCCL gradient exchange ({args.exchange})"
    else:
        cam_cpu = S.make_camera(W, H)
        what = "forward only" if args.forward_only else "fwd+bwd"
        workload = (f"{args.config}: {P} Gaussians (SH {args.sh_degree}, SG {args.sg_degree}), {W}x{H}, {what}, "
                    f"require_depth={geom}")
    raw = S.make_gaussians(P, sh_degree=args.sh_degree, sg_degree=args.sg_degree, aspect=H / W)
    inputs_cpu = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    grads_cpu = S.upstream_grads(H, W)
    cam = cam_cpu.to(dev)
    tanx, tany = math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5)
    params = {k: v.to(dev).requires_grad_(True) for k, v in inputs_cpu.items()}
    means2D = torch.zeros(P, 3, device=dev, requires_grad=True)
    g_color = grads_cpu["color"].to(dev)
    g_mdepth = grads_cpu["mdepth"].to(dev)
    g_normal = grads_cpu["normal"].to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=tanx, tanfovy=tany, kernel_size=0.0, bg=torch.zeros(3, device=dev),
        scale_modifier=1.0, viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform,
        sh_degree=args.sh_degree, sg_degree=args.sg_degree, campos=cam.camera_center, prefiltered=False,
        require_depth=geom, debug=False)
    rasterizer = GaussianRasterizer(settings)
    grad_keys = ["means3D", "shs", "sg_axis", "sg_sharpness", "sg_color", "opacities", "scales", "rotations"]
    reducer = exchanger = overlap = None
    if world > 1 and args.exchange == "overlap":  # the exchange rides inside every rasterizer backward
        from gsr_dist import OverlappedViewGrads
        overlap = OverlappedViewGrads(chunks=args.chunks).install()
    elif world > 1 and args.exchange == "allreduce":
        from gsr_dist import ViewParallelGrads
        reducer = ViewParallelGrads([params[k] for k in grad_keys])
    elif world > 1:  # colour rows rebuilt from the all-gathered DC rows (gsr_dist.FactoredViewGrads)
        from gsr_dist import FactoredViewGrads
        exchanger = FactoredViewGrads(params["means3D"], params["opacities"], params["scales"], params["rotations"],
                                      params["shs"], params["sg_axis"], params["sg_sharpness"], params["sg_color"])
    state = {}

    def step():
        if args.forward_only:  # the forward alone: no autograd graph, nothing saved for a backward
            with torch.no_grad():
                state["radii"] = rasterizer(
                    means3D=params["means3D"], means2D=means2D, opacities=params["opacities"], shs=params["shs"],
                    sg_axis=params["sg_axis"], sg_sharpness=params["sg_sharpness"], sg_color=params["sg_color"],
                    scales=params["scales"], rotations=params["rotations"])[1]
            return
        for t in list(params.values()) + [means2D]:
            t.grad = None
        color, radii, mdepth, alpha, normal = rasterizer(
            means3D=params["means3D"], means2D=means2D, opacities=params["opacities"], shs=params["shs"],
            sg_axis=params["sg_axis"], sg_sharpness=params["sg_sharpness"], sg_color=params["sg_color"],
            scales=params["scales"], rotations=params["rotations"])
        outs, gs = [color], [g_color]
        if geom:
            outs += [mdepth, normal]
            gs += [g_mdepth, g_normal]
        torch.autograd.backward(outs, gs)
        if state.get("no_exchange"):
            return
        if reducer is not None:  # view-parallel gradient exchange
            reducer.all_reduce()
        if exchanger is not None:
            exchanger.exchange(cam.camera_center, args.sh_degree, args.sg_degree)
        state["radii"] = radii

    log(f"[bench] rank {rank}/{world} device {torch.cuda.get_device_name(dev)} P={P} {W}x{H} geom={geom}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # per-stage table: a few untimed steps with every stage bracketed by events
    _C.timing_collect()  # discard
    _C.timing_stages(None)
    _C.timing_enable(True)
    for _ in range(max(1, args.stage_steps)):
        step()
    torch.cuda.synchronize(dev)
    _C.timing_enable(False)
    table = _C.timing_collect()
    table_ms = {k: (ms / n if n else 0.0) for k, (ms, n) in table.items()}
    dom = max(table_ms, key=lambda k: table_ms[k])
    # timed region: events only around the dominant stage (the roofline kernel)
    _C.timing_stages(None if args.all_stage_events else [dom])
    _C.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _C.timing_enable(False)
    _C.timing_stages(None)
    stages = _C.timing_collect()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        _max_over_ranks(t)
        elapsed = float(t.item())
    dist_info = None
    if world > 1:  # the exchange's cost: the same steps without it, and its collectives alone
        if overlap is not None:
            overlap.uninstall()
        state["no_exchange"] = True
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        _max_over_ranks(t)
        ms_noex = float(t.item()) / args.steps * 1e3
        state["no_exchange"] = False
        if overlap is not None:
            overlap.install()
        shm_ = (args.sh_degree + 1) ** 2
        iso = time_exchange(args.exchange, P, shm_, args.sg_degree, world, args.chunks, dev)
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "exchange": args.exchange,
                     "chunks": args.chunks if args.exchange == "overlap" else None,
                     "ms_per_step_without_exchange": round(ms_noex, 4),
                     "exposed_exchange_ms": round(elapsed / args.steps * 1e3 - ms_noex, 4), **iso}

    # K of this view (one extra forward, outside the timed region)
    with torch.no_grad():
        K = _C.rasterize_gaussians(settings.bg, params["means3D"], torch.Tensor([]), params["opacities"],
                                   params["scales"], params["rotations"], torch.Tensor([]), params["shs"],
                                   params["sg_axis"], params["sg_sharpness"], params["sg_color"], args.sh_degree,
                                   args.sg_degree, 1.0, cam.world_view_transform, cam.full_proj_transform, tanx,
                                   tany, 0.0, H, W, cam.camera_center, False, geom, False)[0]
    # instances that survive tile culling (the units the raster kernels process)
    with torch.no_grad():
        fo = _C.rasterize_gaussians(settings.bg, params["means3D"], torch.Tensor([]), params["opacities"],
                                    params["scales"], params["rotations"], torch.Tensor([]), params["shs"],
                                    params["sg_axis"], params["sg_sharpness"], params["sg_color"], args.sh_degree,
                                    args.sg_degree, 1.0, cam.world_view_transform, cam.full_proj_transform, tanx,
                                    tany, 0.0, H, W, cam.camera_center, False, geom, False)
        plist_, ranges_ = _C.debug_binning(fo[7], fo[9], fo[0], H, W, with_list=True)
        K_live = int(ranges_[:, 1].max())
        E_rows = row_entries(plist_, ranges_, (W + 15) // 16)
        del plist_, ranges_
        K_contrib = int(_C.debug_max_contrib(fo[9], H, W).astype("int64").sum())
    ms_per_step = elapsed / args.steps * 1e3
    value = world * args.steps / elapsed
    shm = (args.sh_degree + 1) ** 2
    algo = stage_bytes(P, K, K_live, W * H, shm, args.sg_degree, geom, K_contrib, E_rows)
    algo_upper = stage_bytes(P, K, K_live, W * H, shm, args.sg_degree, geom, None, E_rows)
    per_launch = {k: (ms / n if n else 0.0) for k, (ms, n) in stages.items()}
    if not args.all_stage_events:  # the other stages from the untimed table
        per_launch = {k: (per_launch[k] if k == dom else v) for k, v in table_ms.items()}
    achieved = algo[dom] / (per_launch[dom] * 1e-3) / 1e9
    traffic, valu_insts, trans_insts, valu_active, pmc_file = (
        load_pmc(args.workload_key, dom) if args.preset_workload else (None, None, None, None, None))
    hbm_frac = achieved / HBM_PEAK_GBPS
    # VALU-issue fraction of the same launch: the PMC pass's VALU instruction counts for this kernel
    # (per-launch constants of the workload) at their peak issue cost — 2 SIMD cycles per wave64
    # instruction, 4 per transcendental — over the SIMD-cycles of the launch duration measured live here
    simd_cycles = per_launch[dom] * 1e-3 * CLOCK_HZ * SIMDS
    valu_frac = pipe_busy = None
    if valu_insts:
        tr = trans_insts or 0
        valu_frac = (valu_insts * VALU_PEAK_CYCLES + tr * (TRANS_PEAK_CYCLES - VALU_PEAK_CYCLES)) / simd_cycles
    if valu_active:  # cycles the SIMDs' arbiters spent on VALU instructions (4-cycle units), measured
        pipe_busy = valu_active * 4 / simd_cycles
    # the bound is the measured pipe occupancy against the HBM fraction (the datasheet-rate fraction
    # understates what binds: the box issues plain fp32 at ~4.4 cycles, not 2)
    busy = pipe_busy if pipe_busy is not None else valu_frac
    bound = "valu" if busy is not None and busy > hbm_frac else "hbm"
    roofline = {"bound": bound, "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(hbm_frac, 5),
                "traffic": traffic, "algorithmic_bytes_per_launch": int(algo[dom]),
                "algorithmic_units": ("instances read up to each tile's max contributor (sum of max_contrib: "
                                      f"{K_contrib}) x (4 + {64 if geom else 36}) B + pixels x "
                                      f"{(36 if geom else 20) if dom == 'render_fwd' else (56 if geom else 24)} B"
                                      if dom in ("render_fwd", "render_bwd") else "SURVEY §8(d) per-unit bytes"),
                "upper_bound_bytes_per_launch": int(algo_upper[dom]),
                "avg_launch_ms": round(per_launch[dom], 4),
                "valu": None if valu_frac is None else {
                    "frac": round(valu_frac, 4), "insts_per_launch": int(valu_insts),
                    "trans_insts_per_launch": None if trans_insts is None else int(trans_insts),
                    "peak_cycles_per_inst": VALU_PEAK_CYCLES, "peak_cycles_per_trans": TRANS_PEAK_CYCLES,
                    "clock_hz": CLOCK_HZ, "simds": SIMDS,
                    "pipe_busy": None if pipe_busy is None else round(pipe_busy, 4),
                    "pipe_busy_source": "SQ_ACTIVE_INST_VALU x 4 / SIMD-cycles of the live launch time",
                    "bound_from": "pipe_busy" if pipe_busy is not None else "frac"},
                "pmc_source": None if pmc_file is None else f"profiles/{pmc_file}",
                "stage_ms": {k: round(v, 4) for k, v in per_launch.items()},
                "stage_algorithmic_bytes": {k: int(v) for k, v in algo.items() if per_launch.get(k, 0.0) > 0.0},
                "tile_list_row_entries": E_rows}
    total_algo = sum(v for k, v in algo.items() if per_launch.get(k, 0.0) > 0.0)  # the stages this step ran
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, inputs_cpu, cam_cpu, tanx, tany, grads_cpu, raw)
        except Exception as e:  # noqa: BLE001 - report, never hide
            cpu = {"value": None, "error": repr(e)}
    if rank == 0:
        line = {
            "metric": "train iters/sec (fwd+bwd raster) at 1080p, 1M Gaussians; HBM GB/s vs peak",
            "value": round(value, 3), "unit": "forward iters/s" if args.forward_only else "iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload, "P": P, "width": W, "height": H, "sh_degree": args.sh_degree,
                       "sg_degree": args.sg_degree, "require_depth": geom, "num_rendered": int(K), "instances_after_tile_culling": K_live,
                       "instances_to_max_contributor": K_contrib,
                       "parallelism": f"view-parallel dp{world}" if world > 1 else "single",
                       "step_algorithmic_GBps": round(total_algo / (ms_per_step * 1e-3) / 1e9, 2)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "dist": dist_info,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
