"""View-parallel training step: one process per GPU, RCCL over xGMI.

The reference trains on one GPU, one view per iteration (utils/general_utils.py:135,
train.py:142-192).  The MI355X build shards *views* across ranks (SURVEY §5,
§8(e)): every rank holds a full replica of the Gaussians, rasterises its own
view forward + backward with no communication, and the per-Gaussian gradients
are summed with all_reduce(SUM) — the only exchange step.  The step gradient is
then the sum over the ranks' views, i.e. the gradient of sum_v L_v.

By default (`inplace=True`) the .grad tensors are summed where they lie: one
coalesced all-reduce (a single RCCL group call over the per-parameter
gradients, every one of them MBs long) with no packing, so the step moves no
extra HBM bytes beyond the collective itself (packing into and out of a flat
bucket costs 4 x 236 MB of copies per step at 1M Gaussians / SH3).  With
`inplace=False` gradients are packed into a few large flat fp32 buckets
(bucket_mb, default 256 MB).  xGMI links are point-to-point, so few large
collectives keep every link busy.  With `async_op=True` the collective is
posted and `finish()` waits (and, for buckets, scatters the sums back into
the .grad tensors).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


def _host_staged(group, *tensors) -> bool:
    """gloo with device tensors (the one-GPU rehearsal of the N > 1 path; the product backend is RCCL):
    the collective is staged through host memory here, by blocking copies, instead of by the backend.
    torch's own staging of device tensors for gloo (an asynchronous copy into a pinned buffer on a side
    stream) was observed to hand the reduction stale data — at 8 ranks, 6 of 1200 trials of the
    exchange's pattern wrong without the rasterizer, always the first slice posted after the previous
    trial's works were dropped, identically on every rank; 0 of 1200 staged by blocking copies
    (tools/dbg/gloo_reuse_probe.py) — which is what the C4 test's rare wrong sum was."""
    return any(t.is_cuda for t in tensors) and dist.get_backend(group) == "gloo"


class _StagedWork:
    """An async collective on host copies: wait() waits for it, then copies the result back to the device
    tensor (stream-ordered on the caller's stream)."""

    def __init__(self, work, dst: torch.Tensor, host: torch.Tensor):
        self._work, self._dst, self._host = work, dst, host

    def wait(self):
        self._work.wait()
        if self._dst is not None:
            self._dst.copy_(self._host)
            self._dst = None
        return True


def _all_reduce(t: torch.Tensor, op, group, async_op: bool = False):
    if not _host_staged(group, t):
        return dist.all_reduce(t, op=op, group=group, async_op=async_op)
    h = t.cpu()  # (blocking: after the work queued on the stream before it)
    w = _StagedWork(dist.all_reduce(h, op=op, group=group, async_op=True), t, h)
    if async_op:
        return w
    w.wait()
    return None


def _all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group, async_op: bool = False):
    if not _host_staged(group, out, inp):
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    hi = inp.cpu()
    ho = torch.empty(out.shape, dtype=out.dtype)
    w = _StagedWork(dist.all_gather_into_tensor(ho, hi, group=group, async_op=True), out, ho)
    if async_op:
        return w
    w.wait()
    return None


def _coalescing(group, tensors):
    """torch's coalescing manager (one allreduce_coalesced for several
    tensors) where the backend has it for these tensors: RCCL does; gloo
    only for host tensors (gloo with device tensors is the one-GPU
    rehearsal of the N > 1 path).  None: one all_reduce per tensor."""
    cm_fn = getattr(dist, "_coalescing_manager", None)
    if cm_fn is not None and dist.get_backend(group) == "gloo" and any(t.is_cuda for t in tensors):
        return None
    return cm_fn


class ViewParallelGrads:
    def __init__(self, params: Iterable[torch.Tensor], bucket_mb: float = 256.0,
                 group: Optional[dist.ProcessGroup] = None, average: bool = False, inplace: bool = True):
        self.params: List[torch.Tensor] = [p for p in params if p.requires_grad]
        self.group = group
        self.average = average
        self.inplace = inplace
        self._cm = None
        cap = max(1, int(bucket_mb * 1024 * 1024 // 4))
        self.buckets: List[List[torch.Tensor]] = []
        cur, n = [], 0
        for p in self.params:
            if cur and n + p.numel() > cap:
                self.buckets.append(cur)
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        if cur:
            self.buckets.append(cur)
        self._flat: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._work = []

    def _pack(self, i: int) -> torch.Tensor:
        ps = self.buckets[i]
        n = sum(p.numel() for p in ps)
        dev = ps[0].device
        if self._flat[i] is None or self._flat[i].numel() != n or self._flat[i].device != dev:
            self._flat[i] = torch.empty(n, dtype=torch.float32, device=dev)
        flat = self._flat[i]
        off = 0
        for p in ps:
            k = p.numel()
            if p.grad is None:
                flat[off:off + k].zero_()
            else:
                flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        return flat

    def all_reduce(self, async_op: bool = False):
        """Sum every parameter's .grad over the ranks of the group."""
        cm_fn = _coalescing(self.group, self.params)
        self._work = []
        if self.inplace:
            grads = []
            for p in self.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                if p.numel():
                    grads.append(p.grad)
            if cm_fn is None or len(grads) < 2:
                for g in grads:
                    self._work.append((None, _all_reduce(g, dist.ReduceOp.SUM, self.group, async_op)))
            else:
                with cm_fn(group=self.group, async_ops=async_op) as cm:  # fast path: allreduce_coalesced
                    for g in grads:
                        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
                self._cm = cm if async_op else None
            if not async_op:
                self.finish()
            return
        for i in range(len(self.buckets)):
            flat = self._pack(i)
            w = _all_reduce(flat, dist.ReduceOp.SUM, self.group, async_op)
            self._work.append((i, w))
        if not async_op:
            self.finish()

    def finish(self):
        ws = dist.get_world_size(self.group) if self.average else 1
        if self.inplace:
            if self._cm is not None:
                self._cm.wait()
                self._cm = None
            for _, w in self._work:
                if w is not None:
                    w.wait()
            self._work = []
            if self.average:
                for p in self.params:
                    p.grad.div_(ws)
            return
        for i, w in self._work:
            if w is not None:
                w.wait()
            flat = self._flat[i]
            if self.average:
                flat.div_(ws)
            off = 0
            for p in self.buckets[i]:
                k = p.numel()
                src = flat[off:off + k].view_as(p)
                if p.grad is None:
                    p.grad = src.clone()
                else:
                    p.grad.copy_(src)
                off += k
        self._work = []

    @property
    def bucket_bytes(self) -> List[int]:
        return [4 * sum(p.numel() for p in b) for b in self.buckets]


class FactoredViewGrads:
    """The view-parallel gradient exchange with the colour rows factored.

    Per view, every SH / SG gradient row of a Gaussian is a function of three
    numbers — the clamp-masked dL/dRGB, which is dL/dsh[:, 0, :] / SH_C0 — and
    of the view direction (CR/render_backward.cu:56-191; view_grads.hip).  So
    instead of all-reducing those rows (192 B per Gaussian at SH 3, 388 B with
    SG 7), the ranks all-gather each view's DC row and camera centre (12 B per
    Gaussian per view, one collective) and every rank rebuilds the summed rows
    with one HIP kernel (gsr_view_color_grads, views summed in rank order, so
    the replicas stay bit-identical).  Only the geometry gradients (means3D,
    opacity, scales, rotations: 44 B per Gaussian) are all-reduced.  At 8
    ranks and SH 3 the xGMI bytes per rank drop from 2 * 7/8 * 236 MB = 413 MB
    (ring all-reduce of every row) to 2 * 7/8 * 44 + 7 * 12 = 161 MB per 1M
    Gaussians.

    `exchange(campos, sh_degree, sg_degree)` after the backward: `campos` is
    this rank's camera centre (the rasterizer settings' `campos`), the degrees
    are the active ones of that backward.  `expand` replaces the HIP kernel
    (same signature as `_C.view_color_grads`; CPU tests only).

    The SH rows may be the rasterizer's `shs` input or the reference's two
    parameters `(features_dc, features_rest)` (gaussian_model.py:165-169: the
    activation is a concatenation, so their .grad are the two slices of
    dL/dshs).  SG tensors must be the rasterizer inputs (the SG activations
    are not linear in the rows, so raw SG parameters go in `extra`, which is
    all-reduced with the geometry rows).

    Contract: between two exchanges this rank's SH / SG gradients come from
    exactly ONE rasterizer colour backward for the camera `campos` names —
    no accumulation over several renders, no gradients left over from a
    missing zero_grad, and no other loss or regularizer on the SH / SG rows.
    The rows are rebuilt from the DC row, so anything else that wrote into
    them would be silently replaced.  Two guards:
      * `guard` (default on with the HIP kernel): raise unless exactly one
        rasterizer SH backward ran since the previous exchange (a counter in
        diff_gaussian_rasterization; catches several renders per step);
      * `verify` (opt-in, one extra kernel per exchange): rebuild this rank's
        own rows from its own DC row and raise unless they equal the rows in
        .grad (catches stale gradients and extra SH / SG losses too).
    """

    def __init__(self, means3D: torch.Tensor, opacities: torch.Tensor, scales: torch.Tensor,
                 rotations: torch.Tensor, shs, sg_axis: Optional[torch.Tensor] = None,
                 sg_sharpness: Optional[torch.Tensor] = None, sg_color: Optional[torch.Tensor] = None,
                 group: Optional[dist.ProcessGroup] = None, expand=None, extra: Iterable[torch.Tensor] = (),
                 guard: Optional[bool] = None, verify: bool = False):
        self.means3D = means3D
        self.split = isinstance(shs, (tuple, list))
        self.shs = tuple(shs) if self.split else shs
        self.sg = [t if t is not None and t.numel() else None for t in (sg_axis, sg_sharpness, sg_color)]
        self.group = group
        self.geometry = ViewParallelGrads([means3D, opacities, scales, rotations, *extra], group=group)
        self.guard = (expand is None) if guard is None else guard
        self.verify = verify
        if expand is None:
            from diff_gaussian_rasterization import _C
            expand = _C.view_color_grads
        self.expand = expand
        self._buf = None
        self._gathered = None
        self._calls = self._backward_count() if self.guard else 0

    @staticmethod
    def _backward_count() -> int:
        import diff_gaussian_rasterization as dgr
        return dgr.colour_backward_count()

    def _check_contract(self, sh_degree: int, sg_degree: int) -> None:
        if self.guard:
            n = self._backward_count()
            ran, self._calls = n - self._calls, n
            if ran != 1:
                raise RuntimeError(f"FactoredViewGrads: {ran} rasterizer SH backwards since the last exchange; the "
                                   "factored exchange needs exactly one per step (use ViewParallelGrads otherwise)")
        if not self.verify:
            return
        mine = torch.cat([t.grad for t in self.shs], 1) if self.split else self.shs.grad
        rows = torch.empty_like(mine)
        sgo = [None if t is None else torch.empty_like(t) for t in self.sg]
        self.expand(self._buf, 1, self.means3D.detach(), sh_degree, rows, sg_degree,
                    *[None if t is None else t.detach() for t in self.sg], *sgo)
        pairs = [("sh", mine, rows)]
        for name, t, o in zip(("sg_axis", "sg_sharpness", "sg_color"), self.sg, sgo):
            if t is not None:
                pairs.append((name, torch.zeros_like(t) if t.grad is None else t.grad, o))
        for name, want, got in pairs:
            tol = 1e-5 * max(float(want.abs().max()), 1e-30) if want.numel() else 0.0
            if want.numel() and float((want - got).abs().max()) > tol:
                raise RuntimeError(f"FactoredViewGrads(verify): this rank's {name} gradient rows are not those of "
                                   "its one rasterizer backward (stale .grad or another loss on them?)")

    def exchange(self, campos: torch.Tensor, sh_degree: int, sg_degree: int = 0) -> None:
        world = dist.get_world_size(self.group)
        P = self.means3D.shape[0]
        for t in (self.shs if self.split else (self.shs,)):
            if t.grad is None:
                t.grad = torch.zeros_like(t)
        dev = self.means3D.device
        n = 3 * P + 4
        if self._buf is None or self._buf.numel() != n or self._buf.device != dev:
            self._buf = torch.zeros(n, dtype=torch.float32, device=dev)
            self._gathered = torch.empty(world * n, dtype=torch.float32, device=dev)
        dc = self.shs[0].grad if self.split else self.shs.grad
        self._buf[:3 * P].view(P, 3).copy_(dc[:, 0, :])
        self._buf[3 * P:3 * P + 3].copy_(campos.reshape(3))
        self._check_contract(sh_degree, sg_degree)
        work = _all_gather_into_tensor(self._gathered, self._buf, self.group, async_op=True)
        self.geometry.all_reduce()
        work.wait()
        sgo = []
        for t in self.sg:
            if t is not None and t.grad is None:
                t.grad = torch.zeros_like(t)
            sgo.append(None if t is None else t.grad)
        if self.split:
            dc_t, rest_t = self.shs
            rows = torch.empty(P, dc_t.shape[1] + rest_t.shape[1], 3, dtype=torch.float32, device=dev)
        else:
            rows = self.shs.grad
        self.expand(self._gathered, world, self.means3D.detach(), sh_degree, rows, sg_degree,
                    *[None if t is None else t.detach() for t in self.sg], *sgo)
        if self.split:
            k = dc_t.shape[1]
            dc_t.grad.copy_(rows[:, :k])
            rest_t.grad.copy_(rows[:, k:])


class OverlappedViewGrads:
    """The view-parallel gradient exchange run INSIDE each rasterizer
    backward, overlapped with its per-Gaussian tail ("chunk the
    preprocess-bwd over Gaussian ranges and post per-chunk all-reduces on a
    side stream").

    Installed (`install()` or `with OverlappedViewGrads(...):`), every
    _RasterizeGaussians backward runs its per-Gaussian backward in `chunks`
    Gaussian ranges (gsr_rasterize_backward_ex).  As each range is queued,
    this posts, asynchronously (RCCL runs them on its own stream, after the
    range's kernel, while the next range computes):
      * one coalesced all-reduce of the range's geometry gradients (means3D,
        opacity, scales + rotations or cov3D; colours when no SH is given);
      * one all-gather of the range's DC gradient rows (12 B per Gaussian;
        the kernel writes them to a compact [P][3] buffer and skips the SH /
        SG rows).
    Before the backward returns, its stream waits for the collectives and
    gsr_view_color_grads_chunked rebuilds every SH / SG row as the sum over
    the views (FactoredViewGrads' factorisation, the views summed in rank
    order on every rank, so the replicas stay bit-identical).  The gradients
    the rasterizer hands to autograd are then already summed over the
    ranks' views; autograd carries them through the getters as usual.

    Failure: a rank whose backward fails part-way posts its remaining
    ranges on NaN rows (no peer blocks) and re-raises.  Every backward ends
    with one more tiny all-reduce (MAX) of a failure flag on every rank, so
    the PEERS raise too ("a peer rank's rasterizer backward failed").  When
    they raise is `sync_check`'s choice:
      * False (the default for device tensors): the flag is copied to pinned
        host memory behind an event and read at the next `begin()` (the next
        rasterizer backward) or by an explicit `check()` — no host
        synchronisation per backward, so the host keeps queueing the rest of
        the backward and the optimizer step while the GPU works.  A training
        loop that must never apply a step with a failed peer calls `check()`
        before `optimizer.step()` (one wait on an event the GPU has long
        passed by then, since the step's gradients are complete);
      * True (the default for host tensors, where the read costs nothing):
        `finish()` reads the flag and raises in the same backward, at the
        price of one host synchronisation per backward after its last
        collective.

    Semantics: each rasterizer backward exchanges its own gradients, so
    several renders per step and gradient accumulation sum correctly (the
    exchange is linear).  Gradients of other loss terms on the same
    parameters are NOT exchanged: reduce those yourself (or compute them on
    every rank identically and scale).  means2D gradients (densification
    statistics) stay per view.  `expand` replaces the HIP rebuild kernel (same
    signature as _C.view_color_grads_chunked; CPU tests only).
    """

    def __init__(self, group: Optional[dist.ProcessGroup] = None, chunks: int = 4, expand=None,
                 sync_check: Optional[bool] = None):
        self.group = group
        self.sync_check = sync_check
        self._status = None  # one float per backward: MAX over the ranks of "this rank's backward failed"
        self._pending = None  # (pinned host copy of the flag, event) of the last backward, read by check()
        self.chunks = max(1, int(chunks))
        self.world = dist.get_world_size(group)
        if expand is None:
            from diff_gaussian_rasterization import _C
            expand = _C.view_color_grads_chunked
        self.expand = expand
        self._dc = self._gathered = None
        self._campos_local = self._campos_all = None
        self._works = []
        self._scales = self._sh = True
        self._P = self._cs = self._next = 0
        self._ar_done = False  # the current range's all-reduce is posted, its all-gather not yet
        self._active = False
        self._error = None

    # ---- installation -------------------------------------------------
    def install(self) -> "OverlappedViewGrads":
        import diff_gaussian_rasterization as dgr
        dgr.set_view_exchange(self)
        return self

    def uninstall(self) -> None:
        import diff_gaussian_rasterization as dgr
        if dgr._view_exchange is self:
            dgr.set_view_exchange(None)

    def __enter__(self):
        return self.install()

    def __exit__(self, *exc):
        self.uninstall()

    # ---- the rasterizer backward's protocol ---------------------------
    def dc_rows(self, P: int, device) -> torch.Tensor:
        """The compact [P * 3] DC-row buffer the kernel writes (allocated once)."""
        n = 3 * P
        if self._dc is None or self._dc.numel() != n or self._dc.device != torch.device(device):
            self._dc = torch.empty(n, dtype=torch.float32, device=device)
            self._gathered = torch.empty(self.world * n, dtype=torch.float32, device=device)
        return self._dc

    def chunk_size(self, P: int) -> int:
        """The backward's Gaussian range size, from the library that runs it
        (gsr_backward_chunk_size): the gathered DC rows are laid out by it."""
        from diff_gaussian_rasterization import _C
        return _C.backward_chunk_size(P, self.chunks)

    def check(self) -> None:
        """Raise if the last backward's failure flag (MAX over the ranks) is
        set: a peer rank's rasterizer backward failed and the summed
        gradients of that step are invalid.  Waits only for the event behind
        the flag's copy (the last collective of that backward)."""
        pending, self._pending = self._pending, None
        if pending is None:
            return
        flag, event = pending
        if event is not None:
            event.synchronize()
        if float(flag[0]) > 0.0:
            raise RuntimeError("OverlappedViewGrads: a peer rank's rasterizer backward failed; this step's summed "
                               "gradients are invalid (NaN in that rank's ranges)")

    def begin(self, campos: torch.Tensor, P: int, scales_path: bool, sh_path: bool) -> None:
        if self._active:  # a backward that neither finished nor failed cleanly: settle its collectives first
            self.abort()
        self.check()  # (the previous backward's deferred failure flag)
        self._works = []
        self._P, self._scales, self._sh = P, scales_path, sh_path
        self._cs = self.chunk_size(P) if P else 1
        self._next, self._ar_done, self._error = 0, False, None
        dev = campos.device
        if self._campos_local is None or self._campos_local.device != dev:
            self._campos_local = torch.zeros(4, dtype=torch.float32, device=dev)
            self._campos_all = torch.empty(4 * self.world, dtype=torch.float32, device=dev)
        self._campos_local[:3].copy_(campos.reshape(3))
        self._active = True
        if sh_path:
            self._works.append(_all_gather_into_tensor(self._campos_all, self._campos_local, self.group,
                                                       async_op=True))

    def _post(self, b: int, e: int, rows, dc_in) -> None:
        """One range's collectives, in the order every rank posts them."""
        if not self._ar_done:
            cm_fn = _coalescing(self.group, rows)
            if cm_fn is None:
                self._works += [_all_reduce(t, dist.ReduceOp.SUM, self.group, async_op=True) for t in rows]
            else:
                with cm_fn(group=self.group, async_ops=True) as cm:
                    for t in rows:
                        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                self._works.append(cm)
            self._ar_done = True
        if self._sh:
            W = self.world
            self._works.append(_all_gather_into_tensor(self._gathered[3 * W * b:3 * W * e], dc_in, self.group,
                                                       async_op=True))
        self._ar_done = False
        self._next = e

    def on_chunk(self, b: int, e: int, grads) -> None:
        if b != self._next or e != min(self._P, b + self._cs):
            raise RuntimeError(f"OverlappedViewGrads: backward range [{b}, {e}) does not follow the range layout "
                               f"(next {self._next}, size {self._cs}, P {self._P})")
        (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dsg_axis, dsg_sharpness, dsg_color, dscales,
         drotations) = grads[:11]
        rows = [dmeans3D[b:e], dopacity[b:e]]
        rows += [dscales[b:e], drotations[b:e]] if self._scales else [dcov3D[b:e]]
        if not self._sh:
            rows.append(dcolors[b:e])
        self._post(b, e, rows, self._dc[3 * b:3 * e] if self._sh else None)

    def hook(self, grads):
        """The per-range callback for the backward: errors are held (the C
        backward keeps launching its ranges) until `settle`."""
        def cb(b: int, e: int) -> None:
            if self._error is None:
                try:
                    self.on_chunk(b, e, grads)
                except BaseException as ex:  # noqa: BLE001 - re-raised by settle()
                    self._error = ex
        return cb

    def settle(self, ok: bool) -> None:
        """After the backward's launches: on a failed backward (`ok` False) or
        a range whose exchange raised, keep the group in lockstep (`abort`)
        and re-raise the range's error."""
        if ok and self._error is None:
            return
        err = self._error
        self.abort()
        if err is not None:
            raise err

    def abort(self) -> None:
        """The error path: post the collectives of every range not yet posted
        — on NaN-filled rows, so the peers' summed gradients for those ranges
        are NaN (visibly invalid) instead of silently missing this view —
        then wait for every outstanding work and reset.  Every rank thus
        posts the same collectives per backward, and no peer blocks."""
        if not self._active:
            return
        self._active = False
        try:
            P, cs = self._P, self._cs
            dev = self._campos_local.device
            b = self._next
            while b < P:
                e = min(P, b + cs)
                n = e - b
                nan = lambda *shape: torch.full(shape, float("nan"), dtype=torch.float32, device=dev)  # noqa: E731
                rows = [nan(n, 3), nan(n, 1)] + ([nan(n, 3), nan(n, 4)] if self._scales else [nan(n, 6)])
                if not self._sh:
                    rows.append(nan(n, 3))
                if self._sh and (self._gathered is None or self._gathered.numel() < 3 * self.world * P):
                    self._gathered = torch.empty(3 * self.world * P, dtype=torch.float32, device=dev)
                self._post(b, e, rows, nan(3 * n) if self._sh else None)
                b = e
        finally:
            try:
                self._post_status(True)
            finally:
                works, self._works = self._works, []
                for w in works:
                    try:
                        w.wait()
                    except Exception:  # noqa: BLE001 - already failing; the original error is what is raised
                        pass
                if not self._sync():  # deferred: this rank's next begin() raises as its peers' do (lockstep)
                    self._defer_flag()

    def _sync(self) -> bool:
        return self.sync_check if self.sync_check is not None else not self._status.is_cuda

    def _defer_flag(self) -> None:
        """The deferred check: the all-reduced flag copied behind the
        backward's last collective, read by check() / the next begin()."""
        if self._status.is_cuda:
            flag = torch.empty(1, dtype=torch.float32, pin_memory=True)
            flag.copy_(self._status, non_blocking=True)
            event = torch.cuda.Event()
            event.record()
            self._pending = (flag, event)
        else:
            self._pending = (self._status.clone(), None)

    def _post_status(self, failed: bool) -> None:
        """The backward's last collective, posted by every rank exactly once
        per backward (by finish, or by abort on the failing rank): MAX of the
        ranks' failure flags."""
        dev = self._campos_local.device if self._campos_local is not None else "cpu"
        if self._status is None or self._status.device != torch.device(dev):
            self._status = torch.zeros(1, dtype=torch.float32, device=dev)
        self._status.fill_(1.0 if failed else 0.0)
        self._works.append(_all_reduce(self._status, dist.ReduceOp.MAX, self.group, async_op=True))

    def finish(self, grads, means3D, sg_axis, sg_sharpness, sg_color, sh_degree: int, sg_degree: int) -> None:
        """`grads`: the backward's 11 gradients (+ dsh_rest, the split SH layout)."""
        if self._next != self._P:
            msg = f"OverlappedViewGrads: the backward's ranges covered [0, {self._next}) of {self._P} Gaussians"
            self.abort()
            raise RuntimeError(msg)
        self._active = False
        self._post_status(False)
        for w in self._works:
            w.wait()  # (RCCL: the backward's stream waits for the collective)
        self._works = []
        if self._sync():
            self._pending = (self._status, None)
            self.check()  # host read of the flag: every rank learns that one failed
        else:
            self._defer_flag()
        if not self._sh or self._P == 0:
            return
        (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dsg_axis, dsg_sharpness, dsg_color, dscales,
         drotations) = grads[:11]
        kw = {} if len(grads) < 12 else {"dL_dsh_rest": grads[11]}  # (the split SH layout)
        sg = [None if t is None or not t.numel() else t.detach() for t in (sg_axis, sg_sharpness, sg_color)]
        self.expand(self._gathered, self._campos_all.view(self.world, 4), self.world, self._cs,
                    means3D.detach(), sh_degree, dsh, sg_degree, *sg,
                    *[None if t is None or not t.numel() else t for t in (dsg_axis, dsg_sharpness, dsg_color)], **kw)

    def verify_replicas(self, params: Iterable[torch.Tensor]) -> None:
        """Opt-in check after a training step's whole backward: every rank's
        .grad must be identical (this exchange sums only the rasterizer's own
        gradients; another loss term on the same parameters that was not
        reduced makes the replicas drift).  One small all-reduce (MAX and
        -MIN of float64 checksums) and a host synchronisation."""
        sums = []
        for p in params:
            g = p.grad
            sums += [0.0, 0.0] if g is None else [float(g.double().sum()), float(g.double().abs().sum())]
        if not sums:
            return
        dev = self._campos_local.device if self._campos_local is not None else "cpu"
        t = torch.tensor(sums + [-x for x in sums], dtype=torch.float64, device=dev)
        _all_reduce(t, dist.ReduceOp.MAX, self.group)
        n = len(sums)
        hi, lo = t[:n], -t[n:]
        if not bool(torch.equal(hi, lo)):
            bad = int(torch.nonzero(hi != lo)[0]) // 2
            raise RuntimeError(f"OverlappedViewGrads.verify_replicas: parameter {bad}'s gradients differ across "
                               "ranks (a loss term outside the rasterizer was not reduced?)")


def reduce_densification_stats(grad_norm_accum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                               group: Optional[dist.ProcessGroup] = None) -> None:
    """Densification statistics of the views seen since the last densify step
    (gaussian_model.py:818-821, train.py:236): sums for the accumulated
    screen-space gradient norms and visibility counts, max for the radii.
    Called only at densification steps (every 100 iterations), not per step."""
    _all_reduce(grad_norm_accum, dist.ReduceOp.SUM, group)
    _all_reduce(denom, dist.ReduceOp.SUM, group)
    _all_reduce(max_radii2D, dist.ReduceOp.MAX, group)
