"""Data-parallel training loop for GuideDepth on MI355X (drop-in for src/train.py).

    python -m monocular_depth_estimation_amd.train --epochs 30 --lr 1e-4 --bs 3 --cp 0
    torchrun --nproc-per-node 8 -m monocular_depth_estimation_amd.train --synthetic ...

Keeps the reference CLI (train.py:26-31: --epochs --lr --bs --cp), its loss
(train.py:89-100: DepthNorm target, 1.0*SSIM + 0.1*L1 — here one fused HIP
pass that also yields the gradient), Adam, the checkpoint dict
(train.py:147-153) and, by default, its BatchNorm quirk: LogProgress calls
model.eval() at loader_pos % 300 == 0 and never switches back
(train.py:134-136,161), so from step 1 of every epoch BN uses running stats.

New (the reference is single-GPU): one process per GPU, torch.distributed
over RCCL ("nccl" backend on ROCm; "gloo" on CPU for tests), DDP gradient
all-reduce bucketed and overlapped with backward.  Each rank normalises its
own shard's depth (DepthNorm is batch-global in the reference, utils.py:7-8)
and keeps per-rank BN batch statistics (no SyncBN: DDRNet_23_slim.py:15 has it
commented out).  The host loop never synchronises per step: losses are
accumulated on device and read at log points only.  Silog_loss_variance is
evaluated by the reference every step but never used (train.py:98-100); it
is skipped here.

The NYU CSV-in-zip pipeline (src/data.py) is outside this build's scope;
--synthetic (the default when no dataset is given) feeds on-device uniform
images and depths with per-rank seeds.
"""
from __future__ import annotations

import argparse
import atexit
import json
import os
import time
import weakref
from dataclasses import dataclass

import torch
import torch.distributed as dist


# ------------------------------------------------------------ distributed
@dataclass
class World:
    rank: int = 0
    local_rank: int = 0
    size: int = 1
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_world(backend: str | None = None, use_gpu: bool | None = None,
               device_index: int | None = None) -> World:
    """Join the torchrun job (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), one GPU per process.

    Defaults: RCCL ("nccl") on GPUs, gloo on CPU.  Tests may run gloo over GPU
    tensors (use_gpu=True, several ranks on one device via device_index)."""
    size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if use_gpu is None:
        use_gpu = backend != "gloo"
    use_cuda = torch.cuda.is_available() and use_gpu
    device = torch.device("cuda", local if device_index is None else device_index) \
        if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    if size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        be = backend or ("nccl" if use_cuda else "gloo")
        dist.init_process_group(be, rank=rank, world_size=size,
                                device_id=device if (use_cuda and be == "nccl") else None)
    return World(rank, local, size, device)


def wrap_ddp(model: torch.nn.Module, world: World, bucket_cap_mb: float = 8.0):
    """DDP over RCCL: ~23 MB of fp32 grads in 8 MB buckets -> 3+ all-reduces
    overlapped with backward; BN buffers broadcast from rank 0 each forward."""
    if world.size == 1:
        return model
    kw = dict(bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, broadcast_buffers=True)
    if world.device.type == "cuda":
        kw["device_ids"] = [world.device.index]
    return torch.nn.parallel.DistributedDataParallel(model, **kw)


def unwrap(model):
    return model.module if hasattr(model, "module") else model


# ------------------------------------------------------------------ data
def synthetic_batch(batch: int, height: int, width: int, rank: int, step: int,
                    device, base_seed: int = 0):
    """image U[0,1), depth U[0.1,10); per-rank seed 1000*rank."""
    gen = torch.Generator(device="cpu")
    gen.manual_seed(base_seed + 1000 * rank + 2 * step)
    image = torch.rand((batch, 3, height, width), generator=gen)
    gen.manual_seed(base_seed + 1000 * rank + 2 * step + 1)
    depth = 0.1 + 9.9 * torch.rand((batch, 1, height, width), generator=gen)
    return image.to(device, non_blocking=True), depth.to(device, non_blocking=True)


# ------------------------------------------------------------------ step
def amp_context(amp: str, device: torch.device):
    """`--amp bf16` (BASELINE cfg3): convolutions / GEMMs autocast to bf16 on
    MIOpen / hipBLASLt; the HIP BatchNorm, BN-ReLU-1x1, skip-fusion, SE-over-BN
    and x2-resize kernels read and write bf16 activations (fp32 statistics and
    accumulation); the other HIP kernels compute in fp32 (their Functions cast
    their inputs, functional._amp_fwd).  Weight-cast caching is off so the
    casts stay inside a captured graph."""
    if amp not in ("", "fp32", "bf16"):
        raise ValueError(f"unsupported --amp {amp!r} (fp32 or bf16)")
    return torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp == "bf16",
                          cache_enabled=False)


class Trainer:
    """One reference training step (train.py:86-114) with a device-side loss log."""

    def __init__(self, model, optimizer, loss_fn, world: World, eval_quirk: bool = True,
                 amp: str = "", buckets: "GradBuckets | None" = None):
        self.model, self.optimizer, self.loss_fn, self.world = model, optimizer, loss_fn, world
        self.buckets = buckets  # data parallel by GradBuckets instead of a DDP wrapper
        self.eval_quirk = eval_quirk
        self.amp = amp
        self.loss_sum = torch.zeros((), device=world.device)
        self.loss_count = 0
        self.last_loss = None

    def begin_epoch(self):
        self.model.train()  # train.py:79

    def step(self, image, depth):
        if self.buckets is not None:
            self.buckets.begin()  # zeroes the bucket-view gradients
        with amp_context(self.amp, self.world.device):
            pred = self.model(image)
            loss = self.loss_fn(pred, depth)
        if self.buckets is None:
            self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        if self.buckets is not None:
            self.buckets.finish()
        self.optimizer.step()
        self.loss_sum += loss.detach()
        self.loss_count += 1
        self.last_loss = loss.detach()
        return loss

    def after_step(self, loader_pos: int):
        # LogProgress (train.py:134-136,161): model.eval() that is never undone
        if self.eval_quirk and loader_pos % 300 == 0:
            self.model.eval()


def bucket_groups(params, bucket_bytes: int):
    """All-reduce buckets: the parameters in REVERSE registration order (about
    the order backward finishes their gradients) cut into consecutive groups
    of at least `bucket_bytes` (the last one may be smaller); every parameter
    lands in exactly one group."""
    groups, cur, nbytes = [], [], 0
    for p in reversed(list(params)):
        cur.append(p)
        nbytes += p.numel() * p.element_size()
        if nbytes >= bucket_bytes:
            groups.append(cur)
            cur, nbytes = [], 0
    if cur:
        groups.append(cur)
    return groups


class GradBuckets:
    """Bucketed gradient all-reduce overlapped with backward (the DP exchange).

    The parameters (reverse registration order, about the order backward
    finishes them) are cut into ~`bucket_bytes` groups; every .grad becomes a
    view of its group's flat buffer for good.  A post-accumulate-grad hook
    counts each bucket's parameters; when the last one is final, the bucket
    is averaged over the ranks at once -- on `stream` (a side stream forked
    from the backward stream at that point) when given, so the collective
    overlaps the rest of the backward and, inside a capture, is captured INTO
    the step graph.  The collective is issued whenever the buckets exist,
    also in a one-rank group.  RCCL ("nccl"): one all_reduce(AVG) per bucket;
    gloo (no AVG): scale by 1/N, then all_reduce(SUM).  The collective order
    is the hook order, identical on every rank.

    Per step: begin() before the forward (zeroes the buffers, arms the
    counters), backward, finish() (launches buckets whose parameters got no
    gradient, joins the side stream)."""

    def __init__(self, params, world: World, bucket_bytes: int, stream=None):
        if not dist.is_initialized():
            raise RuntimeError("GradBuckets needs an initialised torch.distributed process group")
        self.world, self.stream = world, stream
        self.avg = dist.get_backend() == "nccl"
        self.groups = bucket_groups(params, bucket_bytes)
        self.buffers, self.bucket_of = [], {}
        for i, ps in enumerate(self.groups):
            flat = torch.zeros(sum(p.numel() for p in ps), device=ps[0].device, dtype=ps[0].dtype)
            off = 0
            for p in ps:
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
                self.bucket_of[p] = i
                p.register_post_accumulate_grad_hook(self._grad_ready)
            self.buffers.append(flat)
        self.pending = [-1] * len(self.groups)
        self.launched = []  # bucket order of the last step (the hook order)

    def __len__(self):
        return len(self.groups)

    def __iter__(self):
        return iter(zip(self.groups, self.buffers))

    def begin(self):
        for flat in self.buffers:
            flat.zero_()
        self.pending = [len(ps) for ps in self.groups]
        self.launched = []

    def _grad_ready(self, p):
        b = self.bucket_of.get(p)
        if b is None or self.pending[b] < 0:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._launch(b)

    def _launch(self, b):
        self.pending[b] = -1
        self.launched.append(b)
        flat = self.buffers[b]
        if self.stream is None:
            self._collective(flat)
            return
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            self._collective(flat)

    def _collective(self, flat):
        if self.avg:
            dist.all_reduce(flat, op=dist.ReduceOp.AVG)
        else:
            flat.mul_(1.0 / self.world.size)
            dist.all_reduce(flat)

    def finish(self):
        for b in range(len(self.groups)):  # parameters that got no gradient this step
            if self.pending[b] >= 0:
                self._launch(b)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)


def dp_exchange_scheme(world_size: int, backend: str | None, dp_overlap: bool | None = None,
                       dp_collectives: bool | None = None, env=None) -> str | None:
    """Which gradient exchange GraphTrainer runs: None (no exchange: one rank),
    "flat" (graph A -> ONE eager all_reduce -> graph B; no collective is ever
    captured) or "overlap" (bucket all-reduces captured INTO the step graph,
    overlapping the backward).  Flat is the N > 1 default.  Overlap is opt-in
    -- MDE_DP_OVERLAP=1 over RCCL, or dp_overlap=True -- because a captured
    multi-rank RCCL collective has not run on hardware in this repo's testing
    (the pool gives one GPU per call); a gloo group cannot capture collectives
    (GraphTrainer then runs the bucket path eagerly only).  dp_collectives
    forces the exchange on (or off) regardless of the world size (tests: the
    same calls in a one-rank group)."""
    env = os.environ if env is None else env
    dp = world_size > 1 if dp_collectives is None else bool(dp_collectives)
    if dp_overlap is None:
        dp_overlap = dp and backend == "nccl" and env.get("MDE_DP_OVERLAP", "0") == "1"
    if dp_overlap:
        return "overlap"
    return "flat" if dp else None


class GraphTrainer:
    """The same training step captured into HIP graphs and replayed.

    The step (forward, DepthNorm + loss, backward, Adam) is a fixed sequence of
    ~700 kernel launches on one stream; replaying it from a hipGraph removes
    the per-launch host cost and the gaps between kernels.  Every call of
    step() performs exactly one training step: the first `eager_steps` calls
    run eagerly on a side stream (MIOpen / hipBLASLt pick and compile their
    kernels, the caching allocator settles), the next call captures and then
    replays.

    Gradients are allocated by the captured backward itself (grads set to None
    before capture, so autograd hands its result buffers to .grad without a
    copy; replays reuse those static buffers).  N == 1: one graph (forward,
    loss, backward, fused capturable Adam).

    N > 1, the default (dp_exchange_scheme "flat"): graph A (forward,
    backward, the gradients packed into one buffer and scaled by 1/N) -> ONE
    eager all_reduce(SUM) outside any graph -> graph B (unpack, Adam); no
    collective is ever captured.  Opt-in over RCCL (MDE_DP_OVERLAP=1 or
    dp_overlap=True, "overlap"): the gradients are views of ~6 MB bucket
    buffers (parameters in reverse registration order, i.e. about the order
    backward finishes them); a post-accumulate hook counts each bucket's
    parameters and, when the last one is final, all-reduces the bucket with
    ReduceOp.AVG on a side stream forked from the backward stream, so the
    RCCL collectives are captured INTO the step graph and overlap the rest of
    the backward (one graph; the Adam step joins the side stream).  The
    captured multi-rank collective has only run through RCCL's one-rank path
    on this pool, hence opt-in.  The BN running statistics live in one flat
    buffer, broadcast from rank 0 at start, when the eval-mode quirk switches
    BN to running statistics (every rank then normalises with rank 0's, as
    under DDP's broadcast_buffers), and by sync_buffers() -- not every step: a
    train-mode forward never reads them, and rank 0's, the ones a checkpoint
    saves, come out bitwise the same as under DDP's per-forward broadcast
    (rank 0 receives its own).  Inputs are copied into static device buffers.

    The reference's BatchNorm quirk (eval_quirk, default on as in Trainer):
    LogProgress calls model.eval() at loader_pos % 300 == 0 and never switches
    back (src/train.py:79,134-136,161), so from step 1 of every epoch BN uses
    running statistics.  Each BN mode has its own captured step (graphs keyed
    by model.training, each captured the first time that mode runs after the
    warm-up), so an epoch replays the train-mode step once and the eval-mode
    step after it.  CUDA only.  close() frees the captured graphs and runs no
    collective (it is also the atexit hook: a rank that gets there alone must
    not block); it must run before dist.destroy_process_group() (a graph
    holding captured RCCL collectives references the communicator).
    """

    BUCKET_BYTES = 6 << 20

    def __init__(self, model, loss_fn, world: World, lr=1e-4, eager_steps=2, amp: str = "",
                 dp_overlap: bool | None = None, dp_collectives: bool | None = None,
                 eval_quirk: bool = True):
        if world.device.type != "cuda":
            raise RuntimeError("GraphTrainer needs a GPU (use Trainer on CPU)")
        self.model, self.loss_fn, self.world = model, loss_fn, world
        self.amp = amp
        self.eager_steps = eager_steps
        self.eval_quirk = eval_quirk
        self.calls = 0
        self.graphs = {}  # BN mode ("train" / "eval") -> (graph A, graph B or None, static loss)
        # the data-parallel exchange runs at N > 1; dp_collectives=True issues it
        # in a one-rank group too (tests: the same RCCL calls, average = identity)
        self.dp = world.size > 1 if dp_collectives is None else bool(dp_collectives)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.optimizer = torch.optim.Adam(self.params, lr, fused=True, capturable=True)
        self.flat_grad = None
        self.flat_bn = None
        if world.size > 1:
            bufs = [(m, name) for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)
                    for name in ("running_mean", "running_var") if getattr(m, name) is not None]
            n = sum(getattr(m, name).numel() for m, name in bufs)
            self.flat_bn = torch.empty(n, device=world.device)
            off = 0
            for m, name in bufs:
                b = getattr(m, name)
                view = self.flat_bn[off:off + b.numel()].view_as(b)
                view.copy_(b)
                m._buffers[name] = view
                off += b.numel()
            for p in self.params:  # identical start on every rank (DDP does this at wrap time)
                dist.broadcast(p.data, 0)
            dist.broadcast(self.flat_bn, 0)
        self.static_image = self.static_depth = None
        # Capture streams and eager streams are disjoint.  A synchronous
        # collective records its completion event on the stream it was issued
        # on, and ProcessGroupNCCL's watchdog thread polls that event until it
        # has seen it complete; if the stream has joined a capture by then, HIP
        # refuses the query (hipErrorCapturedEvent), which invalidates the
        # capture and kills the watchdog (SIGABRT).  So no stream that ever
        # carries an eager collective is captured: warm-up steps and
        # eager_step() run on eager_stream (bucket collectives on eager_side),
        # captures on stream (bucket collectives on side).
        self.stream = torch.cuda.Stream(device=world.device)  # capture stream
        self.eager_stream = torch.cuda.Stream(device=world.device)
        # the exchange (dp_exchange_scheme): flat by default at N > 1; the
        # bucketed all-reduce captured into the step graph on request over
        # RCCL.  dp_overlap=True with a one-rank group issues the same
        # collectives (tests).
        backend = dist.get_backend() if dist.is_initialized() else None
        self.scheme = dp_exchange_scheme(world.size, backend, dp_overlap, dp_collectives)
        self.buckets = None
        if self.scheme == "overlap":
            self.side = torch.cuda.Stream(device=world.device)
            self.eager_side = torch.cuda.Stream(device=world.device)
            self.buckets = GradBuckets(self.params, world, self.BUCKET_BYTES, stream=self.eager_side)
        self.last_loss = None
        self.loss_sum = torch.zeros((), device=world.device)
        self.loss_count = 0
        # graphs with captured collectives must not outlive the communicator:
        # free them at exit even if the caller never calls close()
        ref = weakref.ref(self)
        self._atexit = lambda: (ref() is not None and ref().close())
        atexit.register(self._atexit)

    def begin_epoch(self):
        self.model.train()  # train.py:79

    # -- the step's pieces (each runs eagerly or inside a capture) ----------
    def _forward_backward(self):
        if self.buckets is not None:
            self.buckets.begin()
        with amp_context(self.amp, self.world.device):
            loss = self.loss_fn(self.model(self.static_image), self.static_depth)
        loss.backward()
        if self.buckets is not None:
            self.buckets.finish()
        elif self.dp:
            grads = [p.grad for p in self.params if p.grad is not None]
            if self.flat_grad is None:
                self.flat_grad = torch.empty(sum(g.numel() for g in grads),
                                             device=self.world.device)
            torch.cat([g.reshape(-1) for g in grads], out=self.flat_grad)
            self.flat_grad.mul_(1.0 / self.world.size)
        return loss.detach()

    def _unpack_and_update(self):
        if self.dp and self.buckets is None:
            grads = [p.grad for p in self.params if p.grad is not None]
            flat = self.flat_grad.split([g.numel() for g in grads])
            torch._foreach_copy_(grads, [f.view_as(g) for f, g in zip(flat, grads)])
        self.optimizer.step()

    def sync_buffers(self):
        """Rank 0's BN running statistics to every rank (DDP's broadcast_buffers,
        on demand: before evaluating or checkpointing on a rank other than 0)."""
        if self.world.size > 1 and self.flat_bn is not None and dist.is_initialized():
            dist.broadcast(self.flat_bn, 0)

    def _allreduce(self):
        if self.dp and self.buckets is None:
            dist.all_reduce(self.flat_grad)

    def _zero_grad(self):
        if self.buckets is None:  # bucket views stay; _forward_backward zeroes them
            self.optimizer.zero_grad(set_to_none=True)

    def _side_stream(self, captured: bool):
        if self.buckets is not None:
            self.buckets.stream = self.side if captured else self.eager_side

    def _eager(self):
        self._side_stream(False)
        self._zero_grad()
        loss = self._forward_backward()
        self._allreduce()
        self._unpack_and_update()
        return loss

    def step(self, image, depth):
        if self.static_image is None:
            self.static_image = torch.empty_like(image)
            self.static_depth = torch.empty_like(depth)
        self.static_image.copy_(image)
        self.static_depth.copy_(depth)
        self.calls += 1
        if self.calls <= self.eager_steps:
            cur = torch.cuda.current_stream()
            self.eager_stream.wait_stream(cur)
            with torch.cuda.stream(self.eager_stream):
                loss = self._eager()
            cur.wait_stream(self.eager_stream)
        else:
            mode = "train" if self.model.training else "eval"
            if mode not in self.graphs:
                self.graphs[mode] = self._capture()
            ga, gb, loss = self.graphs[mode]
            ga.replay()
            if gb is not None:
                self._allreduce()
                gb.replay()
        self.last_loss = loss
        self.loss_sum += loss
        self.loss_count += 1
        return loss

    def eager_step(self, image, depth):
        """One uncaptured step (the same kernels the graph replays), e.g. for
        per-kernel HIP-event timing, which graph replay bypasses.  Only valid
        before capture or for measurement: it re-allocates the gradients."""
        self.static_image.copy_(image)
        self.static_depth.copy_(depth)
        loss = self._eager()
        self.last_loss = loss
        return loss

    def _capture(self):
        """Capture the step in the model's current BN mode; returns (graph A,
        graph B or None, static loss).  Every memset node the capture recorded
        (ATen's multi-block reductions zero their semaphores with one) is
        replaced by a fill kernel before instantiation: captured memsets are
        only correct on a graph's first replay on this ROCm stack
        (csrc/graph.hip).  Each capture gets its own memory pool and its own
        gradient buffers (grads are set to None first), so the train-mode and
        eval-mode graphs can be replayed in any order: the Adam state is
        shared, each graph's optimizer step reads the gradients its own
        backward wrote."""
        from . import _abi
        if self.buckets is not None and dist.get_backend() != "nccl":
            raise RuntimeError("the overlapped bucket all-reduce is captured into the step graph "
                               "over RCCL only; a gloo group runs GraphTrainer eagerly "
                               "(eager_steps >= the number of steps)")
        torch.cuda.synchronize()
        self._side_stream(True)
        self._zero_grad()  # backward allocates .grad in the graph pool (non-bucket mode)
        one_graph = not self.dp or self.buckets is not None

        def part_a():
            loss = self._forward_backward()
            if one_graph:
                self.optimizer.step()
            return loss

        ga, static_loss, na = _abi.capture_graph(part_a, self.stream)
        gb, nb = None, 0
        if not one_graph:
            gb, _, nb = _abi.capture_graph(self._unpack_and_update, self.stream, pool=ga.pool())
        self.memsets_replaced = na + nb
        return ga, gb, static_loss

    def after_step(self, loader_pos: int):
        # LogProgress (train.py:134-136,161): model.eval() that is never undone.
        # Every rank calls this at the same loader position, so the broadcast of
        # rank 0's running statistics at the switch is a matched collective
        # (eval-mode steps never change them: all ranks then normalise alike).
        if self.eval_quirk and loader_pos % 300 == 0 and self.model.training:
            self.model.eval()
            self.sync_buffers()

    def close(self):
        """Drain the device and free the captured graphs.  Call before
        dist.destroy_process_group(): a graph with captured RCCL collectives
        still references the communicator, and tearing the communicator down
        under a live graph aborts the process on this stack.  Runs no
        collective (sync_buffers() is the caller's, on every rank)."""
        if not self.graphs:
            return
        torch.cuda.synchronize()
        for ga, gb, _ in self.graphs.values():
            for g in (ga, gb):
                if g is not None:
                    g.reset()
        self.graphs = {}
        torch.cuda.synchronize()

    def timed_replays(self, batches, replays: int = 3) -> dict:
        """Per-kernel HIP-event times of the REPLAYED step (measurement only).

        The step is captured once more with the timing registry on, so each
        HIP launch is bracketed by event-record nodes inside the graph; that
        graph is replayed `replays` times and the registry resolved after each
        replay.  Returns _abi.timing_collect()'s {kernel: (ms, launches,
        bytes, flops)} over all replays.  Leaves the trainer on a second set of
        gradient buffers: call it after the timed loop."""
        from . import _abi
        torch.cuda.synchronize()
        _abi.timing_reset()
        self._side_stream(True)
        self._zero_grad()
        one_graph = not self.dp or self.buckets is not None

        def part():
            loss = self._forward_backward()
            if one_graph:
                self.optimizer.step()
            return loss

        _abi.timing_enable(True)
        try:
            graph, _, _ = _abi.capture_graph(part, self.stream)
        finally:
            _abi.timing_enable(False)
        for i in range(replays):
            image, depth = batches[i % len(batches)]
            self.static_image.copy_(image)
            self.static_depth.copy_(depth)
            graph.replay()
            torch.cuda.synchronize()
            _abi.call("mde_timing_collect")
        out = _abi.timing_collect(resolve=False)
        _abi.timing_reset()
        graph.reset()  # its RCCL nodes must not outlive the communicator (see close())
        return out


class DeviceLossMeter:
    """The reference's per-epoch `losses` AverageMeter (train.py:75,112,141),
    updated every step without a host sync: the trainer accumulates each
    step's loss on the device (loss_sum, one add per step) and the meter
    keeps the epoch's starting point; read() -- at the log points only --
    returns (last loss, epoch average).  The sample weight n is constant
    within an epoch (fixed per-rank batch, drop_last), so the weighted
    average of train.py:112 is the plain mean of the epoch's step losses."""

    def __init__(self, trainer):
        self.trainer = trainer
        self.sum0 = trainer.loss_sum.detach().clone()
        self.count0 = trainer.loss_count
        self.n = 0

    def update(self, n=1):
        self.n = n

    def read(self):
        steps = self.trainer.loss_count - self.count0
        val = float(self.trainer.last_loss.detach())
        avg = float((self.trainer.loss_sum - self.sum0).detach()) / steps if steps else 0.0
        return val, avg


def make_adam(model, lr=1e-4):
    kw = {}
    if next(model.parameters()).is_cuda:
        kw["fused"] = True  # one multi-tensor launch per step on ROCm
    return torch.optim.Adam(model.parameters(), lr, **kw)


def save_checkpoint(path, epoch, model, optimizer, loss):
    """train.py:147-153 dict format, rank 0 only, DDP unwrapped."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    torch.save({"epoch": epoch, "model_state_dict": unwrap(model).state_dict(),
                "optimizer_state_dict": optimizer.state_dict(), "loss": loss}, path)


def load_checkpoint(path, model, optimizer, capturable: bool = False):
    """Resume (train.py:59-68): restarts AT the saved epoch (it is re-run).

    Optimizer.load_state_dict replaces the param groups with the saved ones,
    so a checkpoint written by the eager trainer (fused Adam) or by the
    reference (plain Adam) would turn GraphTrainer's capturable Adam into a
    non-capturable one, whose step() refuses to be captured.  capturable=True
    restores fused + capturable on every group and puts each `step` counter
    on the parameter's device as fp32, as a capturable Adam keeps it."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    unwrap(model).load_state_dict(ckpt["model_state_dict"])
    optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    if capturable:
        for group in optimizer.param_groups:
            group["capturable"] = True
            group["fused"] = True
            group["foreach"] = None
            for p in group["params"]:
                st = optimizer.state.get(p)
                if st and "step" in st:
                    st["step"] = torch.as_tensor(st["step"], dtype=torch.float32).to(p.device)
    return int(ckpt["epoch"]), ckpt["loss"]


def build_parser():
    p = argparse.ArgumentParser(description="GuideDepth training on MI355X (drop-in for src/train.py)")
    p.add_argument("--epochs", default=30, type=int, help="number of total epochs to run")
    p.add_argument("--lr", "--learning-rate", default=0.0001, type=float, help="initial learning rate")
    p.add_argument("--bs", default=3, type=int, help="batch size (per GPU)")
    p.add_argument("--cp", default=0, type=int, help="1 to resume from the last checkpoint")
    p.add_argument("--height", default=480, type=int)
    p.add_argument("--width", default=640, type=int)
    p.add_argument("--steps-per-epoch", default=100, type=int, help="synthetic epoch length")
    p.add_argument("--data", default="", help="NYU CSVdata.zip (data.py:172); empty = synthetic batches")
    p.add_argument("--workers", default=4, type=int, help="decode workers of the NYU loader")
    p.add_argument("--checkpoint", default="checkpoints/global_checkpoint.pth")
    p.add_argument("--no-eval-quirk", action="store_true",
                   help="keep BN in train mode all epoch (the reference switches to eval after step 0)")
    p.add_argument("--log", default="", help="JSONL file for Train/Loss scalars (rank 0)")
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--amp", default="fp32", choices=("fp32", "bf16"),
                   help="bf16 = autocast (BASELINE cfg3): convs / GEMMs in bf16 on MIOpen / hipBLASLt, "
                        "HIP BN / BN-ReLU-1x1 / skip / SE-over-BN / x2-resize kernels on bf16 "
                        "activations (fp32 statistics), other HIP kernels fp32")
    p.add_argument("--pretrained", action="store_true",
                   help="GuideDepth(True) as the reference's train.py:34: load the DDRNet-23-slim "
                        "ImageNet blob (DDRNet_23_slim.py:357-365) non-strictly into the encoder")
    p.add_argument("--weights", default="",
                   help="path of DDRNet23s_imagenet.pth (default: the reference's relative path "
                        "./GuideDepth/model/weights/DDRNet23s_imagenet.pth)")
    p.add_argument("--graph", action="store_true",
                   help="replay the step from HIP graphs (GraphTrainer; one captured step per BN "
                        "mode, so the eval-mode quirk runs replayed too)")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    world = init_world()
    from . import GuideDepth  # noqa: E402  (loads the HIP library)
    from . import gemm_table
    if world.device.type == "cuda":
        gemm_table.enable()  # the vendor GEMMs' tuned solution table
    from .loss import SSIML1

    torch.manual_seed(args.seed)
    if args.weights:
        os.environ["MDE_DDRNET_WEIGHTS"] = args.weights
    model = GuideDepth(pretrained=args.pretrained).to(world.device)
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    if args.graph:
        trainer = GraphTrainer(model, loss_fn, world, lr=args.lr, amp=args.amp,
                               eval_quirk=not args.no_eval_quirk)
        optimizer, ddp = trainer.optimizer, model
    else:
        optimizer = make_adam(model, args.lr)
        ddp = wrap_ddp(model, world)
        trainer = Trainer(ddp, optimizer, loss_fn, world, eval_quirk=not args.no_eval_quirk,
                          amp=args.amp)
    start_epoch = 0
    if args.cp == 1:  # train.py:59-68: restarts AT the saved epoch
        start_epoch, _ = load_checkpoint(args.checkpoint, model, optimizer, capturable=args.graph)
    log = open(args.log, "a") if (args.log and world.is_main) else None
    loader = None
    if args.data:  # data.py:171-179 on the GPU path; each rank reads a disjoint 1/size of the rows
        from .data import NYUBatchLoader, loadZipToMem
        data, nyu2_train, _ = loadZipToMem(args.data)
        loader = NYUBatchLoader(data, nyu2_train[world.rank::world.size], args.bs, train=True,
                                shuffle=True, num_workers=args.workers, device=world.device,
                                drop_last=True)

    def batches(epoch):
        if loader is not None:
            for b in loader:
                yield b["image"], b["depth"]
            return
        for pos in range(args.steps_per_epoch):
            yield synthetic_batch(args.bs, args.height, args.width, world.rank,
                                  epoch * args.steps_per_epoch + pos, world.device, args.seed)

    for epoch in range(start_epoch, args.epochs):
        trainer.begin_epoch()
        losses, t0 = DeviceLossMeter(trainer), time.time()
        n_steps = len(loader) if loader is not None else args.steps_per_epoch
        for pos, (image, depth) in enumerate(batches(epoch)):
            loss = trainer.step(image, depth)
            losses.update(image.size(0))  # every step, as train.py:112 (no host sync)
            trainer.after_step(pos)
            if pos % 5 == 0 and world.is_main:  # train.py:123-132 (host read at log points only)
                v, avg = losses.read()
                dt = time.time() - t0
                print(f"Epoch: [{epoch}][{pos}/{n_steps}]\tTime {dt:.3f}\t"
                      f"Loss {v:.4f} ({avg:.4f})", flush=True)
                if log:
                    log.write(json.dumps({"tag": "Train/Loss", "value": v,
                                          "step": epoch * n_steps + pos}) + "\n")
        if world.is_main:
            if log:  # train.py:141: the mean of EVERY step's loss of the epoch
                log.write(json.dumps({"tag": "Train/Loss.avg", "value": losses.read()[1],
                                      "step": epoch}) + "\n")
                log.flush()
            save_checkpoint(args.checkpoint, epoch, ddp, optimizer, trainer.last_loss.cpu())
    if hasattr(trainer, "close"):
        trainer.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
