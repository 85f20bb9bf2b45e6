"""Training throughput of GuideDepth at 640x480, bs=32 per GPU (BASELINE.json metric, cfg2).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` (N > 1) outside a torchrun job launches the N
ranks itself: the parent starts `torch.distributed.run` as a child process
before anything touches the GPU and exits with its code; rank 0's JSON line
is the child's stdout.  `--device cpu` (gloo) runs the same launcher and
data-parallel plumbing on a small plain-torch stand-in net on the CPU: a
launcher smoke test, not a measurement.

One step = the src/train.py step (train.py:86-114) on one synthetic batch
already resident in HBM: GuideDepth forward (BN in train mode), DepthNorm +
1.0*SSIM + 0.1*L1 (one fused HIP pass), backward, DDP all-reduce over RCCL
(N > 1), Adam step.  Rank 0 prints ONE JSON line.  Extra fields:
  roofline     — the dominant hand-written HIP kernel of the step (HIP events
                 captured into the replayed step graph; algorithmic bytes /
                 flops per SURVEY §8(d)); traffic = rocprofv3 PMC HBM bytes
                 per launch from profiles/ (traffic_ratio = traffic / algorithmic).
  roofline_leaders — the top HBM-bound and the top MFMA-bound hand kernels.
  path_roofline — north_star's depthwise+upsample path (resizes + depthwise).
  cpu_baseline — the CPU oracle's train step (rank 0, N=1 only), bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFS = 157.3  # fp32-input MFMA dense peak (= fp32 vector rate, MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFS = 16 * MFMA_F32_PEAK_TFS  # bf16 MFMA dense peak (~2.5 PF, 16x the f32 rate)
# rocprofv3 PMC HBM bytes per launch (tools/pmc_traffic.py), newest round first.
# Counters are per workload and precision: a kernel's bytes in the cfg2 fp32
# step say nothing about its bytes in the bf16 or the NewCRF step.
def pmc_files(workload: str, amp: str) -> list[str]:
    tag = f"{workload}_{amp}"
    files = [os.path.join(REPO, "profiles", f"r0{r}_pmc_traffic_{tag}.json") for r in (6, 5, 4, 3)]
    if tag == "guidedepth_fp32":  # rounds 1-2 profiled the cfg2 fp32 step only
        files += [os.path.join(REPO, "profiles", f"r0{r}_pmc_traffic.json") for r in (2, 1)]
    return files


AMP_DTYPE = ("bf16 autocast: every 3x3 / 1x1 conv with 32k channels (DDRNet's stride-1 / stride-2 "
             "convs, the 32-640-channel decoder / DAPPM convs) on the HIP bf16 implicit-GEMM kernels "
             "(convbf, v_mfma_f32_32x32x16_bf16, fp32 accumulation, fp32 weight gradients), the "
             "16->16 / 32->32 3x3 convs on the HIP bf16 MFMA kernels, the 3-channel stem and "
             "guide convs bf16 on HIP (stem.hip / in-kernel); the BN-ReLU-1x1 pointwise convs with "
             "bf16 products (pwbf.hip, v_mfma_f32_16x16x32_bf16); BatchNorm, skip fusion, "
             "SE-over-BN and every resize on bf16 activations with fp32 statistics / "
             "accumulation; SSIM + L1 loss fp32")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                   help="cpu: launcher / data-parallel smoke over gloo on a plain-torch stand-in "
                        "net (no HIP; not a measurement)")
    p.add_argument("--backend", choices=("nccl", "gloo"), default=None,
                   help="process-group backend (default: nccl = RCCL on cuda, gloo on cpu)")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=("guidedepth", "newcrf", "sam"), default="guidedepth",
                   help="guidedepth = BASELINE cfg2 (the headline line); newcrf = cfg4, "
                        "PTModel (MobileNetV3-L + NewCRF decoder), the swap-in at train.py:36; "
                        "sam = the MobileNetV3-L + SAM model test.py evaluates (frozen encoder)")
    p.add_argument("--bs", type=int, default=None, help="per-GPU batch (32 cfg2, 16 cfg4)")
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--amp", choices=("fp32", "bf16"), default="fp32",
                   help="bf16: BASELINE cfg3 autocast (convs / GEMMs bf16; BN HIP kernels bf16 I/O)")
    p.add_argument("--cpu-bs", type=int, default=0, help="CPU-baseline batch (0 = the GPU batch)")
    p.add_argument("--cpu-steps", type=int, default=2)
    p.add_argument("--cudnn-benchmark", type=int, default=0)
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--graph", type=int, default=1,
                   help="1: replay the captured step from HIP graphs (GraphTrainer); 0: eager")
    p.add_argument("--timing-steps", type=int, default=3,
                   help="replays of the step (graph mode) / eager steps timed per kernel with HIP "
                        "events after the timed loop")
    args = p.parse_args()
    if args.bs is None:
        args.bs = 32 if args.workload == "guidedepth" else 16
    return args


def _cpu_model_name() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _usable_cpus() -> tuple[int, str]:
    """Every core this process may run on: the CPU affinity set, capped by the
    cgroup's CPU quota (cpu.max) when one is set.  On the GPU box
    os.cpu_count() reports the whole host (256 logical CPUs) while the job's
    quota is a fraction of it; more threads than the quota only time-slice."""
    n = len(os.sched_getaffinity(0))
    how = f"affinity {n}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(-(-int(quota) // int(period))))
            how += f", cgroup quota {int(quota) / int(period):g}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, how


def _lscpu() -> str:
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return ""
    keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)")
    return "; ".join(" ".join(l.split()) for l in out.splitlines() if l.split(":")[0] in keep)


def cpu_baseline(args):
    """The oracle (CPU restatement, the same ATen CPU convs / BN as the reference,
    pinned to it by tests/golden) timed on the host: the metric's own shape
    (640x480, bs 32 = cfg2) for 1 warm-up + `cpu_steps` steps, and (GuideDepth)
    BASELINE cfg1 beside it -- 320x240 bs 4, 1 warm-up + 10 steps (SURVEY
    §8(d)).  Threads: every usable core (_usable_cpus)."""
    from oracle import guidedepth as og
    from oracle import mobilenetv3 as om
    from oracle import ops as oops
    threads, how = _usable_cpus()
    torch.set_num_threads(threads)
    if args.workload == "sam":
        from oracle import sam as osam
        model = om.PTModel().train()
        model.Unet[1] = osam.Decoder()
        for p in model.Unet[0].parameters():
            p.requires_grad_(False)
    else:
        model = (og.GuideDepth() if args.workload == "guidedepth" else om.PTModel()).train()
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], 1e-4)

    def timed(bs, h, w, steps):
        g = torch.Generator().manual_seed(0)
        img = torch.rand((bs, 3, h, w), generator=g)
        dep = 0.1 + 9.9 * torch.rand((bs, 1, h, w), generator=g)

        def step():
            loss = oops.train_loss(model(img), dep)
            opt.zero_grad()
            loss.backward()
            opt.step()

        step()  # warm-up
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        return time.perf_counter() - t0

    bs = args.cpu_bs or args.bs
    dt = timed(bs, args.height, args.width, args.cpu_steps)
    name = "GuideDepth" if args.workload == "guidedepth" else "PTModel"
    out = {"value": round(bs * args.cpu_steps / dt, 3), "unit": "images/s",
           "cores": torch.get_num_threads(), "kind": "port",
           "host_cpu": f"{_cpu_model_name()} ({os.cpu_count()} logical CPUs on the host; "
                       f"usable: {how})",
           "lscpu": _lscpu(),
           "sample": f"oracle {name} train step (SSIM+0.1*L1, Adam), {args.width}x{args.height} "
                     f"bs={bs}, fp32, {args.cpu_steps} timed steps after 1 warm-up ({dt:.1f} s)"}
    if args.workload == "guidedepth":  # BASELINE cfg1: 320x240 bs 4
        dt1 = timed(4, 240, 320, 10)
        out["cfg1"] = {"value": round(4 * 10 / dt1, 3), "unit": "images/s",
                       "s_per_step": round(dt1 / 10, 4), "cores": torch.get_num_threads(),
                       "sample": f"oracle GuideDepth train step, 320x240 bs=4, fp32, 10 timed "
                                 f"steps after 1 warm-up ({dt1:.1f} s)"}
    return out


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) outside a torchrun job: run this script under
    torch.distributed.run as a CHILD process, one rank per GPU, and return
    its exit code.  The parent makes no HIP call before or after (the ranks
    own the devices; a process that initialised the GPU must not exec), and
    rank 0's JSON line reaches stdout through the child."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
    env.setdefault("OMP_NUM_THREADS", "1" if args.device == "cpu" else env.get("OMP_NUM_THREADS", "8"))
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


class _StandInNet(torch.nn.Module):
    """`--device cpu` only: a small plain-torch conv net standing in for the
    HIP model, so the launcher and the data-parallel exchange (GradBuckets
    over gloo) can run without a GPU.  Not a workload of the metric."""

    def __init__(self):
        super().__init__()
        nn = torch.nn
        self.body = nn.Sequential(nn.Conv2d(3, 16, 3, 2, 1), nn.BatchNorm2d(16), nn.ReLU(),
                                  nn.Conv2d(16, 16, 3, 1, 1), nn.BatchNorm2d(16), nn.ReLU(),
                                  nn.Conv2d(16, 1, 1))

    def forward(self, x):
        return torch.nn.functional.interpolate(self.body(x), scale_factor=2, mode="bilinear")


def params_fingerprint(params) -> torch.Tensor:
    """float64 sum of every parameter's float64 sum: equal bitwise across ranks
    iff (for all practical purposes) the replicas hold the same weights."""
    return torch.stack([p.detach().double().sum() for p in params]).sum().reshape(1)


def params_in_sync(params, world) -> bool | None:
    if world.size == 1:
        return None
    fp = params_fingerprint(params)
    every = [torch.empty_like(fp) for _ in range(world.size)]
    dist.all_gather(every, fp)
    return all(bool((e == every[0]).all()) for e in every)


def cpu_smoke(args, world):
    """The launcher / data-parallel plumbing on the CPU over gloo (see
    _StandInNet): rank 0's weights broadcast, per-rank shards, the bucketed
    gradient exchange, Adam; rank 0 prints one JSON line with n_gpus from the
    process group and whether every rank ends with the same parameters."""
    from monocular_depth_estimation_amd.train import GradBuckets, Trainer, synthetic_batch
    torch.manual_seed(world.rank)  # different init per rank: the broadcast must fix it
    model = _StandInNet().train()
    params = list(model.parameters())
    if world.size > 1:
        for p in params:
            dist.broadcast(p.data, 0)
    buckets = GradBuckets(params, world, 4 << 10) if world.size > 1 else None
    opt = torch.optim.Adam(params, 1e-3)
    trainer = Trainer(model, opt, lambda pred, d: torch.nn.functional.l1_loss(pred, d / 10.0),
                      world, eval_quirk=False, buckets=buckets)
    trainer.begin_epoch()
    batches = [synthetic_batch(args.bs, args.height, args.width, world.rank, s, "cpu")
               for s in range(2)]
    for i in range(args.warmup):
        trainer.step(*batches[i % 2])
    if world.size > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.step(*batches[i % 2])
    if world.size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world.size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    in_sync = params_in_sync(params, world)
    if world.is_main:
        out = {"metric": "launcher smoke (CPU, gloo): training images/sec of a stand-in net",
               "value": round(world.size * args.bs * args.steps / elapsed, 2), "unit": "images/s",
               "n_gpus": world.size, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(elapsed * 1e3 / max(args.steps, 1), 2),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic; --device cpu launcher smoke on a plain-torch stand-in net, "
                       "NOT a measurement of the metric",
               "config": {"workload": "stand-in net (bench._StandInNet), CPU",
                          "global_batch": world.size * args.bs, "per_gpu_batch": args.bs,
                          "resolution": f"{args.width}x{args.height}",
                          "parallelism": f"dp{world.size}"},
               "dp_exchange": (f"{len(buckets)} gradient buckets, gloo all_reduce (1/N + SUM) "
                               "from post-accumulate hooks" if buckets is not None else None),
               "params_in_sync": in_sync,
               "params_fingerprint": float(params_fingerprint(params)),
               "loss_last": round(float(trainer.last_loss), 6)}
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))  # before any GPU call: the ranks own the devices
    from monocular_depth_estimation_amd.train import init_world
    backend = args.backend or ("gloo" if args.device == "cpu" else None)
    world = init_world(backend=backend, use_gpu=args.device == "cuda")
    if world.size != args.gpus and world.is_main:
        print(f"[bench] warning: --gpus {args.gpus} but the job has {world.size} ranks; "
              f"n_gpus reports the process group's size", file=sys.stderr, flush=True)
    if args.device == "cpu":
        return cpu_smoke(args, world)
    if world.device.type != "cuda":
        raise RuntimeError("bench.py measures on a ROCm GPU (no GPU visible); "
                           "--device cpu runs the CPU launcher smoke instead")
    from monocular_depth_estimation_amd import _abi
    from monocular_depth_estimation_amd.train import Trainer, make_adam, synthetic_batch, wrap_ddp
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    from monocular_depth_estimation_amd import gemm_table
    gemm_path = gemm_table.enable()  # the vendor GEMMs' tuned solution table
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1

    torch.manual_seed(0)
    if args.workload == "guidedepth":
        model = GuideDepth(pretrained=False).to(world.device)
    elif args.workload == "newcrf":
        from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
        model = PTModel().to(world.device)
    else:
        from monocular_depth_estimation_amd.model_mobileV3_large_SAM import PTModel
        model = PTModel().to(world.device)
    loss_fn = SSIML1(1.0, 0.1, depth_norm=True)
    use_graph = bool(args.graph) and world.device.type == "cuda"
    if use_graph:
        from monocular_depth_estimation_amd.train import GraphTrainer
        # the measured step keeps BN in train mode (batch statistics every step),
        # the heavier of the reference's two modes (DESIGN.md "BatchNorm mode")
        trainer = GraphTrainer(model, loss_fn, world, lr=1e-4, amp=args.amp, eval_quirk=False)
        args.warmup = max(args.warmup, trainer.eager_steps + 1)  # capture happens in warm-up
    else:
        trainer = Trainer(wrap_ddp(model, world), make_adam(model, 1e-4), loss_fn, world,
                          eval_quirk=False, amp=args.amp)
    trainer.begin_epoch()
    batches = [synthetic_batch(args.bs, args.height, args.width, world.rank, s, world.device)
               for s in range(2)]

    def barrier():
        if world.size > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def log(msg):
        if world.is_main:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    log(f"model on {world.device}, world {world.size}, bs {args.bs}, {args.height}x{args.width}")
    for i in range(args.warmup):
        ts = time.perf_counter()
        trainer.step(*batches[i % 2])
        torch.cuda.synchronize()
        log(f"warmup step {i}: {time.perf_counter() - ts:.3f} s")
    barrier()
    # per-step HIP events on the launch stream (between graph replays: they do
    # not perturb the step) for the median; `value` is the whole timed region
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] \
        if world.device.type == "cuda" else None
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for i in range(args.steps):
        trainer.step(*batches[i % 2])
        if evs:
            evs[i + 1].record()
    barrier()
    elapsed = time.perf_counter() - t0
    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)) if evs else []
    median_ms = step_ms[len(step_ms) // 2] if step_ms else None
    # Per-kernel HIP-event timing (the registry brackets every ABI launch on its
    # stream).  Graph mode: the step is captured once more with the events as
    # graph nodes and that graph is replayed `timing_steps` times, so the times
    # are those of the REPLAYED step; eager mode: the timed loop is re-run.
    kernels = {}
    timing_steps = args.timing_steps if use_graph else args.steps
    if not args.no_kernel_timing:
        if use_graph:
            kernels = trainer.timed_replays(batches, args.timing_steps)
        else:
            _abi.timing_reset()
            _abi.timing_enable(True)
            for i in range(args.steps):
                trainer.step(*batches[i % 2])
            barrier()
            _abi.timing_enable(False)
            kernels = _abi.timing_collect()
    if world.size > 1:
        t = torch.tensor([elapsed], device=world.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss = float(trainer.last_loss)
    backend = dist.get_backend() if dist.is_initialized() else None
    if world.size == 1:
        dp_exchange = None
    elif not use_graph:
        dp_exchange = f"DDP buckets over {backend} (eager, overlapped with backward)"
    elif trainer.scheme == "overlap":
        dp_exchange = (f"overlap (opt-in, MDE_DP_OVERLAP=1): {len(trainer.buckets)} gradient "
                       f"buckets, all_reduce(AVG) over {backend} captured into the step graph, "
                       "overlapped with backward (a captured multi-rank RCCL collective has not "
                       "run on hardware in this repo's testing: the pool gives one GPU per call)")
    else:
        dp_exchange = (f"flat (default): graph A (forward, backward, gradients packed x 1/N) -> "
                       f"one eager all_reduce(SUM) over {backend} -> graph B (unpack, Adam); "
                       "no captured collective")
    in_sync = params_in_sync(trainer.params if use_graph else list(model.parameters()), world)
    if use_graph:
        trainer.close()  # free the graphs (captured RCCL nodes) before the group goes
    if not world.is_main:
        if dist.is_initialized():
            dist.destroy_process_group()
        return

    images = world.size * args.bs * args.steps
    pmc = {}
    pmc_file = next((f for f in pmc_files(args.workload, args.amp) if os.path.exists(f)), None)
    if pmc_file:
        with open(pmc_file) as f:
            pmc = json.load(f)

    def roof(name):
        ms, launches, nbytes, flops = kernels[name]
        per_launch = nbytes / launches
        # PMC HBM bytes of this registry name per step (all its launches), per launch
        per_step = pmc.get(name, {}).get("bytes_per_step")
        if per_step is None:  # one kernel behind several ids ("a+b"): split by algorithmic bytes
            for key, val in pmc.items():
                parts = key.split("+")
                if len(parts) > 1 and name in parts and isinstance(val, dict):
                    alg = sum(kernels[p][2] for p in parts if p in kernels)
                    per_step = val.get("bytes_per_step", 0) * nbytes / alg if alg else None
        traffic = per_step / (launches / timing_steps) if per_step else None
        common = {"kernel": name, "traffic": traffic,
                  "traffic_ratio": round(traffic / per_launch, 3) if traffic else None,
                  "bytes_per_launch": per_launch, "avg_launch_us": round(ms * 1e3 / launches, 2),
                  "launches_per_step": launches / timing_steps,
                  "ms_per_step": round(ms / timing_steps, 3)}
        if flops > 0:  # MFMA kernels: the fp32 MFMA peak, or bf16's for the *_bf16 ids
            achieved = flops / (ms * 1e-3) / 1e12
            peak = MFMA_BF16_PEAK_TFS if name.endswith("_bf16") else MFMA_F32_PEAK_TFS
            return dict({"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1),
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "flops_per_launch": flops / launches}, **common)
        achieved = nbytes / (ms * 1e-3) / 1e9
        return dict({"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4)}, **common)

    roofline, leaders = None, {}
    if kernels:
        by_time = sorted(kernels, key=lambda k: -kernels[k][0])
        roofline = roof(by_time[0])
        for bound in ("hbm", "mfma"):
            name = next((k for k in by_time if (kernels[k][3] > 0) == (bound == "mfma")), None)
            if name:
                leaders[bound] = roof(name)
        roofline["timing"] = ("HIP events captured into the replayed step graph, "
                              f"{timing_steps} replays" if use_graph else
                              f"HIP events over {timing_steps} eager steps")
        roofline["pmc_source"] = os.path.relpath(pmc_file, REPO) if pmc_file else None
    # north_star's "depthwise+upsample path": every resize (bilinear, nearest)
    # and depthwise-conv launch of the step, aggregated (sum bytes / sum time)
    path = {k: v for k, v in kernels.items()
            if k.startswith(("bilinear", "nearest", "dwconv"))}
    path_roofline = None
    if path:
        ms = sum(v[0] for v in path.values())
        nbytes = sum(v[2] for v in path.values())
        achieved = nbytes / (ms * 1e-3) / 1e9
        path_roofline = {"bound": "hbm", "kernels": sorted(path), "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "ms_per_step": round(ms / timing_steps, 3)}
    if args.workload == "guidedepth":
        metric = "training images/sec at 640x480 bs=32/GPU (GuideDepth, SSIM+0.1*L1, Adam)"
        workload = ("GuideDepth (DDRNet-23-slim + 3 guided upsampling blocks) train step, "
                    "BASELINE cfg2, BN in train mode")
    elif args.workload == "newcrf":
        metric = "training images/sec at 640x480 bs=16/GPU (MobileNetV3-L + NewCRF, SSIM+0.1*L1, Adam)"
        workload = ("PTModel (MobileNetV3-Large encoder + NewCRF decoder, window attention on "
                    "MFMA) train step, BASELINE cfg4, BN in train mode")
    else:
        metric = "training images/sec at 640x480 bs=16/GPU (MobileNetV3-L + SAM, SSIM+0.1*L1, Adam)"
        workload = ("PTModel of model_mobileV3_large_SAM (frozen MobileNetV3-Large encoder + SAM "
                    "cross-window attention decoder on MFMA) train step, BN in train mode")
    if args.amp == "bf16":
        workload += "; bf16 autocast (BASELINE cfg3 precision)"
    out = {
        "metric": metric,
        "value": round(images / elapsed, 2), "unit": "images/s", "n_gpus": world.size,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "ms_per_step_median": round(median_ms, 3) if median_ms else None,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if args.amp == "fp32" else AMP_DTYPE,
        "data": "synthetic (U[0,1) images, U[0.1,10) depths, resident in HBM), random-init weights",
        "config": {"workload": workload,
                   "global_batch": world.size * args.bs, "per_gpu_batch": args.bs,
                   "resolution": f"{args.width}x{args.height}", "parallelism": f"dp{world.size}"},
        "loss_last": round(loss, 6),
        "execution": ("hipGraph replay of the whole step (GraphTrainer)" if use_graph
                      else "eager (Trainer + DDP)"),
        "dp_exchange": dp_exchange,
        "gemm_table": os.path.relpath(gemm_path, REPO) if gemm_path else None,
        "params_in_sync": in_sync,
        "roofline": roofline,
        "roofline_leaders": leaders,
        "path_roofline": path_roofline,
        "hip_kernels_note": (f"ms_total / launches summed over {timing_steps} timed "
                             f"steps; ms_per_step = ms_total / {timing_steps}"),
        "hip_kernels": {k: dict({"ms_total": round(v[0], 3), "launches": v[1],
                                 "ms_per_step": round(v[0] / max(timing_steps, 1), 4),
                                 "GBps": round(v[2] / (v[0] * 1e-3) / 1e9, 1) if v[0] > 0 else None},
                                **({"TFLOPs": round(v[3] / (v[0] * 1e-3) / 1e12, 2)} if v[3] > 0 else {}))
                        for k, v in sorted(kernels.items(), key=lambda kv: -kv[1][0])},
    }
    if world.size == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
