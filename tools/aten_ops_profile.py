"""Which ATen ops launch the remaining non-HIP, non-conv kernels of one eager
cfg2 GuideDepth train step (fp32, bs 32, 640x480): torch.profiler with input
shapes, self device time per (op, shapes), top entries.  Used to find the
`vectorized_elementwise_kernel` launches of the steady-state profile."""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--amp", default="")
    ap.add_argument("--workload", choices=("guidedepth", "newcrf"), default="guidedepth")
    args = ap.parse_args()
    from monocular_depth_estimation_amd import GuideDepth
    from monocular_depth_estimation_amd.loss import SSIML1
    from monocular_depth_estimation_amd.train import Trainer, init_world, make_adam, synthetic_batch
    world = init_world()
    torch.manual_seed(0)
    if args.workload == "newcrf":  # cfg4 (bs 16)
        from monocular_depth_estimation_amd.model_mobileV3_large_newCRFs import PTModel
        model = PTModel().to(world.device)
    else:
        model = GuideDepth(pretrained=False).to(world.device)
    tr = Trainer(model, make_adam(model, 1e-4), SSIML1(1.0, 0.1, depth_norm=True), world,
                 eval_quirk=False, amp=args.amp)
    tr.begin_epoch()
    batch = synthetic_batch(args.bs, 480, 640, 0, 0, world.device)
    for _ in range(3):
        tr.step(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.step(*batch)
        torch.cuda.synchronize()
    table = prof.key_averages(group_by_input_shape=True)
    rows = [e for e in table if e.self_device_time_total > 0 and e.key.startswith("aten::")]
    rows.sort(key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in rows)
    print(f"aten self device time: {tot / 1e3:.3f} ms/step over {len(rows)} (op, shape) rows")
    for e in rows[:args.top]:
        print(f"{e.self_device_time_total / 1e3:8.3f} ms {e.count:4d}x  {e.key:32s} {str(e.input_shapes)[:150]}")
    other = [e for e in rows if not any(k in e.key for k in ("mm", "convolution", "miopen"))]
    print("other aten ops (no GEMM / convolution):")
    for e in other[:args.top]:
        print(f"{e.self_device_time_total / 1e3:8.3f} ms {e.count:4d}x  {e.key:32s} {str(e.input_shapes)[:150]}")
    # the vendor convolutions: which module shapes still reach MIOpen, and its kernels
    conv = [e for e in prof.key_averages(group_by_input_shape=True)
            if ("convolution" in e.key or "miopen" in e.key) and e.device_time_total > 0]
    conv.sort(key=lambda e: -e.device_time_total)
    print("convolution ops reaching ATen (total device time incl. children):")
    for e in conv[:args.top]:
        print(f"{e.device_time_total / 1e3:8.3f} ms {e.count:4d}x  {e.key:32s} {str(e.input_shapes)[:200]}")
    kern = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and (
                "miopen" in ev.name.lower() or "transpose" in ev.name.lower()
                or "Sp3" in ev.name or "naive_conv" in ev.name):
            kern[ev.name[:90]] += ev.device_time_total
    # which CPU op launched each vendor conv kernel (innermost op with the kernel)
    owners = collections.Counter()
    for ev in prof.events():
        for k in getattr(ev, "kernels", []) or []:
            if "miopen" in k.name.lower() or "Sp3" in k.name or "igemm" in k.name:
                owners[(ev.name, str(ev.input_shapes)[:120], k.name[:48])] += 1
    print("vendor conv kernels by launching op:")
    for (op, shapes, kn), c in owners.most_common(args.top):
        print(f"{c:4d}x  {op:28s} {kn:48s} {shapes}")
    print("vendor conv / transpose kernels:")
    for name, t in kern.most_common(args.top):
        print(f"{t / 1e3:8.3f} ms  {name}")


if __name__ == "__main__":
    main()
