"""Headline benchmark: IntentNetViT training step (fwd + loss + bwd + AdamW) on synthetic
BEV tensors of the constants.py grid — BASELINE.json metric "BEV samples/sec (fwd+bwd)
IntentNetViT at 1/2/4/8 MI355X; attn MFMA util %", config 2 (bf16, batch 8 per GPU) at
N=1 and config 3 (DDP over RCCL) for N>1.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without torchrun's environment, ``--gpus N > 1`` starts the N ranks itself (child processes with
RANK / LOCAL_RANK / WORLD_SIZE set, started before this process touches the GPU) and exits with
their status; a WORLD_SIZE that disagrees with --gpus, or fewer visible GPUs than N, is an error.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "visiontransformer-intention-prediction_amd")
sys.path.insert(0, PKG)

PEAK_BF16_TFLOPS = 2516.6  # 256 CU x 2.4 GHz x 4096 dense bf16 flop/clk (MI355X_MICROARCH.md)


def step_flops(B, H, W, depth=12, D=384, C_l=290, C_m=9, planes=512, A=5, K=8, adapter=192):
    """Algorithmic fwd+bwd FLOPs of one train step (2*MAC; bwd = 2 x fwd except patch-embed dgrad)."""
    Np = (H // 8) * (W // 8)
    N = Np + 1
    per_block = 2 * N * D * (3 * D) + 2 * N * D * D + 2 * 2 * N * D * 4 * D + 2 * 2 * N * N * D
    vit = 2 * depth * per_block
    patch = 2 * Np * D * 64 * (C_l + C_m)
    adapters = 2 * 2 * Np * D * adapter
    cin = 2 * adapter
    fusion = 2 * Np * planes * (9 * cin + 9 * planes + cin + 9 * planes + 9 * planes)
    heads = 2 * Np * 9 * planes * A * (7 + K)
    fwd = vit + patch + adapters + fusion + heads
    return B * (3 * fwd - patch), B * (3 * vit), B * fwd


# The dominant kernels of the bf16 step (profiles/r02_*_bench_kernel_stats.csv): the attention
# backward pair of ivit_attn_bwd_q2 (attn_bwd_dq_v3 + attn_bwd_dkv_v3, ~31 % of GPU time), then the
# attention forward (ivit_attn_fwd_q2, ~13 %). The roofline object reports whichever of the two has
# the larger measured time per step: kernel execution time from HIP event pairs bound to the kernel
# launches themselves (ivit_ktime_*: hipExtLaunchKernel start / stop events, the interval rocprofv3's
# kernel trace reports), inside the timed loop. The stream-span figure (events recorded around the
# launch on the launching stream) is reported beside it: it also counts time the kernel waited
# behind the other ViT stream's kernels.
ATTN = {
    "attn_bwd": {"kernels": ["attn_bwd_dq_v4_kernel", "attn_bwd_dkv_v4_kernel"], "entry": "ivit_attn_bwd_q2",
                 "tags": (1, 2),
                 "flops_note": "8*B*H*N^2*64 (dQ, dK, dV, dP products; the S recompute is not counted)"},
    "attn_fwd": {"kernels": ["attn_fwd_bf16_v6_kernel"], "entry": "ivit_attn_fwd_q2", "tags": (0,),
                 "flops_note": "4*B*H*N^2*64 (QK^T, PV)"},
}


def kernel_exec_ms(ops, name):
    """-> (busy ms per launch, mean kernel-sum ms per launch, launches) for one ATTN entry from its
    kernels' recorded execution intervals (ivit_ktime_read, both ViT streams): busy = the union of
    the intervals (time at least one of its kernels was executing) / launches — the device time per
    launch when the two streams' launches overlap each other; the mean interval sum counts a
    shared stretch once per launch."""
    iv = []
    n0 = None
    for tag in ATTN[name]["tags"]:
        r = ops.ktime_read(tag)
        iv += r
        n0 = len(r) if n0 is None else n0
    if not n0:
        return float("nan"), float("nan"), 0
    return ops.busy_ms(iv) / n0, sum(b - a for a, b in iv) / n0, n0


def write_intervals(ops, path):
    """The attention kernels' execution intervals recorded in the timed region (ivit_ktime_read),
    as a rocprofv3-kernel-trace-shaped CSV (Kernel_Name, Start_Timestamp, End_Timestamp in ns from
    the first recorded launch, Launch = index within the kernel): the input of tools/kunion.py."""
    import csv
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Launch", "Start_Timestamp", "End_Timestamp"])
        for name in ATTN:
            for tag, kern in zip(ATTN[name]["tags"], ATTN[name]["kernels"]):
                for i, (a, b) in enumerate(ops.ktime_read(tag)):
                    w.writerow([kern, i, int(round(a * 1e6)), int(round(b * 1e6))])


def rocprof_union(name):
    """(us per launch, source, generated) of the newest committed rocprofv3-trace union of an ATTN
    entry's kernels (profiles/*_<name>_union.json, written by tools/kunion.py --json from the kernel
    trace of a profiled bench command), or (None, None, None). A file whose matched kernel names
    (``kernel_names``) are not exactly the entry's current kernels is stale and skipped; files
    older than that field are skipped too."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"*_{name}_union.json")),
                   key=lambda p: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(p))])
    want = ATTN[name]["kernels"]
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            if d.get("source_kind") != "rocprofv3":
                continue
            got = d.get("kernel_names", [])
            if not (got and all(any(w in k for w in want) for k in got) and all(any(w in k for k in got) for w in want)):
                continue
            return float(d["union_us_per_launch"]), os.path.relpath(f, HERE), d.get("generated_utc")
        except (OSError, ValueError, KeyError):
            continue
    return None, None, None


def warm_time_ms(fn, warm_s=2.0, iters=20, reps=3):
    """Launch time of fn the way tools/attn_bench.py and DESIGN quote isolated kernels: >= warm_s
    seconds of back-to-back launches first (the clock ramps under sustained MFMA load,
    MI355X_MICROARCH.md "DVFS"; one warm launch read 0.81-0.83 ms where the warm pair runs
    0.71-0.73), then the median over ``reps`` of the mean of ``iters`` launches (HIP events).
    -> (median ms, [ms per rep])."""
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    res = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters)
    return sorted(res)[len(res) // 2], res


def attn_flops(name, B, N, H, Dh=64):
    return (8.0 if name == "attn_bwd" else 4.0) * B * H * N * N * Dh


def attn_bytes(name, B, N, H, Dh=64):
    """Algorithmic HBM bytes per launch: forward reads qkv, writes out + lse; backward reads qkv, out,
    dO, lse and writes dqkv (bf16), plus the padded f32 row constants written and read once."""
    if name == "attn_fwd":
        return B * N * 3 * H * Dh * 2 + B * N * H * Dh * 2 + B * H * N * 4
    return B * N * 3 * H * Dh * 2 * 2 + 2 * B * N * H * Dh * 2 + B * H * N * 4 + 2 * 2 * B * H * N * 4


def pmc_traffic(kernel_prefix):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (profiles/*_pmc_hbm.json, written by tools/pmc_summary.py from separate rocprofv3
    FETCH_SIZE / WRITE_SIZE passes of this same bench command, gfx950 corrections applied)."""
    import glob
    # newest = highest round / version number (natural order: r01_v10 after r01_v9)
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc_hbm.json")),
                   key=lambda p: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(p))])
    if not files:
        return None, None
    try:
        with open(files[-1]) as fh:
            kern = json.load(fh)["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    prefixes = [kernel_prefix] if isinstance(kernel_prefix, str) else list(kernel_prefix)
    tot, found = 0.0, 0
    for pre in prefixes:
        for name, v in kern.items():
            if name.startswith(pre) and v.get("hbm_bytes_avg") is not None:
                tot += float(v["hbm_bytes_avg"])
                found += 1
                break
    if found != len(prefixes):
        return None, None
    return tot, os.path.relpath(files[-1], HERE)


def isolated_attn_ms(name, B, N, H, dev):
    """ivit_attn_fwd_q2 / ivit_attn_bwd_q2 alone at the bench shape, warm (warm_time_ms)."""
    import ops
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * N, 3 * H * 64, device=dev, generator=g).to(torch.bfloat16)
    qkv[:, : H * 64] = (qkv[:, : H * 64].float() * ops.Q2_SCALE).to(torch.bfloat16)
    dout = torch.randn(B * N, H * 64, device=dev, generator=g).to(torch.bfloat16)
    o, lse = ops.attn_fwd_q2(qkv, B, N, H)
    fn = (lambda: ops.attn_fwd_q2(qkv, B, N, H)) if name == "attn_fwd" else \
        (lambda: ops.attn_bwd_q2(qkv, o, dout, lse, B, N, H))
    return warm_time_ms(fn)


def cpu_model_name():
    """lscpu's "Model name" (the first /proc/cpuinfo model name line)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def granted_cpus():
    """(threads to use, how the number was found): the cgroup CPU quota (cpu.max) when one is set
    — the host cores this job may actually use — else the scheduler affinity mask."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        if q != "max":
            n = max(1, int(int(q) // int(p)))
            return min(n, aff), f"cgroup cpu.max quota {q}/{p} = {int(q) / int(p):g} CPUs"
    except (OSError, ValueError):
        pass
    return aff, "sched_getaffinity (no cgroup CPU quota)"


def cpu_baseline(steps=3):
    """The reference's CPU path restated by the oracle (timm semantics with the fused
    F.scaled_dot_product_attention, as timm's Attention.fused_attn runs it): f32 train step
    (forward, loss, backward, torch AdamW), B=1, full grid, on this host's cores; median of
    ``steps`` timed steps after one warm-up."""
    sys.path.insert(0, HERE)
    from oracle import ivit_oracle as O
    from oracle.weights import make_state_dict, model_cfg
    threads, why = granted_cpus()
    torch.set_num_threads(threads)
    cfg = model_cfg()
    sd = {k: (v.requires_grad_(True) if v.is_floating_point() and "running" not in k else v)
          for k, v in make_state_dict(cfg, seed=0).items()}
    opt = torch.optim.AdamW([v for v in sd.values() if v.requires_grad], lr=1e-4, weight_decay=1e-4)
    lidar, mp, gts = O.synthetic_batch(1, seed=1234)
    anchors = O.generate_anchors()

    def step():
        opt.zero_grad()
        c, b, i = O.intentnet_forward(sd, lidar, mp, cfg, training=True, attn="sdpa")
        d = O.detection_loss(c, b, i, anchors, gts, downsampling=True)
        d["loss"].backward()
        opt.step()

    step()  # warm-up
    ts = []
    for _ in range(steps):
        t0 = time.time()
        step()
        ts.append(time.time() - t0)
    med = sorted(ts)[len(ts) // 2]
    return {"value": 1.0 / med, "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu": cpu_model_name(), "os_cpu_count": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "cores_source": why,
            "sample": f"oracle f32 train step (fwd with SDPA attention + loss + bwd + AdamW), B=1, 400x720, "
                      f"median of {steps} after 1 warm-up",
            "step_s": med, "steps_s": [round(t, 3) for t in ts]}


def visible_gpus():
    """GPUs this process may use, counted without initialising HIP: torch.cuda.device_count() reads
    the device count without creating a context on this image — checked here, because the parent
    of the rank processes must never touch the GPU (it would be forked / exec'd around a live
    context)."""
    n = torch.cuda.device_count()
    if torch.cuda.is_initialized():
        raise RuntimeError("bench.py: counting GPUs initialised HIP in the launcher process")
    return n


def launch_ranks(n, argv=None, have=None, poll_s=0.2):
    """Start ranks 0..n-1 of this same command (or ``argv``) as child processes with torchrun's
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR / MASTER_PORT on 127.0.0.1) and return
    the first non-zero exit status (the other ranks are terminated then), else 0. ``have``: the
    visible GPU count (default visible_gpus()); fewer than n is refused with status 2."""
    import socket
    import subprocess
    have = visible_gpus() if have is None else have
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs, {have} visible", file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    argv = argv if argv is not None else [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(poll_s)
    return rc


def time_forced_buckets(model, opt, lf, anchors, batch, args, plain_ms):
    """The DDP leg of configs 3 / 5 on one GPU: the same step through Trainer(force_buckets=True)
    on a world-1 RCCL process group — every gradient a view into the 64-MB buckets, one event per
    parameter on its producing ViT stream, the bucket all-reduces on the comm stream overlapping
    backward, finish() waiting — timed exactly as the plain step, right after it."""
    from trainer import Trainer
    tr = Trainer(model, lf, opt, anchors, world=1, bucket_mb=args.bucket_mb, check_nan=False, force_buckets=True)
    if tr.buckets is None or not tr.buckets.active:
        raise RuntimeError("--force-collectives: the bucketed collective path is not active")
    import ddp
    n0 = ddp.GradBuckets.launched
    for _ in range(args.warmup):
        tr.step(batch)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step(batch)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    per_step = (ddp.GradBuckets.launched - n0) / (args.warmup + args.steps)
    ms = el / args.steps * 1e3
    tr.buckets.remove()
    return {"backend": dist.get_backend(), "world": dist.get_world_size(), "buckets": len(tr.buckets.buckets),
            "bucket_mb": args.bucket_mb, "grad_mb": round(tr.buckets.numel * 4 / 2 ** 20, 1),
            "all_reduces_per_step": per_step, "ms_per_step_buckets": round(ms, 3),
            "ms_per_step_plain": round(plain_ms, 3), "overhead_ms": round(ms - plain_ms, 3),
            "note": "same process, same batch, timed right after the plain step (which is `value`): "
                    "Trainer(force_buckets=True) on a world-1 RCCL group, so every bucket is all-reduced "
                    "(a world-1 ring moves no bytes over xGMI; this is the launch / stream / event cost "
                    "of the DDP path inside the step)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["train", "eval"], default="train",
                    help="train: configs 2/3/5 (fwd+loss+bwd+AdamW); eval: config 4 (inference + decode + NMS)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (configs 2/3/5: 8; config 4: 32)")
    ap.add_argument("--grid", type=str, default="400x720")
    ap.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--augment", action="store_true",
                    help="train mode: run the training-time augment_bev (dataset.py:352-353) on the batch "
                         "inside every timed step (ivit_bev_augment passes)")
    ap.add_argument("--intervals-out", type=str, default=None,
                    help="write the attention kernels' recorded execution intervals of the timed region (the "
                         "roofline's device time) as a kernel-trace CSV; tools/kunion.py recomputes the union")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the isolated attention leg (profiled runs: its warm-up launches would enter the "
                         "kernel trace's union and averages)")
    ap.add_argument("--bucket-mb", type=float, default=64)
    ap.add_argument("--ddp", choices=["buckets", "torch"], default="buckets",
                    help="gradient exchange: ddp.GradBuckets (default) or torch DistributedDataParallel")
    ap.add_argument("--force-collectives", action="store_true",
                    help="N=1 train mode: also time the bucketed RCCL path (a world-1 process group, "
                         "Trainer(force_buckets=True): comm stream, per-parameter events, the all-reduces) "
                         "right after the plain step in the same process; both go into the line")
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')} ranks were launched")

    sys.path.insert(0, PKG)
    from ddp import init_distributed
    force = args.force_collectives and args.gpus == 1 and args.mode == "train"
    if force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            so = socket.socket()
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(so.getsockname()[1])
            so.close()
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("LOCAL_RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    # RCCL prints its version banner to stdout (C level) when the communicator comes up: route fd 1 to
    # stderr around the group's creation and first collective, so stdout carries only the JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        rank, local, world, dev = init_distributed(force_group=force)
        if dist.is_initialized():
            dist.barrier()
            if dev.type == "cuda":
                torch.cuda.synchronize()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    if dev.type != "cuda":
        raise RuntimeError("bench.py needs a ROCm GPU (the HIP kernels have no CPU path)")
    world = dist.get_world_size() if dist.is_initialized() else 1
    backend = dist.get_backend() if dist.is_initialized() else "none (single process)"

    import loss as L
    import model_vit
    import ops
    import utils
    from optim import FusedAdamW
    from synthetic import synthetic_batch
    from trainer import Trainer

    H, W = (int(v) for v in args.grid.split("x"))
    train = args.mode == "train"
    B = args.batch if args.batch is not None else (8 if train else 32)
    cd = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    model = model_vit.IntentNetViT(backbone_cfg={"img_size": (H, W)}).to(dev).set_compute_dtype(cd)
    model.train(train)
    anchors = utils.generate_anchors(H, W, 8, device=dev)
    # inputs resident in HBM before the timed region (SURVEY.md §8d primary placement)
    batch = synthetic_batch(B, (H, W), torch.Generator().manual_seed(1234 + rank), device=dev)
    if train:
        net = model
        if world > 1 and args.ddp == "torch":
            net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], bucket_cap_mb=args.bucket_mb,
                                                            gradient_as_bucket_view=True, broadcast_buffers=False)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
        lf = L.DetectionIntentionLoss(use_rotated_iou=False, apply_intention_downsampling=True)
        trainer = Trainer(net, lf, opt, anchors, world=world if args.ddp == "buckets" else 1,
                          bucket_mb=args.bucket_mb, check_nan=False)
        if trainer.buckets is None and world > 1 and args.ddp == "buckets":
            raise RuntimeError("gradient buckets missing for world > 1")

        if args.augment:
            import random
            random.seed(1234 + rank)
            aug_out = (torch.empty_like(batch["lidar_bev"]), torch.empty_like(batch["map_bev"]))

            def step():
                lo, mo, gts, _ = utils.augment_bev_batch(batch["lidar_bev"], batch["map_bev"], batch["gt_list"],
                                                         out=aug_out)
                return trainer.step({"lidar_bev": lo, "map_bev": mo, "gt_list": gts})
        else:
            def step():
                return trainer.step(batch)
    else:
        kept = []
        # eval_vit.run_inference's loop: a batch's post-processing runs on its own stream beside the
        # next batch's forward (utils.PostPipeline); flush() before and at the end of the timed
        # region, so it holds exactly `steps` forwards and `steps` post-processings
        pipe = utils.PostPipeline(anchors, 0.1, 0.2)

        def collect(preds):
            if preds is not None:
                kept.append(sum(int(p["pred_scores"].numel()) for p in preds))

        def step():  # eval_vit.py:144-180: forward, sigmoid >= 0.1, decode, NMS(0.2), argmax intention
            with torch.inference_mode():
                cls, box, it = model(batch["lidar_bev"], batch["map_bev"])
                collect(pipe.push(cls, box, it))
            return {"loss": torch.zeros(())}

    for _ in range(args.warmup):
        step()
    if args.mode == "eval":
        collect(pipe.flush())
    torch.cuda.synchronize()
    timing = os.environ.get("IVIT_BENCH_KTIME", "1") != "0"  # 0: no attention timing in the loop (A/B of its cost)
    ops.KernelTimer.enabled = set(ATTN) if timing else set()
    ops.KernelTimer.records = {}
    ops.ktime_arm(timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        d = step()
    if args.mode == "eval":
        collect(pipe.flush())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ops.ktime_arm(False)
    if args.intervals_out and timing:
        write_intervals(ops, args.intervals_out)
    span_ms = {k: ops.KernelTimer.mean_ms(k) for k in ATTN}
    kexec = {k: kernel_exec_ms(ops, k) for k in ATTN}
    attn_ms = {k: kexec[k][0] for k in ATTN}
    attn_n = {k: kexec[k][2] for k in ATTN}
    ops.KernelTimer.enabled = set()
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    loss_v = float(d["loss"].detach())
    gb = B * world
    value = gb * args.steps / el
    ms = el / args.steps * 1e3
    fl_step, fl_vit, fl_fwd = step_flops(B, H, W)
    if not train:
        fl_step = fl_fwd
    N = (H // 8) * (W // 8) + 1
    peak = PEAK_BF16_TFLOPS if cd == torch.bfloat16 else 157.3
    # dominant attention kernel(s): larger measured time per step
    per_step = {k: (attn_ms[k] * attn_n[k] / args.steps if attn_n[k] else 0.0) for k in ATTN}
    roof = max(per_step, key=per_step.get) if any(per_step.values()) else "attn_fwd"
    afl = attn_flops(roof, B, N, 6)
    achieved = afl / (attn_ms[roof] * 1e-3) / 1e12 if attn_n[roof] else float("nan")
    # PMC traffic was collected on the default train configuration only
    default_cfg = train and (H, W) == (400, 720) and B == 8 and cd == torch.bfloat16 and not args.augment
    traffic, traffic_src = pmc_traffic(ATTN[roof]["kernels"]) if default_cfg else (None, None)
    # attention MFMA utilisation (BASELINE metric "attn MFMA util %"): attention fwd + bwd algorithmic
    # flops per step / their measured kernel time per step; ViT attention + MLP block flops per step /
    # the whole step's wall time (a lower bound for the blocks' own utilisation)
    at_ms = sum(per_step.values())
    at_fl = sum(attn_flops(k, B, N, 6) * attn_n[k] / args.steps for k in ATTN)
    if train:
        workload = f"IntentNetViT train step (fwd+loss+bwd+AdamW), {args.dtype}, {H}x{W}, batch {B}/GPU"
        if args.augment:
            workload = "augment_bev (GPU) + " + workload
        metric = "BEV samples/sec (fwd+bwd) IntentNetViT at 1/2/4/8 MI355X; attn MFMA util %"
    else:
        workload = (f"IntentNetViT eval_vit.py inference (fwd + sigmoid/threshold 0.1 + decode + NMS 0.2 + argmax; "
                    f"a batch's post-processing beside the next batch's forward, as eval_vit.run_inference), "
                    f"{args.dtype}, {H}x{W}, batch {B}/GPU")
        metric = "BEV samples/sec inference (eval_vit.py path) IntentNetViT on MI355X"
    out = {
        "metric": metric,
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "backend": backend, "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (random BEV rasters U[0,1)/Bernoulli(0.1), 20 random GT/sample; "
                                     "random-init weights)",
        "config": {"workload": workload, "global_batch": gb, "per_gpu_batch": B, "grid": [H, W],
                   "tokens_per_stream": N, "parallelism": f"dp{world}"},
        "roofline": {"kernel": " + ".join(ATTN[roof]["kernels"]) + f" ({ATTN[roof]['entry']})", "bound": "mfma",
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "per_launch": f"{ATTN[roof]['flops_note']} = {afl:.4g} flop (B={B}, H=6, N={N}); "
                                   f"{attn_ms[roof]:.4f} ms of device time per launch = the union of the "
                                   f"execution intervals of its kernels over {attn_n[roof]} launches (both ViT "
                                   f"streams; hipExtLaunchKernel start/stop events bound to each kernel) / launches",
                     "launch_ms": round(kexec[roof][1], 4),
                     "launch_note": "mean execution interval of one launch (its kernels summed): when the two "
                                    "streams' launches overlap, each one's interval covers the shared stretch",
                     "stream_span_ms": round(span_ms[roof], 4),
                     "stream_span_note": "events recorded before / after the entry point on its stream: also "
                                         "counts the wait behind the other stream's kernels",
                     "traffic_note": (f"HBM bytes per launch from {traffic_src} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                      f"gfx950-corrected, summed over the kernels); algorithmic bytes "
                                      f"{attn_bytes(roof, B, N, 6):.4g}")
                     if traffic is not None else "no PMC summary for this configuration",
                     "per_step_ms": {k: round(v, 3) for k, v in per_step.items()}},
        "attn_mfma_util": {
            "attention_fwd_bwd": round(at_fl / (at_ms * 1e-3) / 1e12 / peak, 4) if at_ms else None,
            "vit_blocks_lower_bound": round((fl_vit if train else fl_vit / 3) / (el / args.steps) / 1e12 / peak, 4),
            "note": "attention_fwd_bwd: 12*B*H*N^2*64 flops per block pass (fwd 4 + bwd 8, no recompute) per step / "
                    "the measured attention kernel time per step; vit_blocks_lower_bound: ViT attention + MLP "
                    "block fwd+bwd flops per step / the whole step's wall time; peak = dense bf16 MFMA"},
        "step_mfma": {"achieved": round(fl_step * world / el * args.steps / 1e12 / world, 2), "unit": "TFLOP/s/GPU",
                      "frac": round(fl_step / (el / args.steps) / 1e12 / peak, 4),
                      "flops_per_step_per_gpu": fl_step},
    }
    if default_cfg:
        # the same launches' device time from a committed rocprofv3 kernel trace of the profiled
        # bench command (tools/kunion.py --json): the figure the profile files reproduce
        us, src, gen = rocprof_union(roof)
        if us is not None:
            out["roofline"]["frac_rocprof"] = round(afl / (us * 1e-6) / 1e12 / peak, 4)
            out["roofline"]["frac_rocprof_source"] = {"file": src, "generated_utc": gen}
            out["roofline"]["frac_rocprof_note"] = (f"{us:.1f} us per launch = the union of the kernels' intervals in "
                                                    f"the rocprofv3 kernel trace summarised in {src} (a committed "
                                                    f"profile of the same kernels, not this run; profiled command: "
                                                    f"the profiler lowers the clock, MI355X_MICROARCH.md DVFS item 2)")
    if args.intervals_out and timing:
        out["roofline"]["intervals_file"] = os.path.relpath(os.path.abspath(args.intervals_out), HERE)
    if default_cfg and world == 1 and not args.no_isolated:
        # the same kernel(s) alone on the same shape (outside the timed region): the frac without the
        # other ViT stream's kernels sharing the CUs
        iso, reps = isolated_attn_ms(roof, B, N, 6, dev)
        out["roofline"]["isolated"] = {"ms": round(iso, 4), "achieved": round(afl / (iso * 1e-3) / 1e12, 2),
                                       "frac": round(afl / (iso * 1e-3) / 1e12 / peak, 4),
                                       "reps_ms": [round(r, 4) for r in reps],
                                       "note": "warm: 2 s of back-to-back launches, then the median of 3 x the mean "
                                               "of 20 launches (HIP events) on random bf16 inputs of the bench shape "
                                               "(prescaled Q), nothing else running — the protocol of "
                                               "tools/attn_bench.py and DESIGN's kernel table"}
    if force:
        out["collectives_world1"] = time_forced_buckets(model, opt, lf, anchors, batch, args, ms)
    if train:
        out["loss"] = loss_v
    else:
        out["kept_boxes_per_step"] = kept[-1] if kept else 0
    if rank == 0 and world == 1 and train and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
