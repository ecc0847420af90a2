#!/usr/bin/env python3
"""Headline benchmark: ResNet-18, CIFAR-10-shape synthetic data, PowerSGD r=4 (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One process per GPU, RCCL over xGMI through the framework's native communicator
(csrc/comm.cpp; c10d only bootstraps).  Each timed step is the full reference training
step (ddp_powersgd_guide_cifar10/ddp_init.py:142-178): forward, cross-entropy, backward,
EF pack, PowerSGD compress + all-reduces, decompress, error memory, momentum, SGD update.
The whole step is ONE hipGraph; the PowerSGD group pipelines (gfx950 kernels + RCCL
collectives) run on a side stream that overlaps backward.  fp32 everywhere (the
reference's dtype), random-init weights, synthetic device-resident data.

Launch + failure model (utils/supervisor.py).  The process started by the user or by
torchrun is a SUPERVISOR that never touches the GPU: it starts the GPU worker(s) as child
processes (``python bench.py --gpus N`` alone starts all N ranks itself; under torchrun
each rank's supervisor starts its one worker), each worker running ONE configuration
level of the fallback ladder below.  A worker fails its attempt by exiting non-zero
(exception, failed health check) or by stalling past the allowance of its current phase
(heartbeat file); then every worker of the attempt is killed and all ranks restart at the
next level on a fresh rendezvous.  Health checks after warm-up and after the timed steps:
RCCL async errors, the compute/comm graph flag-wait error word, finite loss, and a
cross-rank fp64 checksum of the parameters (``replicas_equal``).  A number is printed
only for a verified step; if every level fails the exit code is non-zero.

Scaling: **strong** by default for the CIFAR workloads, exactly like the reference — the
global batch is fixed at 512 (PowerSGD, ddp_powersgd_guide_cifar10/ddp_init.py:52) and
each of the N ranks trains on 512/N.  DistilBERT is weak in the reference (16 per rank,
ddp_powersgd_distillBERT_IMDb/ddp_init.py:92).

Rank 0 prints ONE JSON line.  ``value`` = whole-job samples/s (max step time over ranks).
``bytes_per_step`` = bytes all-reduced per rank per step with the reference's accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "samples/sec + bytes/step all-reduced, ResNet18 CIFAR10 PowerSGD r=4, 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE from a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet18", help="resnet18/34/50/101/152 | distilbert")
    ap.add_argument("--num-classes", type=int, default=None, help="default: 1000 (ResNet, reference head) / 2")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="strong: global batch fixed, per-GPU = global/N (CIFAR default, the reference); "
                         "weak: per-GPU batch fixed (DistilBERT default, the reference)")
    ap.add_argument("--global-batch", type=int, default=512, help="strong scaling: global batch (reference 512)")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch; implies weak scaling. Default 512 ResNet, 16 DistilBERT (reference)")
    ap.add_argument("--weak-too", choices=["on", "off"], default="off",
                    help="strong runs: also time the weak config (per-GPU 512) as an extra field")
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--reducer", choices=["powersgd", "dense", "dense-ref", "powersgd-ref", "powersgd-api"],
                    default="powersgd")
    ap.add_argument("--rank", type=int, default=4)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--no-fused-bn", action="store_true", help="use nn.BatchNorm2d + ReLU (MIOpen) instead")
    ap.add_argument("--no-gemm-convs", action="store_true", help="run every conv on MIOpen")
    ap.add_argument("--no-fused-attn", action="store_true", help="DistilBERT: explicit attention math")
    ap.add_argument("--stock", action="store_true",
                    help="stock PyTorch-ROCm model ops (MIOpen conv/BN, explicit attention): with "
                         "--reducer powersgd-ref this is the eager reference-semantics arm")
    ap.add_argument("--amp", choices=["none", "bf16"], default="none",
                    help="opt-in bf16 autocast for model math (NOT the headline: the reference is fp32)")
    ap.add_argument("--link", default="none", help="none|1g|10g|100g link emulation")
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="charge the link model for an N-rank ring even on 1 GPU (bandwidth curves)")
    ap.add_argument("--bucket-mb", type=float, default=None, help="dense arm bucket size (default 8 MB)")
    ap.add_argument("--psgd-groups", type=int, default=None, help="PowerSGD overlap groups (default 4)")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="gradient sync overlapped with backward on the side stream (auto: when N > 1 or a "
                         "link is emulated)")
    ap.add_argument("--no-overlap", action="store_true", help="= --overlap off")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-supervise", action="store_true",
                    help="run the step in this process (no supervisor / fallback; for profilers)")
    ap.add_argument("--level", type=int, default=0, help="first fallback level to try (see FALLBACKS_*)")
    ap.add_argument("--graph-mode", default="auto", choices=["auto", "full", "piecewise", "none"],
                    help="hipGraph capture of the step: full (native RCCL / N=1), piecewise (collectives "
                         "eager between captured compute; c10d data plane), none")
    a = ap.parse_args(argv)
    if a.no_overlap:
        a.overlap = "off"
    bert = a.model.startswith("distilbert")
    if a.stock:
        a.no_fused_bn = a.no_gemm_convs = a.no_fused_attn = True
    if a.scaling is None:
        a.scaling = "weak" if (bert or a.batch is not None) else "strong"
    if a.batch is None and a.scaling == "weak":
        a.batch = 16 if bert else 512
    if a.lr is None:
        a.lr = 5e-5 if bert else 1e-3
    return a


def metric_name(args) -> str:
    if args.amp != "none":
        return f"[non-headline, {args.amp} autocast] " + metric_name(argparse.Namespace(**{**vars(args), "amp": "none"}))
    if args.model == "resnet18" and args.reducer.startswith("powersgd") and args.rank == 4:
        return METRIC
    what = "DistilBERT IMDb" if args.model.startswith("distilbert") else f"{args.model} CIFAR10"
    red = f"PowerSGD r={args.rank}" if args.reducer.startswith("powersgd") else "dense all-reduce"
    return f"samples/sec + bytes/step all-reduced, {what} {red}"


class Workload:
    """Model + gradient sync + a timed-step factory for one per-GPU batch size."""

    def __init__(self, args, device, world, rank):
        import torch

        from network_distributed_pytorch_amd.models import build_model
        from network_distributed_pytorch_amd.parallel.comm import LINK_PRESETS, Communicator
        from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync

        self.args, self.device, self.world, self.rank = args, device, world, rank
        self.is_bert = args.model.startswith("distilbert")
        from network_distributed_pytorch_amd.ops import gemm_tuning

        self.tuned_gemms = gemm_tuning.enable()  # measured hipBLASLt/rocBLAS solutions (ops/gemm_tuning.py)
        self.model = build_model(args.model, args.num_classes, fused_bn=not args.no_fused_bn,
                                 gemm_convs=not args.no_gemm_convs,
                                 fused_attention=not args.no_fused_attn).to(device)
        if args.channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        link = None if args.link == "none" else LINK_PRESETS[args.link]
        native = None if getattr(args, "native_comm", True) else False
        self.comm = Communicator(link=link, emulate_world=args.emulate_world, device=device, native=native)
        kw = {}
        if args.reducer in ("powersgd", "dense"):
            if args.overlap != "auto":  # auto: overlap when a step has wire time (N > 1 / link emulation)
                kw["overlap"] = args.overlap == "on"
            if args.psgd_groups is not None and args.reducer == "powersgd":
                kw["groups"] = args.psgd_groups
        self.sync = build_grad_sync(args.reducer, self.model, self.comm, lr=args.lr, momentum=0.9,
                                    rank=args.rank, bucket_mb=args.bucket_mb, **kw)
        from network_distributed_pytorch_amd.ops.loss import CrossEntropyLoss

        # fused gfx950 softmax cross-entropy (ops/loss.py); --stock keeps PyTorch-ROCm's
        self.crit = torch.nn.CrossEntropyLoss() if args.stock else CrossEntropyLoss()
        self.loss_acc = torch.zeros((), device=device)
        # the fused loss kernel adds each step's loss into loss_acc itself (no add launch)
        self.crit_acc = not args.stock and args.amp != "bf16" and not self.is_bert
        if self.crit_acc:
            self.crit.accumulate = self.loss_acc
        self.graph_mode = None
        self.runner = None

    def make_step(self, batch: int):
        import torch

        args, device, model = self.args, self.device, self.model
        g = torch.Generator(device=device)
        g.manual_seed(1234 + self.rank)
        n_pool = 4
        if self.is_bert:
            from network_distributed_pytorch_amd.utils.data import SyntheticIMDb

            ds = SyntheticIMDb(n=n_pool * batch, seq_len=args.seq_len, seed=1234 + self.rank, device=device)
            pool = [{k: v[i * batch:(i + 1) * batch].contiguous() for k, v in ds.columns.items()}
                    for i in range(n_pool)]

            def loss_of(b):
                return model(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"])[0]
        else:
            # CIFAR-10-shape images in [-1, 1] (what ToTensor+Normalize(0.5, 0.5) yields)
            xs = (torch.rand(n_pool, batch, 3, 32, 32, device=device, generator=g) * 2 - 1)
            if args.channels_last:
                xs = torch.stack([x.contiguous(memory_format=torch.channels_last) for x in xs])
            ys = torch.randint(0, 10, (n_pool, batch), device=device, generator=g)
            pool = [{"x": xs[i], "y": ys[i]} for i in range(n_pool)]

            def loss_of(b):
                return self.crit(model(b["x"]), b["y"])

        if args.amp == "bf16":  # opt-in mixed precision: bf16 model math, fp32 params/grads/reducer
            fp32_loss_of = loss_of

            def loss_of(b):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return fp32_loss_of(b).float()

        sync, loss_acc, crit_acc = self.sync, self.loss_acc, self.crit_acc
        graph_mode = args.graph_mode
        if graph_mode == "auto" and "ref" in args.reducer:
            graph_mode = "none"  # reference-semantics arms are eager by definition
        if graph_mode != "none":
            from network_distributed_pytorch_amd.utils.graph import StepRunner

            # every batch (images + labels, or ids + mask + labels) packed in ONE byte buffer:
            # loading a batch into the graph's static inputs is one device copy, not one per tensor
            if args.channels_last:  # packing would drop the memory format: one copy per tensor
                packed = None
                static = {k: v.clone() for k, v in pool[0].items()}
            else:
                packed = [_pack(b) for b in pool]
                static_buf = packed[0][0].clone()
                static = _views(static_buf, packed[0][1])
            one = torch.ones((), device=device)  # backward seed outside the graph: no fill kernel

            def pre():
                sync.zero_grad()
                loss = loss_of(static)
                loss.backward(one)
                if not crit_acc:
                    loss_acc.add_(loss.detach())  # one add, no copy into a static loss

            runner = StepRunner(pre, sync, mode=graph_mode, warmup=3,
                                state_tensors=list(model.buffers()))
            graph_mode = runner.mode
            self.runner = runner

            def step(i):
                if packed is None:
                    for k, v in pool[i % n_pool].items():
                        static[k].copy_(v, non_blocking=True)
                else:
                    static_buf.copy_(packed[i % n_pool][0], non_blocking=True)
                runner()
        else:
            def step(i):
                sync.zero_grad()
                loss = loss_of(pool[i % n_pool])
                loss.backward()
                sync.step()
                if not crit_acc:
                    loss_acc.add_(loss.detach())
        self.graph_mode = graph_mode
        return step

    def time(self, step, steps: int, warmup: int, start: int = 0) -> float:
        import torch
        import torch.distributed as dist

        for i in range(start, start + warmup):
            step(i)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        self.comm.stats.reset()
        t0 = time.perf_counter()
        for i in range(start + warmup, start + warmup + steps):
            step(i)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([elapsed], device=self.device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed



def _pack(batch: dict):
    """(uint8 buffer, layout) holding every tensor of a batch at 16-B aligned offsets."""
    import torch

    layout, off = [], 0
    for k, v in batch.items():
        n = v.numel() * v.element_size()
        layout.append((k, off, v.dtype, tuple(v.shape)))
        off += (n + 15) // 16 * 16
    buf = torch.empty(off, dtype=torch.uint8, device=next(iter(batch.values())).device)
    for (k, o, dt, shape), v in zip(layout, batch.values()):
        buf[o: o + v.numel() * v.element_size()].view(dt).copy_(v.reshape(-1))
    return buf, layout


def _views(buf, layout) -> dict:
    import torch

    out = {}
    for k, o, dt, shape in layout:
        n = 1
        for s in shape:
            n *= s
        out[k] = buf[o: o + n * torch.empty((), dtype=dt).element_size()].view(dt).view(shape)
    return out


# Fallback ladder (one level per supervised attempt).  N > 1: native RCCL communicator with
# the step captured as compute + comm graphs overlapping backward -> collectives captured
# serially in the step graph -> c10d data plane with eager collectives between captured
# phases -> eager.  N = 1: captured (as configured) -> no overlap -> eager.
FALLBACKS_MULTI = [{}, {"overlap": "off"}, {"native_comm": False, "graph_mode": "auto"},
                   {"native_comm": False, "graph_mode": "none"}]
FALLBACKS_SINGLE = [{}, {"overlap": "off"}, {"overlap": "off", "graph_mode": "none"}]


def fallbacks(world: int):
    return FALLBACKS_MULTI if world > 1 else FALLBACKS_SINGLE


class HealthError(RuntimeError):
    pass


def health_check(wl, world: int, where: str) -> dict:
    """Fail loudly unless the step just run is trustworthy on every rank (see module doc)."""
    import math

    import torch
    import torch.distributed as dist

    from network_distributed_pytorch_amd.ops import checksum

    if wl.runner is not None:
        wl.runner.join()
    torch.cuda.synchronize()
    flag_errors = wl.comm.flag_error()
    wl.comm.check()  # RCCL async error / flag-wait timeout -> raises
    if hasattr(wl.sync, "check_errors"):
        wl.sync.check_errors()  # MGS barrier timeouts
    flat = getattr(getattr(wl.sync, "opt", None), "x", None)
    if flat is None:
        flat = getattr(getattr(wl.sync, "ddp", None), "x", None)
    if flat is None:
        flat = torch.cat([p.detach().reshape(-1) for p in wl.model.parameters()])
    local = checksum(flat)
    sums = [local]
    if world > 1:
        on = "cpu" if dist.get_backend() == "gloo" else wl.device
        t = torch.tensor([local], dtype=torch.float64, device=on)
        outs = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        sums = [float(o.item()) for o in outs]
    equal = all(s == sums[0] for s in sums) and math.isfinite(sums[0])
    loss = float(wl.loss_acc.item())
    if not equal:
        raise HealthError(f"{where}: replicas differ (parameter checksums {sums})")
    if not math.isfinite(loss):
        raise HealthError(f"{where}: non-finite loss accumulator {loss}")
    return {"replicas_equal": equal, "flag_errors": flag_errors, "checksum": sums[0]}


def worker(args, level: int, world: int, rank: int, local: int) -> None:
    """One configuration level on this rank (a supervised child, or in-process unsupervised)."""
    from network_distributed_pytorch_amd.utils.supervisor import Heartbeat

    hb = Heartbeat(rank)
    hb.beat("import", 900)
    import torch
    import torch.distributed as dist

    over = fallbacks(world)[level]
    a = argparse.Namespace(**{**vars(args), **over})
    # one process per GPU; NDP_BACKEND=gloo lets several ranks share one GPU (testing only)
    backend = os.environ.get("NDP_BACKEND", "nccl")
    hb.beat("init", 600)
    dev_index = local % max(1, torch.cuda.device_count())
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)
    # NDP_FORCE_COLLECTIVES=1: 1-rank process group whose collectives are still issued (a
    # one-GPU rehearsal of the N > 1 RCCL path, parallel/comm.py Communicator.active)
    if world > 1 or os.environ.get("NDP_FORCE_COLLECTIVES") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    torch.manual_seed(714)
    torch.backends.cudnn.benchmark = True
    if os.environ.get("NDP_BENCH_FAIL") in (f"{level}:{rank}", f"{level}:*"):  # test hook
        raise RuntimeError(f"injected failure, level {level} rank {rank}")

    if args.scaling == "strong":
        assert args.global_batch % world == 0, "global batch must divide by the world size"
        per_gpu = args.global_batch // world   # reference: bsz = int(512 / float(size))
    else:
        per_gpu = args.batch
    hb.beat("build+capture", 300)
    wl = Workload(a, device, world, rank)
    step = wl.make_step(per_gpu)
    for j in range(args.warmup):
        step(j)
        torch.cuda.synchronize()
        hb.beat(f"warmup {j + 1}/{args.warmup}", 120)
    hb.beat("check:warmup", 120)
    health_check(wl, world, "after warm-up")
    hb.beat("timed", 120 + 10 * args.steps)
    elapsed = wl.time(step, args.steps, 0, start=args.warmup)  # warmed up above
    hb.beat("check:timed", 120)
    health = health_check(wl, world, "after the timed steps")
    comm_stats = wl.comm.stats.as_dict()
    final_loss = float(wl.loss_acc.item()) / max(1, args.warmup + args.steps)

    weak = None
    if args.weak_too == "on" and args.scaling == "strong" and not wl.is_bert:
        hb.beat("weak arm", 600 + 30 * args.steps)
        wb = args.global_batch  # per-GPU batch of the N=1 config, fixed as N grows
        wstep = wl.make_step(wb)
        we = wl.time(wstep, args.steps, args.warmup)
        health_check(wl, world, "after the weak-scaling arm")
        weak = {"value": round(wb * world * args.steps / we, 2), "unit": "samples/s",
                "ms_per_step": round(1e3 * we / args.steps, 4), "per_gpu_batch": wb, "global_batch": wb * world}

    if rank == 0:
        line = json.dumps(record(args, a, wl, world, per_gpu, elapsed, comm_stats, final_loss, health, level,
                                 weak))
        hb.result(line)
        if not hb.enabled:
            print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    hb.done()
    hb.beat("teardown", 120)
    wl.comm.close()
    if dist.is_initialized():
        dist.destroy_process_group()


def record(args, a, wl, world, per_gpu, elapsed, comm_stats, final_loss, health, level, weak) -> dict:
    global_batch = per_gpu * world
    sps = global_batch * args.steps / elapsed
    is_bert = wl.is_bert
    native = wl.comm.native
    rec = {
        "metric": metric_name(args),
        "value": round(sps, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "fp32" if args.amp == "none" else "bf16-autocast (fp32 params/grads/reducer)",
        "data": ("synthetic IMDb-shape (512-token ids + masks, 2 labels)" if is_bert else
                 "synthetic CIFAR-10-shape (3x32x32, 10 labels)") + ", random-init weights",
        "bytes_per_step": wl.sync.bytes_per_step,
        "dense_bytes_per_step": 4 * sum(p.numel() for p in wl.model.parameters()),
        "collectives_per_step": wl.sync.collectives_per_step,
        "comm_backend": wl.comm.backend,
        "rccl_nranks": native.nranks if native is not None else None,
        "replicas_equal": health["replicas_equal"],
        "flag_errors": health["flag_errors"],
        "param_checksum": health["checksum"],
        "fallback": ({"level": level, "config": fallbacks(world)[level]} if level else None),
        "config": {
            "model": args.model,
            "num_classes": args.num_classes if args.num_classes is not None else (2 if is_bert else 1000),
            "global_batch": global_batch,
            "per_gpu_batch": per_gpu,
            "seq_len": args.seq_len if is_bert else None,
            "image": None if is_bert else [3, 32, 32],
            "parallelism": f"dp{world}",
            "reducer": args.reducer,
            "powersgd_rank": args.rank if "powersgd" in args.reducer else None,
            "overlap": getattr(getattr(wl.sync, "opt", getattr(wl.sync, "ddp", None)), "overlap", None),
            "link_emulation": args.link,
            "emulate_world": args.emulate_world,
            "channels_last": args.channels_last,
            "stock_model_ops": bool(a.no_fused_bn and a.no_gemm_convs),
            "hip_graph": wl.graph_mode,
            "tuned_gemms": wl.tuned_gemms,
            "fused_attention": (not args.no_fused_attn) if is_bert else None,
        },
        "comm_stats_timed": comm_stats,
        "collective_payloads": wl.sync.collective_payloads() if hasattr(wl.sync, "collective_payloads") else None,
        "link_model_s_per_step": (sum(wl.comm.link.seconds(b, wl.comm.paced_world)
                                      for b in wl.sync.collective_payloads())
                                  if wl.comm.link is not None and hasattr(wl.sync, "collective_payloads")
                                  else None),
        "mean_loss": round(final_loss, 5),
    }
    if weak is not None:
        rec["weak_scaling"] = weak
    return rec


def resolve_world(args) -> int:
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        if args.gpus is not None and int(env) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env} (launcher and flag disagree)")
        return int(env)
    return args.gpus if args.gpus is not None else 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    from network_distributed_pytorch_amd.utils.supervisor import run_supervised, worker_env_info

    role, level, _ = worker_env_info()
    world = resolve_world(args)
    if role == "worker":
        rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
        try:
            worker(args, level, world, rank, local)
        except BaseException as e:  # noqa: BLE001 - report, then fail the attempt
            import traceback

            from network_distributed_pytorch_amd.utils.supervisor import Heartbeat

            tb = traceback.format_exc()
            print(tb, file=sys.stderr, flush=True)
            Heartbeat(rank).error(f"{type(e).__name__}: {str(e)[:1500]}")
            os._exit(1)  # no teardown: a peer may be stuck in a collective with us
        return 0
    if args.no_supervise:  # in-process, one level, no fallback (debugging / profilers)
        if os.environ.get("WORLD_SIZE") is None and world > 1:
            raise SystemExit("--no-supervise with --gpus N > 1 needs a launcher (torchrun)")
        worker(args, args.level, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
        return 0
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + argv
    levels = fallbacks(world)
    start = max(0, min(args.level, len(levels) - 1))
    code = run_supervised(cmd, world, len(levels), describe=lambda i: str(levels[i]),
                          first_level=start)
    return code


if __name__ == "__main__":
    sys.exit(main())
