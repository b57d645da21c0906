"""Workloads of ``bench.py``: one builder per BASELINE.json config, all measured under the same contract (W untimed
warm-up steps, EXACTLY K timed full optimizer steps bracketed by barrier + device synchronize, MAX over ranks, one
JSON line from rank 0).

| layout        | BASELINE.json config                                                  | reference path                       |
|---------------|-----------------------------------------------------------------------|--------------------------------------|
| ``dp``        | headline: tokens/s + DDP/FSDP scaling, Llama-2-7B at 1/2/4/8 MI355X   | fsdp_tp/fsdp_tp_example.py (dp part) |
| ``tp``        | Llama-2 7B TP=8 over xGMI                                             | fsdp_tp/tensor_parallel_example.py   |
| ``hybrid``    | Llama-2 7B hybrid FSDP(2) x TP(4) via DeviceMesh                      | fsdp_tp/fsdp_tp_example.py:103-187   |
| ``pp``        | Llama-2 7B PP 4 stages x DDP 2 (send/recv micro-batch pipeline)       | scripts/04_pipeline_parallel_pp/03   |
| ``resnet-fsdp`` | ResNet-50 FSDP bf16 on 8 x MI355X                                   | scripts/main.py + resnet_fsdp_training.py |
| ``unet-ddp``  | SimpleUNet DDP, ERA5 65 x 181 x 360, B = 4 per GPU (samples/s)        | scripts/01_data_parallel_ddp/multinode_ddp_unet.py |

Each builder returns a ``Workload``: the step function, the engine to synchronise, the group whose ranks hold
replicas of the same flat parameters (checked bitwise after warm-up), the work per step and the JSON ``config``.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch
import torch.distributed as dist

BASELINE_METRIC = "tokens/sec + DDP/FSDP scaling efficiency, Llama-2-7B at 1/2/4/8 MI355X"
LAYOUTS = ("dp", "tp", "hybrid", "pp", "resnet-fsdp", "unet-ddp")


@dataclass
class Workload:
    step: Callable[[int], Optional[torch.Tensor]]
    engine: object
    metric: str
    unit: str
    items_per_step: int                  # tokens (or images) processed per step by the whole job
    scaling: str                         # "weak" | "strong"
    config: dict
    replica_group: object = None         # ranks holding identical flat parameters (None: every rank / n.a.)
    replica_flat: Optional[torch.Tensor] = None
    flops_per_item: float = 0.0
    extra: dict = field(default_factory=dict)
    # (name, group) pairs whose all-reduces may take the direct-peer xGMI path below a measured crossover
    # (bench.py probes each before timing; comm/custom_allreduce.py)
    ar_groups: list = field(default_factory=list)


def _bucket(args, world_dp: int, grad_bytes: float, sharded: bool, group, dev, log) -> tuple[float, dict]:
    """Bucket size for the data-parallel engine: a number (MiB), 'auto' ($DPH_COMM_FIT / nominal prior) or
    'calibrate' (in-run alpha-beta probe of reduce-scatter / all-gather on ``group``; default for dp > 1)."""
    from ..comm import cost_model
    from ..runtime import preflight

    spec = str(args.bucket_mb)
    if spec == "calibrate" and world_dp <= 1:
        return 256.0, {"bucket_source": "default (no data-parallel collectives at dp = 1)"}
    if spec == "calibrate":
        sizes = (4, 16, 64, 256) if dev.type == "cuda" else (0.0625, 0.25, 1.0)
        fits = preflight.probe_alpha_beta(group, dev, sizes_mib=sizes,
                                          dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
        mib = preflight.calibrated_bucket_mb(fits, grad_bytes, sharded,
                                             lo_mib=32.0 if dev.type == "cuda" else 0.01)
        log(f"[bench] alpha-beta probe: " + ", ".join(
            f"{k} alpha {1e6 * v.alpha_s:.1f} us, busbw {v.beta_bus_Bps / 1e9:.1f} GB/s" for k, v in fits.items())
            + f" -> bucket {mib:.1f} MiB")
        return mib, {"bucket_source": "in-run alpha-beta probe", "comm_fit": preflight.fits_json(fits)}
    if spec == "auto":
        mib = cost_model.auto_bucket_mb(grad_bytes, world_dp, sharded)
        return mib, {"bucket_source": "cost model ($DPH_COMM_FIT or nominal prior)"}
    return float(spec), {"bucket_source": "fixed"}


def _llama(args, dev, dtype, n_layers=None):
    from ..models.llama2 import build_llama, get_preset

    over = {"max_seq_len": max(args.seq_len, 4096 if dev.type == "cuda" else args.seq_len)}
    if n_layers:
        over["n_layers"] = n_layers
    margs = get_preset(args.model, **over)
    return margs, build_llama(margs, device=dev, dtype=dtype, seed=1234)


def _tokens(margs, B, S, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return [torch.randint(0, margs.vocab_size, (B, S + 1), device=dev, generator=g) for _ in range(4)]


def _model_name(args):
    return {"llama2-7b": "Llama-2-7B", "llama2-13b": "Llama-2-13B", "llama2-1b": "Llama-2-1B"}.get(args.model,
                                                                                                 args.model)


def build_dp(args, rank, world, dev, log) -> Workload:
    """Headline: every rank trains the full model on its own batch; N > 1 = sharded engine (reduce-scatter of bf16
    gradient buckets overlapped with backward, 1/N fp32 AdamW, parameter all-gather overlapped with the next
    forward).  N = 1 takes the same engine class (its collectives are no-ops in a world of one)."""
    from ..parallel.data_parallel import DataParallelEngine, MixedPrecision, OptimConfig

    cpu = dev.type == "cpu"
    dtype = torch.float32 if cpu else torch.bfloat16
    margs, model = _llama(args, dev, dtype)
    ac_every = 0
    if args.ac != "none":
        from ..parallel.activation_checkpoint import apply_llama_checkpointing, plan_llama_checkpointing

        static_gb = margs.num_params() * (4 + (12 / world if world > 1 else 12)) / 1e9
        ac_every = (plan_llama_checkpointing(margs, args.micro_batch, args.seq_len, static_gb=static_gb)
                    if args.ac == "auto" else int(args.ac))
        apply_llama_checkpointing(model, ac_every)
    mode = args.parallel
    if mode == "auto":
        mode = "fsdp" if dist.is_initialized() else "ddp"
    if args.fp8 and not cpu:
        from ..ops import fp8 as fp8_mod

        fp8_mod.enable_for_llama(model)
    reduce_dtype = torch.bfloat16 if args.grad_dtype == "bf16" and not cpu else torch.float32
    grad_bytes = sum(p.numel() for p in model.parameters()) * torch.empty((), dtype=reduce_dtype).element_size()
    bucket_mb, binfo = _bucket(args, world, grad_bytes, mode == "fsdp", None, dev, log)
    engine = DataParallelEngine(model, shard=(mode == "fsdp"),
                                mixed_precision=MixedPrecision(param_dtype=dtype, reduce_dtype=reduce_dtype),
                                bucket_cap_mb=bucket_mb)
    engine.configure_optimizer(OptimConfig(name="adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    B, S = args.micro_batch, args.seq_len
    batches = _tokens(margs, B, S, dev, 1000 + rank)

    def step(i):
        t = batches[i % len(batches)]
        loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        engine.step()
        engine.zero_grad()
        return loss

    cfg = {"model": _model_name(args), "global_batch": world * B, "seq_len": S, "parallelism": f"{mode}{world}",
           "micro_batch_per_gpu": B, "tokens_per_step": world * B * S, "kernels": args.kernels,
           "bucket_mb": round(engine.bucket_cap_mb, 1), "activation_checkpoint_every": ac_every, **binfo}
    return Workload(step, engine, BASELINE_METRIC, "tokens/s", world * B * S, "weak", cfg,
                    replica_group=None, replica_flat=engine.flat_param,
                    flops_per_item=margs.flops_per_token(S))


def _tp_hybrid(args, rank, world, dev, log, tp: int, layout: str) -> Workload:
    from ..comm.mesh import DeviceMesh2D
    from ..parallel.data_parallel import DataParallelEngine, MixedPrecision, OptimConfig
    from ..parallel.tensor_parallel import parallelize_llama

    assert world % tp == 0, f"world {world} is not divisible by tp {tp}"
    dp = world // tp
    cpu = dev.type == "cpu"
    dtype = torch.float32 if cpu else torch.bfloat16
    mesh = DeviceMesh2D(dp, tp) if world > 1 else None
    margs, model = _llama(args, dev, dtype)
    if tp > 1:
        parallelize_llama(model, mesh.tp_group, sequence_parallel=True, loss_parallel=True, async_tp=args.async_tp)
    dp_group = mesh.dp_group if mesh is not None else None
    reduce_dtype = torch.bfloat16 if not cpu else torch.float32
    grad_bytes = sum(p.numel() for p in model.parameters()) * torch.empty((), dtype=reduce_dtype).element_size()
    bucket_mb, binfo = _bucket(args, dp, grad_bytes, dp > 1, dp_group, dev, log)
    engine = DataParallelEngine(model, dp_group, shard=dp > 1,
                                mixed_precision=MixedPrecision(param_dtype=dtype, reduce_dtype=reduce_dtype),
                                bucket_cap_mb=bucket_mb)
    engine.configure_optimizer(OptimConfig(name="adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
    B, S = args.micro_batch, args.seq_len
    dp_rank = mesh.dp_rank if mesh is not None else 0
    batches = _tokens(margs, B, S, dev, 1000 + dp_rank)   # TP peers see the same batch

    def step(i):
        t = batches[i % len(batches)]
        loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        engine.step()
        engine.zero_grad()
        return loss

    par = f"tp{tp}" if dp == 1 else f"fsdp{dp}xtp{tp}"
    cfg = {"model": _model_name(args), "global_batch": dp * B, "seq_len": S, "parallelism": par, "tp": tp, "dp": dp,
           "sequence_parallel": tp > 1, "loss_parallel": tp > 1, "async_tp": args.async_tp if tp > 1 else 0,
           "micro_batch_per_dp_replica": B, "tokens_per_step": dp * B * S, "bucket_mb": round(engine.bucket_cap_mb, 1),
           **binfo}
    metric = ("tokens/sec, Llama-2 7B TP=8 over xGMI" if layout == "tp"
              else "tokens/sec, Llama-2 7B hybrid FSDP(2) x TP(4) via DeviceMesh")
    # strong scaling for pure TP (the batch is fixed as N grows), weak over the dp dimension for the hybrid
    return Workload(step, engine, metric, "tokens/s", dp * B * S, "strong" if layout == "tp" else "weak", cfg,
                    replica_group=dp_group, replica_flat=engine.flat_param if dp > 1 else None,
                    flops_per_item=margs.flops_per_token(S),
                    ar_groups=[("tp", mesh.tp_group)] if tp > 1 else [])


def build_tp(args, rank, world, dev, log) -> Workload:
    return _tp_hybrid(args, rank, world, dev, log, args.tp or world, "tp")


def build_hybrid(args, rank, world, dev, log) -> Workload:
    return _tp_hybrid(args, rank, world, dev, log, args.tp or (4 if world % 4 == 0 else world), "hybrid")


class _EngineSet:
    """The per-chunk data-parallel engines of an interleaved pipeline rank, driven as one."""

    def __init__(self, engines):
        self.engines = list(engines)

    def synchronize(self):
        for e in self.engines:
            e.synchronize()

    def step(self):
        for e in self.engines:
            e.step()

    def zero_grad(self):
        for e in self.engines:
            e.zero_grad()

    @property
    def bucket_cap_mb(self):
        return self.engines[0].bucket_cap_mb

    @property
    def flat_param(self):
        return torch.cat([e.flat_param.reshape(-1) for e in self.engines])


def build_pp(args, rank, world, dev, log) -> Workload:
    from ..comm.mesh import Mesh
    from ..parallel.data_parallel import DataParallelEngine, MixedPrecision, OptimConfig
    from ..parallel.pipeline import PipelineSchedule, make_lm_loss, split_llama, split_llama_virtual

    pp = args.pp or (4 if world % 4 == 0 else world)
    assert world % pp == 0, f"world {world} is not divisible by pp {pp}"
    dp = world // pp
    cpu = dev.type == "cpu"
    dtype = torch.float32 if cpu else torch.bfloat16
    if world > 1:
        mesh = Mesh((pp, dp), ("pp", "dp"))
        stage, dp_rank = mesh.local_rank("pp"), mesh.local_rank("dp")
        pp_group, dp_group = mesh.group("pp"), mesh.group("dp")
    else:
        stage = dp_rank = 0
        pp_group = dp_group = None
    margs, model = _llama(args, dev, dtype)
    M = args.microbatches
    B, S = args.micro_batch, args.seq_len
    assert B % M == 0, f"--micro-batch {B} (sequences per dp replica) must be divisible by --microbatches {M}"
    # interleaved 1F1B (v model chunks per rank) where it applies: >= 3 stages, M % pp == 0, a layer per chunk
    schedule, v = args.schedule, max(1, args.virtual_stages)
    if schedule == "auto":
        ok = pp >= 3 and M % pp == 0 and margs.n_layers >= pp * v and v > 1
        schedule, v = ("interleaved", v) if ok else ("1f1b", 1)
    if schedule != "interleaved":
        v = 1
    assert margs.n_layers >= pp * v
    # stages split by modelled cost (embedding on the first, norm + LM head + loss on the last)
    if schedule == "interleaved":
        chunks = split_llama_virtual(model, pp, v, stage, seq_len=S)
    else:
        chunks = [split_llama(model, pp, stage, seq_len=S)]
    del model
    reduce_dtype = torch.bfloat16 if not cpu else torch.float32
    grad_bytes = sum(p.numel() for c in chunks for p in c.parameters()) * \
        torch.empty((), dtype=reduce_dtype).element_size()
    bucket_mb, binfo = _bucket(args, dp, grad_bytes, dp > 1, dp_group, dev, log)
    engines = []
    for c in chunks:
        e = DataParallelEngine(c, dp_group, shard=dp > 1,
                               mixed_precision=MixedPrecision(param_dtype=dtype, reduce_dtype=reduce_dtype),
                               bucket_cap_mb=bucket_mb)
        e.configure_optimizer(OptimConfig(name="adamw", lr=args.lr, betas=(0.9, 0.95), weight_decay=0.1))
        engines.append(e)
    engine = engines[0] if len(engines) == 1 else _EngineSet(engines)
    sched = PipelineSchedule(chunks[0] if v == 1 else chunks, stage, pp, M, loss_fn=make_lm_loss(None),
                             group=pp_group, schedule=schedule, device=dev,
                             dp_engine=engines[0] if v == 1 else engines)
    batches = _tokens(margs, B, S, dev, 1000 + dp_rank)
    first, last = stage == 0, stage == pp - 1

    def step(i):
        t = batches[i % len(batches)]
        losses = sched.step(inputs=t[:, :-1] if first else None, target=t[:, 1:] if last else None)
        engine.step()
        engine.zero_grad()
        return torch.stack(losses).mean() if losses else None

    layers = [sum(len(c.layers) for c in chunks)]
    cfg = {"model": _model_name(args), "global_batch": dp * B, "seq_len": S, "parallelism": f"pp{pp}xddp{dp}",
           "pp": pp, "dp": dp, "microbatches": M, "schedule": schedule, "virtual_stages": v,
           "layers_on_rank0": layers[0], "bubble_fraction": round(sched.bubble, 4), "tokens_per_step": dp * B * S,
           "bucket_mb": round(engine.bucket_cap_mb, 1), **binfo}
    return Workload(step, engine, "tokens/sec, Llama-2 7B PP 4 stages x DDP 2 (1F1B send/recv pipeline)",
                    "tokens/s", dp * B * S, "weak", cfg, replica_group=dp_group,
                    replica_flat=engine.flat_param if dp > 1 else None, flops_per_item=margs.flops_per_token(S),
                    extra={"loss_on_rank0": last})


def build_resnet_fsdp(args, rank, world, dev, log) -> Workload:
    import torch.nn.functional as F

    from ..models import resnet
    from ..models.resnet import BasicBlock, Bottleneck
    from ..parallel.data_parallel import MixedPrecision
    from ..parallel.fsdp import FSDP, ModuleWrapPolicy

    cpu = dev.type == "cpu"
    arch = args.arch
    torch.backends.cudnn.benchmark = not cpu   # MIOpen find mode: solvers timed once per shape during warm-up
    torch.manual_seed(1234)
    model = resnet(arch, num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if not cpu else None
    model32 = copy.deepcopy(model) if not cpu else None   # the witness's fp32 reference (freed after it)
    wrapped = FSDP(model, mixed_precision=mp, auto_wrap_policy=ModuleWrapPolicy({BasicBlock, Bottleneck}))
    opt = wrapped.make_optimizer("sgd", lr=0.1, momentum=0.9, weight_decay=1e-5)
    B, R = args.micro_batch, args.image_size
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = torch.rand(B, 3, R, R, device=dev, generator=g, dtype=torch.float32 if cpu else torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev, generator=g)
    witness = _first_step_witness(wrapped, model32, x, y) if not cpu else "n/a (CPU)"
    del model32

    def step(i):
        out = wrapped(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    cfg = {"model": {"resnet50": "ResNet-50"}.get(arch, arch), "global_batch": world * B, "image_size": R,
           "parallelism": f"fsdp{world}", "micro_batch_per_gpu": B, "sharding": "FULL_SHARD per bottleneck",
           "mixed_precision": "bf16 params / reduce / buffers" if not cpu else "fp32", "channels_last": True,
           "optimizer": "SGD m=0.9 wd=1e-5 (scripts/main.py)"}
    return Workload(step, wrapped.engine, "images/sec, ResNet-50 FSDP bf16 on 8 x MI355X", "images/s", world * B,
                    "weak", cfg, replica_group=None, replica_flat=None,
                    extra={"replica_check": "n/a (FULL_SHARD: no replicated parameters)",
                           "first_step_witness": witness})


def _first_step_witness(wrapped, model32, x, y) -> dict:
    """The untrained model's first forward on the benchmark batch three ways, same weights: the framework's bf16
    kernels, stock ATen / MIOpen in bf16 (reference mode) and stock ATen in fp32.  The loss after many lr-0.1 steps
    on one batch is chaotic (it moves by whole units between equivalent runs); this is not.  A random-init
    ResNet-50 in training-mode BatchNorm amplifies rounding (the two bf16 paths each land ~0.1 rel L2 from fp32 in
    the logits), so the witness is differential: a broken bf16 conv / BN kernel shows up as ``dph_vs_fp32`` well
    above ``aten_bf16_vs_fp32``.  BatchNorm running statistics take three extra updates (never read in training
    mode)."""
    import torch.nn.functional as F

    from ..ops import _lib

    def rel(a, b):
        return round(((a - b).norm() / b.norm().clamp_min(1e-20)).item(), 5)

    with torch.no_grad():
        out_dph = wrapped(x).float()
        _lib.set_reference_mode(True)
        try:
            out_bf = wrapped(x).float()
            out_32 = model32(x.float()).float()
        finally:
            _lib.set_reference_mode(False)
        return {"loss_dph": round(F.cross_entropy(out_dph, y).item(), 5),
                "loss_aten_bf16": round(F.cross_entropy(out_bf, y).item(), 5),
                "loss_aten_fp32": round(F.cross_entropy(out_32, y).item(), 5),
                "logits_dph_vs_fp32": rel(out_dph, out_32), "logits_aten_bf16_vs_fp32": rel(out_bf, out_32),
                "logits_dph_vs_aten_bf16": rel(out_dph, out_bf)}


def build_unet_ddp(args, rank, world, dev, log) -> Workload:
    """SimpleUNet data-parallel training on ERA5-shaped fields (scripts/01_data_parallel_ddp/multinode_ddp_unet.py:
    B = 4 per GPU, AdamW lr 1e-4 wd 1e-5, latitude-weighted MSE, 65 channels on the 181 x 360 grid).  MI355X path:
    channels-last activations and the engine's mixed precision -- bf16 parameters / activations / gradient
    buckets with the fp32 master weights and AdamW state in the fused optimizer (as the ResNet FSDP path), so no
    per-step cast or layout-flip kernels run (``--unet-precision bf16-autocast`` = bf16 autocast over fp32 weights,
    ``fp32`` = the reference's precision); DDP engine with one gradient bucket all-reduced during backward."""
    from ..models.unet import SimpleUNet, to_channels_last
    from ..ops.loss import latitude_weighted_mse
    from ..parallel.data_parallel import DDP, MixedPrecision

    cpu = dev.type == "cpu"
    C = 65 if not cpu else 5
    lat, lon = (181, 360) if not cpu else (19, 36)
    base = 64 if not cpu else 8
    torch.backends.cudnn.benchmark = not cpu
    torch.manual_seed(1234)
    model = to_channels_last(SimpleUNet(C, C, base).to(dev))
    n_params = sum(p.numel() for p in model.parameters())
    prec = args.unet_precision if not cpu else "fp32"
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if prec == "bf16" else None
    grad_bytes = n_params * (2 if mp is not None else 4)
    bucket_mb, binfo = _bucket(args, world, grad_bytes, False, None, dev, log)
    ddp = DDP(model, bucket_cap_mb=bucket_mb, mixed_precision=mp)
    opt = ddp.make_optimizer("adamw", lr=1e-4, weight_decay=1e-5)
    B = args.micro_batch
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = torch.randn(B, C, lat, lon, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    y = (x + 0.1 * torch.randn(B, C, lat, lon, device=dev, generator=g)).contiguous(memory_format=torch.channels_last)
    if mp is not None:   # the data loader hands bf16 fields over (one cast per batch, outside the step)
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = y.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    amp = prec == "bf16-autocast"

    def step(i):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = ddp(x)
        loss = latitude_weighted_mse(out, y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    cfg = {"model": "SimpleUNet (7,742,849 params)" if not cpu else f"SimpleUNet-mini ({n_params} params)",
           "global_batch": world * B, "grid": f"{C} x {lat} x {lon}", "parallelism": f"ddp{world}",
           "micro_batch_per_gpu": B,
           "precision": {"bf16": "bf16 params / activations / grads, fp32 master weights + AdamW",
                         "bf16-autocast": "bf16 autocast over fp32 weights", "fp32": "fp32"}[prec],
           "channels_last": True, "optimizer": "AdamW lr 1e-4 wd 1e-5 (multinode_ddp_unet.py:316)",
           "loss": "latitude-weighted MSE", "bucket_mb": round(bucket_mb, 1)}
    return Workload(step, ddp.engine, "samples/sec, SimpleUNet DDP ERA5 65x181x360", "samples/s", world * B,
                    "weak", cfg, replica_group=None, replica_flat=ddp.engine.flat_param, extra=binfo,
                    ar_groups=[("world", None)] if world > 1 else [])


BUILDERS = {"dp": build_dp, "tp": build_tp, "hybrid": build_hybrid, "pp": build_pp, "resnet-fsdp": build_resnet_fsdp,
            "unet-ddp": build_unet_ddp}
