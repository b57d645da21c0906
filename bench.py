#!/usr/bin/env python3
"""Headline benchmark: Llama-2-7B training throughput (tokens/s) on 1..8 MI355X, weak scaling.

Metric and config come from BASELINE.json ("tokens/sec + DDP/FSDP scaling efficiency, Llama-2-7B at
1/2/4/8 MI355X").  Every rank trains the full Llama-2-7B architecture (random init, synthetic tokens)
with a fixed per-GPU batch on the sharded data-parallel engine (reduce-scatter of bf16 gradient buckets
overlapped with backward, sharded fp32 AdamW state, parameter all-gather overlapped with the next forward) over
RCCL.  N = 1 runs the same engine in a world of one (RCCL process group created; its collectives are no-ops), so
T_1 and T_N come from the same code.
The timed region holds EXACTLY --steps full optimizer steps (forward + backward + gradient collectives +
AdamW + parameter all-gather), bracketed by a barrier and a device synchronize on both sides; the
reported time is the MAX over ranks; rank 0 prints one JSON line.

Before anything is timed, a run with N > 1 (runtime/preflight.py):
  * self-tests every collective the engines use (all-reduce / reduce-scatter / all-gather in fp32 and bf16, a P2P
    ring) with exact known values on the real group -- a mismatch or timeout aborts with exit code 3;
  * sizes the gradient buckets from a ~1-2 s alpha-beta probe of reduce-scatter / all-gather (--bucket-mb
    calibrate, the default); the fit and the chosen size go into the JSON;
  * after the warm-up, checks that the flat parameters of every replica agree bitwise (exit code 4 if not).

Other BASELINE.json configs run under the same contract with --layout (train/bench_layouts.py):
tp (Llama-2 7B TP=N + SP), hybrid (FSDP(N/4) x TP(4)), pp (PP 4 x DDP N/4, 1F1B), resnet-fsdp (ResNet-50 FSDP bf16),
unet-ddp (SimpleUNet DDP on ERA5-shaped 65 x 181 x 360 fields, B = 4 per GPU).  Every line also carries the median
and spread of rank 0's per-step device times ("step_ms", CUDA events between consecutive timed steps).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--layout dp|tp|hybrid|pp|resnet-fsdp|unet-ddp]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Ranks: under a launcher (torchrun, runtime/launch.py, mpiexec, srun) its world size must equal --gpus, or the run
exits 2 before any work.  Without one, --gpus N > 1 starts its own N ranks (runtime/launch.py, one per GPU, before
this process touches a GPU) and exits non-zero if any rank fails or if fewer than N GPUs are visible for RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from distributed_pytorch_hpc_amd.train.bench_layouts import BASELINE_METRIC, BUILDERS, LAYOUTS  # noqa: F401


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layout", choices=LAYOUTS, default="dp",
                    help="dp: headline weak-scaling FSDP; tp / hybrid / pp / resnet-fsdp: BASELINE configs 3 / 4 / 5 / 2")
    ap.add_argument("--model", default=None, help="llama preset (default llama2-7b)")
    ap.add_argument("--arch", default="resnet50", help="resnet-fsdp layout: ResNet depth")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--unet-precision", choices=["bf16", "bf16-autocast", "fp32"], default="bf16",
                    help="unet-ddp layout: bf16 parameters / activations / gradients with fp32 master weights in the "
                         "engine (default: 834 / 927 vs 796 / 799 samples/s for bf16 autocast over fp32 weights in "
                         "alternating runs on one box, profiles/r4/unet/), or the reference's fp32")
    ap.add_argument("--micro-batch", type=int, default=None,
                    help="sequences (images) per GPU / per dp replica per step; default 8 (dp, tp, hybrid), 16 (pp), "
                         "256 (resnet-fsdp).  8 x 4096 tokens: ~249 GB peak on one 288 GB MI355X")
    ap.add_argument("--tp", type=int, default=None, help="tp / hybrid layouts: tensor-parallel degree")
    ap.add_argument("--async-tp", type=int, default=2, help="tp / hybrid: micro-collectives per SP collective")
    ap.add_argument("--pp", type=int, default=None, help="pp layout: pipeline stages (default 4)")
    ap.add_argument("--microbatches", type=int, default=16, help="pp layout: micro-batches per step")
    ap.add_argument("--schedule", choices=["auto", "1f1b", "gpipe", "interleaved"], default="auto",
                    help="pp layout: auto = interleaved 1F1B with --virtual-stages chunks per rank where it applies")
    ap.add_argument("--virtual-stages", type=int, default=2, help="pp layout: model chunks per rank (interleaved)")
    ap.add_argument("--parallel", choices=["auto", "fsdp", "ddp"], default="auto",
                    help="dp layout: auto = the sharded (FSDP / ZeRO-2) engine; ddp = replicated optimizer state")
    ap.add_argument("--bucket-mb", default="calibrate",
                    help="gradient bucket size in MiB; 'calibrate' (in-run alpha-beta probe, default); 'auto' "
                         "(comm/cost_model.py fit from $DPH_COMM_FIT or the nominal prior)")
    ap.add_argument("--grad-dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--kernels", choices=["dph", "aten"], default="dph",
                    help="dph: CDNA4 HIP kernels (default); aten: stock PyTorch-ROCm ops (comparator)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--ac", default="none",
                    help="activation checkpointing: none | auto (fit 288 GB) | N (every N-th block)")
    ap.add_argument("--no-dist", action="store_true",
                    help="N = 1 without a process group (the engine is the same; no RCCL communicator)")
    ap.add_argument("--force-dist", action="store_true", help=argparse.SUPPRESS)   # the default now; kept for scripts
    ap.add_argument("--no-preflight", action="store_true", help="skip the collective self-test and replica check")
    ap.add_argument("--xgmi-probe", type=int, default=1,
                    help="multi-GPU layouts with all-reducing groups (tp, hybrid, unet-ddp): time the direct-peer "
                         "xGMI all-reduce against RCCL and route messages below the crossover to it (0: RCCL only)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None,
                    help="process-group backend (default: nccl = RCCL on GPU); gloo lets several ranks share one GPU "
                         "to rehearse the N > 1 path (tests/test_bench_gpu.py)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--no-telemetry", action="store_true",
                    help="do not sample GPU clock / power / temperature (amdsmi host thread) during the run")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="replay each step as one HIP graph after the warm-up (runtime/graphs.py; one rank only).  "
                         "Default: on for the one-rank unet-ddp layout, whose eager step is launch-bound (243 launches "
                         "in 3.25 ms: graph 1 229 / 1 232 samples/s at stdev 0.02 ms vs eager 1 044 / 1 230 at "
                         "0.13-0.19 ms, profiles/r6/unet_graph/) and the one-rank resnet-fsdp layout (575 launches: "
                         "11 505 / 11 516 vs 11 367 / 11 351 img/s eager, profiles/r6/resnet_graph/), off otherwise")
    ap.add_argument("--fp8", action="store_true",
                    help="opt-in FP8 GEMMs for the projections (ops/fp8.py; e4m3 activations/weights, e5m2 gradients, "
                         "LM head bf16). Reported with dtype 'bf16+fp8-gemm' -- not the bf16 headline number")
    ap.add_argument("--attn-variant", type=int, default=0,
                    help="flash-attention kernels for head dim 128: 0 = 32x32x16 MFMA forms (default), 2 = the "
                         "16x16x32 forms (faster in isolation, not in the power-limited step: profiles/r6/attn16/)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: gloo + eager reference ops (tests of the N > 1 code path with tiny models only)")
    args = ap.parse_args(argv)
    if args.model is None:
        args.model = "llama2-7b"
    if args.micro_batch is None:
        args.micro_batch = {"pp": 16, "resnet-fsdp": 256, "unet-ddp": 4}.get(args.layout, 8)
    return args


def _spread(v):
    """Median and spread of rank 0's per-step times (device events between consecutive steps)."""
    if not v:
        return None
    s = sorted(v)

    def q(f):
        return s[min(len(s) - 1, max(0, round(f * (len(s) - 1))))]

    mean = sum(s) / len(s)
    sd = (sum((x - mean) ** 2 for x in s) / max(len(s) - 1, 1)) ** 0.5
    return {"median": round(q(0.5), 3), "p10": round(q(0.1), 3), "p90": round(q(0.9), 3), "min": round(s[0], 3),
            "max": round(s[-1], 3), "mean": round(mean, 3), "stdev": round(sd, 3), "n": len(s)}


def _fail(code: int, msg: str):
    print(f"[bench] FATAL: {msg}", file=sys.stderr, flush=True)
    sys.stderr.flush()
    os._exit(code)   # a rank that failed a check must not wait in a collective the others never reach


def _self_launch(args, argv) -> int:
    """``--gpus N > 1`` with no launcher around us: start N fresh ranks through the framework's own launcher.

    This process never touches the GPU (``torch.cuda.device_count()`` does not initialise HIP on this image): it checks
    that N ranks can each own a device, spawns N children of this same script with the torchrun environment
    (runtime/launch.py: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT, NUMA binding),
    waits, and returns the gang's exit code -- non-zero as soon as any rank fails (the watchdog tears the others down,
    so no rank is left in a collective).  Rank 0 prints the one JSON line to the shared stdout.
    (Reference: scripts/torchrun_multigpu_pbs.sh:152 wraps every multi-GPU run in an external torchrun.)"""
    import types

    from distributed_pytorch_hpc_amd.runtime import launch

    backend = "gloo" if args.device == "cpu" else (args.backend or "nccl")
    if args.device != "cpu" and backend == "nccl":
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            _fail(2, f"--gpus {args.gpus}: only {visible} GPU(s) visible; RCCL needs one GPU per rank "
                     f"(no N=1 number is reported in place of an N={args.gpus} one)")
    argv = list(sys.argv[1:] if argv is None else argv)
    largs = types.SimpleNamespace(nproc=args.gpus, master_addr="127.0.0.1", master_port=0, backend=None,
                                  log_dir=None, max_restarts=0, timeout=0.0, grace=10.0, omp_threads=0,
                                  cpu_bind="numa" if args.device != "cpu" else "none",
                                  script=os.path.abspath(__file__), script_args=argv)
    if not args.quiet:
        print(f"[bench] launching {args.gpus} ranks (runtime/launch.py, backend {backend})", file=sys.stderr,
              flush=True)
    code = launch.run(largs)
    if code != 0:
        print(f"[bench] FATAL: the {args.gpus}-rank run failed (exit {code})", file=sys.stderr, flush=True)
    return code


def main(argv=None):
    args = parse(argv)
    from distributed_pytorch_hpc_amd.runtime import env as rt
    from distributed_pytorch_hpc_amd.runtime import preflight

    info = rt.get_rank_info()
    if args.gpus < 1:
        _fail(2, f"--gpus {args.gpus}: need at least one rank")
    if info.launcher == "single" and args.gpus > 1:
        sys.exit(_self_launch(args, argv))
    if info.world_size != args.gpus:
        # an N=1 number must never be reported as N=8 (nor the reverse): a launcher / flag mismatch is fatal
        _fail(2, f"--gpus {args.gpus} but the launcher ({info.launcher}) started {info.world_size} rank(s)")
    world_env = info.world_size

    cpu = args.device == "cpu"
    if world_env > 1 or not args.no_dist:
        if world_env == 1 and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(rt.free_port())   # a world of one needs no fixed rendezvous port
        rank, world, local = rt.init_distributed(backend="gloo" if cpu else args.backend, verbose=not args.quiet)
    else:
        rank, world, local = 0, 1, 0
        if not cpu:
            torch.cuda.set_device(0)
    if world != args.gpus:
        _fail(2, f"rank {rank}: --gpus {args.gpus} but the process group has {world} ranks")
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    def log(msg):
        if rank == 0 and not args.quiet:
            print(msg, file=sys.stderr, flush=True)

    from distributed_pytorch_hpc_amd.ops import _lib

    if not cpu:
        _lib.require()
        if args.attn_variant:
            _lib.ops().attn_variant(args.attn_variant)
    if args.kernels == "aten":
        _lib.set_reference_mode(True)

    # ---- pre-flight collective self-test on the real group (outside the timed region) ----
    pre = {"preflight_ok": None}
    if world > 1 and not args.no_preflight:
        try:
            rep = preflight.collective_selftest(None, dev)
            pre = {"preflight_ok": True, "preflight_checked": rep["checked"]}
            log(f"[bench] pre-flight OK on {world} ranks: {', '.join(rep['checked'])}")
        except preflight.PreflightError as e:
            _fail(3, f"rank {rank}: collective self-test failed: {e}")

    wl = BUILDERS[args.layout](args, rank, world, dev, log)
    # ---- direct-peer all-reduce: measured crossover per all-reducing group (small messages, RCCL above) ----
    xgmi = {}
    if world > 1 and not cpu and not args.no_preflight and args.xgmi_probe and wl.ar_groups and \
            dist.get_backend() == "nccl":
        from distributed_pytorch_hpc_amd.comm import custom_allreduce as car_mod

        for name, grp in wl.ar_groups:
            res = car_mod.probe_crossover(grp)
            car_mod.set_policy(grp, res["crossover_bytes"])
            xgmi[name] = {"crossover_bytes": res["crossover_bytes"], "verified": res["verified"],
                          "samples_us": [(b, round(1e6 * tr, 1), None if tx is None else round(1e6 * tx, 1))
                                         for b, tr, tx in res["samples"]]}
            log(f"[bench] xGMI all-reduce vs RCCL on {name}: crossover {res['crossover_bytes']} B")
    graph_info = {}
    if args.graph is None:   # auto: the one-rank SimpleUNet / ResNet steps replay as one graph (fewer launch gaps)
        args.graph = args.layout in ("unet-ddp", "resnet-fsdp") and world == 1 and not cpu and args.warmup >= 2
    if args.graph:
        if world > 1 or cpu:
            _fail(2, "--graph: whole-step graph capture is a one-rank GPU option")
        import types

        from distributed_pytorch_hpc_amd.runtime.graphs import GraphedStep

        eager_step = wl.step
        # the captured step returns a detached loss: an autograd graph kept alive across the capture (the loss of
        # the previous step) makes AccumulateGrad run on the wrong stream
        runner = GraphedStep(lambda: eager_step(0).detach(), optimizer=types.SimpleNamespace(engine=wl.engine),
                             warmup=max(1, args.warmup - 1))
        wl.step = lambda i: runner()
        graph_info = {"graph": "whole step replayed as one HIP graph (captured during the warm-up)"}
        if args.warmup < 2:
            _fail(2, "--graph needs --warmup >= 2 (eager warm-up + capture)")

    def sync_all():
        sync()
        if dist.is_initialized():
            rt.barrier()
        sync()

    # clock / power / temperature of this rank's GPU on a host thread (amdsmi; never touches a stream)
    tel = None
    if not cpu and not args.no_telemetry:
        from distributed_pytorch_hpc_amd.utils.telemetry import GpuTelemetry

        tel = GpuTelemetry(torch.cuda.current_device())
    loss = None
    log(f"[bench] {args.layout}: workload built, {args.warmup} warm-up + {args.steps} timed steps")
    for i in range(args.warmup):
        loss = wl.step(i)
    first_loss = float(loss.detach()) if loss is not None else None
    log(f"[bench] warm-up done (loss {first_loss})")
    wl.engine.synchronize()
    sync_all()
    # ---- replicas must hold bitwise-identical parameters after the warm-up updates ----
    replica = {"param_checksum_ok": None}
    if world > 1 and wl.replica_flat is not None and not args.no_preflight and args.warmup:
        try:
            rep = preflight.replicas_agree(wl.replica_flat, wl.replica_group)
            replica = {"param_checksum_ok": True}
            log(f"[bench] replicas agree after warm-up (checksum {rep['checksum'][0]:.6e})")
        except preflight.PreflightError as e:
            _fail(4, f"rank {rank}: {e}")
        sync_all()

    # per-step device-time marks: events recorded between steps (no host synchronisation inside the timed region)
    marks = [] if cpu else [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    host_marks = []
    if tel is not None:
        tel.mark("timed_start")
    t0 = time.perf_counter()
    for i in range(args.steps):
        if marks:
            marks[i].record()
        else:
            host_marks.append(time.perf_counter())
        loss = wl.step(args.warmup + i)
    if marks:
        marks[-1].record()
    wl.engine.synchronize()
    host_marks.append(time.perf_counter())
    sync_all()
    elapsed = time.perf_counter() - t0
    telem = {}
    if tel is not None:
        tel.mark("timed_end")
        tel.stop()
        flops = (wl.flops_per_item or 0) * wl.items_per_step * args.steps / max(world, 1)
        telem = tel.summary("timed_start", "timed_end", flops=flops or None)
        if dist.is_initialized() and world > 1:
            per_rank = [None] * world
            dist.all_gather_object(per_rank, {k: telem.get(k) for k in ("sclk_mhz", "power_w", "energy_j")})
            telem["per_rank"] = [{"sclk_median": (r.get("sclk_mhz") or {}).get("median"),
                                  "power_median": (r.get("power_w") or {}).get("median"),
                                  "energy_j": r.get("energy_j")} for r in per_rank]
    step_ms = ([marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)] if marks else
               [1000.0 * (host_marks[i + 1] - host_marks[i]) for i in range(args.steps)])
    last_loss = float(loss.detach()) if loss is not None else None
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    items = wl.items_per_step * args.steps
    rate = items / elapsed
    ms = 1000.0 * elapsed / args.steps
    peak_gb = 0.0 if cpu else torch.cuda.max_memory_allocated() / 1e9
    if rank == 0:
        rec = {
            "metric": wl.metric,
            "value": round(rate, 2),
            "unit": wl.unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": wl.scaling,
            "vs_baseline": None,
            "dtype": "fp32" if cpu else ("bf16+fp8-gemm" if args.fp8 else "bf16"),
            "data": "synthetic (random tokens / images, random-init weights)",
            "config": {**wl.config, "layout": args.layout},
            f"{wl.unit.split('/')[0]}_per_sec_per_gpu": round(rate / world, 2),
            "step_ms": _spread(step_ms),
            "peak_hbm_gb": round(peak_gb, 2),
            "loss_first_warmup": round(first_loss, 4) if first_loss is not None else None,
            "loss_last": round(last_loss, 4) if last_loss is not None else None,
            "world": world,
            "process_group": dist.get_backend() if dist.is_initialized() else None,
            "rccl_version": preflight.rccl_version() if not cpu else None,
            **pre, **replica, **wl.extra, **graph_info,
            **({"xgmi_allreduce": xgmi} if xgmi else {}),
            **telem,
        }
        if wl.flops_per_item:
            rec["mfu_vs_2.5PF_bf16_dense"] = round(rate / world * wl.flops_per_item / 2.5e15, 4)
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if dist.is_initialized():
        rt.cleanup_distributed()


if __name__ == "__main__":
    main()
