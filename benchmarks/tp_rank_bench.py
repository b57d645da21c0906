#!/usr/bin/env python3
"""One tensor-parallel rank's compute of the Llama-2-7B TP=8 (or FSDP x TP) step on ONE GPU, collectives stubbed.

The BASELINE configs 3-4 (TP = 8 over xGMI, FSDP(2) x TP(4)) need an 8-GPU node; what a single rank computes does
not: this runs the real ``parallelize_llama`` plan (sequence parallel, loss parallel, the fused SwiGLU / QKV paths
on the local shards) inside a ``fake`` process group of world size tp -- every all-gather / reduce-scatter /
all-reduce returns at once without touching data -- so the timed step is exactly one rank's kernels at the shard
shapes (w13 2752 x 4096, w2 4096 x 1376, the 4000-row vocab shard, 4 local heads ...).  Run it under rocprofv3 to
see which kernels a TP rank spends its time in (reference: fsdp_tp/tensor_parallel_example.py,
fsdp_tp/fsdp_tp_example.py:146-177).

    python benchmarks/tp_rank_bench.py [--tp 8] [--batch 8] [--seq 4096] [--steps 5] [--gemm-nt all]

The data is garbage-in (stubbed collectives leave their outputs uninitialised), so the loss is meaningless; the
kernel sequence and shapes are the real ones.  tokens/s is the TP group's rate if communication were free.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Done:
    def wait(self, *a, **kw):
        return True

    def is_completed(self):
        return True


def _null_collectives():
    def null(*args, async_op=False, **kw):
        return _Done() if async_op else None

    for name in ("all_gather_into_tensor", "reduce_scatter_tensor", "all_reduce", "all_to_all_single",
                 "broadcast", "all_gather"):
        setattr(dist, name, null)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8, help="sequences per TP group")
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gemm-nt", default=None, choices=["fused", "all", "0"])
    ap.add_argument("--fused-qkv", type=int, default=None)
    ap.add_argument("--torch-profile", action="store_true",
                    help="after the timed steps, profile one step with torch.profiler and print where device memcpys "
                         "and copy kernels come from (Python call sites)")
    ap.add_argument("--fake-pg-copies", action="store_true",
                    help="keep the fake process group's own all-gather (a device memcpy per rank slot) instead of the "
                         "null collectives that return without touching data")
    ap.add_argument("--stack-dump", type=int, default=0, metavar="S",
                    help="diagnostics: dump every thread's Python stack each S seconds and mark each phase")
    a = ap.parse_args(argv)

    from torch.testing._internal.distributed.fake_pg import FakeStore

    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.ops import _lib
    from distributed_pytorch_hpc_amd.parallel import fused_layers
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, MixedPrecision, OptimConfig
    from distributed_pytorch_hpc_amd.parallel.tensor_parallel import parallelize_llama

    _lib.require()
    if a.stack_dump:   # diagnostics: the Python stack of every thread every S seconds
        import faulthandler

        faulthandler.dump_traceback_later(a.stack_dump, repeat=True, file=sys.stderr)
    if a.gemm_nt is not None or a.fused_qkv is not None:
        fused_layers.set_enabled(gemm_nt=a.gemm_nt, qkv=None if a.fused_qkv is None else bool(a.fused_qkv))
    dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=a.tp)
    if not a.fake_pg_copies:
        # torch's fake backend implements all_gather_into_tensor as one device memcpy per rank slot
        # (benchmarks/probes/fake_pg_copies.py): 1 413 copy launches / 13.9 ms per TP = 8 step that a real rank runs
        # as RCCL kernels instead.  Null collectives keep the timed step to the rank's own compute.
        _null_collectives()
    tp_group = dist.new_group(list(range(a.tp)))
    dp_group = dist.new_group([0])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    margs = get_preset(a.model)
    model = build_llama(margs, device=dev, dtype=torch.bfloat16, seed=0)
    parallelize_llama(model, tp_group, sequence_parallel=True, loss_parallel=True)
    engine = DataParallelEngine(model, dp_group, shard=False,
                                mixed_precision=MixedPrecision(param_dtype=torch.bfloat16, reduce_dtype=torch.bfloat16))
    engine.configure_optimizer(OptimConfig(name="adamw", lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1))
    ff = model.layers[0].feed_forward
    x_probe = torch.zeros(a.batch, a.seq // a.tp, margs.dim, device=dev, dtype=torch.bfloat16)
    info = {"tp": a.tp, "w13_local": list(ff.w13.weight.shape), "w2_local": list(ff.w2.weight.shape),
            "fused_mlp": fused_layers.swiglu_mlp_ok(x_probe, ff.w13, ff.w2),
            "fused_qkv": fused_layers.qkv_rope_attention_ok(x_probe, model.layers[0].attention.wqkv,
                                                             margs.head_dim),
            "gemm_nt_all": fused_layers.nt_enabled()}
    g = torch.Generator(device=dev).manual_seed(0)
    t = torch.randint(0, margs.vocab_size, (a.batch, a.seq + 1), device=dev, generator=g)

    debug = bool(a.stack_dump)

    def mark(what):
        if debug:
            torch.cuda.synchronize()
            print(f"[tp_rank] {what} done", flush=True)

    def step():
        loss = model(t[:, :-1], t[:, 1:])
        mark("forward")
        loss.backward()
        mark("backward")
        engine.step()
        mark("optimizer step")
        engine.zero_grad()

    print(f"[tp_rank] model built and sharded (tp {a.tp}): {info}", flush=True)
    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()
        print(f"[tp_rank] warm-up step {i} done", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / a.steps
    info.update(ms_per_step=round(ms, 2), tokens_per_s_tp_group_no_comm=round(a.batch * a.seq / (ms / 1000), 1),
                peak_gb=round(torch.cuda.max_memory_allocated() / 1e9, 1))
    if a.torch_profile:
        _copy_sites(step)
    print(json.dumps(info), flush=True)
    dist.destroy_process_group()
    return info


def _copy_sites(step):
    """Which Python call sites issue copy kernels / device memcpys in one step (TorchDispatchMode: every copy-like
    ATen op with its innermost framework frame, counted with its bytes)."""
    import collections
    import traceback

    from torch.utils._python_dispatch import TorchDispatchMode

    cnt, nbytes = collections.Counter(), collections.Counter()
    names = ("copy_", "clone", "contiguous", "_to_copy", "cat.", "index_copy", "fill_", "zero_", "empty_like")

    class _M(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            n = str(func)
            if any(x in n for x in names):
                st = [f for f in traceback.extract_stack() if "distributed_pytorch_hpc_amd" in f.filename
                      or "benchmarks" in f.filename]
                where = f"{st[-1].filename.rsplit('/', 2)[-2]}/{st[-1].filename.rsplit('/', 1)[-1]}:{st[-1].lineno}" \
                    if st else "?"
                cnt[(n, where)] += 1
                o = out if isinstance(out, torch.Tensor) else (args[0] if args and isinstance(args[0], torch.Tensor)
                                                               else None)
                if o is not None:
                    nbytes[(n, where)] += o.numel() * o.element_size()
            return out

    with _M():
        step()
    torch.cuda.synchronize()
    print("[tp_rank] copy-like ops in one step (calls, MB, op, call site):", flush=True)
    for key in sorted(cnt, key=lambda k: -nbytes[k])[:30]:
        print(f"  {cnt[key]:6d} {nbytes[key] / 1e6:10.1f}  {key[0]}  {key[1]}", flush=True)


if __name__ == "__main__":
    main()
