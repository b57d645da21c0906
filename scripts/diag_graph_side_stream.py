#!/usr/bin/env python3
"""Root-cause harness for the whole-step HIP-graph divergence seen with side-stream warm-up (runtime/graphs.py).

Runs ResNet (FSDP units, bf16, channels-last) with MIOpen's deterministic algorithms so two eager runs agree
bitwise, then replays a captured step under combinations of:

  * warm-up stream: current (default) / side (GraphedStep(warmup_side_stream=True), the configuration that diverged);
  * interference between replays: none / "alloc" (fresh allocations of assorted sizes + GPU writes into them, the
    caching allocator may hand out any block it considers free) / "noalloc" (the same writes into ONE buffer
    allocated before the run -- no allocator traffic) / "sync" (alloc, but the host synchronises first);

and reports the first step whose loss departs bitwise from the eager run.  "alloc" diverging while "noalloc" holds
means the graph touches memory the allocator regards as free (a lifetime bug); both diverging means ordering.

    python scripts/diag_graph_side_stream.py [--arch resnet50] [--steps 8] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


CIFAR_STEM = True


def make(arch, dev):
    from distributed_pytorch_hpc_amd.models import resnet

    torch.manual_seed(0)
    return resnet(arch, num_classes=10, cifar_stem=CIFAR_STEM).to(dev).to(memory_format=torch.channels_last)


def run(arch, batches, graphed, interference, side, extra_env=None):
    from distributed_pytorch_hpc_amd.parallel.data_parallel import MixedPrecision
    from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP
    from distributed_pytorch_hpc_amd.runtime import graphs

    for k, v in (extra_env or {}).items():
        os.environ[k] = v
    dev = torch.device("cuda")
    model = make(arch, dev)
    f = FSDP(model, mixed_precision=MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16))
    opt = f.make_optimizer("sgd", lr=0.002, momentum=0.9, weight_decay=1e-4)

    def step_fn(x, y):
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(f(x).float(), y)
        loss.backward()
        opt.step()
        return loss.detach()

    runner = graphs.GraphedStep(step_fn, optimizer=opt, warmup=2, warmup_side_stream=side) if graphed else None
    scratch = torch.empty(64 << 20, dtype=torch.uint8, device=dev)   # "noalloc" interference target
    g = torch.Generator(device=dev).manual_seed(77)
    losses = []
    keep = []
    for i, (x, y) in enumerate(batches):
        out = runner(x, y) if runner is not None else step_fn(x, y)
        losses.append(out.clone())
        if interference == "sync":
            torch.cuda.synchronize()
        if interference in ("alloc", "sync"):
            keep.clear()
            for n in (1 << 20, 3 << 19, 7 << 18, 1 << 22, 5 << 20):   # assorted sizes, fresh blocks
                t = torch.empty(n, dtype=torch.float32, device=dev)
                t.uniform_(-1e4, 1e4, generator=g)
                keep.append(t)
            keep = keep[-2:]
        elif interference == "noalloc":
            scratch.random_(0, 255, generator=g)
    torch.cuda.synchronize()
    for k in (extra_env or {}):
        os.environ.pop(k, None)
    return [float(v) for v in losses], torch.stack(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--image-size", type=int, default=32)
    ap.add_argument("--imagenet-stem", action="store_true", help="7x7/2 stem + 3x3/2 max pool (224 px -> 56/28/14/7)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    global CIFAR_STEM
    CIFAR_STEM = not a.imagenet_stem
    from distributed_pytorch_hpc_amd.ops import _lib

    _lib.require()
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dev = torch.device("cuda")
    torch.manual_seed(3)
    batches = [(torch.randn(a.batch, 3, a.image_size, a.image_size, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last), torch.randint(0, 10, (a.batch,), device=dev)) for _ in range(a.steps)]
    ref, ref_t = run(a.arch, batches, False, "none", False)
    ref2, ref2_t = run(a.arch, batches, False, "alloc", False)
    res = {"eager": ref, "eager_reproducible": bool(torch.equal(ref_t, ref2_t)), "cases": {}}
    print(f"eager losses {ref}; second eager run bitwise equal: {res['eager_reproducible']}", flush=True)
    cases = [("current", "none", {}), ("current", "alloc", {}), ("side", "none", {}), ("side", "alloc", {}),
             ("side", "noalloc", {}), ("side", "sync", {}), ("side", "alloc", {"DPH_CONV": "miopen"})]
    refs = {}
    for side, inter, env in cases:
        name = f"warmup={side} interference={inter}" + (f" {env}" if env else "")
        key = tuple(sorted(env.items()))
        if key not in refs:   # another kernel set changes the eager numbers: its own eager reference
            refs[key] = run(a.arch, batches, False, "none", False, env) if env else (ref, ref_t)
        cref, cref_t = refs[key]
        try:
            got, got_t = run(a.arch, batches, True, inter, side == "side", env)
            first = next((i for i in range(len(got)) if got[i] != cref[i]), None)
            res["cases"][name] = {"losses": got, "first_divergent_step": first,
                                  "max_abs_loss_diff": float((got_t - cref_t).abs().max())}
            print(f"{name:60s} first divergent step: {first}  max |dloss| {res['cases'][name]['max_abs_loss_diff']:.3e}",
                  flush=True)
        except Exception as e:  # keep going: a failing case is a result too
            res["cases"][name] = {"error": repr(e)}
            print(f"{name}: ERROR {e!r}", flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
