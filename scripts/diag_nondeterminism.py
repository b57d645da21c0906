#!/usr/bin/env python3
"""Where does run-to-run nondeterminism of a training step come from?  (GPU diagnostic.)

Runs the same few SGD steps of a bf16 channels-last ResNet (FSDP world 1, as tests/test_graphs.py) twice per
configuration and prints, per configuration, the global and the worst per-parameter relative difference of the fp32
master-weight UPDATES between the two runs, with the offending parameter names.  Configurations toggle one
ingredient at a time: MIOpen determinism, the framework kernels (reference mode = stock PyTorch ops), the direct
gradient-bucket writes, fp32 parameters and the engine (FSDP vs DDP).

    python scripts/diag_nondeterminism.py [--arch resnet18] [--steps 6]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_hpc_amd.models import resnet  # noqa: E402
from distributed_pytorch_hpc_amd.ops import _lib, batchnorm, conv  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import (DataParallelEngine, MixedPrecision,  # noqa: E402
                                                                OptimConfig)
from distributed_pytorch_hpc_amd.parallel.fsdp import FSDP  # noqa: E402
from distributed_pytorch_hpc_amd.utils.flat import align_up  # noqa: E402


def masters(eng):
    out = []
    for g in eng.groups:
        v = eng.master[eng.opt_slice(g)]
        o = 0
        for p in g.params:
            out.append(v[o:o + p.numel()].detach().clone())
            o += align_up(p.numel())
    return out


def run(arch, steps, batches, engine="fsdp", bf16=True):
    torch.manual_seed(0)
    model = resnet(arch, num_classes=10, cifar_stem=True).cuda().to(memory_format=torch.channels_last)
    names = {id(p): n for n, p in model.named_parameters()}
    mp = MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16) if bf16 else None
    if engine == "fsdp":
        f = FSDP(model, mixed_precision=mp)
        eng = f.engine
    else:
        f = model
        eng = DataParallelEngine(model, mixed_precision=mp)
    eng.configure_optimizer(OptimConfig("sgd", lr=0.002, momentum=0.9, weight_decay=1e-4))
    order = [names[id(p)] for g in eng.groups for p in g.params]
    m0 = masters(eng)
    losses = []
    for i in range(steps):
        x, y = batches[i]
        if not bf16:
            x = x.float()
        eng.zero_grad()
        out = f(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        eng.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return [a - b for a, b in zip(masters(eng), m0)], order, losses


def compare(tag, arch, steps, batches, **kw):
    d1, order, l1 = run(arch, steps, batches, **kw)
    d2, _, l2 = run(arch, steps, batches, **kw)
    num = sum(((a - b).double().norm() ** 2).item() for a, b in zip(d1, d2)) ** 0.5
    den = sum((b.double().norm() ** 2).item() for b in d2) ** 0.5
    per = sorted(((((a - b).norm() / (b.norm() + 1e-30)).item(), n, b.norm().item(), b.numel())
                  for a, b, n in zip(d1, d2, order)), reverse=True)
    print(f"== {tag}: global update rel diff {num / den:.3e}; losses {l1[-1]:.6f} vs {l2[-1]:.6f}; "
          f"loss diff per step {[round(a - b, 6) for a, b in zip(l1, l2)]}", flush=True)
    for r, n, nb, k in per[:6]:
        print(f"     {r:.3e}  {n}  (|update| {nb:.3e}, {k} elems)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    _lib.require()
    torch.manual_seed(3)
    batches = [(torch.randn(16, 3, 32, 32, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last), torch.randint(0, 10, (16,), device="cuda")) for _ in range(a.steps)]
    cfgs = {
        "default": lambda: compare("default (as tests/test_graphs.py)", a.arch, a.steps, batches),
        "miopen_det": lambda: compare("MIOpen deterministic", a.arch, a.steps, batches),
        "reference": lambda: compare("stock PyTorch ops (reference mode)", a.arch, a.steps, batches),
        "no_direct": lambda: compare("no direct bucket writes", a.arch, a.steps, batches),
        "ddp": lambda: compare("DDP engine", a.arch, a.steps, batches, engine="ddp"),
        "fp32": lambda: compare("fp32 parameters", a.arch, a.steps, batches, bf16=False),
    }
    for k, fn in cfgs.items():
        if a.only and k not in a.only.split(","):
            continue
        torch.backends.cudnn.deterministic = k == "miopen_det"
        torch.backends.cudnn.benchmark = False
        _lib.set_reference_mode(k == "reference")
        conv._DIRECT = batchnorm._DIRECT = k != "no_direct"
        try:
            fn()
        finally:
            _lib.set_reference_mode(False)
            conv._DIRECT = batchnorm._DIRECT = True


if __name__ == "__main__":
    main()
