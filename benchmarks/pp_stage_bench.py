#!/usr/bin/env python3
"""Per-stage cost of a Llama pipeline split, measured on ONE GPU: each stage (or interleaved chunk) of the
``bench.py --layout pp`` split runs forward + backward of one micro-batch at the real stage shapes, so the balance of
the split (parallel/pipeline.py partition_by_cost: embedding on the first stage, norm + LM head + cross-entropy on the
last) is checked without an 8-GPU node.  Reference: scripts/04_pipeline_parallel_pp/03_pipeline_training.py:180-201
(which splits 2 layers per stage with no cost model).

    python benchmarks/pp_stage_bench.py [--model llama2-7b] [--pp 4] [--virtual-stages 1] [--mb 1] [--seq 4096]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--pp", type=int, default=4)
    ap.add_argument("--virtual-stages", type=int, default=1)
    ap.add_argument("--mb", type=int, default=1, help="sequences per micro-batch")
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--split", choices=["cost", "layers"], default="cost")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)

    from distributed_pytorch_hpc_amd.models.llama2 import build_llama, get_preset
    from distributed_pytorch_hpc_amd.parallel.pipeline import (LlamaStage, _split_bounds, llama_costs, lm_loss)

    dev = torch.device("cuda")
    margs = get_preset(a.model)
    model = build_llama(margs, device=dev, dtype=torch.bfloat16, seed=0)
    n_parts = a.pp * a.virtual_stages
    bounds = _split_bounds(model, n_parts, a.seq if a.split == "cost" else None, None)
    blocks, emb, head = llama_costs(margs, a.seq)
    parts = [LlamaStage(model, lo, hi, i == 0, i == n_parts - 1) for i, (lo, hi) in enumerate(bounds)]
    g = torch.Generator(device=dev).manual_seed(1)
    tokens = torch.randint(0, margs.vocab_size, (a.mb, a.seq + 1), device=dev, generator=g)
    hidden = torch.randn(a.mb, a.seq, margs.dim, device=dev, dtype=torch.bfloat16, generator=g)

    def run(i):
        st = parts[i]
        x = tokens[:, :-1] if st.first else hidden.detach().requires_grad_()
        y = st(x)
        if st.last:
            lm_loss(y, tokens[:, 1:]).backward()
        else:
            y.backward(torch.ones_like(y))
        for p in st.parameters():
            p.grad = None

    times = {i: [] for i in range(n_parts)}
    for i in range(n_parts):
        run(i)   # warm-up
    torch.cuda.synchronize()
    for _ in range(a.rounds):            # interleaved rounds (rule 24): every part in every round
        for i in range(n_parts):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run(i)
            e.record()
            e.synchronize()
            times[i].append(s.elapsed_time(e) / a.iters)
    ms = [min(times[i]) for i in range(n_parts)]
    # rank r runs parts r, r + pp, ...: its per-micro-batch work is their sum
    rank_ms = [sum(ms[c * a.pp + r] for c in range(a.virtual_stages)) for r in range(a.pp)]
    model_cost = [sum(blocks[lo:hi]) + (emb if i == 0 else 0) + (head if i == n_parts - 1 else 0)
                  for i, (lo, hi) in enumerate(bounds)]
    res = {"model": a.model, "pp": a.pp, "virtual_stages": a.virtual_stages, "split": a.split,
           "bounds": bounds, "part_ms": [round(t, 3) for t in ms], "rank_ms": [round(t, 3) for t in rank_ms],
           "rank_max_over_min": round(max(rank_ms) / min(rank_ms), 4),
           "rank_max_over_mean": round(max(rank_ms) / (sum(rank_ms) / len(rank_ms)), 4),
           "modelled_part_cost_rel": [round(c / model_cost[0], 4) for c in model_cost],
           "measured_part_ms_rel": [round(t / ms[0], 4) for t in ms]}
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return res


if __name__ == "__main__":
    main()
