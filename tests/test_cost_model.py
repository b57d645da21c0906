"""alpha-beta collective cost model (comm/cost_model.py) and the bucket sizes it drives."""
import json

import torch

from dist_utils import run_distributed


def test_fit_recovers_alpha_beta():
    from distributed_pytorch_hpc_amd.comm.cost_model import AlphaBeta, fit_alpha_beta

    true = AlphaBeta("all_reduce", 8, 25e-6, 250e9)
    samples = [(b, true.time(b)) for b in (1 << 16, 1 << 20, 1 << 24, 1 << 28)]
    fit = fit_alpha_beta("all_reduce", 8, samples)
    assert abs(fit.alpha_s - 25e-6) < 1e-9 and abs(fit.beta_bus_Bps / 250e9 - 1) < 1e-6


def test_fit_clamps_nonphysical():
    from distributed_pytorch_hpc_amd.comm.cost_model import fit_alpha_beta

    fit = fit_alpha_beta("all_gather", 4, [(1e3, 5e-3), (1e6, 1e-3)])   # noisy: time falls with size
    assert fit.alpha_s >= 0 and fit.beta_bus_Bps > 0


def test_bucket_choice_latency_and_overlap_bounds():
    from distributed_pytorch_hpc_amd.comm.cost_model import AlphaBeta, choose_bucket_bytes

    m = AlphaBeta("reduce_scatter", 8, 30e-6, 300e9)
    b = choose_bucket_bytes(m, total_bytes=13.5e9)
    # alpha is at most 10 % of t(B) ...
    assert m.alpha_s <= 0.1 * m.time(b) + 1e-12
    # ... and the smallest such bucket (one granule less violates it)
    assert m.alpha_s > 0.1 * m.time(b - (1 << 20))
    # a small model keeps >= 4 buckets in flight
    small = choose_bucket_bytes(m, total_bytes=40e6)
    assert small <= 40e6 / 4 + (1 << 20)
    # higher latency -> larger buckets
    assert choose_bucket_bytes(AlphaBeta("reduce_scatter", 8, 300e-6, 300e9), 13.5e9) > b


def _measure_and_fit(rank, world, path):
    from distributed_pytorch_hpc_amd.comm.cost_model import fit_alpha_beta, load_fits, measure, save_fits

    fits = {}
    for op in ("all_reduce", "all_gather", "reduce_scatter"):
        s = measure(op, [1 << 12, 1 << 16, 1 << 20], dtype=torch.float32, iters=3, warmup=1)
        assert len(s) == 3 and all(t > 0 for _, t in s)
        fits[op] = fit_alpha_beta(op, world, s)
    if rank == 0:
        save_fits(fits, path)
    torch.distributed.barrier()
    back = load_fits(path)
    return {k: [v.alpha_s, v.beta_bus_Bps] for k, v in back.items()}


def test_measure_fit_roundtrip_gloo(tmp_path):
    path = str(tmp_path / "fit.json")
    res = run_distributed(_measure_and_fit, 2, path)
    assert set(res[0]) == {"all_reduce", "all_gather", "reduce_scatter"}
    raw = json.load(open(path))
    assert all(v["beta_bus_Bps"] > 0 and v["alpha_s"] >= 0 for v in raw.values())


def _engine_auto(rank, world, path):
    import os

    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine

    os.environ["DPH_COMM_FIT"] = path
    torch.manual_seed(0)
    m = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(8)])
    eng = DataParallelEngine(m, shard=True, bucket_cap_mb="auto")
    return {"mb": eng.bucket_cap_mb, "n": len(eng.buckets)}


def test_engine_auto_buckets(tmp_path):
    from distributed_pytorch_hpc_amd.comm.cost_model import AlphaBeta, save_fits

    path = str(tmp_path / "fit.json")
    save_fits({"reduce_scatter": AlphaBeta("reduce_scatter", 2, 1e-3, 1e9),
               "all_reduce": AlphaBeta("all_reduce", 2, 1e-3, 1e9)}, path)
    res = run_distributed(_engine_auto, 2, path)[0]
    # 8 x (256*256 + 256) fp32 params = 2.1 MB: the overlap bound (>= 4 buckets) wins -> 1 MiB granule buckets
    assert res["mb"] == 1.0 and res["n"] >= 2


def test_sharded_step_prediction_weak_scaling():
    """predict_sharded_step: N=1 is the 1-GPU step; the optimizer sweep shrinks 1/N; with collectives that fit under
    the compute windows only the first / last bucket is exposed; starving the bus makes communication exposed."""
    from distributed_pytorch_hpc_amd.comm.cost_model import AlphaBeta, predict_sharded_step

    fits = {op: AlphaBeta(op, 8, 30e-6, 300e9) for op in ("reduce_scatter", "all_gather")}
    g = p = 13.5e9
    one = predict_sharded_step(1110.0, 35.0, g, p, 1, 256 * 2 ** 20, fits)
    assert one.ms_per_step == 1145.0 and one.efficiency == 1.0
    eight = predict_sharded_step(1110.0, 35.0, g, p, 8, 256 * 2 ** 20, fits)
    assert eight.optimizer_ms == 35.0 / 8
    assert 0.0 < eight.exposed_comm_ms < 5.0                   # one 256 MiB bucket each way
    assert eight.efficiency > 1.0                              # sharded optimizer: N > 1 can beat N = 1 per GPU
    slow = {op: AlphaBeta(op, 8, 30e-6, 10e9) for op in ("reduce_scatter", "all_gather")}
    starved = predict_sharded_step(1110.0, 35.0, g, p, 8, 256 * 2 ** 20, slow)
    assert starved.exposed_comm_ms > 500.0 and starved.efficiency < 0.7
