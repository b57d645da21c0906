"""bench.py contract (one JSON line with the driver's fields) on its N = 1 and N > 1 (sharded engine over gloo)
code paths, with a tiny Llama on CPU -- the same script the round-end driver runs on 1..8 MI355X."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
ARGS = ["--device", "cpu", "--model", "tiny", "--seq-len", "64", "--micro-batch", "2", "--steps", "2",
        "--warmup", "1", "--quiet"]


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_bench_contract(n, tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + ARGS
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", str(n)] + ARGS
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _lines(p.stdout)
    assert len(recs) == 1, p.stdout          # rank 0 only, exactly one line
    r = recs[0]
    assert KEYS <= set(r)
    assert r["n_gpus"] == n and r["steps"] == 2 and r["warmup"] == 1 and r["value"] > 0
    assert r["config"]["parallelism"] == f"fsdp{n}"     # N = 1 runs the same engine in a world of one
    assert r["world"] == n and r["process_group"] == "gloo"
    if n > 1:
        assert r["preflight_ok"] is True and "p2p_ring" in r["preflight_checked"]
        assert r["param_checksum_ok"] is True
        assert r["config"]["bucket_source"] == "in-run alpha-beta probe"
        assert set(r["config"]["comm_fit"]) == {"reduce_scatter", "all_gather"}
        assert r["config"]["comm_fit"]["reduce_scatter"]["alpha_s"] >= 0
    assert r["config"]["global_batch"] == 2 * n and r["config"]["seq_len"] == 64
    assert abs(r["value"] - n * 2 * 64 * 2 / (r["ms_per_step"] * 2 / 1000)) / r["value"] < 1e-3


def test_scaling_sweep_harness(tmp_path):
    """benchmarks/scaling_sweep.py runs bench.py at N = 1 and 2 (gloo, tiny model) and derives E(N) itself."""
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import scaling_sweep

    out = tmp_path / "scaling"
    rows = scaling_sweep.main(["--ns", "1", "2", "--steps", "2", "--warmup", "1", "--out", str(out), "--"] + ARGS[:-5]
                              + ["--quiet"])
    assert [r["n_gpus"] for r in rows] == [1, 2]
    assert rows[0]["scaling_efficiency"] == 1.0
    assert rows[1]["parallelism"] == "fsdp2" and rows[1]["global_batch"] == 4
    assert abs(rows[1]["scaling_efficiency"] - rows[1]["tokens_per_s"] / (2 * rows[0]["tokens_per_s"])) < 1e-3
    assert (out / "scaling.json").exists() and (out / "n2.log").exists()
    assert "| 2 | fsdp2 |" in (out / "scaling.md").read_text()


ARGS8 = ["--device", "cpu", "--model", "tiny8", "--seq-len", "64", "--steps", "2", "--warmup", "1", "--quiet"]


@pytest.mark.parametrize("layout,extra,par,scaling,batch", [
    ("tp", ["--micro-batch", "4"], "tp8", "strong", 4),
    ("hybrid", ["--micro-batch", "4"], "fsdp2xtp4", "weak", 8),
    ("pp", ["--micro-batch", "8", "--microbatches", "4", "--model", "tiny8-deep"], "pp4xddp2", "weak", 16),
])
def test_bench_baseline_layouts_world8(layout, extra, par, scaling, batch, tmp_path):
    """BASELINE configs 3-5 (TP=8, FSDP(2) x TP(4), PP4 x DDP2) under bench.py's JSON contract at world 8 (gloo)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "8",
           "--layout", layout] + ARGS8 + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _lines(p.stdout)
    assert len(recs) == 1, p.stdout
    r = recs[0]
    assert KEYS <= set(r) and r["n_gpus"] == 8 and r["unit"] == "tokens/s"
    assert r["config"]["parallelism"] == par and r["scaling"] == scaling and r["config"]["layout"] == layout
    assert r["config"]["global_batch"] == batch
    assert r["preflight_ok"] is True
    if layout != "tp":   # replicas exist only over a dp dimension
        assert r["param_checksum_ok"] is True
    if layout == "pp":   # default schedule: interleaved 1F1B, 2 chunks per rank
        assert r["config"]["schedule"] == "interleaved" and r["config"]["virtual_stages"] == 2
        assert abs(r["config"]["bubble_fraction"] - round(3 / (2 * 4 + 3), 4)) < 1e-9
    assert abs(r["value"] - batch * 64 * 2 / (r["ms_per_step"] * 2 / 1000)) / r["value"] < 1e-3


def test_bench_resnet_fsdp_layout(tmp_path):
    """BASELINE config 2 (ResNet-50 FSDP bf16) under the contract; a ResNet-18 at 32 px keeps it CPU-sized."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--layout", "resnet-fsdp", "--device", "cpu", "--arch", "resnet18", "--image-size", "32",
           "--micro-batch", "2", "--steps", "2", "--warmup", "1", "--quiet"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    r = _lines(p.stdout)[0]
    assert r["unit"] == "images/s" and r["config"]["parallelism"] == "fsdp2" and r["config"]["global_batch"] == 4
    assert r["preflight_ok"] is True and r["images_per_sec_per_gpu"] > 0


def test_bench_unet_ddp_layout(tmp_path):
    """SimpleUNet DDP under the contract (CPU: a narrow UNet on a 19 x 36 grid); per-step spread reported."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--layout", "unet-ddp", "--device", "cpu", "--steps", "4", "--warmup", "1", "--quiet"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    r = _lines(p.stdout)[0]
    assert r["unit"] == "samples/s" and r["config"]["parallelism"] == "ddp2" and r["config"]["global_batch"] == 8
    assert r["preflight_ok"] is True and r["param_checksum_ok"] is True
    st = r["step_ms"]
    assert st["n"] == 4 and st["min"] <= st["median"] <= st["max"] and st["p10"] <= st["p90"]


# ---- pre-flight failure injection: a corrupted collective / diverged replica must abort, not publish ----
def _selftest_corrupt_worker(rank, world, which):
    import torch.distributed as dist

    from distributed_pytorch_hpc_amd.runtime import preflight

    real = getattr(dist, which)

    def bad(*a, **kw):
        w = real(*a, **kw)
        if w is not None:
            w.wait()
        if rank == 1:
            a[0].add_(1)     # rank 1's result (after the collective completed) is off by one everywhere
        return None

    setattr(dist, which, bad)
    try:
        preflight.collective_selftest(None, None)
    except preflight.PreflightError as e:
        return str(e)
    finally:
        setattr(dist, which, real)
    return "no error"


@pytest.mark.parametrize("which", ["all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor"])
def test_preflight_detects_corrupted_collective(which):
    from dist_utils import run_distributed

    outs = run_distributed(_selftest_corrupt_worker, 2, which)
    # rank 1 names its mismatch; rank 0 either finishes or fails on the next collective its peer never joins
    assert "mismatch on rank 1" in outs[1], outs
    assert outs[0] == "no error" or "mismatch" not in outs[0], outs


def _replica_worker(rank, world, diverge):
    import torch

    from distributed_pytorch_hpc_amd.runtime import preflight

    flat = torch.linspace(-1, 1, 1000)
    if diverge and rank == world - 1:
        flat[[10, 20]] = flat[[20, 10]]    # a swapped pair: same plain sum, different position-weighted sum
    try:
        return preflight.replicas_agree(flat)["ok"]
    except preflight.PreflightError as e:
        return str(e)


def test_replica_checksum_detects_divergence():
    from dist_utils import run_distributed

    assert run_distributed(_replica_worker, 4, False) == [True] * 4
    outs = run_distributed(_replica_worker, 4, True)
    assert all(isinstance(o, str) and "diverged" in o for o in outs), outs


def _probe_worker(rank, world):
    from distributed_pytorch_hpc_amd.runtime import preflight

    fits = preflight.probe_alpha_beta(None, None, sizes_mib=(0.0625, 0.25), budget_s=5.0)
    mib = preflight.calibrated_bucket_mb(fits, 64 * 2 ** 20, True, lo_mib=1.0, hi_mib=64.0)
    return {k: (v.alpha_s, v.beta_bus_Bps) for k, v in fits.items()}, mib


def test_alpha_beta_probe_and_bucket_choice():
    from dist_utils import run_distributed

    outs = run_distributed(_probe_worker, 2)
    fits, mib = outs[0]
    assert set(fits) == {"reduce_scatter", "all_gather"}
    for a, b in fits.values():
        assert a >= 0 and b > 0
    assert 1.0 <= mib <= 64.0


def _probe_skew_worker(rank, world):
    import time

    from distributed_pytorch_hpc_amd.runtime import preflight

    # rank 1 arrives late: a stop rule on each rank's own wall clock would let rank 0 quit the sweep while rank 1
    # enters the next size's collective (deadlock); the rule on the max-reduced measured times is the same everywhere
    if rank == 1:
        time.sleep(1.0)
    fits = preflight.probe_alpha_beta(None, None, sizes_mib=(0.0625, 0.125, 0.25), budget_s=0.5)
    return {k: (v.alpha_s, v.beta_bus_Bps, v.source) for k, v in fits.items()}


def test_alpha_beta_probe_stop_rule_is_rank_consistent():
    from dist_utils import run_distributed

    outs = run_distributed(_probe_skew_worker, 2)
    assert outs[0] == outs[1], outs


def _selftest_worker(rank, world):
    from distributed_pytorch_hpc_amd.runtime import preflight

    return preflight.collective_selftest(None, None, numel=1 << 12)["checked"]


def test_preflight_selftest_exact_at_world_16():
    """The bf16 self-test values stay exact past 8 ranks (two-node jobs): every partial sum has <= 8 significant
    bits whatever the reduction order (3 * (1 + ... + 13) = 273 needs 9)."""
    from dist_utils import run_distributed

    outs = run_distributed(_selftest_worker, 16, timeout=400)
    assert all("all_reduce[bfloat16]" in o and "reduce_scatter[bfloat16]" in o for o in outs), outs


def test_bench_self_launches_its_ranks(tmp_path):
    """`python bench.py --gpus 2` with no launcher starts its own 2 ranks (runtime/launch.py) and reports world 2 --
    never an N = 1 number labelled N = 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _lines(p.stdout)
    assert len(recs) == 1, p.stdout
    r = recs[0]
    assert r["n_gpus"] == 2 and r["world"] == 2 and r["config"]["parallelism"] == "fsdp2"
    assert r["preflight_ok"] is True and r["param_checksum_ok"] is True


def test_bench_rank_count_mismatch_is_fatal(tmp_path):
    """An external launcher whose world size disagrees with --gpus: exit 2 on every rank, no JSON line."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "4"] + ARGS
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert p.returncode != 0 and not _lines(p.stdout)
    assert "--gpus 4 but the launcher" in p.stderr


def test_bench_too_few_gpus_is_fatal(tmp_path):
    """--gpus N over RCCL with fewer than N visible GPUs (none here; one on the 1-GPU test box): exit 2 before any
    rank starts."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this machine has enough GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny", "--quiet"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert p.returncode == 2 and not _lines(p.stdout), p.stderr[-2000:]
    assert "RCCL needs one GPU per rank" in p.stderr
