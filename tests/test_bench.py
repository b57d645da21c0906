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


@pytest.mark.parametrize("n", [1, 2, 4])
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
    assert r["config"]["parallelism"] == ("ddp1" if n == 1 else f"fsdp{n}")
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
