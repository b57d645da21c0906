"""Auxiliary utilities of SURVEY.md §2.1 / §2.7 / §2.8 that the other tests do not reach: the environment checker
(T-env / T-env1: world-1 and world-2 gloo all-reduce smoke), per-rank stdio redirection (A7), the GPU-count guard
(R9) and the shell launch scripts (L-PBS / L-TR, syntax only: no scheduler here)."""
import glob
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _report(stdout: str) -> dict:
    start = stdout.index("{")
    depth = 0
    for i, ch in enumerate(stdout[start:], start):
        depth += ch == "{"
        depth -= ch == "}"
        if depth == 0:
            return json.loads(stdout[start:i + 1])
    raise AssertionError("no JSON report")


def test_check_env_world1_cpu():
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "check_env.py")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rep = _report(p.stdout)
    assert rep["gloo"] is True and "native_extension" in rep and rep["gpus"] == []
    assert "✓ world-1 all_reduce" in p.stdout


def test_check_env_world2_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="1")   # no GPU here: default_backend() is gloo
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "benchmarks", "check_env.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rep = _report(p.stdout)
    assert [r["rank"] for r in rep["ranks"]] == [0, 1]
    assert "✓ all_reduce over 2 ranks" in p.stdout


def test_redirect_writes_per_rank_files(tmp_path):
    code = ("import os, sys; sys.path.insert(0, %r)\n"
            "from distributed_pytorch_hpc_amd.utils.redirect import redirect\n"
            "redirect(%r, 'worker', rank=3)\n"
            "print('to stdout'); print('to stderr', file=sys.stderr)\n"
            "os.write(1, b'native fd1\\n')\n") % (ROOT, str(tmp_path))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout == "" and p.stderr == ""
    out = (tmp_path / "worker.3.out").read_text()
    assert "to stdout" in out and "native fd1" in out
    assert "to stderr" in (tmp_path / "worker.3.err").read_text()


def test_verify_min_gpu_count_without_gpus():
    import torch

    from distributed_pytorch_hpc_amd.utils import verify_min_gpu_count

    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    assert verify_min_gpu_count(1) is False and verify_min_gpu_count(2) is False


@pytest.mark.parametrize("script", sorted(glob.glob(os.path.join(ROOT, "scripts", "*.sh"))
                                      + glob.glob(os.path.join(ROOT, "scripts", "*.sbatch"))),
                         ids=os.path.basename)
def test_shell_scripts_parse(script):
    p = subprocess.run(["bash", "-n", script], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr


def test_gpu_telemetry_summary_without_device(monkeypatch):
    """bench.py's clock / power sampler: spreads over the samples inside the timed marks, energy from the accumulator
    delta, throttle residency as a fraction of the SMU accumulation counter.  Fed synthetic readings (no GPU here)."""
    from distributed_pytorch_hpc_amd.utils import telemetry as tm

    t = tm.GpuTelemetry.__new__(tm.GpuTelemetry)
    t.samples, t.marks, t.error, t._smi = [], {}, None, object()
    t.marks["a"] = {"t": 0.0, "energy_j": 100.0, "accumulation_counter": 1000, "ppt_residency_acc": 500}
    t.marks["b"] = {"t": 2.0, "energy_j": 2900.0, "accumulation_counter": 3000, "ppt_residency_acc": 2300}
    for i, (clk, pw) in enumerate([(1700, 1390), (1750, 1395), (1800, 1380), (2400, 200)]):
        t.samples.append({"t": 0.5 * i if i < 3 else 5.0, "sclk": clk, "sclk_min_xcd": clk - 50, "power": pw,
                          "temp_hot": 60, "temp_mem": 50})
    out = t.summary("a", "b", flops=2.8e15)
    assert out["sclk_mhz"]["median"] == 1750 and out["sclk_mhz"]["n"] == 3   # the idle sample after "b" is excluded
    assert out["power_w"]["max"] == 1395
    assert out["energy_j"] == 2800.0 and out["avg_power_w"] == 1400.0
    assert abs(out["tflop_per_joule"] - 1.0) < 1e-9
    assert out["ppt_limited_frac"] == 0.9
    # no amdsmi / no GPU: the bench line says so instead of failing
    u = tm.GpuTelemetry.__new__(tm.GpuTelemetry)
    u._smi, u.error = None, "ImportError: x"
    assert "unavailable" in u.summary("a", "b")["telemetry"]
