"""Communication microbenchmarks run end-to-end on gloo (the reference runs its tests/*.py by hand under PBS:
SURVEY.md T-bench / T-ar / T-sr / T-p2p).  Tiny sizes; checks the JSON/log outputs they produce."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(script, nproc, args, cwd):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, script)] + args
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=cwd)
    assert p.returncode == 0, f"{script} failed:\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p.stdout


def test_all_reduce_test_gloo(tmp_path):
    log = tmp_path / "bench.log"
    out = _torchrun("benchmarks/all_reduce_test.py", 2, ["--backend", "gloo", "--tensor-sizes", "1000,20000",
                                                         "--iters", "3", "--log-file", str(log),
                                                         "--json", str(tmp_path / "ar.json")], str(tmp_path))
    lines = log.read_text().splitlines()
    assert len(lines) == 4 and all("GB/s" in ln for ln in lines)          # 2 ops x 2 sizes (sizes honoured)
    rows = json.loads((tmp_path / "ar.json").read_text())["rows"]
    assert {r["numel"] for r in rows} == {1000, 20000}
    assert all(r["busbw_GBps"] > 0 for r in rows)
    assert '"benchmark": "all_reduce_test"' in out


def test_comm_bench_gloo(tmp_path):
    _torchrun("benchmarks/comm_bench.py", 2, ["--backend", "gloo", "--sizes", "1e3,1e4", "--iters", "2",
                                              "--warmup", "1", "--json", str(tmp_path / "c.json"),
                                              "--csv", str(tmp_path / "c.csv")], str(tmp_path))
    res = json.loads((tmp_path / "c.json").read_text())["results"]
    ops = {r["op"] for r in res}
    assert {"broadcast", "all_reduce", "all_gather", "reduce_scatter", "all_to_all", "send_recv"} <= ops
    assert (tmp_path / "c.csv").read_text().startswith("#")


def test_send_recv_smoke_gloo(tmp_path):
    _torchrun("benchmarks/send_recv_test.py", 3, ["--backend", "gloo", "--smoke", "--numel", "1000", "--iters", "2",
                                                  "--json", str(tmp_path / "s.json")], str(tmp_path))
    res = json.loads((tmp_path / "s.json").read_text())
    assert res["smoke"] == "ok" and res["world"] == 3 and res["fanout_s"] > 0


def test_torch_baseline_comparator_gloo(tmp_path):
    """The stock-PyTorch comparator (torch DDP over gloo, ATen ops, torch AdamW) on a tiny Llama."""
    out = _torchrun("benchmarks/torch_baseline.py", 2, ["--device", "cpu", "--model", "tiny", "--seq-len", "32",
                                                        "--micro-batch", "2", "--steps", "2", "--warmup", "1",
                                                        "--gpus", "2", "--json-out", str(tmp_path / "t.json")],
                    str(tmp_path))
    rec = json.loads((tmp_path / "t.json").read_text())
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "torch-ddp2" and rec["value"] > 0
    assert sum(ln.startswith("{") for ln in out.splitlines()) == 1   # rank 0 only


def test_prof_summary_idle_launches_categories():
    """benchmarks/prof_summary.py: per-category time, launches per step and idle share of the span."""
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import prof_summary

    ms = 1_000_000
    ev = [("void dph::conv3_k<64, 3, 2, false>(...)", 0, 2 * ms),          # 2 ms
          ("igemm_wrw_gtcx35_nhwc_bf16", 3 * ms, 4 * ms),                  # 1 ms after 1 ms idle
          ("dph::bn_apply_k<...>", 4 * ms, 5 * ms)]
    out = prof_summary.summarise(ev, steps=1)
    assert out["launches_per_step"] == 3
    assert abs(out["idle_pct"] - 20.0) < 1e-6
    cats = out["categories_ms_per_step"]
    assert cats["conv3x3(dph)"] == 2.0 and cats["conv(miopen/ck)"] == 1.0 and cats["batchnorm(dph)"] == 1.0


def test_prof_summary_step_marker_window():
    """Steps counted by a per-step marker kernel, not a time window: a traced run of 6 steps whose last steps are
    slower than the un-traced step still yields exactly the last 2 steps' kernels, and idle vs the un-traced step."""
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import prof_summary

    ms = 1_000_000
    ev, t = [], 0
    for step in range(6):
        for name in ("dph::conv3_k<64>", "dph::c3w_k<128>", "dph::adamw_k<bf16>", "dph::adamw_k<bf16>"):
            ev.append((name, t, t + ms))
            t += 2 * ms   # 1 ms busy + 1 ms gap per kernel
    out = prof_summary.summarise(list(ev), last_ms=3.0, steps=2, marker="adamw_k", run_steps=6, step_ms=6.0)
    assert out["window"] == "marker"
    assert out["launches_per_step"] == 4 and out["kernel_busy_ms_per_step"] == 4.0
    assert abs(out["idle_vs_step_pct"] - 100 * 2 / 6) < 0.01
    # without the marker the 3 ms window holds only part of a step
    assert prof_summary.summarise(list(ev), last_ms=3.0, steps=2)["launches_per_step"] < 4
