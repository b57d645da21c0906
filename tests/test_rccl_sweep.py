"""benchmarks/rccl_sweep.py: summary logic on synthetic comm_bench rows, and the driver end to end on gloo (the RCCL
knobs are inert there; this checks the per-variant jobs, the JSON merge and the recommended-env file)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

import rccl_sweep  # noqa: E402


def _run(name, bw):
    rows = [{"op": op, "bytes": nb, "busbw_GBps": bw(op, nb)}
            for op in ("reduce_scatter", "all_gather", "all_reduce") for nb in (1 << 10, 64 << 20, 256 << 20)]
    return {"name": name, "env": rccl_sweep.VARIANTS[name], "ok": True, "results": rows}


def test_summary_picks_bucket_winner_and_noise_floor():
    runs = [_run("base", lambda op, nb: 100.0),
            _run("ch32", lambda op, nb: 150.0 if nb > 1 << 20 else 90.0),   # wins the bucket sizes only
            _run("ll128", lambda op, nb: 300.0 if nb == 1 << 10 else 80.0),  # wins small messages only
            {"name": "tree", "env": {}, "ok": False, "rc": 1}]
    s = rccl_sweep.summarise(runs)
    assert s["recommended"] == "ch32"
    best = {(r["op"], r["bytes"]): r for r in s["best_per_size"]}
    assert best[("all_gather", 1 << 10)]["best"] == "ll128"
    assert best[("reduce_scatter", 256 << 20)]["speedup_vs_base"] == 1.5
    assert s["failed"] == [{"name": "tree", "rc": 1}]
    # a 1 % "win" is noise: the defaults stay
    s = rccl_sweep.summarise([_run("base", lambda op, nb: 100.0), _run("ch32", lambda op, nb: 101.0)])
    assert s["recommended"] == "base"


def test_sweep_driver_gloo(tmp_path):
    out = str(tmp_path / "sweep")
    s = rccl_sweep.main(["--nproc", "2", "--backend", "gloo", "--variants", "base,ch16", "--ops",
                         "reduce_scatter,all_gather", "--sizes", "1e3,1e4", "--iters", "2", "--warmup", "1",
                         "--out", out, "--timeout", "240"])
    assert not s["failed"]
    assert {r["op"] for r in s["best_per_size"]} == {"reduce_scatter", "all_gather"}
    with open(os.path.join(out, "summary.json")) as fh:
        assert json.load(fh)["nproc"] == 2
    assert os.path.exists(os.path.join(out, "base.json")) and os.path.exists(os.path.join(out, "ch16.json"))


def test_env_file_only_for_real_winners(tmp_path):
    import subprocess

    out = str(tmp_path)
    p = rccl_sweep.write_env_file(out, "ch32", 8, {"ch32": 1.2})
    text = open(p).read()
    assert "DPH_RCCL_SWEEP_NPROC=8" in text
    k, v = next(iter(rccl_sweep.VARIANTS["ch32"].items()))
    assert f": ${{{k}:={v}}}; export {k}" in text
    # a user's explicit value survives sourcing; an unset knob takes the sweep's value
    r = subprocess.run(["bash", "-c", f"export {k}=user; . {p}; echo ${k}"], capture_output=True, text=True)
    assert r.stdout.strip() == "user"
    r = subprocess.run(["bash", "-c", f"unset {k}; . {p}; echo ${k}"], capture_output=True, text=True)
    assert r.stdout.strip() == str(v)
    # gloo rehearsals and no-winner sweeps remove a stale file
    assert rccl_sweep.write_env_file(out, "ch32", 8, {"ch32": 1.2}, backend="gloo") is None
    assert not os.path.exists(p)
    rccl_sweep.write_env_file(out, "ch32", 8, {"ch32": 1.2})
    assert rccl_sweep.write_env_file(out, "base", 8, {}) is None and not os.path.exists(p)


def test_env_script_checks_rank_count(tmp_path):
    import subprocess

    p = rccl_sweep.write_env_file(str(tmp_path), "ch32", 2, {"ch32": 1.2})
    k, v = next(iter(rccl_sweep.VARIANTS["ch32"].items()))
    script = os.path.join(ROOT, "scripts", "env_mi355x.sh")
    r = subprocess.run(["bash", "-c", f"unset {k}; DPH_RCCL_ENV={p} DPH_NPROC=8 . {script}; echo ${k}"],
                       capture_output=True, text=True)
    assert r.stdout.strip() == "" and "ignoring" in r.stderr
    r = subprocess.run(["bash", "-c", f"unset {k}; DPH_RCCL_ENV={p} DPH_NPROC=2 . {script}; echo ${k}"],
                       capture_output=True, text=True)
    assert r.stdout.strip() == str(v)
