"""Multi-GPU tier (SURVEY.md §7.5 tests/multigpu): one rank per DISTINCT MI355X over RCCL / xGMI.

Skipped unless at least 2 GPUs are visible, so it runs on an 8-GPU node and is skipped on the 1-GPU test box.  Every
case launches its ranks through the framework's own launcher (runtime/launch.py; the watchdog tears the gang down on
the first failure) and runs tests/scripts/multigpu_worker.py:

* RCCL collectives (all-reduce sum/max, all-gather, reduce-scatter, all-to-all, broadcast, send/recv, P2P ring) on
  exact integer data, fp32 / bf16 / int64, at world 2 and at every visible GPU (up to 8);
* the direct-peer xGMI all-reduce across distinct devices: bitwise equal to RCCL on integer-valued data and to the
  fp32 rank-order sum on random data; the crossover probe; the stream-ordered step guard;
* Llama TP = 2 (+SP, loss parallel, async TP) and PP = 2 (1F1B) against one rank;
* ``bench.py --gpus 2`` self-launching its ranks, with the replica checksum.
Reference counterparts: tests/torch_comm_bench.py:40-89, tests/pbs_run_tests.sh:128-158,
scripts/torchrun_multigpu_pbs.sh:152.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count()

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(NGPU < 2, reason=f"needs >= 2 GPUs ({NGPU} visible)")]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    return env


def _launch(case: str, world: int, timeout: float = 240.0):
    cmd = [sys.executable, "-m", "distributed_pytorch_hpc_amd.runtime.launch", "--nproc", str(world),
           "--cpu-bind", "none", "--timeout", str(timeout - 20), os.path.join(ROOT, "tests", "scripts",
                                                                          "multigpu_worker.py"), case]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert f"MGPU_RESULT case={case} world={world} failures=0" in out, out[-4000:]
    return out


@pytest.mark.parametrize("world", sorted({2, min(NGPU, 8)}))
def test_rccl_collectives_exact(world):
    _launch("collectives", world)


@pytest.mark.parametrize("world", sorted({2, min(NGPU, 8)}))
def test_xgmi_allreduce_matches_rccl_on_distinct_devices(world):
    _launch("xgmi", world)


def test_tp2_matches_one_rank():
    _launch("tp", 2)


def test_pp2_matches_one_rank():
    _launch("pp", 2)


def test_bench_two_gpus_self_launched(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny", "--seq-len", "128",
           "--micro-batch", "2", "--steps", "2", "--warmup", "1", "--quiet"]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1, p.stdout
    r = recs[0]
    assert r["n_gpus"] == 2 and r["world"] == 2 and r["process_group"] == "nccl"
    assert r["preflight_ok"] is True and r["param_checksum_ok"] is True
