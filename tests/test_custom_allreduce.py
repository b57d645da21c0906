"""Direct-peer-read xGMI all-reduce (csrc/custom_allreduce.hip, comm/custom_allreduce.py).

GPU: 2 and 4 processes share the box's single MI355X -- the IPC mapping, barriers, one-/two-shot data paths,
in-place / out-of-place, avg scaling and HIP-graph replay are the same code that runs across 8 GPUs; results must
be bit-identical to an fp32 rank-order sum.  CPU: the routing in comm.functional stays on the collective backend.
"""
import os
import subprocess
import sys

import pytest
import torch

from distributed_pytorch_hpc_amd.runtime.env import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_processes_share_one_gpu(world):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.join(ROOT, "tests", "scripts", "car_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert f"CAR_RESULT world={world}" in out and "failures=0" in out, out[-4000:]


def test_custom_allreduce_not_used_on_cpu(monkeypatch):
    from distributed_pytorch_hpc_amd.comm import functional as F
    from distributed_pytorch_hpc_amd.comm.custom_allreduce import get_custom_allreduce

    monkeypatch.setenv("DPH_CUSTOM_ALLREDUCE", "1")
    assert get_custom_allreduce(None) is None          # no process group
    x = torch.ones(16)
    assert F.all_reduce_(x, None) is x                 # world 1: untouched
