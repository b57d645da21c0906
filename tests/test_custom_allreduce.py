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


def test_choose_crossover_rule():
    from distributed_pytorch_hpc_amd.comm.custom_allreduce import choose_crossover

    KiB = 1 << 10
    # direct-peer wins up to 256 KiB, then RCCL: the crossover is the last winning size
    s = [(4 * KiB, 20e-6, 8e-6), (64 * KiB, 22e-6, 10e-6), (256 * KiB, 30e-6, 25e-6), (1 << 20, 40e-6, 45e-6),
         (4 << 20, 80e-6, 70e-6)]
    assert choose_crossover(s) == 256 * KiB          # a later win after a loss does not count
    assert choose_crossover(list(reversed(s))) == 256 * KiB
    assert choose_crossover([(4 * KiB, 5e-6, 9e-6)]) == 0          # RCCL wins from the start: nothing changes
    assert choose_crossover([(4 * KiB, 5e-6, None)]) == 0          # no direct-peer arm on this group
    assert choose_crossover([]) == 0


def test_policy_routing_is_size_and_env_driven(monkeypatch):
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as C

    monkeypatch.delenv("DPH_CUSTOM_ALLREDUCE", raising=False)
    C.clear_policy(None)
    assert C.policy_max_bytes(None) == 0                       # no measurement: RCCL
    C.set_policy(None, 1 << 20)
    try:
        assert C.policy_max_bytes(None) == 1 << 20
        monkeypatch.setenv("DPH_CUSTOM_ALLREDUCE", "0")
        assert C.policy_max_bytes(None) == 0                   # forced off
        monkeypatch.setenv("DPH_CUSTOM_ALLREDUCE", "1")
        monkeypatch.setenv("DPH_CUSTOM_ALLREDUCE_MAX_BYTES", str(4 << 20))
        assert C.policy_max_bytes(None) == 4 << 20             # forced on
        monkeypatch.delenv("DPH_CUSTOM_ALLREDUCE")
        assert C.use_custom(torch.ones(16), None) is None      # CPU tensors never take the IPC path
    finally:
        C.clear_policy(None)


def test_check_health_raises_and_disables_path(monkeypatch):
    """Advisor r4: a timed-out direct-peer barrier must stop training at the next step boundary (not leave wrong
    sums in the gradients) and turn the path off for that group."""
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as car

    class _Fake:
        _guard_event = None   # no engine guard ran: the rank's own timeout word decides

        def __init__(self, err):
            self.err = err
            self.closed = False

        def errors(self):
            return self.err

        def close(self):
            self.closed = True

    bad = _Fake(1)
    monkeypatch.setattr(car, "_CACHE", {"world": _Fake(0), 123: bad})
    monkeypatch.setattr(car, "_POLICY", {"world": 1 << 20, 123: 1 << 20})
    monkeypatch.setattr(car, "_DEAD", set())
    with pytest.raises(car.XgmiAllReduceError):
        car.check_health()
    assert 123 not in car._POLICY and car._POLICY["world"] == 1 << 20
    assert car._CACHE[123] is None and bad.closed and 123 in car._DEAD
    car.check_health()   # healthy groups: no error


def test_check_health_reads_the_agreed_verdict_after_the_guard(monkeypatch):
    """With an engine guard in flight the host check waits for that guard's event and reads the group-agreed word,
    not this rank's own one: every rank raises at the same step (advisor r5)."""
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as car

    class _Ev:
        waited = False

        def synchronize(self):
            _Ev.waited = True

    class _Guarded:
        def __init__(self, own, agreed):
            self.own, self.agreed = own, agreed
            self._guard_event = _Ev()

        def errors(self):
            return self.own

        def agreed_error(self):
            return self.agreed

        def close(self):
            pass

    monkeypatch.setattr(car, "_POLICY", {"world": 1 << 20})
    monkeypatch.setattr(car, "_DEAD", set())
    monkeypatch.setattr(car, "_CACHE", {"world": _Guarded(own=0, agreed=1)})   # a peer timed out, not this rank
    with pytest.raises(car.XgmiAllReduceError):
        car.check_health()
    assert _Ev.waited and "world" in car._DEAD
    monkeypatch.setenv("DPH_CUSTOM_ALLREDUCE", "1")
    assert car.policy_max_bytes(None) == 0          # dead groups stay off, whatever the environment says
    monkeypatch.setattr(car, "_CACHE", {"world": _Guarded(own=1, agreed=0)})   # own word alone does not raise
    car._DEAD.clear()
    car.check_health()


def test_engine_step_checks_xgmi_health(monkeypatch):
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as car
    from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig

    m = torch.nn.Linear(8, 8)
    eng = DataParallelEngine(m, shard=False)
    eng.configure_optimizer(OptimConfig(lr=1e-3))
    m(torch.randn(4, 8)).sum().backward()
    eng.synchronize()

    class _Bad:
        _guard_event = None

        def errors(self):
            return 1

        def close(self):
            pass

    monkeypatch.setattr(car, "_CACHE", {"world": _Bad()})
    monkeypatch.setattr(car, "_POLICY", {})
    monkeypatch.setattr(car, "_DEAD", set())
    with pytest.raises(car.XgmiAllReduceError):
        eng.step()


def test_failed_probe_drops_the_instance(monkeypatch):
    """A direct-peer path that fails the crossover probe (wrong sums or a barrier timeout; probe_crossover calls
    drop() on every rank) is never used again, and its recorded timeout does not stop training at the first engine
    step."""
    from distributed_pytorch_hpc_amd.comm import custom_allreduce as car

    class _Bad:
        closed = False

        def errors(self):
            return 1

        def close(self):
            _Bad.closed = True

    monkeypatch.setattr(car, "_CACHE", {"world": _Bad()})
    monkeypatch.setattr(car, "_POLICY", {"world": 1 << 20})
    car.drop(None)
    assert car._CACHE["world"] is None and "world" not in car._POLICY and _Bad.closed
    car.check_health()   # no error: the failed instance is gone
    assert car.get_custom_allreduce(None) is None   # cached as unusable (no process group here either)
