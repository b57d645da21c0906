"""Tiny gloo training job used by the launcher fault-injection test.

Attempt 0: rank 2 dies with os._exit(3) at step 3 (after the step-2 checkpoint).  The launcher must tear down the
gang and restart; attempt 1 resumes from the latest checkpoint and finishes, writing DONE markers.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_pytorch_hpc_amd.models.llama2 import ModelArgs, build_llama  # noqa: E402
from distributed_pytorch_hpc_amd.parallel.data_parallel import DataParallelEngine, OptimConfig  # noqa: E402
from distributed_pytorch_hpc_amd.runtime import env as rt  # noqa: E402
from distributed_pytorch_hpc_amd.utils.checkpointing import ShardedCheckpointer  # noqa: E402

out_dir = sys.argv[1]
rank, world, _ = rt.init_distributed(backend="gloo", verbose=False, timeout_s=60)
torch.manual_seed(0)
m = build_llama(ModelArgs(dim=32, n_layers=1, n_heads=2, vocab_size=64, max_seq_len=32, multiple_of=16),
                device="cpu", dtype=torch.float32)
eng = DataParallelEngine(m, shard=True)
eng.configure_optimizer(OptimConfig(lr=1e-2))
ck = ShardedCheckpointer(os.path.join(out_dir, "ckpt"), m, eng)
start = ck.load()
attempt = int(os.environ.get("DPH_RESTART_COUNT", "0"))
g = torch.Generator().manual_seed(1)
data = [torch.randint(0, 64, (world * 2, 9), generator=g) for _ in range(6)]
for step in range(start, 6):
    if attempt == 0 and step == 3 and rank == 2:
        os._exit(3)
    t = data[step].chunk(world)[rank]
    loss = m(t[:, :-1], t[:, 1:])
    loss.backward()
    eng.step()
    eng.zero_grad()
    if step == 1:
        ck.save(step + 1)
with open(os.path.join(out_dir, f"DONE.{rank}"), "w") as fh:
    fh.write(f"{start} {attempt}\n")
rt.cleanup_distributed()
