#!/usr/bin/env python3
"""Do the stub ("fake") process group's collectives launch device copies?  tp_rank_bench.py stubs every collective
with torch's fake process group; its rocprof trace shows ~1400 __amd_rocclr_copyBuffer per step that no framework
op issues.  This times each stubbed collective kind on GPU tensors under torch.profiler and prints the device
activities it launched."""
import torch
import torch.distributed as dist
from torch.profiler import ProfilerActivity, profile
from torch.testing._internal.distributed.fake_pg import FakeStore

dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=8)
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
out = torch.empty(8 * 4096, 4096, device="cuda", dtype=torch.bfloat16)
small = torch.empty(512, 4096, device="cuda", dtype=torch.bfloat16)
for name, fn in (("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(out, x)),
                 ("reduce_scatter_tensor", lambda: dist.reduce_scatter_tensor(small, x)),
                 ("all_reduce", lambda: dist.all_reduce(x))):
    fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    dev = [e for e in prof.events() if e.device_type.name == "CUDA"]
    print(f"{name}: {len(dev)} device activities in 10 calls: "
          f"{sorted(set(e.name for e in dev))[:4]}", flush=True)
