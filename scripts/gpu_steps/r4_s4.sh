#!/bin/bash
# round 4 step 4: same-batch stock comparator, UNet host overhead (both precisions) with cProfile
set -o pipefail
O=gpurun_out/r4s4; mkdir -p $O
timeout -k 10 400 python -u bench.py --micro-batch 4 --steps 10 --warmup 3 > $O/bench_b4.log 2>&1 || { tail -20 $O/bench_b4.log; exit 1; }
tail -1 $O/bench_b4.log | cut -c1-220
timeout -k 10 400 python -u benchmarks/torch_baseline.py --micro-batch 4 --steps 6 --warmup 2 > $O/torch_b4_fp32.log 2>&1 || { tail -5 $O/torch_b4_fp32.log; exit 1; }
tail -1 $O/torch_b4_fp32.log | cut -c1-220
timeout -k 10 400 python -u benchmarks/torch_baseline.py --params bf16 --micro-batch 4 --steps 6 --warmup 2 > $O/torch_b4_bf16.log 2>&1 || { tail -5 $O/torch_b4_bf16.log; exit 1; }
tail -1 $O/torch_b4_bf16.log | cut -c1-220
timeout -k 10 400 python -u benchmarks/torch_baseline.py --params bf16 --micro-batch 8 --steps 6 --warmup 2 > $O/torch_b8_bf16.log 2>&1
tail -2 $O/torch_b8_bf16.log | cut -c1-300
for prec in bf16 bf16-autocast; do
  timeout -k 10 300 python -u benchmarks/probes/host_overhead.py --layout unet-ddp --unet-precision $prec --steps 20 --warmup 5 --cprofile 5 --top 40 > $O/unet_host_$prec.log 2>&1 || { tail -20 $O/unet_host_$prec.log; exit 1; }
  head -60 $O/unet_host_$prec.log
done
