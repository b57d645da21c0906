#!/usr/bin/env bash
# round 3 step 10: 3x3 LDS-DMA conv kernel (parity + per-pass bench vs MIOpen and the old path), dQ prefetch A/B,
# UNet up-path tests, smoke, unet-ddp bench A/B
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s10_conv3_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv3x3 or bottleneck" || exit 1
run r3_s10_conv3_bench python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench.json || exit 1
DPH_CONV3_ZERO=oob run r3_s10_conv3_tests_oob python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv3x3 or bottleneck" || exit 1
DPH_CONV3_ZERO=oob run r3_s10_conv3_bench_oob python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench_oob.json || exit 1
DPH_CONV3_KERNEL=ts run r3_s10_conv3_bench_old python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench_old.json || exit 1
DPH_ATTN_DQ_VAR=1 run r3_s10_attn_dqpf_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_dropout.py -k "flash or attention or attn" || exit 1
for rep in 1 2; do for v in 0 1; do
  DPH_ATTN_DQ_VAR=$v run r3_s10_attn_bwd_dq${v}_rep$rep python -u benchmarks/probes/attn_one.py --which bwd --iters 20 || exit 1
done; done
grep -H "bwd" $O/r3_s10_attn_bwd_dq*_rep*.log
run r3_s10_upsample python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_upsample_gpu.py
run r3_s10_smoke python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run r3_s10_unet_fused python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_fused.json || exit 1
DPH_FUSED_UPCAT=0 run r3_s10_unet_unfused python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_unfused.json || exit 1
