#!/usr/bin/env bash
# round 3 step 9: dQ prefetch A/B (+ parity), UNet up-path tests, smoke, unet-ddp bench A/B + rocprof
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
DPH_ATTN_DQ_VAR=1 run r3_s9_attn_dqpf_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_dropout.py -k "flash or attention or attn" || exit 1
for rep in 1 2; do for v in 0 1; do
  DPH_ATTN_DQ_VAR=$v run r3_s9_attn_bwd_dq${v}_rep$rep python -u benchmarks/probes/attn_one.py --which bwd --iters 20 || exit 1
done; done
grep -H "bwd" $O/r3_s9_attn_bwd_dq*_rep*.log
run r3_s9_upsample python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_upsample_gpu.py
run r3_s9_smoke python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run r3_s9_unet_fused python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_fused.json || exit 1
DPH_FUSED_UPCAT=0 run r3_s9_unet_unfused python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_unfused.json || exit 1
run r3_s9_unet_fp32 python -u bench.py --layout unet-ddp --unet-precision fp32 --steps 100 --warmup 10 --json-out $O/r3_unet_fp32.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_unet -o unet -- python3 bench.py --layout unet-ddp --steps 20 --warmup 5 > $O/r3_s9_unet_prof.log 2>&1; echo "prof rc=$?"
