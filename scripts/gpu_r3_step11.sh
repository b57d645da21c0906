#!/usr/bin/env bash
# round 3 step 11: 3x3 path defaults (OOB zero, MIOpen wgrad) + native up-path GEMMs: parity, ResNet-50 / UNet A/B
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s11_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_upsample_gpu.py -k "conv3x3 or bottleneck or up_concat or unet" || exit 1
for rep in 1 2; do for c in 0 1; do
  DPH_CONV3X3=$c run r3_s11_resnet_c${c}_rep$rep python -u bench.py --layout resnet-fsdp --steps 20 --warmup 5 --json-out $O/r3_resnet_c${c}_rep$rep.json || exit 1
  DPH_CONV3X3=$c run r3_s11_unet_c${c}_rep$rep python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_c${c}_rep$rep.json || exit 1
done; done
DPH_CONV3X3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_unet11 -o unet -- python3 bench.py --layout unet-ddp --steps 30 --warmup 5 > $O/r3_s11_unet_prof.log 2>&1; echo "prof rc=$?"
