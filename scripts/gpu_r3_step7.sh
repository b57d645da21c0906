#!/usr/bin/env bash
# round 3 step 7: UNet up-path kernels, smoke with gradient checks, unet-ddp bench A/B (100 timed steps) + rocprof
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_upsample_gpu.py > $O/r3_s7_upsample.log 2>&1 || { echo "upsample tests failed rc=$?"; exit 1; }
echo "upsample tests ok"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3_s7_smoke.log 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_fused.json > $O/r3_unet_fused.log 2>&1 || { echo "unet fused bench rc=$?"; exit 1; }
echo "unet fused ok"
DPH_FUSED_UPCAT=0 timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 100 --warmup 10 --json-out $O/r3_unet_unfused.json > $O/r3_unet_unfused.log 2>&1 || { echo "unet unfused bench rc=$?"; exit 1; }
echo "unet unfused ok"
timeout -k 10 300 python -u bench.py --layout unet-ddp --unet-precision fp32 --steps 100 --warmup 10 --json-out $O/r3_unet_fp32.json > $O/r3_unet_fp32.log 2>&1 || { echo "unet fp32 bench rc=$?"; exit 1; }
echo "unet fp32 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_unet -o unet -- python3 bench.py --layout unet-ddp --steps 20 --warmup 5 > $O/r3_unet_prof.log 2>&1 || { echo "unet prof rc=$?"; exit 1; }
echo "prof ok"
