#!/bin/bash
# round-6: x16 attention numerics, then SimpleUNet DDP (B = 4, 65 x 181 x 360, bf16) eager vs whole-step HIP graph,
# interleaved, 100 timed steps each
set -o pipefail
out=gpurun_out/r6/unet_graph
mkdir -p $out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "x16_forms" > $out/tests_x16.log 2>&1 || { tail -30 $out/tests_x16.log; exit 1; }
tail -1 $out/tests_x16.log
for r in 1 2; do
  for arm in eager graph; do
    extra=""; [ $arm = graph ] && extra="--graph"
    timeout -k 10 200 python -u bench.py --layout unet-ddp --steps 100 --warmup 5 $extra > $out/${arm}_r$r.log 2>&1 || exit 1
    python3 -c "import json; r=json.loads([l for l in open('$out/${arm}_r$r.log') if l.startswith('{')][0]); print('$arm r$r', r['value'], r['ms_per_step'], r['step_ms']['median'], r['step_ms']['stdev'])"
  done
done
