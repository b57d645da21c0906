#!/bin/bash
# round 4 step 36: grid-tail probe of the 1x1 / 3x3 forward kernels; SimpleUNet eager vs whole-step graph now that its
# kernel time dropped to 3.56 ms (interleaved)
set -o pipefail
O=gpurun_out/r4s36; mkdir -p $O
timeout -k 10 300 python -u benchmarks/probes/grid_tail.py > $O/grid_tail.log 2>&1 || { tail -20 $O/grid_tail.log; exit 1; }
grep -v amdgpu.ids $O/grid_tail.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['kind'], d['N'], d['K'], d['row_tiles'], d['ms'], d['us_per_row_tile'])"
for rep in 1 2; do
  for g in 0 1; do
    flag=""; [ $g = 1 ] && flag=--graph
    timeout -k 10 300 python -u bench.py --layout unet-ddp --steps 40 --warmup 8 $flag > $O/unet_graph${g}_r$rep.log 2>&1 || { tail -20 $O/unet_graph${g}_r$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][0]); print('unet graph', sys.argv[2], d['value'], d['step_ms']['median'], d['step_ms']['stdev'])" $O/unet_graph${g}_r$rep.log $g
  done
done
