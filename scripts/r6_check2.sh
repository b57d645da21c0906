#!/bin/bash
# round 6: graph-default bench test, 1x1 convolution roofline probe
set -o pipefail
out=gpurun_out/r6c2
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bench_gpu.py -k graph > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u benchmarks/probes/conv1x1_fwd_probe.py > $out/c1.log 2>&1 || { tail $out/c1.log; exit 1; }
grep -v amdgpu.ids $out/c1.log
