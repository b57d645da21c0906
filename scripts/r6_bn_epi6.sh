#!/bin/bash
# round 6: conv3_k loads the BatchNorm operands before its K-loop -- tests, probe, A/B (v0 = both off, v2 = default),
# kernel profile of the default
set -o pipefail
out=gpurun_out/r6bn6
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_whole_net_grad_gpu.py > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u benchmarks/probes/bn_epi_probe.py > $out/probe.log 2>&1 || { tail $out/probe.log; exit 1; }
grep -v amdgpu.ids $out/probe.log | grep "conv2\|total"
for r in 1 2; do
  for v in 0 2; do
    e=$([ $v -ge 1 ] && echo 1 || echo 0); m=$([ $v -ge 2 ] && echo 1 || echo 0)
    DPH_BN_EPILOGUE=$e DPH_RES_MASK=$m timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/bench_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/bench_v${v}_r${r}.log | cut -c60-140)"
  done
done
timeout -k 10 500 bash scripts/prof_resnet.sh $out/prof 256 10 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -40 $out/prof/summary.txt | cut -c1-150
