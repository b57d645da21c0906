#!/bin/bash
# round 6: BatchNorm reductions in dgrad epilogues + bn3's masked residual-gradient hand-off -- tests, per-shape probe,
# interleaved ResNet-50 FSDP A/B: v0 both off, v1 reductions only, v2 both (default)
set -o pipefail
out=gpurun_out/r6bn5
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_epilogue_gpu.py \
  tests/test_kernels_gpu.py tests/test_strided_conv_gpu.py -k "bn or conv or bottleneck or slot or resnet or epilogue or mask" \
  > $out/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u benchmarks/probes/bn_epi_probe.py > $out/probe.log 2>&1 || { tail $out/probe.log; exit 1; }
grep -v amdgpu.ids $out/probe.log
for r in 1 2; do
  for v in 0 1 2; do
    e=$([ $v -ge 1 ] && echo 1 || echo 0); m=$([ $v -ge 2 ] && echo 1 || echo 0)
    DPH_BN_EPILOGUE=$e DPH_RES_MASK=$m timeout -k 10 300 python -u bench.py --layout resnet-fsdp --steps 30 --warmup 5 > $out/bench_v${v}_r${r}.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $out/bench_v${v}_r${r}.log | cut -c60-140)"
  done
done
