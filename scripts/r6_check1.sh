#!/bin/bash
# round-6 check 1: new health guard / bench tests on the 1-GPU box, attention probe, 7B bench
set -o pipefail
out=gpurun_out/r6a
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_custom_allreduce.py tests/test_bench_gpu.py tests/test_multigpu.py > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
timeout -k 10 240 python -u benchmarks/probes/attn_one.py --iters 10 --sustain 2 > $out/attn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 3 > $out/bench.log 2>&1 || exit 1
tail -3 $out/tests.log; cat $out/attn.log; tail -1 $out/bench.log | cut -c1-400
