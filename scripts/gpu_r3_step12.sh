#!/usr/bin/env bash
# round 3 step 12: 3x3 weight-gradient kernel parity + per-pass bench (new LDS-DMA vs split-pixel ts_tn_k vs MIOpen)
export TMPDIR=/tmp
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run r3_s12_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv3x3" || exit 1
run r3_s12_conv3_bench python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench_c3w.json || exit 1
DPH_CONV3W_KERNEL=ts run r3_s12_conv3_bench_tsw python -u benchmarks/conv3x3_bench.py --json $O/r3_conv3_bench_tsw.json || exit 1
