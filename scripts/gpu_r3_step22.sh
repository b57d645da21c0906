#!/usr/bin/env bash
# round 3 step 22: dS hand-off v2 (counted dK/dV wait, 8-wave 3-stage dQ pass)
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { local name=$1; local t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | tail -1)"; return $rc; }
run r3_s22_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" || exit 1
for rep in 1 2; do for cfg in "0 8" "1 8" "1 4"; do set -- $cfg
  DPH_ATTN_DS=$1 DPH_ATTN_DS_WAVES=$2 run r3_s22_attn_ds$1_w$2_rep$rep 300 python -u benchmarks/probes/attn_one.py --which bwd --iters 10 || exit 1
  grep bwd $O/r3_s22_attn_ds$1_w$2_rep$rep.log
done; done
run r3_s22_prof 300 rocprofv3 --kernel-trace --stats -d $O/r3_s22_prof -o prof -- python -u benchmarks/probes/attn_one.py --which bwd --iters 3 || exit 1
python benchmarks/rocpd_summary.py $O/r3_s22_prof/prof_results.db | head -8
