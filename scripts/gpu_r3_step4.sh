#!/usr/bin/env bash
# round 3 step 4: ragged wgrad + fused-MLP tests, HIP-graph side-stream diagnosis, in-step A/B of the fused paths
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py "tests/test_kernels_gpu.py" -k "gemm_nt or gemm_tn or llama_fused" > gpurun_out/r3_s4_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/diag_graph_side_stream.py --json gpurun_out/r3_graph_diag.json > gpurun_out/r3_graph_diag.log 2>&1; rc=$?; echo "diag rc=$rc"
[ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for mode in 0 bwd 1; do
    q=0; [ "$mode" = "1" ] && q=1
    DPH_FUSED_MLP=$mode DPH_FUSED_QKV=$q timeout -k 10 300 python bench.py --steps 6 --warmup 2 --quiet > gpurun_out/r3_ab_mlp_${mode}_$rep.log 2>&1 || exit $?
    echo "mode=$mode rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/r3_ab_mlp_${mode}_$rep.log)"
  done
done
