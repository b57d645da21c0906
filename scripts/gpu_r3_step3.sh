#!/usr/bin/env bash
# round 3: gemm_nt variant A/B + PMC of both variants and hipBLASLt on the wqkv shape
export TMPDIR=/tmp
python -c "import torch" > /dev/null 2>&1
timeout -k 10 400 python -u benchmarks/gemm_nt_bench.py --rounds 3 --json gpurun_out/r3_gemm_nt_bench_v01.json > gpurun_out/r3_gemm_nt_bench_v01.log 2>&1 || exit $?
for v in 0 1; do
  rm -rf /tmp/pmc_nt_$v
  DPH_GEMM_NT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/pmc_nt_$v -o p -- python benchmarks/gemm_nt_bench.py --shapes wqkv --rounds 1 --iters 2 --variants $v --no-fused > gpurun_out/r3_pmc_nt_v$v.log 2>&1 || exit $?
  db=$(find /tmp/pmc_nt_$v -name "*results.db" -print -quit)
  python benchmarks/pmc_summary.py "$db" --match "gemm_nt|Cijk" > gpurun_out/r3_pmc_nt_v$v.txt 2>&1
done
