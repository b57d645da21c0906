#!/bin/bash
# round 4 step 18: attention backward with 8-wave workgroups vs 4 (A/B), and PMC of the three attention kernels
set -o pipefail
O=gpurun_out/r4s18; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for w in 4 8; do
    DPH_ATTN_WAVES=$w timeout -k 10 120 python -u benchmarks/probes/attn_one.py --which fwd,bwd --iters 20 > $O/attn_w${w}_r$rep.log 2>&1 || { tail $O/attn_w${w}_r$rep.log; exit 1; }
    echo "waves=$w rep=$rep $(grep -v amdgpu $O/attn_w${w}_r$rep.log | tr '\n' ' ')"
  done
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  -d /tmp/pmc_attn -o p -- python benchmarks/probes/attn_one.py --which fwd,bwd --iters 3 > $O/pmc_attn.run.log 2>&1 || { tail -5 $O/pmc_attn.run.log; exit 1; }
db=$(find /tmp/pmc_attn -name "*results.db" -print -quit)
python benchmarks/pmc_summary.py "$db" > $O/pmc_attention_r4.txt 2>&1
grep -A20 "attn_" $O/pmc_attention_r4.txt | grep -E "==|mfma_busy|clock|_dur"
