#!/usr/bin/env bash
# round 3 step 16: kernel-trace profile of the 7B step on the final tree; PMC counters of the 3x3 kernels and the
# attention backward
export TMPDIR=/tmp
O=gpurun_out
CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
rm -rf /tmp/prof7b && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof7b -o k -- python3 bench.py --steps 4 --warmup 2 > $O/r3_s16_prof7b.log 2>&1 || { echo "prof7b rc=$?"; exit 1; }
db=$(find /tmp/prof7b -name "*results.db" -print -quit); python benchmarks/rocpd_summary.py "$db" --window 0.55 --top 40 > $O/r3_s16_prof7b_summary.txt 2>&1; echo "prof7b ok"
rm -rf /tmp/pmcc3 && timeout -s KILL 200 rocprofv3 --pmc $CTRS -d /tmp/pmcc3 -o p -- python3 benchmarks/conv3x3_bench.py --only resnet50.layer3 > $O/r3_s16_pmc_conv3.log 2>&1 || { echo "pmc conv3 rc=$?"; exit 1; }
db=$(find /tmp/pmcc3 -name "*results.db" -print -quit); python benchmarks/pmc_summary.py "$db" --match "conv3_k|igemm|grouped_conv|c3w_k|ts_tn_k" > $O/r3_s16_pmc_conv3.txt 2>&1; echo "pmc conv3 ok"
rm -rf /tmp/pmcat && timeout -s KILL 200 rocprofv3 --pmc $CTRS -d /tmp/pmcat -o p -- python3 benchmarks/probes/attn_one.py --which fwd,bwd --iters 3 > $O/r3_s16_pmc_attn.log 2>&1 || { echo "pmc attn rc=$?"; exit 1; }
db=$(find /tmp/pmcat -name "*results.db" -print -quit); python benchmarks/pmc_summary.py "$db" --match "attn" > $O/r3_s16_pmc_attn.txt 2>&1; echo "pmc attn ok"
