#!/usr/bin/env bash
# Flash attention at B 8, H 32, S 4096, D 128 causal: TFLOP/s plus a sustained window per kernel under the GPU
# telemetry sampler (clock, power, TFLOP/J), then one rocprofv3 PMC pass (MFMA busy, issue waits, LDS conflicts) with
# the per-kernel summary.  Raw rocprof output stays in /tmp.
#
#   bash scripts/pmc_attn.sh OUTDIR
set -euo pipefail
out=${1:?usage: pmc_attn.sh OUTDIR}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python -u benchmarks/probes/attn_one.py --iters 20 --sustain 3 > "$out/probe.log" 2>&1
cat "$out/probe.log"
ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
raw=/tmp/pmc_attn_$$
rm -rf "$raw"
timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$raw" -o p -- python benchmarks/probes/attn_one.py --iters 4 \
  > "$out/pmc_run.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
python benchmarks/pmc_summary.py "$db" --match "attn_" --json "$out/pmc.json" > "$out/pmc.txt"
cat "$out/pmc.txt"
rm -rf "$raw"
