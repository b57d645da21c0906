#!/usr/bin/env bash
# Any driver under rocprofv3 --kernel-trace, summarised over its last LAST_MS of GPU activity divided by STEPS.
# Raw rocprof output stays in /tmp; the driver log and the summary land in OUTDIR.
#
#   bash scripts/prof_cmd.sh OUTDIR STEPS LAST_MS python examples/01_data_parallel_ddp/ddp_unet.py --amp ...
set -euo pipefail
out=${1:?usage: prof_cmd.sh OUTDIR STEPS LAST_MS cmd...}
steps=${2:?}
last=${3:?}
shift 3
mkdir -p "$out"
export TMPDIR=/tmp
raw=/tmp/prof_cmd_$$
rm -rf "$raw"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$raw" -o p -- "$@" > "$out/run_under_rocprof.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
python benchmarks/prof_summary.py "$db" --steps "$steps" --last-ms "$last" --json "$out/summary.json" > "$out/summary.txt"
head -n 40 "$out/summary.txt"
rm -rf "$raw"
