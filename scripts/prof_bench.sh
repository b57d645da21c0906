#!/usr/bin/env bash
# One bench.py run, then the same bench under rocprofv3 --kernel-trace with a per-kernel / per-category summary.
# Raw rocprof output stays in /tmp (it is large); only the bench lines and the summary land in OUTDIR.
#
#   bash scripts/prof_bench.sh gpurun_out/prof_rNN [extra bench.py args...]
set -euo pipefail
out=${1:?usage: prof_bench.sh OUTDIR [bench args]}
shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 "$@" > "$out/bench.log" 2>&1
grep '^{"metric"' "$out/bench.log"
raw=/tmp/prof_bench_$$
rm -rf "$raw"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$raw" -o p -- python bench.py --steps 4 --warmup 2 "$@" \
  > "$out/bench_under_rocprof.log" 2>&1
db=$(find "$raw" -name "*results.db" -print -quit)
# the last 4 steps of GPU activity: 4 x the un-profiled ms/step, slightly trimmed
ms=$(python -c "import json,sys; print(4 * 0.99 * json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][0])['ms_per_step'])" "$out/bench.log")
step_ms=$(python -c "import json,sys; print(json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric')][0])['ms_per_step'])" "$out/bench.log")
# steps counted by the optimizer kernel (a fixed number of launches per step; 6 steps traced), time window otherwise
python benchmarks/prof_summary.py "$db" --steps 4 --last-ms "$ms" --step-marker "${PROF_STEP_MARKER:-adamw_k|sgd_k}" \
  --run-steps "${PROF_RUN_STEPS:-6}" --step-ms "$step_ms" --json "$out/summary.json" > "$out/summary.txt"
head -n 16 "$out/summary.txt"
rm -rf "$raw"
