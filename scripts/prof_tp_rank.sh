# rocprofv3 kernel trace of one tensor-parallel rank's Llama-2-7B step (collectives stubbed) at TP = 8 and TP = 4,
# plus the un-traced ms/step of each (BASELINE configs 3 / 4; verdict r4 "account for the TP-rank gap").
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5/${TP_OUT:-tp_rank}
mkdir -p $out
for tp in 8 4; do
  timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp $tp --steps 5 > $out/tp${tp}_bench.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_tp$tp -o p -- python3 $R/benchmarks/tp_rank_bench.py --tp $tp --steps 3 --warmup 2 > $out/tp${tp}_prof.log 2>&1 || exit 1
  db=$(ls $out/prof_tp$tp/*/*.db $out/prof_tp$tp/*.db 2>/dev/null | head -1)
  ms=$(python3 -c "import json,sys; print([json.loads(l) for l in open('$out/tp${tp}_bench.log') if l.startswith('{')][-1]['ms_per_step'])")
  last=$(python3 -c "print(3 * $ms * 1.3)")
  python3 $R/benchmarks/prof_summary.py "$db" --steps 3 --last-ms "$last" --json $out/summary_tp$tp.json > $out/summary_tp$tp.txt || exit 1
  rm -rf $out/prof_tp$tp   # the trace database is far larger than what gpurun copies back
  echo "tp $tp: $ms ms/step"; head -25 $out/summary_tp$tp.txt
done
