#!/bin/bash
# round-6: (1) 3 interleaved 7B bench rounds, attention variant 0 (32x32x16, default) vs 2 (16x16x32);
# (2) one TP rank's step (collectives stubbed) at TP 8 and 4 under rocprofv3 + TP 8 with every projection on the NT kernel
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6/tp_ab
mkdir -p $out
for r in 1 2 3; do
  for v in 0 2; do
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --attn-variant $v > $out/bench_v${v}_r$r.log 2>&1 || exit 1
    python3 -c "import json; r=json.loads([l for l in open('$out/bench_v${v}_r$r.log') if l.startswith('{')][0]); print('v$v r$r', r['value'], r['ms_per_step'], r.get('sclk_mhz',{}).get('median'), r.get('avg_power_w'))"
  done
done
for tp in 8 4; do
  timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp $tp --steps 5 > $out/tp${tp}_bench.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_tp$tp -o p -- python3 $R/benchmarks/tp_rank_bench.py --tp $tp --steps 3 --warmup 2 > $out/tp${tp}_prof.log 2>&1 || exit 1
  db=$(find /tmp/prof_tp$tp -name "*results.db" -print -quit)
  ms=$(python3 -c "import json,sys; print([json.loads(l) for l in open('$out/tp${tp}_bench.log') if l.startswith('{')][-1]['ms_per_step'])")
  last=$(python3 -c "print(3 * $ms * 1.3)")
  python3 $R/benchmarks/prof_summary.py "$db" --steps 3 --last-ms "$last" --json $out/summary_tp$tp.json > $out/summary_tp$tp.txt || exit 1
  rm -rf /tmp/prof_tp$tp
  echo "tp $tp: $ms ms/step"; head -22 $out/summary_tp$tp.txt
done
timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp 8 --steps 5 --gemm-nt all > $out/tp8_ntall_bench.log 2>&1 || exit 1
echo "tp 8 gemm-nt all: $(tail -1 $out/tp8_ntall_bench.log)"
timeout -k 10 240 python3 -u $R/benchmarks/tp_rank_bench.py --tp 8 --steps 5 > $out/tp8_bench_r2.log 2>&1 || exit 1
echo "tp 8 default again: $(tail -1 $out/tp8_bench_r2.log)"
