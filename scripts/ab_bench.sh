#!/usr/bin/env bash
# A/B of two environment settings on the headline bench, interleaved in one GPU session (same box, same clock).
# usage: bash scripts/ab_bench.sh OUTDIR "ENV_A" "ENV_B" [rounds]
set -o pipefail
cd /root/repo
out=gpurun_out/$1; mkdir -p $out
A="$2"; B="$3"; R=${4:-2}
for r in $(seq 1 $R); do
  env $A timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 > $out/A_$r.log 2>&1 || exit 1
  env $B timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 > $out/B_$r.log 2>&1 || exit 1
done
for f in $out/A_*.log $out/B_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
