# A/B of the flash-attention forward variants (one process per arm, two interleaved rounds) on the 7B shape.
set -o pipefail
out=${1:-gpurun_out/r5/ab_fwd.log}
: > "$out"
for round in 1 2; do
  for arm in legacy 0 1 2 3; do
    if [ "$arm" = legacy ]; then env="DPH_ATTN_FWD=legacy"; else env="DPH_ATTN_FWD=pipe DPH_ATTN_FWD_VAR=$arm"; fi
    echo "== $arm round $round" >> "$out"
    env $env timeout -k 10 120 python3 -u benchmarks/probes/attn_one.py --iters 20 --which fwd >> "$out" 2>&1 || exit 1
  done
done
