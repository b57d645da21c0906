#!/usr/bin/env bash
# Single-GPU smoke of the example drivers on an MI355X (one rank; RCCL paths need >= 2 GPUs and are covered by the
# gloo tests).  Each step is time-limited; the first failure stops the script.
set -euo pipefail
cd "$(dirname "${BASH_SOURCE[0]}")/.."
OUT=${OUT:-gpurun_out/examples}
mkdir -p "$OUT"
run() {
    local name=$1; shift
    if [[ -n "${ONLY:-}" && " $ONLY " != *" $name "* ]]; then return 0; fi
    echo "== $name"; timeout -k 10 "${T:-300}" python3 "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1; tail -n 1 "$OUT/$name.log"; }
run ddp_unet examples/01_data_parallel_ddp/ddp_unet.py --epochs 2 --steps-per-epoch 10 --amp --channels-last
run fsdp_resnet examples/02_fully_sharded_fsdp/fsdp_resnet.py --use-amp --epochs 2 --steps-per-epoch 10
run tp_vit examples/03_tensor_parallel_tp/tensor_parallel_vit.py --tp 1 --epochs 1 --steps-per-epoch 10 --bf16
run pp_training examples/04_pipeline_parallel_pp/pipeline_training.py --steps 5 --warmup 2
run cp_llama examples/05_sequence_context_parallel/context_parallel_llama.py --mode ring --seq-len 8192 --model llama2-1b --n-layers 4 --steps 3
run hybrid_llama examples/06_hybrid_parallelism/fsdp_tp_hybrid.py --tp 1 --model llama2-1b --batch 4 --seq-len 2048 --iters 4
run domain_unet examples/07_domain_parallel/domain_parallel_unet.py --steps 3 --check
run resnet50_ddp examples/resnet_benchmark.py --arch resnet50 --amp --channels-last --batch-size 256 --epochs 3 --steps-syn 20
