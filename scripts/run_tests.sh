#!/usr/bin/env bash
# Test + diagnostics battery (counterpart of the reference's tests/run_tests.sh and tests/pbs_run_tests.sh:
# send/recv + all-reduce with nccl vs gloo, then the workload drivers).
#   scripts/run_tests.sh [cpu|gpu|comm|all]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
ROOT="$(dirname "$HERE")"
cd "$ROOT"
source "$HERE/env_mi355x.sh"
MODE="${1:-cpu}"
NGPU=$(python3 -c 'import torch; print(torch.cuda.device_count())')
if [[ "$MODE" == cpu || "$MODE" == all ]]; then
    python3 -m pytest tests -q -m "not gpu"
fi
if [[ "$MODE" == gpu || "$MODE" == all ]]; then
    timeout -k 10 900 python3 -m pytest tests -q -m gpu
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.build(); g.smoke()"
fi
if [[ "$MODE" == comm || "$MODE" == all ]]; then
    mkdir -p results
    timeout -k 10 300 python3 benchmarks/check_env.py
    for be in gloo nccl; do
        n=$([[ $be == nccl ]] && echo "$NGPU" || echo 4)
        [[ "$n" -lt 2 ]] && { echo "skip $be (needs >= 2 ranks)"; continue; }
        timeout -k 10 600 "$HERE/torchrun_node.sh" "$n" benchmarks/send_recv_test.py --backend $be --smoke
        timeout -k 10 900 "$HERE/torchrun_node.sh" "$n" benchmarks/comm_bench.py --backend $be \
            --csv "results/comm_${be}_${n}.csv"
    done
fi
