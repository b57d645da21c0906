#!/usr/bin/env bash
# Launch any driver on one MI355X node, one rank per GPU, through the framework launcher (gang watchdog,
# optional restarts, per-rank logs).  Replaces scripts/**/run_*.sh PBS templates and the
# ``mpiexec -n N --ppn 4 python X.py`` / torchrun-under-mpiexec lines of the reference (SURVEY.md L-PBS, L-TR).
#
#   scripts/launch_node.sh [NPROC] DRIVER [driver args...]
#   NPROC=8 MAX_RESTARTS=2 LOG_DIR=logs scripts/launch_node.sh examples/01_data_parallel_ddp/ddp_unet.py --epochs 3
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
ROOT="$(dirname "$HERE")"
source "$HERE/env_mi355x.sh"
if [[ "${1:-}" =~ ^[0-9]+$ ]]; then NPROC="$1"; shift; fi
NPROC="${NPROC:-$(python3 -c 'import torch; print(max(torch.cuda.device_count(), 1))')}"
DRIVER="$1"; shift
EXTRA=()
[[ -n "${LOG_DIR:-}" ]] && EXTRA+=(--log-dir "$LOG_DIR")
[[ -n "${TIMEOUT:-}" ]] && EXTRA+=(--timeout "$TIMEOUT")
exec python3 -m distributed_pytorch_hpc_amd.runtime.launch --nproc "$NPROC" --max-restarts "${MAX_RESTARTS:-0}" \
    "${EXTRA[@]}" "$DRIVER" "$@"
