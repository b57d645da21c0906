#!/usr/bin/env bash
# Same as launch_node.sh with stock torchrun (c10d rendezvous on 127.0.0.1).
#   scripts/torchrun_node.sh [NPROC] DRIVER [args...]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/env_mi355x.sh"
if [[ "${1:-}" =~ ^[0-9]+$ ]]; then NPROC="$1"; shift; fi
NPROC="${NPROC:-8}"
PORT="${MASTER_PORT:-$(python3 -c 'import socket; s=socket.socket(); s.bind(("127.0.0.1",0)); print(s.getsockname()[1])')}"
exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 \
    --master-port "$PORT" --max-restarts "${MAX_RESTARTS:-0}" "$@"
