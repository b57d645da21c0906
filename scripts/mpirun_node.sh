#!/usr/bin/env bash
# Open MPI launch (rank from OMPI_COMM_WORLD_*; runtime/env.py) -- the reference's
# `mpiexec -n 8 --ppn 8 --cpu-bind none python X.py` path without mpi4py.
#   scripts/mpirun_node.sh [NPROC] DRIVER [args...]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
source "$HERE/env_mi355x.sh"
if [[ "${1:-}" =~ ^[0-9]+$ ]]; then NPROC="$1"; shift; fi
export MASTER_ADDR=127.0.0.1
export MASTER_PORT="${MASTER_PORT:-$(python3 -c 'import socket; s=socket.socket(); s.bind(("127.0.0.1",0)); print(s.getsockname()[1])')}"
exec mpirun -np "${NPROC:-8}" --bind-to none -x MASTER_ADDR -x MASTER_PORT -x HSA_ENABLE_IPC_MODE_LEGACY \
    python3 "$@"
