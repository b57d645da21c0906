"""Per-rank stdout/stderr redirection (utils/redirect.py:5-38 of the reference).

``redirect(path, prefix)`` sends this rank's Python AND native output (fd 1/2, e.g. RCCL / HIP runtime
messages) to ``{path}/{prefix}.{rank}.out`` / ``.err``, line-buffered.  Used by runtime/launch.py.
"""
from __future__ import annotations

import os
import sys


def redirect(path: str, prefix: str = "rank", rank: int | None = None):
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    os.makedirs(path, exist_ok=True)
    out = open(os.path.join(path, f"{prefix}.{rank}.out"), "a", buffering=1)
    err = open(os.path.join(path, f"{prefix}.{rank}.err"), "a", buffering=1)
    sys.stdout.flush()
    sys.stderr.flush()
    os.dup2(out.fileno(), 1)
    os.dup2(err.fileno(), 2)
    sys.stdout, sys.stderr = out, err
    return out, err
