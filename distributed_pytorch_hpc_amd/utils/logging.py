"""Rank-aware logging (utils/logging.py:1-65 and fsdp_tp/log_utils.py of the reference, one module).

Every record carries the rank ("[r3/8]"); ``rank_log`` emits on rank 0 only; ``get_logger(level)`` honours the
``DPH_LOG_LEVEL`` environment variable.  No global ``basicConfig`` side effect at import.
"""
from __future__ import annotations

import logging
import os
import sys

import torch

_FMT = "%(asctime)s [r%(rank)s/%(world)s] %(levelname)s %(name)s: %(message)s"


class _RankFilter(logging.Filter):
    def filter(self, record):
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                record.rank, record.world = dist.get_rank(), dist.get_world_size()
            else:
                record.rank, record.world = os.environ.get("RANK", "0"), os.environ.get("WORLD_SIZE", "1")
        except Exception:  # pragma: no cover
            record.rank, record.world = "?", "?"
        return True


def get_logger(name: str = "dph", level: str | int | None = None) -> logging.Logger:
    logger = logging.getLogger(name)
    if not getattr(logger, "_dph_configured", False):
        h = logging.StreamHandler(sys.stdout)
        h.setFormatter(logging.Formatter(_FMT))
        h.addFilter(_RankFilter())
        logger.addHandler(h)
        logger.propagate = False
        logger._dph_configured = True
    lvl = level if level is not None else os.environ.get("DPH_LOG_LEVEL", "INFO")
    logger.setLevel(lvl if isinstance(lvl, int) else lvl.upper())
    return logger


def rank_log(rank: int, logger: logging.Logger, msg: str, *args):
    """Log only from rank 0 (reference: utils/logging.py rank_log)."""
    if rank == 0:
        logger.info(msg, *args)


def verify_min_gpu_count(min_gpus: int = 2) -> bool:
    return torch.cuda.is_available() and torch.cuda.device_count() >= min_gpus
