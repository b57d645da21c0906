"""Utility façade with the reference package's names (utils/__init__.py:9-16 re-exports its distributed and logging
helpers), so ``from distributed_pytorch_hpc_amd.utils import init_distributed, print_rank0, ...`` replaces
``from utils import ...`` of the reference scripts one to one.

    distributed   get_rank_info, init_distributed, cleanup_distributed, is_main_rank, print_rank0  (runtime/env.py)
    logging       get_logger, rank_log, verify_min_gpu_count                                       (utils/logging.py)
    profiling     training_profiler, print_profiler_summary                                         (utils/profiling.py)
    checkpointing save_checkpoint, load_checkpoint, ShardedCheckpointer                             (utils/checkpointing.py)
    config        TrainingConfig                                                                    (utils/config.py)
    redirect      redirect                                                                          (utils/redirect.py)
"""
from ..runtime.env import cleanup_distributed, get_rank_info, init_distributed, is_main_rank, print_rank0
from .checkpointing import ShardedCheckpointer, load_checkpoint, save_checkpoint
from .config import TrainingConfig
from .logging import get_logger, rank_log, verify_min_gpu_count
from .profiling import print_profiler_summary, training_profiler
from .redirect import redirect

__all__ = [
    "get_rank_info", "init_distributed", "cleanup_distributed", "is_main_rank", "print_rank0",
    "get_logger", "rank_log", "verify_min_gpu_count", "training_profiler", "print_profiler_summary",
    "save_checkpoint", "load_checkpoint", "ShardedCheckpointer", "TrainingConfig", "redirect",
]
