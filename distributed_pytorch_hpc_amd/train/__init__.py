"""Training utilities: fused flat optimizers and the generic epoch loop."""
from .optim import FusedAdamW, FusedSGD, clip_grad_norm_, global_grad_norm
from .trainer import EpochStats, Trainer, setup_run

__all__ = ["FusedAdamW", "FusedSGD", "clip_grad_norm_", "global_grad_norm", "EpochStats", "Trainer", "setup_run"]
