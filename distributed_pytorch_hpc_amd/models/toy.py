"""Small demonstration models used by the walkthroughs and tests.

Same shapes and parameter names as the reference toys so the same TP / PP plans apply:
  ToyMLP        in_proj -> ReLU -> out_proj (16->64->16)       scripts/03_tensor_parallel_tp/02_basic_tensor_parallel.py:46-54
  ToyModel      64 -> 64 -> 64                                 fsdp_tp/tensor_parallel_example.py:76-84
  SimpleModel   fc1 -> ReLU -> fc2 (10->64->2)                 scripts/01_data_parallel_ddp/distributed_dataloader.py:160-172
  LinearModel   Linear(20, 1)                                  scripts/01_data_parallel_ddp/multinode_ddp_basic.py:211-215
  FourBlockMLP  4 x Linear(512, 512) (+ReLU on the first 3)    scripts/04_pipeline_parallel_pp/02_pipeline_schedules.py:45-60
  StageModule   Linear (+ReLU unless last)                     scripts/04_pipeline_parallel_pp/01_manual_model_split.py:38-50
"""
from __future__ import annotations

import torch
from torch import nn


class ToyMLP(nn.Module):
    def __init__(self, in_dim: int = 16, hidden_dim: int = 64, out_dim: int = 16):
        super().__init__()
        self.in_proj = nn.Linear(in_dim, hidden_dim)
        self.relu = nn.ReLU()
        self.out_proj = nn.Linear(hidden_dim, out_dim)

    def forward(self, x):
        return self.out_proj(self.relu(self.in_proj(x)))


class ToyModel(ToyMLP):
    def __init__(self, dim: int = 64):
        super().__init__(dim, dim, dim)


class SimpleModel(nn.Module):
    def __init__(self, input_dim: int = 10, hidden_dim: int = 64, output_dim: int = 2):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, hidden_dim)
        self.relu = nn.ReLU()
        self.fc2 = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        return self.fc2(self.relu(self.fc1(x)))


class LinearModel(nn.Linear):
    def __init__(self, in_features: int = 20, out_features: int = 1):
        super().__init__(in_features, out_features)


class FourBlockMLP(nn.Module):
    def __init__(self, dim: int = 512):
        super().__init__()
        self.block0 = nn.Sequential(nn.Linear(dim, dim), nn.ReLU())
        self.block1 = nn.Sequential(nn.Linear(dim, dim), nn.ReLU())
        self.block2 = nn.Sequential(nn.Linear(dim, dim), nn.ReLU())
        self.block3 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.block3(self.block2(self.block1(self.block0(x))))

    def as_sequential(self) -> nn.Sequential:
        return nn.Sequential(self.block0, self.block1, self.block2, self.block3)


class StageModule(nn.Module):
    def __init__(self, in_features: int, out_features: int, is_last: bool = False):
        super().__init__()
        self.linear = nn.Linear(in_features, out_features)
        self.is_last = is_last

    def forward(self, x):
        x = self.linear(x)
        return x if self.is_last else torch.relu(x)


def manual_split_stages(dims=(128, 256, 256, 256, 64)) -> list[StageModule]:
    """The 4-stage chain of the manual PP walkthrough (01_manual_model_split.py:74-79)."""
    n = len(dims) - 1
    return [StageModule(dims[i], dims[i + 1], is_last=(i == n - 1)) for i in range(n)]
