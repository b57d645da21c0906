"""Typed training configuration: dataclass + YAML + CLI (capability parity with utils/config.py:25-122).

``TrainingConfig`` keeps the reference fields (num_epochs, batch_size, learning_rate, weight_decay, momentum,
seed, backend, use_amp, amp_dtype, save_every, checkpoint_dir, profile, profile_dir) and adds what an
MI355X run needs: model preset, mesh dims (dp/tp/pp/cp), sharding strategy, bucket size, sequence length,
micro-batches, kernel selection.  ``from_yaml`` ignores unknown keys (as the reference) and ``from_args``
accepts hyphenated flags with the ``--lr`` alias, returning the unparsed remainder.
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import asdict, dataclass, fields
from typing import Optional

import yaml


@dataclass
class TrainingConfig:
    # reference fields
    num_epochs: int = 10
    batch_size: int = 32
    learning_rate: float = 1e-3
    weight_decay: float = 0.0
    momentum: float = 0.9
    seed: int = 42
    backend: str = "nccl"
    use_amp: bool = False
    amp_dtype: str = "bfloat16"
    save_every: int = 0
    checkpoint_dir: str = "checkpoints"
    profile: bool = False
    profile_dir: str = "profiler_output"
    # MI355X framework fields
    model: str = "toy"
    seq_len: int = 256
    steps: int = 0
    micro_batches: int = 1
    dp: int = -1
    tp: int = 1
    pp: int = 1
    cp: int = 1
    cp_mode: str = "ulysses"
    sharding: str = "SHARD_GRAD_OP"
    bucket_cap_mb: float = 256.0
    optimizer: str = "adamw"
    grad_clip: Optional[float] = None
    kernels: str = "dph"
    pp_schedule: str = "1f1b"
    log_every: int = 10
    metrics_file: Optional[str] = None

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "TrainingConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in (d or {}).items() if k in names})

    @classmethod
    def from_yaml(cls, path: str) -> "TrainingConfig":
        with open(path) as fh:
            return cls.from_dict(yaml.safe_load(fh))

    def to_yaml(self, path: str):
        with open(path, "w") as fh:
            yaml.safe_dump(self.to_dict(), fh, sort_keys=False)

    @classmethod
    def add_arguments(cls, parser: argparse.ArgumentParser):
        for f in fields(cls):
            flag = "--" + f.name.replace("_", "-")
            names = [flag] + (["--lr"] if f.name == "learning_rate" else [])
            default = f.default if f.default is not dataclasses.MISSING else None
            if f.type in ("bool", bool):
                parser.add_argument(*names, dest=f.name, action=argparse.BooleanOptionalAction, default=default)
            else:
                typ = {"int": int, "float": float, "str": str}.get(str(f.type), None)
                if typ is None:
                    typ = float if "float" in str(f.type) else (int if "int" in str(f.type) else str)
                parser.add_argument(*names, dest=f.name, type=typ, default=default)
        parser.add_argument("--config", default=None, help="YAML file; CLI flags override it")
        return parser

    @classmethod
    def from_args(cls, argv=None):
        ap = cls.add_arguments(argparse.ArgumentParser())
        args, rest = ap.parse_known_args(argv)
        base = cls.from_yaml(args.config).to_dict() if args.config else {}
        defaults = cls().to_dict()
        for k, v in vars(args).items():
            if k == "config":
                continue
            if k not in base or v != defaults.get(k):
                base[k] = v
        return cls.from_dict(base), rest
