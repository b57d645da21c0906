"""Loader for the in-tree native extension ``distributed_pytorch_hpc_amd/_C.so``.

Policy (no silent fallbacks on the GPU):
  * GPU tensors always go through the HIP kernels.  If the extension is missing on a machine with a
    GPU, the first op raises ``NativeExtensionMissing`` instead of quietly running eager PyTorch.
  * CPU tensors run the pure-PyTorch reference implementation of the same op (used by the CPU/gloo
    distributed tests and the CPU ResNet-50 DDP config); those references are also the fp32 oracles of
    the kernel numerics tests.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DPH_NATIVE_SO points at another build of the extension (A/B runs of two kernel versions on one box)
SO_PATH = os.environ.get("DPH_NATIVE_SO") or os.path.join(_PKG, "_C.so")

_lock = threading.Lock()
_loaded = False
_error: str | None = None


class NativeExtensionMissing(RuntimeError):
    pass


def load(build_if_missing: bool = False) -> bool:
    """Load ``_C.so`` once; returns True if the dph ops are registered."""
    global _loaded, _error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(SO_PATH) and build_if_missing:
            from ..csrc import build as _build

            _build.build()
        if not os.path.exists(SO_PATH):
            _error = f"{SO_PATH} not found (run `python -m distributed_pytorch_hpc_amd.csrc.build`)"
            return False
        try:
            torch.ops.load_library(SO_PATH)
        except Exception as e:  # pragma: no cover - only on a broken build
            _error = f"failed to load {SO_PATH}: {e}"
            return False
        from . import _meta  # noqa: F401  (fake/meta kernels for the dispatcher ops)

        if os.environ.get("DPH_GEMM1_LDS", "1") == "0":   # deep-K 1x1 GEMMs back on ts_nt_k (A/B, docs/guide/knobs.md)
            torch.ops.dph.gemm1_lds(0)
        if os.environ.get("DPH_C3W_ROUND"):   # weight-gradient split count: workgroup slots per round (A/B)
            torch.ops.dph.c3w_round(int(os.environ["DPH_C3W_ROUND"]))
        _loaded = True
        return True


def available() -> bool:
    return load()


def require() -> None:
    """Raise loudly if the native extension is unavailable (called on every GPU op path)."""
    if not load():
        raise NativeExtensionMissing(
            "distributed_pytorch_hpc_amd native HIP extension is not available: " + str(_error)
        )


def ops():
    require()
    return torch.ops.dph


# DPH_KERNELS=aten selects the stock-op comparator for a whole process (explicit opt-in, like --kernels aten)
_reference_mode = os.environ.get("DPH_KERNELS", "dph").lower() == "aten"


def set_reference_mode(enabled: bool) -> None:
    """Route GPU tensors through the stock PyTorch-ROCm reference ops instead of the HIP kernels.

    Only for A/B benchmarking (bench.py --kernels aten: the "stock PyTorch" comparator of BASELINE.md) and
    debugging; never enabled implicitly.
    """
    global _reference_mode
    _reference_mode = bool(enabled)


def reference_mode() -> bool:
    return _reference_mode


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU (then the HIP kernel MUST be used)."""
    if t.is_cuda and not _reference_mode:
        require()
        return True
    return False
