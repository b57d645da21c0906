"""Linear layer whose weight gradient is written straight into the data-parallel engine's flat gradient
buffer (``weight.main_grad``) by the backward GEMM itself.

Without this, autograd materialises a fresh dW per weight which then has to be copied (or added) into the
bucket the collective reads -- one extra pass over every gradient byte (13.5 GB per step for Llama-2-7B).
Here dW = dY^T X is computed by hipBLASLt with ``out=`` (first micro-batch) or ``addmm_`` (gradient
accumulation, beta = 1) directly into the bucket view, and the engine is notified that the gradient
is ready (``weight._dph_grad_ready()``), which may launch the bucket's reduce-scatter/all-reduce while the
rest of the backward pass is still running.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from ..ops import fp8 as _fp8

# Opt-in (DPH_WGRAD_STREAM=1): weight-gradient GEMMs on a side stream (per device).  dW is off the backward's
# critical path, so the CDNA4 wgrad kernel could overlap the next dgrad / attention-backward / norm kernels and
# fill their tail waves.  The data-parallel engine orders its collectives after this stream and joins it at the
# end of backward (DataParallelEngine._finalize_backward).  Measured on Llama-2-7B (1 MI355X, B=8 x 4096): 26,642
# (lag 1) / 26,463 (lag 2) vs 27,288 tokens/s single-stream -- both kernels are sized for the whole chip and
# contend for CUs / L2 -- so the default is one stream.
_WGRAD_STREAMS: dict = {}
# In-flight side-stream wgrads: (event, operands).  Operands stay referenced (instead of record_stream, which keeps
# the caching allocator from recycling multi-GB blocks and drives it into synchronising cudaFree/retry cycles
# near the 288 GB limit) and the compute stream waits for the oldest once more than _WGRAD_LAG are in flight.
_WGRAD_PENDING: list = []
_WGRAD_LAG = 1


def join_wgrad_stream(device: torch.device):
    """Order the compute stream after every side-stream wgrad and drop the operands kept alive for them."""
    side = wgrad_stream(device)
    if side is not None:
        torch.cuda.current_stream(device).wait_stream(side)
    _WGRAD_PENDING.clear()


def wgrad_stream(device: torch.device):
    """The side stream the engine-managed weight-gradient GEMMs use on ``device`` (None: disabled / not CUDA)."""
    if device.type != "cuda" or os.environ.get("DPH_WGRAD_STREAM", "0") != "1":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _WGRAD_STREAMS.get(idx)
    if s is None:
        s = _WGRAD_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return s


def _native_wgrad(out: torch.Tensor, g2: torch.Tensor, x2: torch.Tensor, accumulate: bool) -> bool:
    """out[N_out, N_in] (+)= g2^T x2 on the CDNA4 weight-gradient kernel (csrc/gemm.hip) when the shapes fit
    its tiling (M, N % 8 -- ragged tensor-parallel shards run as edge tiles -- and tokens % 64); False -> caller uses
    hipBLASLt."""
    if not (g2.is_cuda and g2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16):
        return False
    from ..ops import _lib

    if _lib.reference_mode():
        return False
    T, M = g2.shape
    N = x2.shape[1]
    if M % 8 or N % 8 or M < 8 or N < 8 or T % 64 or T == 0:
        return False
    if g2.stride(1) != 1 or x2.stride(1) != 1 or g2.stride(0) % 8 or x2.stride(0) % 8:
        return False
    if not out.is_contiguous() or out.dtype not in (torch.bfloat16, torch.float32):
        return False
    if g2.data_ptr() % 16 or x2.data_ptr() % 16:
        return False
    _lib.ops().gemm_tn_(out, g2, x2, accumulate)
    return True


def _nt_ok(a: torch.Tensor, w: torch.Tensor) -> bool:
    """a [..., K] @ w[N, K]^T can run on the CDNA4 NT kernel (csrc/gemm_nt.hip) and DPH_GEMM_NT=all asks for it."""
    from . import fused_layers

    if not fused_layers.nt_enabled():
        return False
    if not (a.is_cuda and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    from ..ops import _lib

    if _lib.reference_mode() or not _lib.use_native(a):
        return False
    K = a.shape[-1]
    rows = a.numel() // K if K else 0
    if not fused_layers._nt_ok(rows, w.shape[0], K) or w.shape[1] != K or not w.is_contiguous():
        return False
    return a.is_contiguous() and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0


def _fwd_gemm(x: torch.Tensor, w: torch.Tensor, b=None) -> torch.Tensor:
    """y = x W^T (+ b): the CDNA4 NT kernel when enabled and tileable, else hipBLASLt (F.linear)."""
    if b is None and _nt_ok(x, w):
        from ..ops import _lib

        return _lib.ops().gemm_nt(x, w)
    if x.dim() > 2 and not x.is_contiguous():
        x = x.contiguous()   # F.linear folds a contiguous input into one 2-D GEMM (see _mm2d)
    return F.linear(x, w, b)


def _dgrad(gy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dY W.  hipBLASLt runs this 10-15 % faster with a K-contiguous W^T operand (mm(dY, W^T.t()):
    profiles/gemm_layout_*.json); the HIP transpose makes that copy at HBM speed (~0.04-0.07 ms for 7B weights)
    and it is freed right after the GEMM.  With DPH_GEMM_NT=all the same W^T feeds the CDNA4 NT kernel."""
    if (gy.is_cuda and w.dtype == torch.bfloat16 and gy.dtype == torch.bfloat16 and w.dim() == 2
            and w.is_contiguous() and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 and w.numel() >= (1 << 22)):
        from ..ops import _lib

        if not _lib.reference_mode():
            wt = _lib.ops().transpose2d(w)
            gyc = gy.contiguous()
            if _nt_ok(gyc, wt):
                return _lib.ops().gemm_nt(gyc, wt)
            return _mm2d(gyc, wt.t())
    return _mm2d(gy, w)


def _mm2d(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [..., K] @ b [K, N] as ONE 2-D GEMM over the folded leading dims.  torch.matmul of a non-contiguous 3-D
    ``a`` (e.g. a sequence-parallel all-gather's view) with a 2-D ``b`` becomes a batched GEMM with ``b`` broadcast
    at batch stride 0, which hipBLASLt on this stack rejects (HIPBLAS_STATUS_INTERNAL_ERROR) and whose rocBLAS
    fallback faulted the GPU (illegal address) on the tensor-parallel w2 input gradient."""
    if a.dim() == 2:
        return torch.mm(a, b)
    lead = a.shape[:-1]
    return torch.mm(a.reshape(-1, a.shape[-1]), b).view(*lead, b.shape[-1])


def weight_grad(w: torch.Tensor, g2: torch.Tensor, x2: torch.Tensor):
    """dW = g2^T x2 for weight ``w`` ([N, K] from g2 [T, N], x2 [T, K]).  When the data-parallel engine owns ``w``
    (``w.main_grad``), dW is written / accumulated straight into the flat gradient bucket (CDNA4 wgrad kernel when
    the shape fits, else hipBLASLt), the engine is notified, and None is returned; otherwise dW is returned."""
    mg = getattr(w, "main_grad", None)
    side = wgrad_stream(g2.device) if mg is not None else None
    if side is not None:
        main = torch.cuda.current_stream(g2.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            launched = _native_wgrad(mg, g2, x2, getattr(w, "_dph_accum", False))
        if launched:
            ev = torch.cuda.Event()
            ev.record(side)
            _WGRAD_PENDING.append((ev, g2, x2))
            while len(_WGRAD_PENDING) > _WGRAD_LAG:
                main.wait_event(_WGRAD_PENDING.pop(0)[0])
            w._dph_accum = True
            w._dph_grad_ready()
            return None
    elif mg is not None and _native_wgrad(mg, g2, x2, getattr(w, "_dph_accum", False)):
        w._dph_accum = True
        w._dph_grad_ready()
        return None
    if mg is not None and mg.dtype != x2.dtype:
        gw_ = g2.t().mm(x2)
        if getattr(w, "_dph_accum", False):
            mg.add_(gw_)
        else:
            mg.copy_(gw_)
            w._dph_accum = True
        w._dph_grad_ready()
        return None
    if mg is not None:
        if getattr(w, "_dph_accum", False):
            mg.addmm_(g2.t(), x2)
        else:
            torch.mm(g2.t(), x2, out=mg)
            w._dph_accum = True
        w._dph_grad_ready()
        return None
    gw = torch.empty(w.shape, dtype=w.dtype, device=w.device)
    if not _native_wgrad(gw, g2, x2, False):
        gw = g2.t().mm(x2)
    return gw


def weight_grad_from(w: torch.Tensor, mm):
    """dW for a GEMM given as ``mm(out)`` (writes into ``out`` when given, else returns a new bf16 tensor), routed like
    ``weight_grad``: written straight into the engine's bucket view (first micro-batch, matching dtype) or added to
    it, the engine notified and None returned; without an engine the gradient itself is returned (ops/fp8.py)."""
    mg = getattr(w, "main_grad", None)
    if mg is None:
        return mm(None)
    if not getattr(w, "_dph_accum", False) and mg.dtype == torch.bfloat16 and mg.is_contiguous():
        mm(mg)
    elif getattr(w, "_dph_accum", False):
        mg.add_(mm(None))
    else:
        mg.copy_(mm(None))
    w._dph_accum = True
    w._dph_grad_ready()
    return None


def _autocast_dtype(t: torch.Tensor):
    dev = t.device.type
    return torch.get_autocast_dtype(dev) if torch.is_autocast_enabled(dev) else None


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        # autocast: cast once here and save the low-precision copies, so backward GEMMs see matching dtypes
        # (the low-precision dW is accumulated into the fp32 main_grad below)
        dt = _autocast_dtype(x)
        if dt is not None and x.is_floating_point():
            x, w = x.to(dt), w.to(dt)
            b = b.to(dt) if b is not None else None
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        with torch.autocast(x.device.type, enabled=False):
            return _fwd_gemm(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gw = gb = None
        g2 = gy.reshape(-1, gy.shape[-1])
        if ctx.needs_input_grad[0]:
            gx = _dgrad(gy, w)
        if ctx.needs_input_grad[1]:
            gw = weight_grad(w, g2, x.reshape(-1, x.shape[-1]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = g2.sum(0)
            if getattr(w, "main_grad", None) is not None and gb is not None:
                pass  # bias handled by the generic post-accumulate hook of the engine
        return gx, gw, gb


def linear(x, w, b=None):
    if b is None and _fp8.fp8_enabled() and _fp8.applicable(x, w):
        return _fp8.fp8_linear(x, w)   # opt-in FP8 GEMMs (ops/fp8.py)
    if getattr(w, "main_grad", None) is not None and torch.is_grad_enabled() and w.requires_grad:
        return _LinearFn.apply(x, w, b)
    if x.is_cuda and x.dim() > 2 and not x.is_contiguous():
        x = x.contiguous()   # one folded 2-D GEMM, not a batched GEMM with the weight broadcast (see _mm2d)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """nn.Linear with the main-grad fast path (identical math and parameters)."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)


def convert_linears_(module: nn.Module) -> nn.Module:
    """Swap every plain nn.Linear of ``module`` for ``Linear`` in place (parameters are kept)."""
    for m in module.modules():
        if type(m) is nn.Linear:
            m.__class__ = Linear
    return module
