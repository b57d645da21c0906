"""1x1 and 3x3 convolutions on channels-last activations through the CDNA4 tall-skinny GEMM kernels
(csrc/conv1x1.hip).

In NHWC a stride-1, bias-free 1x1 convolution is ``Y[M, Cout] = X[M, Cin] W[Cout, Cin]^T`` with M = N*H*W, and
its two gradients are ``dX = dY W`` and ``dW = dY^T X`` -- no im2col, no layout change: the channels-last tensor
IS the row-major [M, C] matrix.  ResNet-50's bottleneck convolutions conv1 / conv3 are of this kind (about 2/3
of its convolution time, benchmarks/conv_bench.py).  Strided 1x1 / 3x3 convolutions run on the gathered implicit GEMM
(``StridedConv2d``, below), the 7x7 stride-2 stem on the same gathered kernel (``StemConv2d``).

One switch covers every convolution here: ``DPH_CONV=miopen`` sends all of them (forward and both gradients) to
ATen / MIOpen -- the comparator of the A/B runs quoted below; the default ``dph`` takes the HIP kernels wherever the
shape qualifies.

``Conv1x1`` is a drop-in ``nn.Conv2d`` (same parameter, same state dict) that takes the kernel path for bf16
(or bf16-autocast) channels-last inputs on the GPU with channel counts that are multiples of 64, and falls back
to ``F.conv2d`` otherwise.

``Conv3x3`` does the same for stride-1 / padding-1 3x3 convolutions as implicit GEMMs (K = 9 * Cin, tap-major):
forward and input gradient on the LDS-DMA kernel of csrc/conv3x3.hip (the input gradient is a 3x3 convolution of dY
with the spatially flipped, channel-transposed weight; padding taps are zero-filled by range-checked buffer DMA; an
epilogue emits the following BatchNorm's statistics or adds a bias): 440-810 TFLOP/s vs MIOpen's 370-780 on the
ResNet-50 / SimpleUNet shapes (profiles/r3/conv3_bench_oob.json).  The
weight gradients run on the LDS-DMA split-pixel kernel (``c3w_k``) by default: 1.20-1.42x MIOpen per shape since round
4 removed its per-piece address divisions and its second, nearly empty round of split-K workgroups (round 3 measured it
at 241-357 TFLOP/s vs MIOpen's 318-491 and kept MIOpen for ResNet, profiles/r3/conv3_bench_c3w_wgrad.json).
Rejected variants (removed from the tree in round 5; their A/B evidence stays under profiles/): round 2's
register-staged 3x3 forward (0.51-0.63 ms vs MIOpen's 0.38-0.53 ms per shape), the 8-wave 3x3 tile, the sub-image copy
for strided 1x1 weight gradients, and ATen copies for the input-gradient weight transposes.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib

# weight gradients go straight into the data-parallel engine's bucket (main_grad) when it exposes one
_DIRECT = True


def _miopen() -> bool:
    """DPH_CONV=miopen: every convolution on ATen / MIOpen (A/B comparator); default dph = the HIP kernels."""
    return os.environ.get("DPH_CONV", "dph").lower() == "miopen"


def _autocast_bf16(t: torch.Tensor) -> bool:
    return t.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


def _nhwc2d(t: torch.Tensor) -> torch.Tensor:
    """[B, C, H, W] (any layout) -> row-major [B*H*W, C] (a view when t is channels-last contiguous)."""
    return t.permute(0, 2, 3, 1).contiguous().view(-1, t.shape[1])


def weight_t(w2: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin] -> [Cin, Cout] for an input-gradient GEMM: the HIP tile transpose (csrc/transpose.hip) instead of
    ATen's element-wise strided copy."""
    if w2.is_cuda and w2.dtype == torch.bfloat16 and w2.stride(1) == 1 and w2.stride(0) % 8 == 0 and \
            w2.shape[0] % 8 == 0 and w2.data_ptr() % 16 == 0:
        return _lib.ops().transpose2d(w2)
    return w2.t().contiguous()


def _main_grad_target(w: torch.Tensor, shape):
    """The engine-owned gradient buffer of parameter ``w`` viewed as ``shape`` (parallel/data_parallel.py keeps
    ``main_grad`` views into its flat bucket), or None when the weight gradient has to be returned to autograd."""
    mg = getattr(w, "main_grad", None)
    if mg is None or not _DIRECT or not mg.is_contiguous() or mg.data_ptr() % 16:
        return None
    return mg.view(shape)


def bias_grad(param, dy2: torch.Tensor, dtype):
    """Per-channel sum of dy (a convolution's bias gradient), written straight into the engine-owned gradient bucket
    view of ``param`` when there is one (engine notified, None returned), else returned in ``dtype``."""
    mg = getattr(param, "main_grad", None) if param is not None else None
    if (mg is not None and _DIRECT and not getattr(param, "_dph_accum", False) and mg.is_contiguous()
            and mg.dtype in (torch.float32, torch.bfloat16)):
        _lib.ops().channel_sum_into_(dy2, mg.view(-1))
        param._dph_zeroed = False
        param._dph_accum = True
        param._dph_grad_ready()
        return None
    return _lib.ops().channel_sum(dy2, dtype)   # in the bias's own dtype: no cast kernel


def zero_bias_grad(param, n: int, dtype, device):
    """The gradient of a bias that a following training-mode BatchNorm cancels: exactly zero, so no channel sum runs
    (SimpleUNet's 14 conv biases: 28 reduction launches per step).  Written into the engine's bucket view when
    there is one (engine notified, None returned): one fill -- or none when the view lives in a persistent bucket
    (``_dph_persistent_grad``: parallel/data_parallel.py) that an earlier step zeroed and no writer has touched since
    (``_dph_zeroed``, cleared by every other write of the parameter's gradient), so it still holds the zeros."""
    mg = getattr(param, "main_grad", None) if param is not None else None
    if mg is not None and _DIRECT:
        if not getattr(param, "_dph_accum", False):
            if not (getattr(param, "_dph_persistent_grad", False) and getattr(param, "_dph_zeroed", False)):
                mg.zero_()
                param._dph_zeroed = bool(getattr(param, "_dph_persistent_grad", False))
            param._dph_accum = True
        param._dph_grad_ready()
        return None
    return torch.zeros(n, dtype=dtype, device=device)


def _wgrad_into_main(w: torch.Tensor, shape, launch) -> bool:
    """Run ``launch(out, accumulate)`` straight into the engine's gradient bucket and notify the engine (no
    autograd gradient, no post-accumulate copy).  False when ``w`` has no engine-owned buffer."""
    mg = _main_grad_target(w, shape)
    if mg is None:
        return False
    launch(mg, bool(getattr(w, "_dph_accum", False)))
    w._dph_accum = True
    w._dph_grad_ready()
    return True


class GradSlot:
    """Hand-off of a residual branch's input gradient into a 1x1 convolution's input-gradient epilogue.

    In an identity ResNet bottleneck the block input x feeds conv1 and the residual add of bn3; autograd would sum
    the two gradients of x with a separate add kernel (2 reads + 1 write of x's size).  With a slot, conv1 (on the
    kernel path) marks itself the ``consumer``, bn3 takes the residual detached, ``arms`` the slot and leaves its
    residual gradient in ``t`` -- bn3's backward runs before conv1's -- and conv1's dgrad kernel adds it in its
    epilogue (``ts_gemm_nt(..., add=)``), so x receives one gradient."""

    __slots__ = ("consumer", "armed", "t", "sub", "mask")

    def __init__(self):
        self.sub = None      # (s, H, W): t is the gradient of the stride-s sub-image of an H x W input
        self.consumer = False
        self.armed = False
        self.t = None
        # ReLU bits of the BatchNorm that left t: the residual gradient is t under this mask -- bn3 hands over its dy
        # and its forward's bits instead of writing the masked copy (DPH_RES_MASK=0 restores the copy)
        self.mask = None


class _GradTapFn(torch.autograd.Function):
    """Identity whose backward parks the incoming gradient in ``slot.t`` (instead of returning it to autograd), for
    the 1x1 convolution that consumes the same tensor to add in its input-gradient epilogue."""

    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ctx.slot.t = g
        return None, None


def grad_tap(x: torch.Tensor, slot: GradSlot) -> torch.Tensor:
    """Route the gradient that flows back into ``x`` through this branch into ``slot`` (armed here); the slot's
    consumer -- a Conv1x1 whose forward ran on ``x`` BEFORE this call, so that autograd runs this branch's backward
    first -- adds it in its dgrad epilogue.  Used for a ResNet downsample branch: x's two gradients (main branch and
    downsample convolution) are then summed inside conv1's kernel instead of by a separate add over x."""
    slot.armed = True
    return _GradTapFn.apply(x, slot)


class StatsSlot:
    """BatchNorm statistics of a 1x1 convolution's output, computed in the convolution's epilogue
    (``ts_gemm_nt_stats``: per-128-row-block [mean | M2 | rows] partials) and consumed by the BatchNorm that
    follows, which then skips its own statistics pass over the activation.  Passing a slot declares that consumer: a
    training-mode BatchNorm applied directly to this output, so a convolution bias cancels in it and gets an exactly
    zero gradient (``zero_bias_grad``)."""

    __slots__ = ("stats", "rows", "cols")

    def __init__(self):
        self.stats = None
        self.rows = self.cols = 0

    def take(self, rows: int, cols: int):
        st, self.stats = self.stats, None
        return st if st is not None and (self.rows, self.cols) == (rows, cols) else None


class BnGradSlot:
    """The backward reduction of a training-mode BatchNorm + ReLU, run in the epilogue of the convolution that consumes
    the BatchNorm's output (``ts_gemm_nt_bnred``; csrc/bn_epilogue.h).

    The BatchNorm backward needs, per channel, sum(dz) and sum(dz * xhat) over its output gradient (dz = dy * ReLU
    mask) before it can write dx -- a pass that re-reads dy, x and the mask.  dy is written by the consumer
    convolution's input-gradient kernel, so that kernel reads x and the mask at the rows it stores and emits the
    per-128-row partials instead (one read of dy fewer, one launch fewer).  The BatchNorm's forward ``fill``s the slot
    (its saved x, mean, invstd and mask source), the consumer's backward leaves ``part`` and the identity of the
    gradient it returned, and the BatchNorm's backward ``take``s the partials -- only if the gradient it received is
    that very tensor, unmodified (``dy_key``): a gradient summed with another consumer's falls back to the reduction
    pass.  ``sole``: the convolution is the output's only consumer; otherwise (a ResNet block input, also the
    residual) it uses the slot only when its GradSlot routes the other gradient into the same epilogue."""

    __slots__ = ("x", "mean", "invstd", "ss", "bits", "part", "dy_key", "sole")

    def __init__(self, sole: bool = True):
        self.sole = sole
        self.x = self.mean = self.invstd = self.ss = self.bits = self.part = self.dy_key = None

    def fill(self, x, mean, invstd, ss=None, bits=None):
        self.x, self.mean, self.invstd, self.ss, self.bits = x, mean, invstd, ss, bits

    def usable(self, rows: int, cols: int, armed: bool = False) -> bool:
        # DPH_BN_EPILOGUE=0: the BatchNorm runs its own reduction pass (A/B comparisons)
        return (self.x is not None and (self.sole or armed) and self.x.dtype == torch.bfloat16
                and os.environ.get("DPH_BN_EPILOGUE", "1") != "0"
                and self.x.numel() == rows * cols and self.x.shape[1] == cols)

    def launch(self, A, B, H=0, W=0, add=None, sub=0):
        """dX = A B^T (+ add) with the reduction epilogue; keeps the partials, returns dX [rows, cols]."""
        dx2, self.part = _lib.ops().ts_gemm_nt_bnred(A, B, H, W, add, sub, self.x, self.mean, self.invstd, self.ss,
                                                     self.bits)
        return dx2

    def mark(self, dx: torch.Tensor):
        self.dy_key = (dx.data_ptr(), dx._version, tuple(dx.shape), tuple(dx.stride()))

    def take(self, dy: torch.Tensor):
        part, key = self.part, self.dy_key
        self.x = self.mean = self.invstd = self.ss = self.bits = self.part = self.dy_key = None
        if part is None or key != (dy.data_ptr(), dy._version, tuple(dy.shape), tuple(dy.stride())):
            return None
        return part


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, slot=None, stats_slot=None, bn_slot=None):
        wdtype = w.dtype
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        wb = w.to(torch.bfloat16) if w.dtype != torch.bfloat16 else w
        B, C, H, W = x.shape
        x2 = _nhwc2d(x)
        w2 = wb.view(wb.shape[0], C)
        if stats_slot is not None:
            y2, stats_slot.stats = _lib.ops().ts_gemm_nt_stats(x2, w2)   # [M, Cout] + BN partials
            stats_slot.rows, stats_slot.cols = y2.shape
        else:
            y2 = _lib.ops().ts_gemm_nt(x2, w2)                      # [M, Cout]
        ctx.save_for_backward(x2, w2)
        ctx.shape, ctx.wdtype, ctx.param, ctx.slot, ctx.bn_slot = (B, C, H, W), wdtype, w, slot, bn_slot
        return y2.view(B, H, W, -1).permute(0, 3, 1, 2)             # channels-last [B, Cout, H, W]

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        B, C, H, W = ctx.shape
        dy2 = _nhwc2d(dy.to(torch.bfloat16))                        # [M, Cout]
        dx = gw = None
        slot = ctx.slot
        if ctx.needs_input_grad[0]:
            add = amask = None
            if slot is not None and slot.armed:
                if slot.t is None:
                    raise RuntimeError("Conv1x1: residual gradient slot armed but empty (backward order)")
                add, amask = slot.t, slot.mask
                slot.t = slot.mask = None
            bn = ctx.bn_slot   # x is a BatchNorm + ReLU output: that BatchNorm's reduction in this epilogue
            bn = bn if bn is not None and bn.usable(B * H * W, C, slot is not None and slot.armed) else None
            if amask is not None:   # the residual gradient is add under the ReLU bits amask (identity block)
                add = _nhwc2d(add.to(torch.bfloat16))
                if bn is not None:
                    dx2, bn.part = _lib.ops().ts_gemm_nt_bnred(dy2, weight_t(w2), 0, 0, add, 0, bn.x, bn.mean,
                                                               bn.invstd, bn.ss, bn.bits, amask)
                else:
                    dx2 = _lib.ops().ts_gemm_nt_addmask(dy2, weight_t(w2), add, amask)
            elif add is not None and slot.sub is not None:   # a strided 1x1 downsample's sub-image gradient
                s_, h_, w_ = slot.sub
                if bn is not None:
                    dx2 = bn.launch(dy2, weight_t(w2), h_, w_, add.to(torch.bfloat16), s_)
                else:
                    dx2 = _lib.ops().ts_gemm_nt_add_sub(dy2, weight_t(w2), add.to(torch.bfloat16), h_, w_, s_)
            else:
                if add is not None:
                    add = _nhwc2d(add.to(torch.bfloat16))
                if bn is not None:
                    dx2 = bn.launch(dy2, weight_t(w2), 0, 0, add)
                else:
                    dx2 = _lib.ops().ts_gemm_nt(dy2, weight_t(w2), 0, 0, add)    # [M, Cin] (+ residual grad)
            dx = dx2.view(B, H, W, C).permute(0, 3, 1, 2)
            if bn is not None:
                bn.mark(dx)
        if ctx.needs_input_grad[1]:
            cout = w2.shape[0]
            if not _wgrad_into_main(ctx.param, (cout, C), lambda out, acc: _lib.ops().ts_gemm_tn_(out, dy2, x2, acc)):
                gw = torch.empty((cout, C), dtype=ctx.wdtype, device=dy.device)
                _lib.ops().ts_gemm_tn_(gw, dy2, x2, False)
                gw = gw.view(cout, C, 1, 1)
        return dx, gw, None, None, None


# 3x3 weight gradients on the c3w_k kernel (wgrad="dph") since its DMA addresses advance incrementally and its split-K
# fills exactly one resident round: 1.20-1.42x MIOpen on the ResNet-50 / SimpleUNet shapes (profiles/r4/c3w_rounds/
# c3.log).  Before that, Conv3x3 (ResNet bottlenecks) kept MIOpen (10 068 / 10 079 img/s vs 9 835 / 9 833 with the
# kernel) while BiasConv2d (SimpleUNet) already took the kernel (1 005 / 984 vs 848 / 826 samples/s,
# profiles/r4/conv_wgrad/).  wgrad="miopen" keeps MIOpen's (comparisons).
# stride-1 3x3 convolutions on csrc/conv3x3.hip: ResNet-50 FSDP bf16 B=256 9 472 / 9 513 vs 9 258 / 9 278 img/s on
# MIOpen (interleaved A/B on one MI355X, profiles/r3/ab_conv3x3/)


def _main_grad_cl(w: torch.Tensor, cout: int, k: int):
    """The engine-owned gradient of a channels-last 4-D weight viewed as [Cout, (kh, kw, Cin)] (its memory order),
    or None."""
    mg = getattr(w, "main_grad", None)
    if (mg is None or not _DIRECT or mg.dim() != 4 or not mg.is_contiguous(memory_format=torch.channels_last)
            or mg.data_ptr() % 16):
        return None
    return mg.permute(0, 2, 3, 1).view(cout, k)


def _conv3_lds_ok(M: int, N: int, K: int, lda: int, ldb: int) -> bool:
    """csrc/conv3x3.hip conv3_supported: the 3x3 shapes the LDS-DMA kernel (and its BatchNorm epilogue) takes."""
    return M > 0 and N % 64 == 0 and K % (9 * 64) == 0 and M * lda * 2 < 2 ** 31 and N * ldb * 2 < 2 ** 31


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stats_slot=None, bias=None, wgrad="dph", bn_slot=None):
        wdtype = w.dtype
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        wb = w.to(torch.bfloat16)
        B, C, H, W = x.shape
        cout = wb.shape[0]
        x2 = _nhwc2d(x)
        wk = wb.permute(0, 2, 3, 1).reshape(cout, 9 * C)             # [Cout, (kh, kw, Cin)]
        if stats_slot is not None:   # + BN partials of the output (of the biased output when there is a bias)
            y2, stats_slot.stats = _lib.ops().ts_gemm_nt_stats(x2, wk, H, W, None, bias)
            stats_slot.rows, stats_slot.cols = y2.shape
        elif bias is not None:   # fp32 bias in the epilogue (SimpleUNet's biased 3x3 convolutions)
            y2 = _lib.ops().ts_gemm_nt(x2, wk, H, W, None, bias)
        else:
            y2 = _lib.ops().ts_gemm_nt(x2, wk, H, W)
        ctx.has_bias = bias is not None
        # a stats slot means a training-mode BatchNorm normalises this output with its own batch statistics: a
        # per-channel constant (the bias) cancels in BN(y + b) = BN(y), so the bias gradient is exactly zero
        ctx.bias_cancels = bias is not None and stats_slot is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.bias_param = bias if isinstance(bias, nn.Parameter) else None
        ctx.wgrad = wgrad
        ctx.bn_slot = bn_slot
        ctx.save_for_backward(x2, wb)
        ctx.shape, ctx.wdtype, ctx.param = (B, C, H, W), wdtype, w
        return y2.view(B, H, W, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, wb = ctx.saved_tensors
        B, C, H, W = ctx.shape
        cout = wb.shape[0]
        dy2 = _nhwc2d(dy.to(torch.bfloat16))
        dx = gw = None
        if ctx.needs_input_grad[0]:
            # dX = conv3x3(dY, W') with W'[ci, (kh, kw), co] = W[co, ci, 2 - kh, 2 - kw]
            if wb.is_contiguous(memory_format=torch.channels_last) and cout % 8 == 0 and C % 8 == 0:
                wf = _lib.ops().conv3x3_dgrad_weight(wb)                  # one launch, HBM-speed tiles
            else:
                wf = wb.flip(2, 3).permute(1, 2, 3, 0).reshape(C, 9 * cout)
            bn = ctx.bn_slot   # x is a BatchNorm + ReLU output: that BatchNorm's reduction in this epilogue
            if (bn is not None and bn.usable(B * H * W, C) and wf.is_contiguous()
                    and _conv3_lds_ok(B * H * W, C, 9 * cout, dy2.stride(0), wf.stride(0))):
                dx = bn.launch(dy2, wf, H, W).view(B, H, W, C).permute(0, 3, 1, 2)
                bn.mark(dx)
            else:
                dx = _lib.ops().ts_gemm_nt(dy2, wf, H, W).view(B, H, W, C).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and ctx.wgrad != "dph":
            # weight gradient on MIOpen: 1.0-1.5x the split-pixel kernel on the ResNet-50 shapes
            # (profiles/r3/conv3_bench_oob.json: 318-485 vs 302-321 TFLOP/s, before round 4's c3w_k rework)
            x4 = x2.view(B, H, W, C).permute(0, 3, 1, 2)
            dy4 = dy2.view(B, H, W, cout).permute(0, 3, 1, 2)
            gw = torch.ops.aten.convolution_backward(dy4, x4, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1].to(ctx.wdtype)
        elif ctx.needs_input_grad[1]:
            w = ctx.param
            mg = _main_grad_cl(w, cout, 9 * C)
            if mg is not None:   # straight into the engine's bucket (channels-last weight = [Cout, (kh, kw, Cin)])
                _lib.ops().ts_gemm_tn_(mg, dy2, x2, bool(getattr(w, "_dph_accum", False)), H, W)
                w._dph_accum = True
                w._dph_grad_ready()
            else:
                gk = torch.empty((cout, 9 * C), dtype=ctx.wdtype, device=dy.device)
                _lib.ops().ts_gemm_tn_(gk, dy2, x2, False, H, W)
                gw = gk.view(cout, 3, 3, C).permute(0, 3, 1, 2).contiguous()
        db = None
        if ctx.has_bias and ctx.needs_input_grad[3]:
            db = (zero_bias_grad(ctx.bias_param, cout, ctx.bias_dtype, dy.device) if ctx.bias_cancels
                  else bias_grad(ctx.bias_param, dy2, ctx.bias_dtype))
        return dx, gw, None, db, None, None


def conv3x3_native_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    if _miopen() or not x.is_cuda or _lib.reference_mode():
        return False
    if not (x.dtype == torch.bfloat16 or _autocast_bf16(x)):
        return False
    cout, cin = w.shape[0], w.shape[1]
    return (x.dim() == 4 and cin % 64 == 0 and cout % 64 == 0 and
            x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


class Conv3x3(nn.Conv2d):
    """Stride-1, padding-1, bias-free 3x3 ``nn.Conv2d`` with the channels-last implicit-GEMM kernel path."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__(in_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False)

    def forward(self, x, stats_slot: StatsSlot | None = None, bn_slot: BnGradSlot | None = None):
        """``bn_slot``: x is the output of a training-mode BatchNorm + ReLU consumed only here; the BatchNorm's backward
        reduction then runs in this convolution's input-gradient epilogue (BnGradSlot)."""
        if conv3x3_native_ok(x, self.weight):
            _lib.require()
            return _Conv3x3Fn.apply(x, self.weight, stats_slot, None, "dph", bn_slot)
        return F.conv2d(x, self.weight, padding=1)


# ------------------------------------------------------------------------------------------------ strided convolutions
def conv_geo(Hs, Ws, Ho, Wo, sy, sx, by, bx, Hd, Wd, ty, tx, tby, tbx, taps) -> list[int]:
    """The 33-integer geometry of the gathered implicit GEMM (csrc/kernels.h ConvGeo): rows (n, oy, ox) over Ho x Wo
    read source pixel (sy oy + by + dy, sx ox + bx + dx) of an Hs x Ws image for tap (dy, dx), and are stored to
    destination pixel (ty oy + tby, tx ox + tbx) of an Hd x Wd image."""
    dy = [t[0] for t in taps] + [0] * (9 - len(taps))
    dx = [t[1] for t in taps] + [0] * (9 - len(taps))
    return [Hs, Ws, Ho, Wo, sy, sx, by, bx, Hd, Wd, ty, tx, tby, tbx, len(taps)] + dy + dx


def strided_out_hw(H, W, k, s, p):
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def strided_fwd_geo(H, W, k, s, p) -> list[int]:
    Ho, Wo = strided_out_hw(H, W, k, s, p)
    taps = [(ky - p, kx - p) for ky in range(k) for kx in range(k)]
    return conv_geo(H, W, Ho, Wo, s, s, 0, 0, Ho, Wo, 1, 1, 0, 0, taps)


def strided_dgrad_classes(H, W, k, s, p):
    """The input gradient of a stride-s convolution as s^2 parity classes: input pixel (s a + py, s b + px) receives
    dY(a + dy, b + dx) W[ky, kx] for every tap with ky = py + p - s dy (0 <= ky < k).  Yields
    (geometry, [(ky, kx)...]) per class with at least one tap; classes without taps receive zero."""
    Ho, Wo = strided_out_hw(H, W, k, s, p)
    for py in range(s):
        for px in range(s):
            Hc, Wc = len(range(py, H, s)), len(range(px, W, s))
            if Hc == 0 or Wc == 0:
                continue
            ys = [((py + p - ky) // s, ky) for ky in range(k) if (py + p - ky) % s == 0]
            xs = [((px + p - kx) // s, kx) for kx in range(k) if (px + p - kx) % s == 0]
            taps = [(dy, dx) for dy, _ in ys for dx, _ in xs]
            if not taps:
                continue
            yield (conv_geo(Ho, Wo, Hc, Wc, 1, 1, 0, 0, H, W, s, s, py, px, taps),
                   [(ky, kx) for _, ky in ys for _, kx in xs])


def strided_dgrad_covers_all(H, W, k, s, p) -> bool:
    """True when every input pixel belongs to a parity class with taps (no zero-fill needed)."""
    return sum(g[2] * g[3] for g, _ in strided_dgrad_classes(H, W, k, s, p)) == H * W


def convg_reference(A: torch.Tensor, B: torch.Tensor, geo: list, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 PyTorch model of ``convg_nt`` (the gathered implicit GEMM) for tests: A [imgs * Hs * Ws, Cin],
    B [N, ntaps * Cin] -> rows per the destination map."""
    Hs, Ws, Ho, Wo, sy, sx, by, bx, Hd, Wd, ty, tx, tby, tbx, nt = geo[:15]
    tdy, tdx = geo[15:15 + nt], geo[24:24 + nt]
    imgs, cin = A.shape[0] // (Hs * Ws), A.shape[1]
    img = A.float().view(imgs, Hs, Ws, cin)
    oy = torch.arange(Ho, device=A.device)
    ox = torch.arange(Wo, device=A.device)
    acc = torch.zeros(imgs, Ho, Wo, B.shape[0], device=A.device)
    for t in range(nt):
        yy, xx = sy * oy + by + tdy[t], sx * ox + bx + tdx[t]
        vy, vx = (yy >= 0) & (yy < Hs), (xx >= 0) & (xx < Ws)
        g = img[:, yy.clamp(0, Hs - 1)][:, :, xx.clamp(0, Ws - 1)]
        g = g * (vy[None, :, None, None] & vx[None, None, :, None])
        acc += g @ B.float()[:, t * cin:(t + 1) * cin].t()
    if out is None:
        out = torch.zeros(imgs * Hd * Wd, B.shape[0], device=A.device)
    dst = out.view(imgs, Hd, Wd, -1)
    dst[:, ty * oy[:, None] + tby, tx * ox[None, :] + tbx] = acc.to(out.dtype)
    return out


# Strided weight gradients on c3w_k since its DMA addresses advance incrementally: 0.90-1.46x MIOpen per shape
# (profiles/r4/c3w_incr/str_ns2.log) and, with the 1x1 identity-row kernel, ResNet-50 10 042 / 10 056 vs 9 912 / 9 927
# img/s (profiles/r4/resnet_wgrad_ab/).


class _StridedConvFn(torch.autograd.Function):
    """Strided, bias-free k x k convolution (ResNet's stride-2 3x3 conv2 and 1x1 downsample) on the gathered implicit
    GEMM: forward = per-lane strided source pixels (csrc/conv3x3.hip conv3_k GEN), input gradient = one GEMM per
    parity class of input pixels with only the taps that reach it, scattered to its pixels, weight gradient = the
    LDS-DMA 3x3 weight-gradient kernel with strided gathered rows (c3w_k GEN; 1x1: the dense 1x1 kernel over the
    strided sub-image)."""

    @staticmethod
    def forward(ctx, x, w, k, s, p, stats_slot=None, grad_slot=None):
        wdtype = w.dtype
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        wb = w.to(torch.bfloat16)
        B, C, H, W = x.shape
        cout = wb.shape[0]
        Ho, Wo = strided_out_hw(H, W, k, s, p)
        x2 = _nhwc2d(x)
        wk = wb.permute(0, 2, 3, 1).reshape(cout, k * k * C)          # [Cout, (kh, kw, Cin)]
        geo = strided_fwd_geo(H, W, k, s, p)
        if stats_slot is not None:
            y2, stats_slot.stats = _lib.ops().convg_nt(x2, wk, geo, True)
            stats_slot.rows, stats_slot.cols = y2.shape
        else:
            y2 = _lib.ops().convg_nt(x2, wk, geo, False)[0]
        ctx.save_for_backward(x2, wb)
        ctx.cfg = (B, C, H, W, k, s, p, Ho, Wo)
        ctx.wdtype, ctx.param, ctx.grad_slot = wdtype, w, grad_slot
        return y2.view(B, Ho, Wo, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, wb = ctx.saved_tensors
        B, C, H, W, k, s, p, Ho, Wo = ctx.cfg
        cout = wb.shape[0]
        dy2 = _nhwc2d(dy.to(torch.bfloat16))
        dx = gw = None
        slot = ctx.grad_slot
        if slot is not None and slot.armed:
            # 1x1 / stride 2 feeding a GradSlot: the sub-image gradient (one dense GEMM over the strided pixels) goes to
            # the block's conv1, whose dgrad epilogue adds it at the even pixels -- no zero-filled full-size tensor
            slot.t = _lib.ops().ts_gemm_nt(dy2, weight_t(wb.view(cout, C)))
            slot.sub = (s, H, W)
        elif ctx.needs_input_grad[0]:
            full = strided_dgrad_covers_all(H, W, k, s, p)
            dx2 = (torch.empty if full else torch.zeros)((B * H * W, C), dtype=torch.bfloat16, device=dy.device)
            wp = wb.permute(1, 2, 3, 0)                                   # [Cin, kh, kw, Cout]
            for geo, kt in strided_dgrad_classes(H, W, k, s, p):
                bk = torch.stack([wp[:, ky, kx, :] for ky, kx in kt], 1).reshape(C, len(kt) * cout)
                _lib.ops().convg_nt_out_(dy2, bk, geo, dx2)
            dx = dx2.view(B, H, W, C).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            w = ctx.param
            mg = _main_grad_cl(w, cout, k * k * C)
            tgt = mg if mg is not None else torch.empty((cout, k * k * C), dtype=ctx.wdtype, device=dy.device)
            acc = bool(getattr(w, "_dph_accum", False)) if mg is not None else False
            # 1x1 included: the weight-gradient kernel gathers the strided rows itself (no sub-image copy)
            _lib.ops().convg_tn_(tgt, dy2, x2, strided_fwd_geo(H, W, k, s, p), acc)
            if mg is not None:
                w._dph_accum = True
                w._dph_grad_ready()
            else:
                gw = tgt.view(cout, k, k, C).permute(0, 3, 1, 2).contiguous()
        return dx, gw, None, None, None, None, None


def strided_native_ok(x: torch.Tensor, m: nn.Conv2d) -> bool:
    if _miopen() or not x.is_cuda or _lib.reference_mode():
        return False
    if not (x.dtype == torch.bfloat16 or _autocast_bf16(x)):
        return False
    k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
    cout, cin = m.weight.shape[0], m.weight.shape[1]
    return (x.dim() == 4 and m.kernel_size == (k, k) and m.stride == (s, s) and m.padding == (p, p)
            and m.dilation == (1, 1) and m.groups == 1 and m.bias is None and k in (1, 3) and s > 1
            and cin % 64 == 0 and cout % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and x.data_ptr() % 16 == 0)


class StridedConv2d(nn.Conv2d):
    """Bias-free strided 1x1 / 3x3 ``nn.Conv2d`` (same parameters and state dict) on the framework's gathered
    implicit-GEMM kernels for channels-last bf16 inputs with 64-multiple channels; MIOpen otherwise
    (``DPH_CONV=miopen`` forces MIOpen).  ResNet-50 FSDP bf16 B=256: 10 066 / 10 106 vs 10 037 / 10 020 img/s
    (profiles/r4/strided_conv/final/)."""

    def forward(self, x, stats_slot: StatsSlot | None = None, grad_slot: GradSlot | None = None):
        """``grad_slot`` (1x1 / stride 2 only, armed by the caller): the input gradient is handed to the slot's
        consumer as the stride-2 sub-image gradient instead of being returned (ResNet downsample, models/resnet.py)."""
        if strided_native_ok(x, self):
            _lib.require()
            gs = grad_slot if (grad_slot is not None and self.kernel_size[0] == 1 and self.stride[0] == 2) else None
            return _StridedConvFn.apply(x, self.weight, self.kernel_size[0], self.stride[0], self.padding[0],
                                        stats_slot, gs)
        if grad_slot is not None:
            raise RuntimeError("StridedConv2d: grad_slot needs the kernel path (check strided_native_ok first)")
        return F.conv2d(x, self.weight, None, self.stride, self.padding)


def conv1x1_native_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    if _miopen() or not x.is_cuda or _lib.reference_mode():
        return False
    if not (x.dtype == torch.bfloat16 or _autocast_bf16(x)):
        return False
    cout, cin = w.shape[0], w.shape[1]
    return (x.dim() == 4 and cin % 64 == 0 and cout % 64 == 0 and
            x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


class Conv1x1(nn.Conv2d):
    """Stride-1, bias-free 1x1 ``nn.Conv2d`` with the channels-last GEMM kernel path (see module docstring)."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__(in_channels, out_channels, kernel_size=1, stride=1, padding=0, bias=False)

    def forward(self, x, grad_slot: GradSlot | None = None, stats_slot: StatsSlot | None = None,
                bn_slot: BnGradSlot | None = None):
        """``bn_slot``: x is a training-mode BatchNorm + ReLU output whose backward reduction may run in this
        convolution's input-gradient epilogue (BnGradSlot: always when the slot is ``sole``, else only when
        ``grad_slot`` carries x's other gradient into the same epilogue)."""
        if conv1x1_native_ok(x, self.weight):
            _lib.require()
            if grad_slot is not None:
                grad_slot.consumer = True
            return _Conv1x1Fn.apply(x, self.weight, grad_slot, stats_slot, bn_slot)
        return F.conv2d(x, self.weight)


# ------------------------------------------------------------------------------------------------ bias convolutions
class _ConvBiasFn(torch.autograd.Function):
    """MIOpen convolution (forward, input and weight gradients through aten.convolution[_backward]) whose bias
    gradient is the deterministic channels-last per-channel sum of csrc/chsum.hip instead of ATen's outer-dimension
    reduction (1.9 ms for the 65-channel output convolution of SimpleUNet at B=4, 181x360)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, dilation, transposed, output_padding, groups):
        y = torch.ops.aten.convolution(x, w, b, stride, padding, dilation, transposed, output_padding, groups)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, padding, dilation, transposed, output_padding, groups)
        ctx.bdtype = b.dtype
        ctx.bias_param = b if isinstance(b, nn.Parameter) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, padding, dilation, transposed, output_padding, groups = ctx.cfg
        dy = dy.contiguous(memory_format=torch.channels_last)
        nx, nw, nb = ctx.needs_input_grad[:3]
        dx = dw = db = None
        if nx or nw:
            dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, stride, padding, dilation, transposed,
                                                            output_padding, groups, [nx, nw, False])
        if nb:
            db = bias_grad(ctx.bias_param, dy, ctx.bdtype)
        return dx, dw, db, None, None, None, None, None, None


def _bias_conv_ok(m: nn.Module, x: torch.Tensor) -> bool:
    return (m.bias is not None and x.is_cuda and x.dim() == 4 and m.padding_mode == "zeros"
            and not isinstance(m.padding, str) and x.dtype in (torch.bfloat16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last) and _lib.use_native(x))


def _bias_conv(m: nn.Module, x: torch.Tensor, transposed: bool, output_padding) -> torch.Tensor:
    w, b = m.weight, m.bias
    args = (list(m.stride), list(m.padding), list(m.dilation), transposed, list(output_padding), m.groups)
    if torch.is_autocast_enabled("cuda"):   # same casts as autocast's conv2d: inputs, weight and bias to its dtype
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _ConvBiasFn.apply(x.to(dt), w.to(dt), b.to(dt), *args)
    return _ConvBiasFn.apply(x, w, b, *args)


def _bias_conv3x3_ok(m: nn.Module, x: torch.Tensor) -> bool:
    return (tuple(m.kernel_size) == (3, 3) and tuple(m.stride) == (1, 1) and tuple(m.padding) == (1, 1)
            and tuple(m.dilation) == (1, 1) and m.groups == 1 and m.padding_mode == "zeros" and m.bias is not None
            and conv3x3_native_ok(x, m.weight))


def _edge_conv_input_ok(x: torch.Tensor) -> bool:
    return (not _miopen() and x.is_cuda and not _lib.reference_mode() and x.dim() == 4
            and (x.dtype == torch.bfloat16 or _autocast_bf16(x))
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


def _bias_conv3x3_padded_ok(m: nn.Module, x: torch.Tensor) -> bool:
    """A stride-1 3x3 biased convolution whose input channel count is not a multiple of 64 (SimpleUNet's 65-channel
    ERA5 input) on the implicit-GEMM kernel, through a zero-padded copy of the input."""
    return (tuple(m.kernel_size) == (3, 3) and tuple(m.stride) == (1, 1) and tuple(m.padding) == (1, 1)
            and tuple(m.dilation) == (1, 1) and m.groups == 1 and m.padding_mode == "zeros" and m.bias is not None
            and m.in_channels % 64 != 0 and m.in_channels <= 512 and m.out_channels % 64 == 0
            and _edge_conv_input_ok(x))


def _bias_conv1x1_ok(m: nn.Module, x: torch.Tensor) -> bool:
    return (tuple(m.kernel_size) == (1, 1) and tuple(m.stride) == (1, 1) and tuple(m.padding) == (0, 0)
            and tuple(m.dilation) == (1, 1) and m.groups == 1 and m.bias is not None and m.in_channels % 64 == 0
            and not isinstance(m, nn.ConvTranspose2d) and _edge_conv_input_ok(x))


class _PadChannelsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cp):
        B, C, H, W = x.shape
        xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
        ctx.c, ctx.dtype = C, x.dtype
        x2 = xb.permute(0, 2, 3, 1).contiguous().view(-1, C)   # a view for channels-last input
        return _lib.ops().pad_cols(x2, cp).view(B, H, W, cp).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        return g[:, :ctx.c].to(ctx.dtype), None


def pad_channels(x: torch.Tensor, cp: int) -> torch.Tensor:
    """Channels-last [B, C, H, W] -> a bf16 channels-last [B, cp, H, W] copy whose channels C..cp-1 are zero (one
    HIP pass, csrc/transpose.hip pad_cols_k); the gradient is the first C channels of the padded one."""
    return _PadChannelsFn.apply(x, cp)


class _BiasConv1x1Fn(torch.autograd.Function):
    """Stride-1 1x1 convolution with a bias and any output-channel count (SimpleUNet's 64 -> 65 ``out``) on the
    gathered implicit GEMM (one tap, bias in the epilogue, csrc/conv3x3.hip): the weight is zero-padded to a multiple
    of 64 rows and the result is the first Cout columns of the [pixels, Np] product, returned as a strided
    channels-last view (no slicing copy).  The backward pads dY the same way, so the input gradient (K = Np) and the
    weight gradient (``ts_gemm_tn_``) run on the 1x1 kernels and the bias gradient is one channel sum."""

    @staticmethod
    def forward(ctx, x, w, bias, bn_slot=None):
        B, C, H, W = x.shape
        cout = w.shape[0]
        npad = -(-cout // 64) * 64
        ctx.bn_slot = bn_slot
        xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
        x2 = _nhwc2d(xb)
        w2 = F.pad(w.reshape(cout, C).to(torch.bfloat16), (0, 0, 0, npad - cout))
        bp = F.pad(bias.float(), (0, npad - cout))
        y2 = _lib.ops().convg_nt(x2, w2, strided_fwd_geo(H, W, 1, 1, 0), False, False, bp)[0]
        ctx.save_for_backward(x2, w2)
        ctx.cfg = (B, C, H, W, cout, npad, w.dtype, bias.dtype)
        ctx.bias_param = bias if isinstance(bias, nn.Parameter) else None
        return y2.view(B, H, W, npad)[..., :cout].permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        B, C, H, W, cout, npad, wdt, bdt = ctx.cfg
        dy2 = _lib.ops().pad_cols(_nhwc2d(dy.to(torch.bfloat16)), npad)   # [pixels, npad], zero columns past Cout
        dx = gw = gb = None
        if ctx.needs_input_grad[0]:
            bn = ctx.bn_slot   # x is a BatchNorm + ReLU output consumed only here: its reduction in this epilogue
            if bn is not None and bn.usable(B * H * W, C):
                dx = bn.launch(dy2, weight_t(w2)).view(B, H, W, C).permute(0, 3, 1, 2)
                bn.mark(dx)
            else:
                dx = _lib.ops().ts_gemm_nt(dy2, weight_t(w2)).view(B, H, W, C).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            gk = torch.empty((npad, C), device=dy.device, dtype=torch.float32)
            _lib.ops().ts_gemm_tn_(gk, dy2, x2, False)
            gw = gk[:cout].to(wdt).view(cout, C, 1, 1)
        if ctx.needs_input_grad[2]:
            gb = _lib.ops().channel_sum(dy2, torch.float32)[:cout]
            p = ctx.bias_param
            mg = getattr(p, "main_grad", None) if p is not None else None
            if mg is not None and _DIRECT and not getattr(p, "_dph_accum", False) and mg.is_contiguous():
                mg.view(-1).copy_(gb)   # straight into the engine's bucket (as bias_grad does)
                p._dph_zeroed = False
                p._dph_accum = True
                p._dph_grad_ready()
                gb = None
            else:
                gb = gb.to(bdt)
        return dx, gw, gb, None


class BiasConv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters and state dict) whose channels-last GPU path computes the bias gradient with
    the per-channel sum kernel; stride-1 3x3 convolutions take the implicit-GEMM kernel of csrc/conv3x3.hip with the
    bias in its epilogue (input channels that are not a multiple of 64 through a zero-padded input copy), stride-1 1x1
    ones the gathered one-tap GEMM (output channels padded to a multiple of 64), everything else the stock MIOpen
    convolution."""

    def forward(self, x, stats_slot: StatsSlot | None = None, bn_slot: BnGradSlot | None = None):
        """``stats_slot``: on the 3x3 kernel path the following BatchNorm's statistics come from this convolution's
        epilogue (SimpleUNet's conv -> BN blocks, models/unet.py); otherwise the slot stays empty.  ``bn_slot``: x is
        a training-mode BatchNorm + ReLU output consumed only here; its backward reduction then runs in this
        convolution's input-gradient epilogue (3x3 and 1x1 kernel paths)."""
        if _bias_conv3x3_ok(self, x):
            _lib.require()
            b = self.bias if self.bias.dtype in (torch.float32, torch.bfloat16) else self.bias.float()
            return _Conv3x3Fn.apply(x, self.weight, stats_slot, b, "dph", bn_slot)
        if _bias_conv3x3_padded_ok(self, x):
            # SimpleUNet's 65-channel input conv: MIOpen's igemm_fwd / igemm_wrw before (0.117 + 0.095 ms per step,
            # profiles/r4/unet_c3w_default/); the padded K costs 2x the MFMAs but keeps the BN-statistics epilogue
            _lib.require()
            cp = -(-self.in_channels // 64) * 64
            b = self.bias if self.bias.dtype in (torch.float32, torch.bfloat16) else self.bias.float()
            wp = F.pad(self.weight, (0, 0, 0, 0, 0, cp - self.in_channels))
            return _Conv3x3Fn.apply(pad_channels(x, cp), wp, stats_slot, b)
        if _bias_conv1x1_ok(self, x):
            _lib.require()
            return _BiasConv1x1Fn.apply(x, self.weight, self.bias, bn_slot)
        if _bias_conv_ok(self, x):
            return _bias_conv(self, x, False, (0, 0))
        return super().forward(x)


class BiasConvTranspose2d(nn.ConvTranspose2d):
    """``nn.ConvTranspose2d`` counterpart of ``BiasConv2d`` (no ``output_size`` argument on the fast path)."""

    def forward(self, x, output_size=None):
        if output_size is None and _bias_conv_ok(self, x):
            return _bias_conv(self, x, True, self.output_padding)
        return super().forward(x, output_size)


# ------------------------------------------------------------------------------------------------ RGB stem
def stem_geometry(H, W, k, p, cin=4):
    """The k x k / stride-2 stem as a chunk-tap implicit GEMM (csrc/conv3x3.hip conv3_k GEN = 2): the input is
    zero-padded by p and stored as pairs of 4-channel pixels (16-B rows of 8 bf16), so output pixel (oy, ox) and kernel
    tap (ky, kx = 2 kxp + px) read pair row (2 oy + ky, ox + kxp); every 16-B chunk of the GEMM's K is one (ky, kxp)
    tap.  Returns (Hp, Wq, Ho, Wo, kxp, ntaps, K, geo)."""
    Hp, Wp = H + 2 * p, W + 2 * p
    Wp += Wp % 2
    Wq = Wp // 2
    Ho, Wo = (H + 2 * p - k) // 2 + 1, (W + 2 * p - k) // 2 + 1
    kxp = (k + 1) // 2
    ntaps = k * kxp
    K = -(-ntaps * 8 // 128) * 128
    geo = conv_geo(Hp, Wq, Ho, Wo, 2, 1, 0, 0, Ho, Wo, 1, 1, 0, 0, [(0, kxp)])
    geo[14] = ntaps
    return Hp, Wq, Ho, Wo, kxp, ntaps, K, geo


def stem_weight(w: torch.Tensor, kxp: int, K: int) -> torch.Tensor:
    """[Cout, C <= 4, k, k] -> the chunk-tap operand [Cout, K]: column (ky kxp + j) 8 + 4 px + c = w[co, c, ky, 2j + px]
    (zero for the 4th channel, kx = k and the K padding)."""
    co, c, k, _ = w.shape
    w4 = F.pad(w, (0, 2 * kxp - k, 0, 0, 0, 4 - c))                 # [Cout, 4, k, 2 kxp]
    wk = w4.view(co, 4, k, kxp, 2).permute(0, 2, 3, 4, 1).reshape(co, k * kxp * 8)
    return F.pad(wk, (0, K - wk.shape[1])).contiguous()


class _StemConvFn(torch.autograd.Function):
    """The RGB stem (k x k / stride 2, 3 -> Cout channels, no bias) on the framework's chunk-tap implicit GEMM:
    forward (with the following BatchNorm's statistics when asked) and weight gradient (c3w_k GEN = 2) from one padded
    pair-pixel copy of the image; the image itself gets no gradient."""

    @staticmethod
    def forward(ctx, x, w, k, p, stats_slot=None):
        B, C, H, W = x.shape
        Hp, Wq, Ho, Wo, kxp, ntaps, K, geo = stem_geometry(H, W, k, p)
        xp = torch.zeros((B, Hp, 2 * Wq, 4), device=x.device, dtype=torch.bfloat16)
        xp[:, p:p + H, p:p + W, :C] = x.permute(0, 2, 3, 1)
        a = xp.view(B * Hp * Wq, 8)
        cout = w.shape[0]
        wk = stem_weight(w.to(torch.bfloat16), kxp, K)
        if stats_slot is not None:
            y2, stats_slot.stats = _lib.ops().convg_nt(a, wk, geo, True, True)
            stats_slot.rows, stats_slot.cols = y2.shape
        else:
            y2 = _lib.ops().convg_nt(a, wk, geo, False, True)[0]
        ctx.save_for_backward(a)
        ctx.cfg = (B, C, H, W, k, p, Ho, Wo, kxp, K, geo, w.shape, w.dtype)
        return y2.view(B, Ho, Wo, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (a,) = ctx.saved_tensors
        B, C, H, W, k, p, Ho, Wo, kxp, K, geo, wshape, wdtype = ctx.cfg
        gw = None
        if ctx.needs_input_grad[1]:
            cout = wshape[0]
            dy2 = _nhwc2d(dy.to(torch.bfloat16))
            gk = torch.empty((cout, K), device=dy.device, dtype=torch.float32)
            _lib.ops().convg_tn_(gk, dy2, a, geo, False, True)
            g5 = gk[:, :k * kxp * 8].view(cout, k, kxp, 2, 4).permute(0, 4, 1, 2, 3).reshape(cout, 4, k, 2 * kxp)
            gw = g5[:, :C, :, :k].to(wdtype).contiguous(memory_format=torch.channels_last)
        return None, gw, None, None, None


def stem_native_ok(x: torch.Tensor, m: nn.Conv2d) -> bool:
    if _miopen() or not x.is_cuda or _lib.reference_mode():
        return False
    if not (x.dtype == torch.bfloat16 or _autocast_bf16(x)) or x.requires_grad:
        return False
    k = m.kernel_size[0]
    return (x.dim() == 4 and m.in_channels <= 4 and m.kernel_size == (k, k) and k % 2 == 1 and m.stride == (2, 2)
            and m.padding == (m.padding[0],) * 2 and m.dilation == (1, 1) and m.groups == 1 and m.bias is None
            and m.padding_mode == "zeros" and m.out_channels % 64 == 0)


class StemConv2d(nn.Conv2d):
    """``nn.Conv2d`` for a 3-channel (RGB) image stem whose channels-last GPU path zero-pads the input channels to 4.

    With 3 channels an NHWC pixel is 6 bytes and MIOpen's implicit-GEMM kernels run the ResNet stem (7x7 / 2, 64
    filters, B=256 x 224 x 224, bf16) in 0.876 ms forward + weight gradient; at 4 channels (8-byte pixels) 0.603 ms,
    at 8 channels 0.777 (`benchmarks/stem_conv_bench.py`, profiles/r2s3/stem_conv_bench.log).  The padded copy of the
    image (written once per step, in the compute dtype) and a zero weight slice make the 4-channel convolution
    exactly the 3-channel one; the parameter keeps its [Cout, 3, k, k] shape (state dicts unchanged) and receives
    the gradient of its own 3 channels."""

    def forward(self, x, stats_slot: StatsSlot | None = None):
        if stem_native_ok(x, self):
            _lib.require()
            return _StemConvFn.apply(x, self.weight, self.kernel_size[0], self.padding[0],
                                     stats_slot)
        if not (self.in_channels == 3 and self.groups == 1 and x.is_cuda and x.dim() == 4
                and self.padding_mode == "zeros" and not isinstance(self.padding, str)
                and x.is_contiguous(memory_format=torch.channels_last) and _lib.use_native(x)):
            return super().forward(x)
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        b, _, h, w = x.shape
        x4 = torch.empty((b, 4, h, w), device=x.device, dtype=dt, memory_format=torch.channels_last)
        x4[:, 3].zero_()
        x4[:, :3].copy_(x)
        wt = self.weight
        w4 = torch.cat([wt, wt.new_zeros((wt.shape[0], 1) + tuple(wt.shape[2:]))], 1)
        return F.conv2d(x4, w4, self.bias, self.stride, self.padding, self.dilation, 1)
