"""Fused BatchNorm + residual add + ReLU for channels-last activations (csrc/batchnorm.hip).

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers and state-dict keys) whose
``forward(x, residual=None)`` computes ``act(bn(x) + residual)``.  On an MI355X with a channels-last input whose
channel count is a power of two in [8, 2048] it runs the fused HIP kernels (one statistics pass + one apply pass
forward; one reduction pass + one dx pass backward, which also emits the residual's gradient; for ReLU without a
residual the backward takes the mask from x and the forward's scale / shift instead of reading y); otherwise the
stock ``F.batch_norm`` + add + ReLU path.  The reference trains torchvision ResNets (scripts/main.py:249,
resnet_fsdp_training.py:186-191) whose conv -> BN -> ReLU (+ identity) blocks this fuses.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from .conv import _DIRECT, weight_t


def _pow2_channels(c: int) -> bool:
    return 8 <= c <= 2048 and (c & (c - 1)) == 0


def _native_ok(x: torch.Tensor, residual) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)):
        return False
    if not _lib.use_native(x):
        return False
    if not (_pow2_channels(x.shape[1]) and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    if x.data_ptr() % 16:
        return False
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype
                                 or residual.stride() != x.stride()):
        return False
    return True


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, slot=None,
                pre_stats=None, nbt=None, bn_slot=None):
        # ReLU without residual: the backward recomputes the mask from x with the forward's scale / shift and
        # never reads y (one activation-sized read less in each backward pass).  ReLU after a residual add: the
        # forward writes [y > 0] as bits (1/16 of y's bytes) and the backward reads those instead of y.
        ctx.xmask = relu and residual is None
        ctx.bmask = relu and residual is not None
        bits = x.new_empty((x.numel() // 8,), dtype=torch.uint8) if ctx.bmask else None
        y, mean, invstd, ss = _lib.ops().bn_act_fwd(x, residual, weight, bias, running_mean, running_var, momentum,
                                                    eps, relu, pre_stats, nbt, bits)
        ctx.save_for_backward(x, ss if ctx.xmask else (bits if ctx.bmask else y), mean, invstd, weight)
        # the consumer convolution may run this BatchNorm's backward reduction in its dgrad epilogue (BnGradSlot)
        ctx.bn_slot = bn_slot if (bn_slot is not None and (ctx.xmask or ctx.bmask)
                                  and x.dtype == torch.bfloat16) else None
        if ctx.bn_slot is not None:
            bn_slot.fill(x, mean, invstd, ss if ctx.xmask else None, bits if ctx.bmask else None)
        ctx.relu, ctx.has_res = relu, residual is not None
        ctx.has_wb = weight is not None
        ctx.params = (weight, bias)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, saved, mean, invstd, weight = ctx.saved_tensors
        part = ctx.bn_slot.take(dy) if ctx.bn_slot is not None else None   # reduced by the consumer's epilogue
        dy = dy.contiguous(memory_format=torch.channels_last)
        need_wb = ctx.has_wb and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        # y is only read by the kernels when neither mask form applies (no ReLU: it is not read at all)
        y = saved if not (ctx.xmask or ctx.bmask) else x
        ss = saved if ctx.xmask else None
        bits = saved if ctx.bmask else None
        # engine-owned parameters (parallel/data_parallel.py main_grad views) on their first gradient of the step:
        # the kernel writes dgamma / dbeta straight into the gradient bucket, autograd gets None
        wp, bp = ctx.params
        direct = (need_wb and bp is not None and _DIRECT and all(
            getattr(p, "main_grad", None) is not None and not getattr(p, "_dph_accum", True)
            and p.main_grad.is_contiguous() and p.main_grad.dtype == p.dtype for p in (wp, bp)))
        # the residual gradient is dy under the ReLU bits: with a consuming 1x1 convolution (GradSlot) hand it dy and
        # the bits -- its dgrad kernel adds dy * mask -- instead of writing the masked copy (one activation-sized
        # write less)
        handoff = (ctx.slot is not None and ctx.has_res and bits is not None and dy.dtype == torch.bfloat16
                   and os.environ.get("DPH_RES_MASK", "1") != "0")
        dx, dres, dw, db = _lib.ops().bn_act_bwd(dy, y, x, mean, invstd, weight if ctx.has_wb else None, ctx.relu,
                                                 ctx.has_res and not handoff, need_wb, ss,
                                                 wp.main_grad if direct else None, bp.main_grad if direct else None,
                                                 bits, part)
        if direct:
            for p in (wp, bp):
                p._dph_accum = True
                p._dph_grad_ready()
            dw = db = None
        if handoff:
            ctx.slot.t, ctx.slot.mask = dy, bits
            dres = None
        elif ctx.slot is not None and ctx.has_res:   # the residual's gradient goes to the consuming 1x1 conv
            ctx.slot.t = dres
            dres = None
        return (dx, dw if need_wb else None, db if need_wb else None, None, None, dres if ctx.has_res else None,
                None, None, None, None, None, None, None)


def _direct_pair(wp, bp, need_wb: bool) -> bool:
    """Write dgamma / dbeta straight into engine-owned gradient buckets (parallel/data_parallel.py main_grad views)
    on the parameters' first gradient of the step."""
    return bool(need_wb and wp is not None and bp is not None and _DIRECT and all(
        getattr(p, "main_grad", None) is not None and not getattr(p, "_dph_accum", True)
        and p.main_grad.is_contiguous() and p.main_grad.dtype == p.dtype for p in (wp, bp)))


def _mark_direct(wp, bp):
    for p in (wp, bp):
        p._dph_accum = True
        p._dph_grad_ready()


class _BNDualActFn(torch.autograd.Function):
    """relu(bn_a(x) + bn_b(z)) for two training-mode BatchNorms: a BatchNorm + residual + ReLU whose residual is itself
    a BatchNorm's output -- ResNet's projection shortcut, bn3(conv3(.)) + bn(downsample(.)).

    Forward: both BatchNorms' statistics (from the producing convolutions' epilogues when given) and running-stat
    updates, then ONE apply pass that reads x and z and writes y and its ReLU bits (csrc/batchnorm.hip bn_apply_k
    RESBN): the shortcut's normalised activation is never written or re-read.  Backward: the gradient reaching both
    BatchNorm outputs is dy under the ReLU bits, so each BatchNorm's backward takes dy and the bits directly (no
    masked residual-gradient copy is written); bn_a's reduction may come from the consumer's epilogue (bn_slot)."""

    @staticmethod
    def forward(ctx, x, z, wa, ba, rma, rva, wb, bb, rmb, rvb, mom_a, eps_a, mom_b, eps_b, pre_a, pre_b, nbt_a, nbt_b,
                bn_slot):
        ops = _lib.ops()
        _, mean_a, inv_a, ss_a = ops.bn_act_fwd(x, None, wa, ba, rma, rva, mom_a, eps_a, True, pre_a, nbt_a, None,
                                                False)
        _, mean_b, inv_b, ss_b = ops.bn_act_fwd(z, None, wb, bb, rmb, rvb, mom_b, eps_b, False, pre_b, nbt_b, None,
                                                False)
        bits = x.new_empty((x.numel() // 8,), dtype=torch.uint8)
        y = ops.bn_act_apply_resbn(x, ss_a, z, ss_b, bits)
        ctx.save_for_backward(x, z, bits, mean_a, inv_a, mean_b, inv_b, wa, wb)
        ctx.params = (wa, ba, wb, bb)
        ctx.bn_slot = bn_slot if bn_slot is not None and x.dtype == torch.bfloat16 else None
        if ctx.bn_slot is not None:
            bn_slot.fill(x, mean_a, inv_a, None, bits)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, bits, mean_a, inv_a, mean_b, inv_b, wa, wb = ctx.saved_tensors
        part = ctx.bn_slot.take(dy) if ctx.bn_slot is not None else None   # reduced by the consumer's epilogue
        dy = dy.contiguous(memory_format=torch.channels_last)
        wpa, bpa, wpb, bpb = ctx.params
        need_a = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        need_b = ctx.needs_input_grad[6] or ctx.needs_input_grad[7]
        da, db_ = _direct_pair(wpa, bpa, need_a), _direct_pair(wpb, bpb, need_b)
        if os.environ.get("DPH_BN_DUAL_DX", "1") != "0":
            # both BatchNorms' dx in one pass over dy, the bits, x and z (csrc/batchnorm.hip bn_bwd_dx2_k)
            dxa, dxb, dwa, dba, dwb, dbb = _lib.ops().bn_act_bwd_dual(
                dy, x, z, bits, mean_a, inv_a, wa, mean_b, inv_b, wb, need_a, need_b,
                wpa.main_grad if da else None, bpa.main_grad if da else None,
                wpb.main_grad if db_ else None, bpb.main_grad if db_ else None, part)
        else:
            dxa, _, dwa, dba = _lib.ops().bn_act_bwd(dy, x, x, mean_a, inv_a, wa, True, False, need_a, None,
                                                     wpa.main_grad if da else None, bpa.main_grad if da else None,
                                                     bits, part)
            dxb, _, dwb, dbb = _lib.ops().bn_act_bwd(dy, z, z, mean_b, inv_b, wb, True, False, need_b, None,
                                                     wpb.main_grad if db_ else None, bpb.main_grad if db_ else None,
                                                     bits, None)
        if da:
            _mark_direct(wpa, bpa)
            dwa = dba = None
        if db_:
            _mark_direct(wpb, bpb)
            dwb = dbb = None
        return (dxa, dxb, dwa if need_a else None, dba if need_a else None, None, None,
                dwb if need_b else None, dbb if need_b else None, None, None, None, None, None, None, None, None,
                None, None, None)


def bn_dual_act(bn_a: "BatchNormAct2d", bn_b: "BatchNormAct2d", x, z, stats_a=None, stats_b=None, bn_slot=None):
    """``bn_a(x, residual=bn_b(z))`` with bn_a's ReLU and bn_b without activation (ResNet's projection-shortcut block
    tail), as one fused op when both are training-mode, tracked, affine BatchNorms on eligible tensors
    (_BNDualActFn); otherwise exactly the two module calls.  ``stats_a`` / ``stats_b``: statistics from the producing
    convolutions' epilogues (ops.conv.StatsSlot); ``bn_slot``: bn_a's reduction from its consumer's epilogue."""
    ok = (all(b.training and b.track_running_stats and b.affine and b.momentum is not None for b in (bn_a, bn_b))
          and bn_a.act and not bn_b.act and x.shape == z.shape and x.stride() == z.stride() and x.dtype == z.dtype
          and _native_ok(x, None) and _native_ok(z, None) and os.environ.get("DPH_BN_DUAL", "1") != "0")
    if not ok:
        return bn_a(x, bn_b(z, stats_slot=stats_b), stats_slot=stats_a, bn_slot=bn_slot)
    ch = x.shape[1]
    pre_a = stats_a.take(x.numel() // ch, ch) if stats_a is not None else None
    pre_b = stats_b.take(z.numel() // ch, ch) if stats_b is not None else None
    return _BNDualActFn.apply(x, z, bn_a.weight, bn_a.bias, bn_a.running_mean, bn_a.running_var, bn_b.weight,
                              bn_b.bias, bn_b.running_mean, bn_b.running_var, bn_a.momentum, bn_a.eps, bn_b.momentum,
                              bn_b.eps, pre_a, pre_b, bn_a.num_batches_tracked, bn_b.num_batches_tracked,
                              bn_slot if torch.is_grad_enabled() else None)


def batch_norm_act(x, weight, bias, running_mean, running_var, training: bool, momentum: float, eps: float,
                   residual=None, relu: bool = True, residual_grad_slot=None, stats_slot=None,
                   num_batches_tracked=None, bn_slot=None):
    """act(batch_norm(x) + residual) with the fused kernels when eligible.  ``residual_grad_slot``
    (ops.conv.GradSlot): hand the residual's gradient to the 1x1 convolution that consumes the same input.
    ``bn_slot`` (ops.conv.BnGradSlot): the convolution consuming the output may run the backward reduction."""
    if _native_ok(x, residual):
        if training:
            # statistics already computed by the producing 1x1 convolution (ops.conv.StatsSlot)
            pre = stats_slot.take(x.numel() // x.shape[1], x.shape[1]) if stats_slot is not None else None
            slot = residual_grad_slot
            if not torch.is_grad_enabled():
                bn_slot = None
            if slot is not None and residual is not None and slot.consumer and torch.is_grad_enabled():
                slot.armed = True
                return _BNActFn.apply(x, weight, bias, running_mean, running_var, residual.detach(), momentum, eps,
                                      relu, slot, pre, num_batches_tracked, bn_slot)
            return _BNActFn.apply(x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, None,
                                  pre, num_batches_tracked, bn_slot)
        with torch.no_grad():
            inv = torch.rsqrt(running_var.float() + eps)
            scale = inv * (weight.float() if weight is not None else 1.0)
            shift = (bias.float() if bias is not None else 0.0) - running_mean.float() * scale
        if not torch.is_grad_enabled() or not x.requires_grad:
            return _lib.ops().bn_act_apply(x, residual, scale.contiguous(), shift.contiguous(), relu)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class BatchNormAct2d(nn.BatchNorm2d):
    """``act(BatchNorm2d(x) + residual)``; ``act=False`` gives plain BatchNorm2d (+ residual)."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, affine: bool = True,
                 track_running_stats: bool = True, act: bool = True, **kw):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, **kw)
        self.act = act

    def forward(self, x, residual=None, residual_grad_slot=None, stats_slot=None, bn_slot=None):
        training = self.training or not self.track_running_stats
        momentum = self.momentum
        nbt = None
        if self.training and self.track_running_stats:
            if momentum is None or not _native_ok(x, residual):
                self.num_batches_tracked.add_(1)
                if momentum is None:   # cumulative moving average, as nn.BatchNorm2d
                    momentum = 1.0 / float(self.num_batches_tracked)
            else:   # the fused kernel increments the counter (one launch per BN layer fewer)
                nbt = self.num_batches_tracked
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        if training and rm is not None and not self.training:
            rm = rv = None
        return batch_norm_act(x, self.weight, self.bias, rm, rv, training, momentum, self.eps, residual, self.act,
                              residual_grad_slot, stats_slot, nbt, bn_slot)

    def extra_repr(self):
        return super().extra_repr() + f", act={'relu' if self.act else 'none'}"


# ------------------------------------------------------------------------------------------------ BN + ReLU -> 1x1 conv
# Off by default since round 4: with bn2 applied by its own pass, conv3's weight gradient runs on the plain 1x1 kernel
# (c3w_k identity rows), which beats the prologue form's register-staged ts_tn_k by more than the extra activation
# write / read costs -- ResNet-50 10 435 / 10 453 / 10 491 vs 10 318 / 10 323 / 10 345 img/s, interleaved
# (profiles/r4/bn_prologue_ab/).  DPH_BN_PROLOGUE=1 restores the fused form.
_PROLOGUE = os.environ.get("DPH_BN_PROLOGUE", "0") == "1"


class _BNReLUConv1x1Fn(torch.autograd.Function):
    """``conv1x1(relu(bn(x)))`` in training mode with the BatchNorm apply + ReLU folded into the convolution's operand
    loads (csrc/conv1x1.hip ``pro_ss``): the statistics pass and the running-stat update run as usual, but the
    normalised activation is never written -- the forward GEMM and the weight-gradient GEMM both read x and apply
    ``relu(x * scale + shift)`` in registers, and the BatchNorm backward takes its ReLU mask from x."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, w3, momentum, eps, pre_stats, nbt, stats_slot3):
        _, mean, invstd, ss = _lib.ops().bn_act_fwd(x, None, weight, bias, running_mean, running_var, momentum, eps,
                                                     True, pre_stats, nbt, None, False)
        B, C, H, W = x.shape
        cout = w3.shape[0]
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)                   # channels-last: a view
        w3b = w3.to(torch.bfloat16) if w3.dtype != torch.bfloat16 else w3
        w2d = w3b.reshape(cout, C)
        if stats_slot3 is not None:
            y2, stats_slot3.stats = _lib.ops().ts_gemm_nt_stats(x2, w2d, 0, 0, ss)
            stats_slot3.rows, stats_slot3.cols = y2.shape
        else:
            y2 = _lib.ops().ts_gemm_nt(x2, w2d, 0, 0, None, None, ss)
        ctx.save_for_backward(x, ss, mean, invstd, weight, w2d)
        ctx.params = (weight, bias, w3)
        ctx.w3dtype = w3.dtype
        return y2.view(B, H, W, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        from .conv import _nhwc2d, _wgrad_into_main

        x, ss, mean, invstd, weight, w2d = ctx.saved_tensors
        wp, bp, w3 = ctx.params
        B, C, H, W = x.shape
        cout = w2d.shape[0]
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
        dy2 = _nhwc2d(dy.to(torch.bfloat16))
        gw3 = None
        if ctx.needs_input_grad[5]:
            def launch(out, acc):
                _lib.ops().ts_gemm_tn_(out, dy2, x2, acc, 0, 0, ss)   # dW3 = dY^T relu(bn(x))

            if not _wgrad_into_main(w3, (cout, C), launch):
                gw3 = torch.empty((cout, C), dtype=ctx.w3dtype, device=dy.device)
                launch(gw3, False)
                gw3 = gw3.view(cout, C, 1, 1)
        dx = dw = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dyb = _lib.ops().ts_gemm_nt(dy2, weight_t(w2d))   # gradient of relu(bn(x)), [M, C]
            dyb = dyb.view(B, H, W, C).permute(0, 3, 1, 2)
            need_wb = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
            direct = (need_wb and bp is not None and _DIRECT and all(
                getattr(p, "main_grad", None) is not None and not getattr(p, "_dph_accum", True)
                and p.main_grad.is_contiguous() and p.main_grad.dtype == p.dtype for p in (wp, bp)))
            dx, _, dw, db = _lib.ops().bn_act_bwd(dyb, x, x, mean, invstd, weight, True, False, need_wb, ss,
                                                  wp.main_grad if direct else None, bp.main_grad if direct else None,
                                                  None)
            if direct:
                for p in (wp, bp):
                    p._dph_accum = True
                    p._dph_grad_ready()
                dw = db = None
            if not need_wb:
                dw = db = None
        return dx, dw, db, None, None, gw3, None, None, None, None, None


def bn_relu_conv1x1_ok(bn: "BatchNormAct2d", conv, x: torch.Tensor) -> bool:
    from .conv import Conv1x1, conv1x1_native_ok

    return (_PROLOGUE and isinstance(conv, Conv1x1) and bn.training and bn.track_running_stats and bn.act
            and bn.momentum is not None and bn.affine and x.dtype == torch.bfloat16 and x.shape[1] <= 2048
            and _native_ok(x, None) and conv1x1_native_ok(x, conv.weight) and torch.is_grad_enabled())


def bn_relu_conv1x1(bn: "BatchNormAct2d", conv, x: torch.Tensor, stats_slot=None, out_stats_slot=None):
    """``conv(bn(x))`` for a training-mode ``BatchNormAct2d`` (ReLU) followed by a stride-1 ``Conv1x1``, the apply
    folded into the convolution (see _BNReLUConv1x1Fn); ``stats_slot`` holds x's statistics from its producer's
    epilogue, ``out_stats_slot`` receives the convolution output's statistics for the next BatchNorm."""
    pre = stats_slot.take(x.numel() // x.shape[1], x.shape[1]) if stats_slot is not None else None
    return _BNReLUConv1x1Fn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, conv.weight, bn.momentum,
                                  bn.eps, pre, bn.num_batches_tracked, out_stats_slot)
