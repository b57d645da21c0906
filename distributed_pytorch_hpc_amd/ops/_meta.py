"""Fake (meta) implementations of the ``torch.ops.dph`` operators.

They let the custom ops flow through FakeTensor tracing (torch.export / meta-device model
construction / shape inference) without running a kernel.
"""
from __future__ import annotations

import torch
from torch.library import register_fake


@register_fake("dph::rmsnorm_fwd")
def _rmsnorm_fwd(x, w, eps, residual=None):
    rows = x.numel() // x.shape[-1]
    h = torch.empty_like(x) if residual is not None else x.new_empty((0,))
    return torch.empty_like(x), x.new_empty((rows,), dtype=torch.float32), h


@register_fake("dph::rmsnorm_bwd")
def _rmsnorm_bwd(dy, x, w, rstd, dres=None):
    return torch.empty_like(x), torch.empty_like(w)


@register_fake("dph::layernorm_fwd")
def _layernorm_fwd(x, w, b, eps):
    rows = x.numel() // x.shape[-1]
    return torch.empty_like(x), x.new_empty((rows,), dtype=torch.float32), x.new_empty((rows,), dtype=torch.float32)


@register_fake("dph::layernorm_bwd")
def _layernorm_bwd(dy, x, w, mean, rstd):
    return torch.empty_like(x), torch.empty_like(w), torch.empty_like(w)


@register_fake("dph::rope_")
def _rope(x, cos, sin, pos_offset, inverse):
    return None


@register_fake("dph::swiglu_fwd")
def _swiglu_fwd(x2):
    return x2.new_empty((*x2.shape[:-1], x2.shape[-1] // 2))


@register_fake("dph::swiglu_bwd")
def _swiglu_bwd(dy, x2):
    return torch.empty_like(x2)


@register_fake("dph::gelu_fwd")
def _gelu_fwd(x, tanh_form):
    return torch.empty_like(x)


@register_fake("dph::gelu_bwd")
def _gelu_bwd(dy, x, tanh_form):
    return torch.empty_like(x)


@register_fake("dph::adamw_step_")
def _adamw(master, m, v, grad, param_out, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale, hyper=None):
    return None


@register_fake("dph::sgd_step_")
def _sgd(master, buf, grad, param_out, lr, momentum, dampening, weight_decay, nesterov, first_step, grad_scale,
         hyper=None):
    return None


@register_fake("dph::sumsq_")
def _sumsq(x, out):
    return None


@register_fake("dph::bn_act_fwd")
def _bn_act_fwd(x, res, w, b, rm, rv, momentum, eps, relu, pre_stats=None, num_batches_tracked=None,
                relu_mask_out=None):
    c = x.shape[1]
    return (torch.empty_like(x), x.new_empty((c,), dtype=torch.float32), x.new_empty((c,), dtype=torch.float32),
            x.new_empty((2 * c,), dtype=torch.float32))


@register_fake("dph::bn_act_apply")
def _bn_act_apply(x, res, scale, shift, relu):
    return torch.empty_like(x)


@register_fake("dph::bn_act_bwd")
def _bn_act_bwd(dy, y, x, mean, invstd, w, relu, need_dres, need_dwb, xmask_ss=None, dw_out=None, db_out=None,
                relu_mask=None):
    c = x.shape[1]
    pdt = w.dtype if w is not None else torch.float32
    return (torch.empty_like(x), torch.empty_like(x) if need_dres else x.new_empty((0,)),
            x.new_empty((c,) if need_dwb else (0,), dtype=pdt), x.new_empty((c,) if need_dwb else (0,), dtype=pdt))


@register_fake("dph::transpose2d")
def _transpose2d(x):
    return x.new_empty((x.shape[1], x.shape[0]))


def _pool_out(n, k):
    return (n - 1) // 2 + 1 if k == 3 else n // 2


@register_fake("dph::maxpool_s2_fwd")
def _maxpool_s2_fwd(x, k):
    n, c, h, w = x.shape
    ho, wo = _pool_out(h, k), _pool_out(w, k)
    y = x.new_empty((n, c, ho, wo)).contiguous(memory_format=torch.channels_last)
    return y, x.new_empty((n, ho, wo, c), dtype=torch.uint8)


@register_fake("dph::maxpool_s2_bwd")
def _maxpool_s2_bwd(dy, tap, H, W, k):
    n, c = dy.shape[:2]
    return dy.new_empty((n, c, H, W)).contiguous(memory_format=torch.channels_last)


@register_fake("dph::channel_sum")
def _channel_sum(x, out_dtype):
    return x.new_empty((x.shape[1],), dtype=out_dtype)
