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
                relu_mask_out=None, apply=True):
    c = x.shape[1]
    return (torch.empty_like(x) if apply else x.new_empty((0,)), x.new_empty((c,), dtype=torch.float32), x.new_empty((c,), dtype=torch.float32),
            x.new_empty((2 * c,), dtype=torch.float32))


@register_fake("dph::bn_act_apply")
def _bn_act_apply(x, res, scale, shift, relu):
    return torch.empty_like(x)


@register_fake("dph::bn_act_apply_resbn")
def _bn_act_apply_resbn(x, ss, z, zss, relu_mask):
    return torch.empty_like(x)


@register_fake("dph::bn_act_bwd_dual")
def _bn_act_bwd_dual(dy, x, z, relu_mask, mean_a, invstd_a, w_a, mean_b, invstd_b, w_b, need_a, need_b, dw_a_out=None,
                     db_a_out=None, dw_b_out=None, db_b_out=None, pre_part_a=None):
    c = x.shape[1]

    def pg(need):
        return x.new_empty((c,) if need else (0,), dtype=w_a.dtype if need else torch.float32)

    return [torch.empty_like(x), torch.empty_like(z), pg(need_a), pg(need_a), pg(need_b), pg(need_b)]


@register_fake("dph::bn_act_bwd")
def _bn_act_bwd(dy, y, x, mean, invstd, w, relu, need_dres, need_dwb, xmask_ss=None, dw_out=None, db_out=None,
                relu_mask=None, pre_part=None):
    c = x.shape[1]
    pdt = w.dtype if w is not None else torch.float32
    return (torch.empty_like(x), torch.empty_like(x) if need_dres else x.new_empty((0,)),
            x.new_empty((c,) if need_dwb else (0,), dtype=pdt), x.new_empty((c,) if need_dwb else (0,), dtype=pdt))


@register_fake("dph::pad_cols")
def _pad_cols(x, cols):
    return x.new_empty((x.shape[0], cols))


@register_fake("dph::transpose2d")
def _transpose2d(x):
    return x.new_empty((x.shape[1], x.shape[0]))


@register_fake("dph::conv3x3_dgrad_weight")
def _conv3x3_dgrad_weight(w):
    return w.new_empty((w.shape[1], 9 * w.shape[0]), memory_format=torch.contiguous_format)


def _pool_out(n, k):
    return (n - 1) // 2 + 1 if k == 3 else n // 2


@register_fake("dph::maxpool_s2_fwd")
def _maxpool_s2_fwd(x, k):
    n, c, h, w = x.shape
    ho, wo = _pool_out(h, k), _pool_out(w, k)
    y = x.new_empty((n, c, ho, wo)).contiguous(memory_format=torch.channels_last)
    return y, x.new_empty((n, ho, wo, c), dtype=torch.uint8)


@register_fake("dph::maxpool_s2_bwd")
def _maxpool_s2_bwd(dy, tap, H, W, k, add=None, add_off=0):
    n, c = dy.shape[:2]
    return dy.new_empty((n, c, H, W)).contiguous(memory_format=torch.channels_last)


@register_fake("dph::upcat_fwd")
def _upcat_fwd(y2, bias, skip, H, W):
    n, cs, ho, wo = skip.shape
    return skip.new_empty((n, y2.shape[1] // 4 + cs, ho, wo)).contiguous(memory_format=torch.channels_last)


@register_fake("dph::upcat_bwd")
def _upcat_bwd(dcat, H, W, Co, want_skip=True):
    n, ct, ho, wo = dcat.shape
    dskip = (dcat.new_empty((n, ct - Co, ho, wo)).contiguous(memory_format=torch.channels_last) if want_skip
             else dcat.new_empty((0,)))
    return dcat.new_empty((n * H * W, 4 * Co)), dskip


@register_fake("dph::channel_sum")
def _channel_sum(x, out_dtype):
    return x.new_empty((x.shape[1],), dtype=out_dtype)


# ---- attention / GEMM / embedding / loss (restored) and serving / FP8 ops ----
@register_fake("dph::flash_attn_fwd")
def _flash_attn_fwd(q, k, v, scale, causal, dropout_p=0.0, seed=0):
    # q [B, S, H, D] -> o [B, S, H, Dv], lse [B, H, S] fp32
    o = q.new_empty(q.shape)
    return o, q.new_empty((q.shape[0], q.shape[2], q.shape[1]), dtype=torch.float32)


@register_fake("dph::flash_attn_bwd")
def _flash_attn_bwd(dout, q, k, v, o, lse, scale, causal, dropout_p=0.0, seed=0):
    return torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)


@register_fake("dph::flash_attn_bwd_into")
def _flash_attn_bwd_into(dout, q, k, v, o, lse, scale, causal, dq, dk, dv, dropout_p=0.0, seed=0, rope_cos=None,
                         rope_sin=None, rope_offset=0):
    return None


@register_fake("dph::cross_entropy_fwd")
def _cross_entropy_fwd(logits, target, inv_count, ignore_index, grad_inplace, smoothing):
    n = logits.shape[0]
    return logits.new_empty((n,), dtype=torch.float32), logits.new_empty((n,), dtype=torch.float32)


@register_fake("dph::embedding_fwd")
def _embedding_fwd(ids, table, vocab_start):
    return table.new_empty((*ids.shape, table.shape[1]))


@register_fake("dph::embedding_bwd")
def _embedding_bwd(ids, dout, vocab_local, vocab_start):
    return dout.new_empty((vocab_local, dout.shape[-1]), dtype=torch.float32)


@register_fake("dph::gemm_tn_")
def _gemm_tn(C, A, B, accumulate):
    return None


@register_fake("dph::ts_gemm_nt")
def _ts_gemm_nt(A, B, H=0, W=0, add=None, bias=None, pro_ss=None):
    return A.new_empty((A.shape[0], B.shape[0]))


@register_fake("dph::ts_gemm_nt_stats")
def _ts_gemm_nt_stats(A, B, H=0, W=0, pro_ss=None, bias=None):
    M, N = A.shape[0], B.shape[0]
    nmb = (M + 127) // 128
    return A.new_empty((M, N)), A.new_empty((2 * nmb * N + nmb,), dtype=torch.float32)


@register_fake("dph::ts_gemm_tn_")
def _ts_gemm_tn(C, A, B, accumulate, H=0, W=0, pro_ss=None):
    return None


@register_fake("dph::convg_nt")
def _convg_nt(A, B, geo, stats=False, chunk_taps=False, bias=None):
    Hs, Ws, Ho, Wo, Hd, Wd = geo[0], geo[1], geo[2], geo[3], geo[8], geo[9]
    imgs = A.shape[0] // (Hs * Ws)
    N = B.shape[0]
    res = [A.new_empty((imgs * Hd * Wd, N))]
    if stats:
        M = imgs * Ho * Wo
        nmb = (M + 127) // 128
        res.append(A.new_empty((2 * nmb * N + nmb,), dtype=torch.float32))
    return res


@register_fake("dph::gemm_nt_swiglu_into")
def _gemm_nt_swiglu_into(x, w13, x13_out, h_out):
    return None


@register_fake("dph::gemm_nt_dswiglu_into")
def _gemm_nt_dswiglu_into(dy, w2t, x13, d13_out):
    return None


@register_fake("dph::convg_nt_out_")
def _convg_nt_out(A, B, geo, out):
    return None


@register_fake("dph::convg_tn_")
def _convg_tn(C, A, B, geo, accumulate, chunk_taps=False):
    return None


@register_fake("dph::ts_gemm_nt_add_sub")
def _ts_gemm_nt_add_sub(A, B, add, H, W, s):
    return A.new_empty((A.shape[0], B.shape[0]))


@register_fake("dph::ts_gemm_nt_bnred")
def _ts_gemm_nt_bnred(A, B, H, W, add, sub, x, mean, invstd, ss=None, bits=None, add_mask=None):
    M, N = A.shape[0], B.shape[0]
    return A.new_empty((M, N)), A.new_empty(((M + 127) // 128, 2 * N), dtype=torch.float32)


@register_fake("dph::ts_gemm_nt_addmask")
def _ts_gemm_nt_addmask(A, B, add, add_mask):
    return A.new_empty((A.shape[0], B.shape[0]))


@register_fake("dph::maxpool_s2_bwd_bnred")
def _maxpool_s2_bwd_bnred(dy, tap, H, W, k, x, mean, invstd, ss, add=None, add_off=0):
    n, c = dy.shape[0], dy.shape[1]
    blocks = min(max((n * H * W * (c // 8) + 255) // 256, 1), 2048)   # csrc/dph_common.h stream_grid
    dx = dy.new_empty((n, c, H, W)).contiguous(memory_format=torch.channels_last)
    return dx, dy.new_empty((blocks, 2 * c), dtype=torch.float32)


@register_fake("dph::latmse_fwd")
def _latmse_fwd(pred, target, n_global, lat_offset):
    return pred.new_empty((), dtype=torch.float32)


@register_fake("dph::latmse_bwd")
def _latmse_bwd(gloss, pred, target, n_global, lat_offset, need_dtarget):
    return torch.empty_like(pred), (torch.empty_like(target) if need_dtarget else pred.new_empty((0,)))


@register_fake("dph::image_augment")
def _image_augment(images, idx, params, mean, inv_std, pad, channels_last, bf16_out):
    _, H, W, C = images.shape
    y = images.new_empty((idx.shape[0], C, H, W), dtype=torch.bfloat16 if bf16_out else torch.float32)
    return y.contiguous(memory_format=torch.channels_last) if channels_last else y


@register_fake("dph::fp8_quantize")
def _fp8_quantize(x, fmt, rowmajor, transposed):
    f8 = torch.float8_e4m3fn if fmt == 0 else torch.float8_e5m2
    R, C = x.shape
    y = x.new_empty((R, C) if rowmajor else (0,), dtype=f8)
    yt = x.new_empty((C, R) if transposed else (0,), dtype=f8)
    return y, yt, x.new_empty((), dtype=torch.float32)


@register_fake("dph::kv_append_")
def _kv_append(qkv, k_cache, v_cache, pos, cos, sin, n_heads, n_kv_heads, kv_scale=1.0):
    return None


@register_fake("dph::decode_attention")
def _decode_attention(qkv, k_cache, v_cache, pos, n_heads, n_kv_heads, scale, max_len, kv_scale=1.0):
    D = k_cache.shape[-1]
    return qkv.new_empty((qkv.shape[0], n_heads * D))


@register_fake("dph::skinny_linear")
def _skinny_linear(x, w):
    return x.new_empty((*x.shape[:-1], w.shape[0]))


@register_fake("dph::gemv_swiglu")
def _gemv_swiglu(x2, w):
    return x2.new_empty((*x2.shape[:-1], w.shape[0]))


@register_fake("dph::gemv_rmsnorm")
def _gemv_rmsnorm(x, res, norm_weight, eps, w):
    return x.new_empty((*x.shape[:-1], w.shape[0])), (torch.empty_like(x) if res is not None else x.new_empty((0,)))


@register_fake("dph::car_allreduce")
def _car_allreduce(ctx, inp, out, algo, scale, max_blocks):
    return None


@register_fake("dph::car_flag")
def _car_flag(ctx, flag):
    return None


@register_fake("dph::car_poison")
def _car_poison(ctx, flag, gscale):
    return None


@register_fake("dph::gemm_nt")
def _gemm_nt(A, B):
    return A.new_empty((*A.shape[:-1], B.shape[0]))


@register_fake("dph::gemm_nt_swiglu")
def _gemm_nt_swiglu(x, w13):
    H = w13.shape[0] // 2
    return x.new_empty((*x.shape[:-1], 2 * H)), x.new_empty((*x.shape[:-1], H))


@register_fake("dph::gemm_nt_dswiglu")
def _gemm_nt_dswiglu(dy, w2t, x13):
    return dy.new_empty((*dy.shape[:-1], 2 * w2t.shape[0]))


@register_fake("dph::gemm_nt_rope")
def _gemm_nt_rope(x, w, cos, sin, S, hd, n_rot, pos_off):
    return x.new_empty((*x.shape[:-1], w.shape[0]))


@register_fake("dph::flash_attn_fwd_merge_")
def _flash_attn_fwd_merge(q, k, v, scale, causal, acc_o, acc_lse):
    return None


@register_fake("dph::channel_sum_into_")
def _channel_sum_into(x, out):
    return None
