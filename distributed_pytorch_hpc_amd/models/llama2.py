"""Llama-2 decoder for MI355X training (capability parity with fsdp_tp/llama2_model.py:1-462).

Same architecture, hyper-parameters and init scheme as the reference ``Transformer``:
pre-norm RMSNorm blocks, interleaved-pair RoPE (theta 1e4), causal MHA/GQA attention, SwiGLU FFN with
hidden = multiple_of * ceil(int(2 * 4 * dim / 3) / multiple_of) (11008 at dim 4096), depth-scaled
truncated-normal init, fp32 logits from ``forward(tokens)``.

MI355X-first changes (numerically equivalent):
  * q/k/v and w1/w3 are FUSED projections (``wqkv``, ``w13``): one GEMM each instead of three / two,
    q/k/v are strided views of the GEMM output fed straight to the flash-attention kernel.
  * RoPE + attention run as one autograd node (ops.rope_attention), RoPE in place on the QKV buffer.
  * The residual add after each sub-block is fused into the following RMSNorm (ops.add_rms_norm):
    a block consumes and produces the pair (residual, pending delta) -- see TransformerBlock.forward.
  * With targets, ``forward`` returns the mean cross-entropy through the fused CE kernel, which never
    materialises fp32 logits.
``convert_reference_state_dict`` maps a reference checkpoint (wq/wk/wv, w1/w3) onto this layout.
Serving (beyond the reference): ``KVCache`` + ``Transformer.forward_inference`` (prefill and single-token decode
through csrc/decode.hip), driven by ``inference.Generator``.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional

import torch
from torch import nn

from .. import ops
from ..ops import decode as decode_ops
from ..ops.rope import precompute_rope_tables
from ..parallel import fused_layers


@dataclass
class ModelArgs:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: Optional[int] = None
    vocab_size: int = -1
    multiple_of: int = 256
    ffn_dim_multiplier: Optional[float] = None
    norm_eps: float = 1e-5
    max_batch_size: int = 32
    max_seq_len: int = 32768
    depth_init: bool = True
    rope_theta: float = 10000.0

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def kv_heads(self) -> int:
        return self.n_heads if self.n_kv_heads is None else self.n_kv_heads

    @property
    def ffn_hidden(self) -> int:
        h = int(2 * (4 * self.dim) / 3)
        if self.ffn_dim_multiplier is not None:
            h = int(self.ffn_dim_multiplier * h)
        return self.multiple_of * ((h + self.multiple_of - 1) // self.multiple_of)

    def num_params(self) -> int:
        d, hd = self.dim, self.head_dim
        attn = d * (self.n_heads + 2 * self.kv_heads) * hd + self.n_heads * hd * d
        ffn = 3 * d * self.ffn_hidden
        return self.n_layers * (attn + ffn + 2 * d) + 2 * self.vocab_size * d + d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token: 6 N (dense) + 6 L S D (causal attention, fwd+bwd, with the 1/2 mask)."""
        n_dense = self.num_params() - self.vocab_size * self.dim  # embedding gather is not a GEMM
        return 6.0 * n_dense + 6.0 * self.n_layers * seq_len * self.dim


PRESETS = {
    # the reference toy config (fsdp_tp/fsdp_tp_example.py:134, scripts/06_hybrid_parallelism/01_fsdp_tp_hybrid.py)
    "toy": ModelArgs(dim=256, n_layers=2, n_heads=16, vocab_size=32000),
    "tiny": ModelArgs(dim=128, n_layers=2, n_heads=4, vocab_size=512, max_seq_len=512),
    # heads, FFN (352), vocab and layers divisible by 8 / 4: rehearses the BASELINE meshes (tp8, dp2 x tp4, pp4 x dp2)
    "tiny8": ModelArgs(dim=128, n_layers=4, n_heads=8, vocab_size=512, multiple_of=32, max_seq_len=512),
    "tiny8-deep": ModelArgs(dim=128, n_layers=8, n_heads=8, vocab_size=512, multiple_of=32, max_seq_len=512),
    "llama2-1b": ModelArgs(dim=2048, n_layers=16, n_heads=16, vocab_size=32000, max_seq_len=4096),
    "llama2-7b": ModelArgs(dim=4096, n_layers=32, n_heads=32, vocab_size=32000, max_seq_len=4096),
    "llama2-13b": ModelArgs(dim=5120, n_layers=40, n_heads=40, vocab_size=32000, max_seq_len=4096),
    # GQA (8 KV heads), FFN 28 672: 69 B parameters, 138 GB in bf16 -- serving fits on ONE 288 GB MI355X
    "llama2-70b": ModelArgs(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, vocab_size=32000, multiple_of=4096,
                            ffn_dim_multiplier=1.3, max_seq_len=4096),
}


def get_preset(name: str, **overrides) -> ModelArgs:
    return replace(PRESETS[name], **overrides)


# ---------------------------------------------------------------------------------------------- rope cache
_ROPE: dict = {}


def rope_tables(head_dim: int, max_pos: int, theta: float, device) -> tuple[torch.Tensor, torch.Tensor]:
    key = (head_dim, max_pos, theta, str(device))
    t = _ROPE.get(key)
    if t is None:
        t = precompute_rope_tables(head_dim, max_pos, theta, device)
        _ROPE[key] = t
    return t


def _proj(mod: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Linear projection; a decode-sized row count without autograd (serving) takes the weight-streaming skinny
    GEMM of csrc/decode.hip, everything else the module itself."""
    if not torch.is_grad_enabled() and type(mod) is nn.Linear and decode_ops.skinny_ok(x, mod):
        return decode_ops.skinny_linear(x, mod.weight)
    return mod(x)


# ---------------------------------------------------------------------------------------------- modules
class Attention(nn.Module):
    def __init__(self, args: ModelArgs):
        super().__init__()
        self.n_heads = args.n_heads
        self.n_kv_heads = args.kv_heads
        self.head_dim = args.head_dim
        self.max_pos = 2 * args.max_seq_len
        self.theta = args.rope_theta
        self.wqkv = nn.Linear(args.dim, (self.n_heads + 2 * self.n_kv_heads) * self.head_dim, bias=False)
        self.wo = nn.Linear(self.n_heads * self.head_dim, args.dim, bias=False)
        # local head counts (changed by the tensor-parallel plan)
        self.n_local_heads = self.n_heads
        self.n_local_kv_heads = self.n_kv_heads
        # optional context-parallel attention implementation (Ulysses / ring), set by parallel.cp
        self.cp_attention = None

    def init_weights(self, init_std: float):
        nn.init.trunc_normal_(self.wqkv.weight, mean=0.0, std=0.02)
        nn.init.trunc_normal_(self.wo.weight, mean=0.0, std=init_std)

    def forward(self, x: torch.Tensor, pos_offset: int = 0, cache: Optional["KVCache"] = None,
                layer: int = 0) -> torch.Tensor:
        if cache is None and self.cp_attention is None and \
                fused_layers.qkv_rope_attention_ok(x, self.wqkv, self.head_dim):
            # projection + RoPE (in the GEMM epilogue) + flash attention as one autograd node (parallel/fused_layers)
            cos, sin = rope_tables(self.head_dim, self.max_pos, self.theta, x.device)
            o = fused_layers.qkv_rope_attention(x, self.wqkv, cos, sin, self.n_local_heads, self.n_local_kv_heads,
                                                self.head_dim, pos_offset)
            return _proj(self.wo, o)
        qkv = _proj(self.wqkv, x)
        cos, sin = rope_tables(self.head_dim, self.max_pos, self.theta, qkv.device)
        if cache is not None:
            return self.decode_from_qkv(qkv, cache, layer)
        if self.cp_attention is not None:
            o = self.cp_attention(qkv, cos, sin, self.n_local_heads, self.n_local_kv_heads, self.head_dim)
        else:
            o = ops.rope_attention(qkv, cos, sin, self.n_local_heads, self.n_local_kv_heads, self.head_dim,
                                   causal=True, pos_offset=pos_offset)
        return _proj(self.wo, o)

    def decode_from_qkv(self, qkv: torch.Tensor, cache: "KVCache", layer: int) -> torch.Tensor:
        """Serving: cached attention of an already projected qkv, then the output projection."""
        cos, sin = rope_tables(self.head_dim, self.max_pos, self.theta, qkv.device)
        return _proj(self.wo, self._cached_attention(qkv.contiguous(), cos, sin, cache, layer))

    def _cached_attention(self, qkv, cos, sin, cache: "KVCache", layer: int) -> torch.Tensor:
        """Serving path: append this step's k / v (RoPE at each sequence's cache position) and attend over the cache.
        One new token per sequence runs the split-KV decode kernel; several (prefill, chunked append) run the flash
        kernel over the cached prefix with the bottom-right causal mask."""
        if self.cp_attention is not None:
            raise NotImplementedError("KV-cache inference with context-parallel attention")
        b, s, _ = qkv.shape
        nh, nkv, hd = self.n_local_heads, self.n_local_kv_heads, self.head_dim
        kc, vc = cache.k[layer], cache.v[layer]
        ops.kv_append_(qkv, kc, vc, cache.pos, cos, sin, nh, nkv, cache.kv_scale)
        if s == 1:
            return ops.decode_attention(qkv, kc, vc, cache.pos, nh, nkv, max_len=cache.attn_bound(),
                                        kv_scale=cache.kv_scale).view(b, 1, -1)
        n = cache.length
        if n is None:
            raise RuntimeError("a multi-token append needs every sequence of the cache at the same, host-known length "
                               "(prefill ragged prompts one sequence at a time through KVCache.slot)")
        q = qkv[:, :, : nh * hd].view(b, s, nh, hd)
        if not cache.fp8:
            o = ops.flash_attention(q, kc[:, : n + s], vc[:, : n + s], causal=True)
        else:
            # FP8 cache: the new tokens attend over bf16 keys / values -- their own (rotated here, in place in qkv;
            # the cache got the quantised copy) after the dequantised prefix
            k = qkv[:, :, nh * hd: (nh + nkv) * hd].view(b, s, nkv, hd)
            v = qkv[:, :, (nh + nkv) * hd:].view(b, s, nkv, hd)
            ops.rope_(k, cos, sin, n)
            if n:
                k = torch.cat([decode_ops.dequantize_kv(kc[:, :n], cache.kv_scale, k.dtype), k], 1)
                v = torch.cat([decode_ops.dequantize_kv(vc[:, :n], cache.kv_scale, v.dtype), v], 1)
            o = ops.flash_attention(q, k, v, causal=True)
        return o.reshape(b, s, nh * hd)


class FeedForward(nn.Module):
    def __init__(self, dim: int, hidden_dim: int):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.w13 = nn.Linear(dim, 2 * hidden_dim, bias=False)   # [w1; w3]
        self.w2 = nn.Linear(hidden_dim, dim, bias=False)

    def init_weights(self, init_std: float):
        h = self.hidden_dim
        with torch.no_grad():
            nn.init.trunc_normal_(self.w13.weight[:h], mean=0.0, std=0.02)          # w1
            nn.init.trunc_normal_(self.w13.weight[h:], mean=0.0, std=init_std)      # w3
        nn.init.trunc_normal_(self.w2.weight, mean=0.0, std=init_std)

    def forward(self, x):
        if fused_layers.swiglu_mlp_ok(x, self.w13, self.w2):
            # SwiGLU in the w13 GEMM's epilogue, its backward in w2's input-gradient epilogue (parallel/fused_layers)
            return fused_layers.swiglu_mlp(x, self.w13, self.w2)
        return _proj(self.w2, ops.swiglu(_proj(self.w13, x)))


class TransformerBlock(nn.Module):
    def __init__(self, layer_id: int, args: ModelArgs):
        super().__init__()
        self.layer_id = layer_id
        self.attention = Attention(args)
        self.feed_forward = FeedForward(args.dim, args.ffn_hidden)
        self.attention_norm = ops.RMSNorm(args.dim, eps=args.norm_eps)
        self.ffn_norm = ops.RMSNorm(args.dim, eps=args.norm_eps)
        if args.depth_init:
            self.weight_init_std = 0.02 / (2 * (layer_id + 1)) ** 0.5
        else:
            self.weight_init_std = 0.02 / (2 * args.n_layers) ** 0.5

    def init_weights(self):
        self.attention_norm.reset_parameters()
        self.ffn_norm.reset_parameters()
        self.attention.init_weights(self.weight_init_std)
        self.feed_forward.init_weights(self.weight_init_std)

    def forward(self, x: torch.Tensor, delta: Optional[torch.Tensor] = None, cache: Optional["KVCache"] = None):
        """Takes the residual stream as (x, delta) with x + delta = reference block input and returns
        (h, ffn_out) with h + ffn_out = reference block output (the final add is deferred into the next
        norm).  ``forward(x)`` with delta None is the plain reference input; ``cache`` selects the serving path."""
        att, ff = self.attention, self.feed_forward
        if cache is not None and decode_ops.fused_decode_ok(x, self.attention_norm, self.ffn_norm, att.wqkv, ff.w13):
            # batch-1 decode: the norms (and SwiGLU where the GEMV covers w2's width) are computed inside the
            # projection kernels (one launch each instead of two; decode_ops.gemv_rmsnorm / gemv_swiglu)
            qkv, r = decode_ops.gemv_rmsnorm(x, delta, self.attention_norm.weight, self.attention_norm.eps,
                                             att.wqkv.weight)
            attn = att.decode_from_qkv(qkv, cache, self.layer_id)
            f13, h = decode_ops.gemv_rmsnorm(r, attn, self.ffn_norm.weight, self.ffn_norm.eps, ff.w13.weight)
            if decode_ops.fused_decode_ok(f13[..., : ff.w2.weight.shape[1]], ff.w2):
                return h, decode_ops.gemv_swiglu(f13, ff.w2.weight)
            return h, _proj(ff.w2, ops.swiglu(f13))
        if delta is None:
            r, a = x, self.attention_norm(x)
        else:
            r, a = self.attention_norm(x, delta)
        attn = self.attention(a) if cache is None else self.attention(a, cache=cache, layer=self.layer_id)
        h, f = self.ffn_norm(r, attn)
        return h, self.feed_forward(f)


class Transformer(nn.Module):
    def __init__(self, args: ModelArgs):
        super().__init__()
        assert args.vocab_size > 0, "vocab_size must be set"
        self.model_args = args
        self.vocab_size = args.vocab_size
        self.n_layers = args.n_layers
        self.tok_embeddings = ops.Embedding(args.vocab_size, args.dim)
        # set by parallel.tensor_parallel.parallelize_llama
        self.tp_group = None
        self.sequence_parallel = False
        self.loss_parallel = False
        self.layers = nn.ModuleList([TransformerBlock(i, args) for i in range(args.n_layers)])
        self.norm = ops.RMSNorm(args.dim, eps=args.norm_eps)
        self.output = nn.Linear(args.dim, args.vocab_size, bias=False)
        # the LM head stays bf16 in FP8-GEMM mode (ops/fp8.py): its logits feed the loss directly
        self.output.weight._dph_fp8_exempt = True
        self.init_weights()

    @classmethod
    def from_model_args(cls, args: ModelArgs) -> "Transformer":
        return cls(args)

    @torch.no_grad()
    def init_weights(self):
        nn.init.normal_(self.tok_embeddings.weight)
        for layer in self.layers:
            layer.init_weights()
        self.norm.reset_parameters()
        std = self.model_args.dim ** -0.5
        nn.init.trunc_normal_(self.output.weight, mean=0.0, std=std, a=-3 * std, b=3 * std)

    def embed(self, tokens: torch.Tensor) -> torch.Tensor:
        return self.tok_embeddings(tokens)

    def head(self, h: torch.Tensor, delta: Optional[torch.Tensor], targets: Optional[torch.Tensor] = None):
        if delta is None:
            x = self.norm(h)
        else:
            _, x = self.norm(h, delta)
        logits = _proj(self.output, x)
        if self.loss_parallel and self.tp_group is not None:
            # vocab-sharded logits [B, S, V/tp] ("loss parallel", no [B, S, V] all-gather)
            vloc = logits.shape[-1]
            vstart = torch.distributed.get_rank(self.tp_group) * vloc
            if targets is None:
                from ..comm.functional import gather_replicated_along_dim

                return gather_replicated_along_dim(logits, logits.dim() - 1, self.tp_group).float()
            return ops.vocab_parallel_cross_entropy(logits.reshape(-1, vloc), targets.reshape(-1), vstart,
                                                    self.tp_group)
        if targets is None:
            return logits.float()
        return ops.fused_cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1))

    def forward(self, tokens: torch.Tensor, targets: Optional[torch.Tensor] = None):
        """tokens [B, S] -> fp32 logits [B, S, V]; with ``targets`` -> scalar mean cross-entropy."""
        h, delta = self.embed(tokens), None
        for layer in self.layers:
            h, delta = layer(h, delta)
        return self.head(h, delta, targets)

    @torch.no_grad()
    def forward_inference(self, tokens: torch.Tensor, cache: "KVCache", last_only: bool = True) -> torch.Tensor:
        """Incremental forward for serving: tokens [B, S] continue each sequence of ``cache`` (prefill: S = prompt
        length on an empty cache; decode: S = 1).  Returns fp32 logits of the last position [B, V] (or of every new
        position [B, S, V]) and advances the cache by S."""
        s = tokens.shape[1]
        if cache.lengths is not None and max(cache.lengths) + s > cache.max_len:
            raise ValueError(f"KV cache full: {max(cache.lengths)} + {s} tokens > capacity {cache.max_len}")
        h, delta = self.embed(tokens), None
        for layer in self.layers:
            h, delta = layer(h, delta, cache=cache)
        if last_only and s > 1:
            h = h[:, -1:].contiguous()
            delta = delta[:, -1:].contiguous() if delta is not None else None
        if not (self.loss_parallel and self.tp_group is not None) and decode_ops.fused_decode_ok(h, self.norm,
                                                                                                  self.output):
            logits = decode_ops.gemv_rmsnorm(h, delta, self.norm.weight, self.norm.eps, self.output.weight)[0].float()
        else:
            logits = self.head(h, delta)
        cache.advance(s)
        return logits[:, -1] if last_only else logits


class KVCache:
    """Per-layer key / value cache of a Transformer for incremental decoding (serving; the reference model is
    training-only).  ``k`` / ``v``: [n_layers, B, max_len, Hkv_local, head_dim]; ``pos``: int32 [B] device tensor =
    tokens cached per sequence, read by the kernels (a captured decode graph advances it on the device alone).
    ``lengths`` mirrors pos on the host while it is known (None inside / after graph replays that the owner
    tracks itself).  ``slot(i)`` is a view of sequence i (prefill of prompts of different lengths).
    ``dtype=torch.float8_e4m3fn`` stores OCP e4m3 keys / values (value / ``kv_scale``): half the cache bytes.
    Sized for HBM: 7B at 4 096 tokens is 2 GiB per sequence in bf16."""

    def __init__(self, model: "Transformer", batch: int, max_len: int, device=None, dtype: torch.dtype | None = None,
                 kv_scale: float = 1.0):
        args = model.model_args
        attn = model.layers[0].attention if len(model.layers) else None
        hkv = attn.n_local_kv_heads if attn is not None else args.kv_heads
        ref = next(model.parameters())
        device = ref.device if device is None else torch.device(device)
        dtype = ref.dtype if dtype is None else dtype
        if max_len > 2 * args.max_seq_len:
            raise ValueError(f"max_len {max_len} exceeds the RoPE table ({2 * args.max_seq_len} positions)")
        n_layers = max((layer.layer_id for layer in model.layers), default=-1) + 1   # pipeline stages keep ids
        shape = (n_layers, batch, max_len, hkv, args.head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        self.pos = torch.zeros(batch, dtype=torch.int32, device=device)
        self.batch, self.max_len = batch, max_len
        # dtype torch.float8_e4m3fn: OCP e4m3 entries holding key / kv_scale (half the bytes of bf16; decode is
        # bound by the cache read at large batch / long context)
        self.fp8 = dtype == decode_ops.FP8_KV
        self.kv_scale = float(kv_scale)
        self.lengths: Optional[list] = [0] * batch
        self._parent, self._index = None, None

    @property
    def length(self) -> Optional[int]:
        """The common length of every sequence when known on the host, else None."""
        if self.lengths is None or len(set(self.lengths)) != 1:
            return None
        return self.lengths[0]

    def attn_bound(self) -> int:
        """Upper bound of pos + 1 over the batch for the decode kernel's launch (the capacity when unknown)."""
        return self.max_len if self.lengths is None else min(max(self.lengths) + 1, self.max_len)

    def advance(self, n: int) -> None:
        self.pos.add_(n)
        if self.lengths is not None:
            self.lengths = [x + n for x in self.lengths]
        if self._parent is not None and self._parent.lengths is not None:
            self._parent.lengths[self._index] += n

    def reset(self) -> None:
        self.pos.zero_()
        self.lengths = [0] * self.batch

    def reset_slot(self, i: int) -> None:
        """Empty sequence slot i (continuous batching: a finished sequence's slot takes the next request)."""
        self.pos[i] = 0
        if self.lengths is not None:
            self.lengths[i] = 0

    def slot(self, i: int) -> "KVCache":
        view = object.__new__(KVCache)
        view.k, view.v, view.pos = self.k[:, i:i + 1], self.v[:, i:i + 1], self.pos[i:i + 1]
        view.batch, view.max_len = 1, self.max_len
        view.fp8, view.kv_scale = self.fp8, self.kv_scale
        view.lengths = None if self.lengths is None else [self.lengths[i]]
        view._parent, view._index = self, i
        return view


def build_llama(args: ModelArgs | str, device=None, dtype: torch.dtype = torch.bfloat16, seed: int = 0,
                **overrides) -> Transformer:
    """Construct and initialise directly on ``device`` (fast for 7B on a GPU), then cast to ``dtype``.

    Models whose fp32 copy would not fit beside the cast (more than 16 B parameters, e.g. 70B: 276 GB fp32) are
    built and initialised in ``dtype`` directly instead -- the same distributions, drawn in the lower precision."""
    if isinstance(args, str):
        args = get_preset(args, **overrides)
    elif overrides:
        args = replace(args, **overrides)
    torch.manual_seed(seed)
    direct = args.num_params() > 16e9 and dtype != torch.float32
    old = torch.get_default_dtype()
    if direct:
        torch.set_default_dtype(dtype)
    try:
        with torch.device(device if device is not None else "cpu"):
            model = Transformer(args)
    finally:
        torch.set_default_dtype(old)
    return model.to(dtype)


def convert_reference_state_dict(sd: dict, args: ModelArgs) -> dict:
    """Map a reference llama2_model.Transformer state dict (wq/wk/wv, w1/w3, freqs_cis) to this layout."""
    out = {}
    for k, v in sd.items():
        if k == "freqs_cis":
            continue
        if ".attention.wq." in k:
            base = k.replace(".wq.", ".")
            out[base.replace(".attention.", ".attention.wqkv.")] = torch.cat(
                [v, sd[k.replace(".wq.", ".wk.")], sd[k.replace(".wq.", ".wv.")]], 0)
        elif ".attention.wk." in k or ".attention.wv." in k:
            continue
        elif ".feed_forward.w1." in k:
            out[k.replace(".w1.", ".w13.")] = torch.cat([v, sd[k.replace(".w1.", ".w3.")]], 0)
        elif ".feed_forward.w3." in k:
            continue
        else:
            out[k] = v
    return out
