"""Context (sequence) parallelism for long sequences: DeepSpeed-Ulysses and ring attention.

The reference only DOCUMENTS these (docs/guide/08_sequence_parallel.md:41-142, SURVEY.md S-ULY / S-RING, C21/C22);
here they are real, tested implementations on top of the CDNA4 flash-attention kernels:

Ulysses (``UlyssesAttention``): the sequence is sharded over the CP group; before attention one all-to-all
turns [B, S/P, H, D] into [B, S, H/P, D] (heads scattered, sequence gathered), attention runs on the full
sequence for H/P heads, and a second all-to-all restores the sequence sharding.  4 all-to-alls per layer
(q/k/v in, o out) map onto the fully connected xGMI mesh: every pair of GPUs is one hop, all 7 links busy.
Requires heads % P == 0.

Ring (``RingAttention``): each rank keeps its query chunk; K/V chunks rotate around the ring (P-1 hops,
batch_isend_irecv posted BEFORE the local block so the xGMI transfer overlaps the flash kernel).  Blocks are
merged with the online-softmax rule on (o, lse) -- the flash forward kernel emits the log-sum-exp.  Backward
re-runs the ring: per block the flash backward kernel, fed the FINAL (o, lse), yields exact dq/dk/dv
contributions; the next K/V hop is posted before the block's kernel (overlapped like the forward), and the dK/dV
accumulators travel one hop behind their K/V chunk, arriving home after P hops.  With causal
attention and contiguous chunks, block (q_r, kv_j) is full for j < r, causal for j == r, skipped for j > r --
rank P-1 does P blocks of work while rank 0 does one.

Zig-zag layout (``layout="zigzag"``, load-balanced causal): the sequence is cut into 2P chunks and rank r holds
chunks r and 2P-1-r.  Against the K/V of rank j every step costs the same half block: j == r is a causal pass
over the local pair, j < r is (all local queries) x (first K/V chunk, full), j > r is (second query chunk) x (both
K/V chunks, full).  ``shard_sequence`` / ``unshard_sequence`` map tokens to and from the layout, and RoPE uses
each chunk's global positions.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

from .. import ops
from ..comm import functional as cf
from ..ops import _lib
from ..ops.rope import rope_reference


def _ws(g):
    return dist.get_world_size(g) if dist.is_initialized() else 1


def _rank(g):
    return dist.get_rank(g) if dist.is_initialized() else 0


def _split_qkv(qkv, nh, nkv, hd):
    b, s, _ = qkv.shape
    q = qkv[:, :, : nh * hd].view(b, s, nh, hd)
    k = qkv[:, :, nh * hd:(nh + nkv) * hd].view(b, s, nkv, hd)
    v = qkv[:, :, (nh + nkv) * hd:].view(b, s, nkv, hd)
    return q, k, v


# ================================================================================================ Ulysses
class UlyssesAttention:
    def __init__(self, group, causal: bool = True):
        self.group, self.causal = group, causal

    def __call__(self, qkv, cos, sin, nh, nkv, hd):
        p = _ws(self.group)
        assert nh % p == 0 and nkv % p == 0, f"Ulysses needs heads ({nh}, kv {nkv}) divisible by cp={p}"
        b, s_loc, _ = qkv.shape
        # [B, S/P, (H + 2 Hkv) hd] -> [B, S, (H + 2 Hkv) / P * hd]: one all-to-all for q, k and v together, landing
        # directly in the packed layout the fused RoPE + attention kernel reads (comm/functional.py ulysses_qkv)
        packed = cf.ulysses_qkv(qkv.contiguous(), nh, nkv, hd, self.group)
        s = packed.shape[1]
        o = ops.rope_attention(packed, cos, sin, nh // p, nkv // p, hd, causal=self.causal)
        o = o.view(b, s, nh // p, hd)
        o = cf.all_to_all(o, 1, 2, self.group)    # back to [B, S/P, H, D]
        return o.reshape(b, s_loc, nh * hd)


# ================================================================================================ ring
def _attn_fwd_lse(q, k, v, causal, scale):
    """(o, lse) for one block; lse natural-log [B, H, S]."""
    if q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (32, 64, 128):
        return _lib.ops().flash_attn_fwd(q, k, v, scale, causal)
    qf, kf, vf = q.float(), k.float(), v.float()
    hq, hk = q.shape[2], k.shape[2]
    if hq != hk:
        kf, vf = kf.repeat_interleave(hq // hk, 2), vf.repeat_interleave(hq // hk, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * scale
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        mask = torch.arange(sk)[None, :] <= torch.arange(sq)[:, None] + (sk - sq)
        s = s.masked_fill(~mask.to(s.device), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.einsum("bhqk,bkhd->bqhd", torch.exp(s - lse[..., None]), vf)
    return o.to(q.dtype), lse


def _attn_bwd(do, q, k, v, o, lse, causal, scale):
    if q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (32, 64, 128):
        return _lib.ops().flash_attn_bwd(do.contiguous(), q, k, v, o, lse, scale, causal)
    qf, kf, vf, dof, of = (t.float() for t in (q, k, v, do, o))
    hq, hk = q.shape[2], k.shape[2]
    rep = hq // hk
    if rep > 1:
        kf, vf = kf.repeat_interleave(rep, 2), vf.repeat_interleave(rep, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * scale
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        mask = torch.arange(sk)[None, :] <= torch.arange(sq)[:, None] + (sk - sq)
        s = s.masked_fill(~mask.to(s.device), float("-inf"))
    p = torch.exp(s - lse[..., None])
    dv = torch.einsum("bhqk,bqhd->bkhd", p, dof)
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, vf)
    delta = (dof * of).sum(-1).transpose(1, 2)[..., None]
    ds = p * (dp - delta) * scale
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, kf)
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, qf)
    if rep > 1:
        dk = dk.view(*dk.shape[:2], hk, rep, dk.shape[-1]).sum(3)
        dv = dv.view(*dv.shape[:2], hk, rep, dv.shape[-1]).sum(3)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


def _fused_merge_ok(q) -> bool:
    """The flash forward can merge into the ring accumulators in its epilogue (bf16 CUDA operands, native head dim)."""
    return (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (32, 64, 128) and _lib.use_native(q))


def _merge(o, lse, o2, lse2):
    """Online-softmax merge of two partial attentions (fp32 accumulators)."""
    new = torch.logaddexp(lse, lse2)
    w1 = torch.exp(lse - new).transpose(1, 2)[..., None]
    w2 = torch.exp(lse2 - new).transpose(1, 2)[..., None]
    return o * w1 + o2.float() * w2, new


class _Ring:
    """Posts the K/V (and optional dK/dV) transfer to the next rank before the local compute."""

    def __init__(self, group):
        self.group = group
        ranks = dist.get_process_group_ranks(group)
        r = _rank(group)
        p = len(ranks)
        self.next, self.prev = ranks[(r + 1) % p], ranks[(r - 1) % p]

    def start(self, tensors):
        bufs = [torch.empty_like(t) for t in tensors]
        ops_ = []
        for t, b in zip(tensors, bufs):
            ops_.append(dist.P2POp(dist.isend, t.contiguous(), self.next, self.group))
            ops_.append(dist.P2POp(dist.irecv, b, self.prev, self.group))
        return dist.batch_isend_irecv(ops_), bufs


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale, zigzag):
        p, r = _ws(group), _rank(group)
        ring = _Ring(group)
        c = q.shape[1] // 2
        o = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        lse = torch.full((q.shape[0], q.shape[2], q.shape[1]), float("-inf"), dtype=torch.float32, device=q.device)

        fused = _fused_merge_ok(q)

        def accumulate(rows, qb, kb, vb, blk_causal):
            """Fold attention(q[rows], kb, vb) into (o, lse)[rows]: in the flash kernel's epilogue on the GPU (the
            running fp32 output and lse are read-modify-written once per step, no separate merge pass), else the
            eager online-softmax merge."""
            if fused:
                _lib.ops().flash_attn_fwd_merge_(qb, kb, vb, scale, blk_causal, o[:, rows], lse[:, :, rows])
                return
            ob, lb = _attn_fwd_lse(qb, kb, vb, blk_causal, scale)
            o_r, l_r = o[:, rows], lse[:, :, rows]
            new_o, new_l = _merge(o_r, l_r, ob, lb)
            o[:, rows], lse[:, :, rows] = new_o, new_l

        kc, vc = k.contiguous(), v.contiguous()
        for i in range(p):
            j = (r - i) % p                       # owner of the K/V chunk held at step i
            works = bufs = None
            if i < p - 1:
                works, bufs = ring.start([kc, vc])
            allq = slice(0, q.shape[1])
            if not causal:
                accumulate(allq, q, kc, vc, False)
            elif not zigzag:
                if j <= r:
                    accumulate(allq, q, kc, vc, j == r)
            elif j == r:
                accumulate(allq, q, kc, vc, True)
            elif j < r:
                accumulate(allq, q, kc[:, :c], vc[:, :c], False)
            else:
                accumulate(slice(c, 2 * c), q[:, c:], kc, vc, False)
            if works is not None:
                for w in works:
                    w.wait()
                kc, vc = bufs
        out = o.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.group, ctx.causal, ctx.scale, ctx.zigzag = group, causal, scale, zigzag
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, causal, scale, zigzag = ctx.group, ctx.causal, ctx.scale, ctx.zigzag
        p, r = _ws(group), _rank(group)
        ring = _Ring(group)
        c = q.shape[1] // 2
        dq = torch.zeros_like(q, dtype=torch.float32)
        kc, vc = k.contiguous(), v.contiguous()
        dkc = torch.zeros_like(k, dtype=torch.float32)
        dvc = torch.zeros_like(v, dtype=torch.float32)
        for i in range(p):
            j = (r - i) % p
            # K/V for the next step need nothing from this one: post them before the block's backward kernel
            kv_works = kv_next = None
            if i < p - 1:
                kv_works, kv_next = ring.start([kc, vc])
            if not causal or (not zigzag and j <= r) or (zigzag and j == r):
                dq_i, dk_i, dv_i = _attn_bwd(do, q, kc, vc, o, lse, causal and j == r, scale)
                dq += dq_i.float()
                dkc += dk_i.float()
                dvc += dv_i.float()
            elif zigzag and j < r:     # all queries x first K/V chunk
                dq_i, dk_i, dv_i = _attn_bwd(do, q, kc[:, :c], vc[:, :c], o, lse, False, scale)
                dq += dq_i.float()
                dkc[:, :c] += dk_i.float()
                dvc[:, :c] += dv_i.float()
            elif zigzag:               # second query chunk x all K/V
                dq_i, dk_i, dv_i = _attn_bwd(do[:, c:], q[:, c:], kc, vc, o[:, c:], lse[:, :, c:].contiguous(), False,
                                             scale)
                dq[:, c:] += dq_i.float()
                dkc += dk_i.float()
                dvc += dv_i.float()
            # the dK / dV accumulators follow their chunk one hop; after p hops every accumulator is home
            works, (dkc_n, dvc_n) = ring.start([dkc, dvc])
            for w in (kv_works or []) + works:
                w.wait()
            dkc, dvc = dkc_n, dvc_n
            if kv_next is not None:
                kc, vc = kv_next
        return dq.to(q.dtype), dkc.to(k.dtype), dvc.to(v.dtype), None, None, None, None


def ring_attention(q, k, v, group, causal: bool = True, scale: float | None = None, layout: str = "contiguous"):
    """Exact attention over a sequence sharded across ``group``: q/k/v [B, S/P, H, D] in ``layout``
    ("contiguous": rank r holds chunk r; "zigzag": chunks r and 2P-1-r, see ``shard_sequence``)."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if _ws(group) == 1:
        return ops.flash_attention(q, k, v, causal, scale)
    assert layout in ("contiguous", "zigzag")
    if layout == "zigzag":
        assert q.shape[1] % 2 == 0, "zig-zag layout needs an even local sequence length"
    return _RingAttnFn.apply(q, k, v, group, causal, scale, layout == "zigzag")


def zigzag_chunks(rank: int, world: int) -> tuple[int, int]:
    return rank, 2 * world - 1 - rank


def shard_sequence(t: torch.Tensor, group, layout: str = "contiguous", dim: int = 1) -> torch.Tensor:
    """This rank's share of a full-sequence tensor (tokens, targets, activations) for the given layout."""
    p, r = _ws(group), _rank(group)
    if layout == "contiguous":
        return t.chunk(p, dim)[r].contiguous()
    ch = t.chunk(2 * p, dim)
    a, b = zigzag_chunks(r, p)
    return torch.cat([ch[a], ch[b]], dim).contiguous()


def unshard_sequence(parts: list, layout: str = "contiguous", dim: int = 1) -> torch.Tensor:
    """Inverse of ``shard_sequence`` given every rank's share (rank order)."""
    if layout == "contiguous":
        return torch.cat(parts, dim)
    p = len(parts)
    chunks = [None] * (2 * p)
    for r, t in enumerate(parts):
        x, y = t.chunk(2, dim)
        a, b = zigzag_chunks(r, p)
        chunks[a], chunks[b] = x, y
    return torch.cat(chunks, dim)


class RingAttention:
    def __init__(self, group, causal: bool = True, layout: str = "contiguous"):
        self.group, self.causal, self.layout = group, causal, layout

    def _rope(self, x, cos, sin, off):
        if x.is_cuda:
            from ..ops.rope import apply_rope

            return apply_rope(x, cos, sin, off)
        return rope_reference(x, cos, sin, off)

    def __call__(self, qkv, cos, sin, nh, nkv, hd):
        b, s_loc, _ = qkv.shape
        q, k, v = _split_qkv(qkv, nh, nkv, hd)
        p, r = _ws(self.group), _rank(self.group)
        if self.layout == "zigzag":
            c = s_loc // 2
            a, bb = zigzag_chunks(r, p)          # global positions of the two local chunks
            q = torch.cat([self._rope(q[:, :c], cos, sin, a * c), self._rope(q[:, c:], cos, sin, bb * c)], 1)
            k = torch.cat([self._rope(k[:, :c], cos, sin, a * c), self._rope(k[:, c:], cos, sin, bb * c)], 1)
        else:
            off = r * s_loc                       # global position of the local chunk
            q, k = self._rope(q, cos, sin, off), self._rope(k, cos, sin, off)
        o = ring_attention(q, k, v.contiguous(), self.group, self.causal, layout=self.layout)
        return o.reshape(b, s_loc, nh * hd)


def apply_context_parallel(model, cp_group, mode: str = "ulysses", layout: str = "contiguous"):
    """Install Ulysses / ring attention in every Attention module of a models.llama2.Transformer.

    The caller shards tokens and targets with ``shard_sequence(t, cp_group, layout)`` (Ulysses: contiguous;
    ring: contiguous or zigzag) and includes the cp ranks in the gradient data-parallel group (each rank's loss
    is a mean over its local tokens).
    """
    if mode == "ulysses":
        assert layout == "contiguous", "Ulysses gathers the sequence in rank order: contiguous layout only"
    impl = UlyssesAttention(cp_group) if mode == "ulysses" else RingAttention(cp_group, layout=layout)
    for layer in model.layers:
        layer.attention.cp_attention = impl
    model.cp_group = cp_group
    return model
