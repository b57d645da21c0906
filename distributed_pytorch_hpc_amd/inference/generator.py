"""Autoregressive generation for the Llama decoder: prefill, then one HIP-graph replay per generated token.

The reference trains only (its llama2_model.py has no KV cache); this is the serving side of the same model:

    gen = Generator(model, batch=8, max_len=4096)          # KV cache for 8 sequences of up to 4096 tokens
    out = gen.generate(prompts, max_new_tokens=256)        # lists of token ids (prompt + continuation)

* prefill: prompts of one length run as one batched ``forward_inference`` (flash kernel over the new tokens);
  prompts of different lengths are prefilled one sequence at a time into their cache slots (``KVCache.slot``).
* decode: a step is memory-bound (every weight and every cached key / value read once), and launch-bound at small
  batch -- ~10 kernels per layer.  The first decode step runs eagerly (lazy library set-up, allocator warm-up), the
  second captures the step into a HIP graph, every later one is a single replay: the kernels read the token buffer
  and the per-sequence positions from device memory, so nothing in the step depends on the host.
* sampling (greedy, temperature, top-k) runs on the logits outside the graph.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from ..models.llama2 import KVCache, Transformer


class Generator:
    def __init__(self, model: Transformer, batch: int, max_len: int, graphs: Optional[bool] = None,
                 dtype: torch.dtype | None = None, kv_scale: float = 1.0):
        """``dtype``: KV-cache element type (default the model's; ``torch.float8_e4m3fn`` halves the cache bytes)."""
        self.model = model
        self.cache = KVCache(model, batch, max_len, dtype=dtype, kv_scale=kv_scale)
        dev = self.cache.pos.device
        self.device = dev
        if graphs is None:
            # multi-rank (tensor-parallel) steps would capture their RCCL all-reduces: eager unless asked for
            multi = torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size() > 1
            graphs = dev.type == "cuda" and not multi
        self.graphs = bool(graphs)
        if self.graphs and dev.type != "cuda":
            raise ValueError("Generator: HIP graphs need the model on a GPU")
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self._tok = torch.zeros(batch, 1, dtype=torch.long, device=dev)
        self._logits: Optional[torch.Tensor] = None
        self._eager_steps = 0

    @property
    def batch(self) -> int:
        return self.cache.batch

    def reset(self) -> None:
        """Empty the cache (the captured graph stays valid: it reads the positions from the cache)."""
        self.cache.reset()

    # ------------------------------------------------------------------------------------------------ steps
    @torch.no_grad()
    def prefill(self, prompts) -> torch.Tensor:
        """Run the prompts (LongTensor [B, S] or B lists of ids) into an empty cache; returns last logits [B, V]."""
        if isinstance(prompts, torch.Tensor):
            if prompts.shape[0] != self.batch:
                raise ValueError(f"prefill: {prompts.shape[0]} prompts for a cache of {self.batch} sequences")
            return self.model.forward_inference(prompts.to(self.device), self.cache)
        if len(prompts) != self.batch:
            raise ValueError(f"prefill: {len(prompts)} prompts for a cache of {self.batch} sequences")
        if any(len(p) == 0 for p in prompts):
            raise ValueError("prefill: empty prompt")
        if len({len(p) for p in prompts}) == 1:
            return self.prefill(torch.tensor(prompts, dtype=torch.long))
        rows = []
        for i, p in enumerate(prompts):
            ids = torch.tensor([p], dtype=torch.long, device=self.device)
            rows.append(self.model.forward_inference(ids, self.cache.slot(i)))
        return torch.cat(rows, 0)

    @torch.no_grad()
    def decode(self, tokens: torch.Tensor) -> torch.Tensor:
        """Append one token per sequence (LongTensor [B]); returns logits [B, V] (the graph's output buffer when
        graphed: consume it before the next call)."""
        lengths = self.cache.lengths
        if lengths is not None and max(lengths) + 1 > self.cache.max_len:
            raise ValueError(f"KV cache full ({self.cache.max_len} tokens)")
        self._tok.copy_(tokens.view(-1, 1))
        if not self.graphs or self._eager_steps < 1:
            self._eager_steps += 1
            return self.model.forward_inference(self._tok, self.cache)
        if self._graph is None:
            self._capture()
        self._graph.replay()
        # the replay advanced pos on the device; mirror it on the host
        self.cache.lengths = None if lengths is None else [x + 1 for x in lengths]
        return self._logits

    def _capture(self) -> None:
        cache = self.cache
        lengths = cache.lengths
        cache.lengths = None   # the captured step must not bake host lengths in (launch bound = capacity)
        try:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._logits = self.model.forward_inference(self._tok, cache)
        finally:
            cache.lengths = lengths
        self._graph = g

    # ------------------------------------------------------------------------------------------------ loop
    @staticmethod
    def sample(logits: torch.Tensor, temperature: float = 0.0, top_k: Optional[int] = None,
               generator: Optional[torch.Generator] = None) -> torch.Tensor:
        if temperature <= 0.0:
            return logits.argmax(-1)
        x = logits.float() / temperature
        if top_k is not None and top_k < x.shape[-1]:
            kth = torch.topk(x, top_k, dim=-1).values[..., -1:]
            x = x.masked_fill(x < kth, float("-inf"))
        return torch.multinomial(torch.softmax(x, -1), 1, generator=generator).view(-1)

    @torch.no_grad()
    def generate(self, prompts: Sequence[Sequence[int]] | torch.Tensor, max_new_tokens: int,
                 temperature: float = 0.0, top_k: Optional[int] = None, eos_id: Optional[int] = None,
                 generator: Optional[torch.Generator] = None) -> list:
        """Prompts (B lists of ids or LongTensor [B, S]) -> B lists of ids: prompt + up to ``max_new_tokens``."""
        rows = prompts.tolist() if isinstance(prompts, torch.Tensor) else [list(p) for p in prompts]
        longest = max(len(p) for p in rows)
        if longest + max_new_tokens > self.cache.max_len + 1:
            raise ValueError(f"prompt {longest} + {max_new_tokens} new tokens exceed the cache ({self.cache.max_len})")
        self.reset()
        logits = self.prefill(prompts if isinstance(prompts, torch.Tensor) else rows)
        done = [False] * len(rows)
        for step in range(max_new_tokens):
            tok = self.sample(logits, temperature, top_k, generator)
            for i, t in enumerate(tok.tolist()):
                if not done[i]:
                    rows[i].append(t)
                    done[i] = eos_id is not None and t == eos_id
            if all(done) or step == max_new_tokens - 1:
                break
            logits = self.decode(tok)
        return rows


@dataclass
class Request:
    prompt: list
    max_new_tokens: int
    eos_id: Optional[int] = None
    output: list = field(default_factory=list)   # generated ids
    done: bool = False

    def _push(self, tok: int) -> None:
        self.output.append(tok)
        self.done = len(self.output) >= self.max_new_tokens or (self.eos_id is not None and tok == self.eos_id)


class ContinuousBatcher:
    """A stream of requests served on the Generator's fixed cache slots.

    Every ``step()`` admits waiting requests into free slots (per-slot prefill into ``KVCache.slot(i)`` while the
    other sequences keep their caches), then runs ONE decode step for the whole batch -- the same captured HIP graph
    every time, since positions live on the device -- and samples the next token of every active sequence.  A
    sequence that reaches its eos or token budget frees its slot for the next request on the following step.  Idle
    slots decode garbage that is never read; their position is reset each step so they never fill up.

        cb = ContinuousBatcher(Generator(model, batch=8, max_len=4096))
        for p in prompts: cb.submit(p, max_new_tokens=128)
        finished = cb.run()
    """

    def __init__(self, generator: Generator, temperature: float = 0.0, top_k: Optional[int] = None,
                 rng: Optional[torch.Generator] = None):
        self.gen = generator
        self.temperature, self.top_k, self.rng = temperature, top_k, rng
        self.slots: list = [None] * generator.batch
        self.queue: list = []
        self._next = torch.zeros(generator.batch, dtype=torch.long, device=generator.device)
        generator.reset()

    def submit(self, prompt: Sequence[int], max_new_tokens: int, eos_id: Optional[int] = None) -> Request:
        if not prompt or max_new_tokens < 1:
            raise ValueError("ContinuousBatcher: empty prompt or no tokens requested")
        if len(prompt) + max_new_tokens > self.gen.cache.max_len + 1:
            raise ValueError(f"request of {len(prompt)} + {max_new_tokens} tokens exceeds the cache "
                             f"({self.gen.cache.max_len})")
        r = Request(list(prompt), max_new_tokens, eos_id)
        self.queue.append(r)
        return r

    @property
    def active(self) -> int:
        return sum(r is not None for r in self.slots)

    @torch.no_grad()
    def step(self) -> list:
        """Admit, decode one token for every active sequence; returns the requests finished in this step."""
        cache, finished = self.gen.cache, []
        for i in range(len(self.slots)):
            if self.slots[i] is None and self.queue:
                r = self.queue.pop(0)
                cache.reset_slot(i)
                ids = torch.tensor([r.prompt], dtype=torch.long, device=self.gen.device)
                logits = self.gen.model.forward_inference(ids, cache.slot(i))
                tok = int(Generator.sample(logits, self.temperature, self.top_k, self.rng)[0])
                r._push(tok)
                if r.done:
                    finished.append(r)
                else:
                    self.slots[i] = r
                    self._next[i] = tok
        if self.active == 0:
            return finished
        for i, r in enumerate(self.slots):
            if r is None:
                cache.reset_slot(i)
        logits = self.gen.decode(self._next)
        toks = Generator.sample(logits, self.temperature, self.top_k, self.rng)
        self._next.copy_(toks)
        for i, t in enumerate(toks.tolist()):
            r = self.slots[i]
            if r is None:
                continue
            r._push(t)
            if r.done:
                finished.append(r)
                self.slots[i] = None
        return finished

    def run(self) -> list:
        """Serve until the queue is empty and every slot is idle; returns the requests in completion order."""
        out = []
        while self.queue or self.active:
            out.extend(self.step())
        return out
