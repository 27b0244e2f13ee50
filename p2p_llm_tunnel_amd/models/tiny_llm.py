"""Llama-style decoder for the on-node inference upstream.

The tunnel's serve side fronts an OpenAI/Ollama-compatible endpoint running
on the MI355X node (BASELINE.json north star). This module is that
endpoint's model: random-init weights (no checkpoints offline), bf16.

Two decode paths over the same weights and caches:

* fused (default, up to 64 token rows per step): ``ops.FusedLlamaDecoder`` — one
  C++ call launching 5 kernels per layer + 2 (decode_fused.hip: MFMA skinny
  GEMMs with RMSNorm prologues and RoPE/KV-append, SwiGLU, residual and
  argmax epilogues; split-K attention with in-kernel merge);
* unfused: the standalone kernels of kernels.hip (residual+RMSNorm,
  RoPE+KV-append, flash-decoding, SwiGLU, argmax) around hipBLASLt GEMMs
  (``torch.nn.functional.linear``) — kept as the cross-check and for batches
  above 64.

``reference_logits`` recomputes the same network in fp32 PyTorch (full
causal attention over the whole sequence) for numerics tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from p2p_llm_tunnel_amd import ops


@dataclass(frozen=True)
class LlamaConfig:
    vocab: int = 32000
    dim: int = 1024
    n_layers: int = 4
    n_heads: int = 16
    n_kv_heads: int = 4
    head_dim: int = 64
    ffn: int = 2816
    max_seq: int = 2048
    eps: float = 1e-5
    rope_theta: float = 10000.0


CONFIGS = {
    "tiny": LlamaConfig(),
    "micro": LlamaConfig(vocab=4096, dim=256, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, max_seq=512),
    "small": LlamaConfig(vocab=32000, dim=2048, n_layers=8, n_heads=16, n_kv_heads=4, head_dim=128, ffn=5632,
                         max_seq=4096),
}


class TinyLlama:
    def __init__(self, cfg: LlamaConfig | str = "tiny", device="cuda", max_batch: int = 8, seed: int = 0,
                 fused: bool = True, weights: dict | None = None):
        """Random-init weights from ``seed``, or ``weights`` (embed, final_norm,
        lm_head, layers[{attn_norm, wqkv, wo, ffn_norm, w_gate_up, w_down}],
        bf16 on ``device``) — see ``checkpoint.load_llama``."""
        self.cfg = CONFIGS[cfg] if isinstance(cfg, str) else cfg
        self.fused = fused
        self._fused = None
        c = self.cfg
        self.device = torch.device(device)
        self.max_batch = max_batch
        if weights is not None:
            self.embed, self.final_norm, self.lm_head = weights["embed"], weights["final_norm"], weights["lm_head"]
            self.layers = weights["layers"]
            self._alloc_caches()
            return
        g = torch.Generator(device="cpu").manual_seed(seed)

        def w(*shape, scale):
            return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(self.device)

        def norm_w(n):
            return (1.0 + 0.1 * torch.randn(n, generator=g)).to(torch.bfloat16).to(self.device)

        qkv_out = (c.n_heads + 2 * c.n_kv_heads) * c.head_dim
        self.embed = w(c.vocab, c.dim, scale=1.0)
        self.layers = []
        for _ in range(c.n_layers):
            self.layers.append({
                "attn_norm": norm_w(c.dim),
                "wqkv": w(qkv_out, c.dim, scale=1 / math.sqrt(c.dim)),
                "wo": w(c.dim, c.n_heads * c.head_dim, scale=1 / math.sqrt(c.n_heads * c.head_dim)),
                "ffn_norm": norm_w(c.dim),
                "w_gate_up": w(2 * c.ffn, c.dim, scale=1 / math.sqrt(c.dim)),
                "w_down": w(c.dim, c.ffn, scale=1 / math.sqrt(c.ffn)),
            })
        self.final_norm = norm_w(c.dim)
        self.lm_head = w(c.vocab, c.dim, scale=1 / math.sqrt(c.dim))
        self._alloc_caches()

    @classmethod
    def from_weights(cls, cfg: LlamaConfig, weights: dict, device="cuda", max_batch: int = 8, fused: bool = True):
        return cls(cfg, device=device, max_batch=max_batch, fused=fused, weights=weights)

    def _alloc_caches(self):
        c = self.cfg
        # One spare slot (index max_batch) absorbs the K/V writes of padding rows.
        self.scratch_slot = self.max_batch
        cache_shape = (c.n_layers, self.max_batch + 1, c.max_seq, c.n_kv_heads, c.head_dim)
        self.k_cache = torch.zeros(cache_shape, dtype=torch.bfloat16, device=self.device)
        self.v_cache = torch.zeros(cache_shape, dtype=torch.bfloat16, device=self.device)

    # ------------------------------------------------------------------ HIP path
    @torch.no_grad()
    def decode_step(self, tokens: torch.Tensor, pos: torch.Tensor, pos_range: tuple[int, int],
                    return_logits: bool = False, slots: torch.Tensor | None = None, emit_rows: int = 0):
        """One step of token rows. tokens: int64 [B]; pos: int32 [B] (cache position of
        each token); slots: int32 [B] cache slot of each row (default: row b -> slot b).
        With ``slots`` (fused path, B <= 64) several rows may feed one sequence at
        consecutive positions: a causal prefill chunk. ``emit_rows`` > 0: only the
        first rows get ids/logits (fused path; the LM head skips the rest).

        Returns next-token ids (int64 [B]) and optionally the bf16 logits.
        """
        c = self.cfg
        B = tokens.shape[0]
        if slots is None and B > self.max_batch:
            raise ValueError("batch exceeds max_batch")
        if slots is not None and not (self.fused and B <= ops.MAX_ROWS):
            raise ValueError(f"row->slot mapping needs the fused path and at most {ops.MAX_ROWS} rows")
        if pos_range[0] < 0 or pos_range[1] >= c.max_seq:
            raise ValueError("positions out of [0, max_seq)")
        ids, logits = self._decode_impl(tokens, pos, pos_range, pos_range[1] + 1, slots, emit_rows)
        return (ids, logits) if return_logits else ids

    def fused_decoder(self) -> ops.FusedLlamaDecoder:
        if self._fused is None:
            c = self.cfg
            dims = ops.LlamaDims(vocab=c.vocab, dim=c.dim, n_layers=c.n_layers, H=c.n_heads, Hkv=c.n_kv_heads,
                                 D=c.head_dim, ffn=c.ffn, max_seq=c.max_seq, max_batch=self.max_batch + 1, eps=c.eps,
                                 theta=c.rope_theta)
            # The fused GEMMs take the RMSNorm weight folded into the following
            # projection's columns (W[n][k] * g[k]), and QKV / gate-up rows
            # interleaved in pairs so a 16-column tile holds both members of a
            # RoPE pair or a SwiGLU pair; see decode_fused.hip.
            def fold(w, g):
                return (w.float() * g.float()[None, :]).to(torch.bfloat16)

            def pairs(n):  # [0, n, 1, n + 1, ...]
                return torch.stack([torch.arange(n), torch.arange(n) + n], 1).flatten().to(self.device)

            heads = c.n_heads + 2 * c.n_kv_heads
            head_perm = (torch.arange(heads, device=self.device)[:, None] * c.head_dim
                         + pairs(c.head_dim // 2)[None, :]).flatten()
            ws = [self.embed, self.final_norm, fold(self.lm_head, self.final_norm)]
            for L in self.layers:
                ws += [L["attn_norm"], fold(L["wqkv"], L["attn_norm"])[head_perm].contiguous(), L["wo"],
                       L["ffn_norm"], fold(L["w_gate_up"], L["ffn_norm"])[pairs(c.ffn)].contiguous(), L["w_down"]]
            self._fused = ops.FusedLlamaDecoder(dims, ws, self.k_cache, self.v_cache)
        return self._fused

    def _decode_impl(self, tokens, pos, pos_range, max_len, slots=None, emit_rows=0):
        B = tokens.shape[0]
        if self.fused and B <= ops.MAX_ROWS:
            tokens, pos = tokens.contiguous(), pos.contiguous()
            slots = slots.contiguous() if slots is not None else None
            logits = torch.empty(B, self.cfg.vocab, dtype=torch.bfloat16, device=self.device)
            ids = torch.empty(B, dtype=torch.int64, device=self.device)
            self.fused_decoder().step(tokens, pos, max_len, logits, ids, slots, emit_rows)
            return ids, logits
        return self._decode_unfused(tokens, pos, pos_range, max_len)

    def _decode_unfused(self, tokens, pos, pos_range, max_len):
        c = self.cfg
        B = tokens.shape[0]
        lens = pos + 1
        x = self.embed.index_select(0, tokens)
        h = ops.rmsnorm(x, self.layers[0]["attn_norm"], c.eps)
        residual = x
        for i, L in enumerate(self.layers):
            kc, vc = self.k_cache[i, :B], self.v_cache[i, :B]
            qkv = F.linear(h, L["wqkv"])
            q = ops.rope_qkv_cache(qkv, pos, kc, vc, c.n_heads, c.n_kv_heads, c.head_dim, c.rope_theta,
                                   pos_range=pos_range)
            a = ops.decode_attention(q, kc, vc, lens, max_len=max_len)
            o = F.linear(a.view(B, -1), L["wo"])
            h, residual = ops.rmsnorm(o, L["ffn_norm"], c.eps, residual=residual)
            m = F.linear(ops.silu_mul(F.linear(h, L["w_gate_up"])), L["w_down"])
            nxt = self.layers[i + 1]["attn_norm"] if i + 1 < len(self.layers) else self.final_norm
            h, residual = ops.rmsnorm(m, nxt, c.eps, residual=residual)
        logits = F.linear(h, self.lm_head)
        return ops.argmax(logits), logits

    # ------------------------------------------------------------------ hipGraph
    def capture_graph(self, rows: int | None = None, emit_rows: int = 0):
        """Capture one step of ``rows`` token rows into a hipGraph (torch.cuda.CUDAGraph).

        Decode at small batch is bound by kernel count; replaying the captured
        graph removes the per-kernel launch cost. The attention is captured for
        the cache capacity (its splits past each row's length exit immediately),
        so one graph serves every step. Fused path: up to 64 rows with a
        row->slot map (padding rows point at the scratch slot); unfused: one row
        per slot. Several row counts may be captured (e.g. 16 for decode-heavy
        steps, 64 for prefill-heavy ones); ``graph_step`` picks the graph by the
        number of rows it is given. ``emit_rows``: rows that get ids (0: all).
        """
        c = self.cfg
        R = rows or (16 if self.fused else self.max_batch)
        self.graph_rows = R
        g_tok = torch.zeros(R, dtype=torch.int64, device=self.device)
        g_pos = torch.zeros(R, dtype=torch.int32, device=self.device)
        g_slot = (torch.full((R,), self.scratch_slot, dtype=torch.int32, device=self.device)
                  if self.fused else None)
        full = (0, c.max_seq - 1)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(2):  # allocator + GEMM heuristics warm-up outside capture
                self._decode_impl(g_tok, g_pos, full, c.max_seq, g_slot, emit_rows)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(graph):
            g_ids, g_logits = self._decode_impl(g_tok, g_pos, full, c.max_seq, g_slot, emit_rows)
        if not hasattr(self, "_graphs"):
            self._graphs = {}
        self._graphs[R] = (graph, g_tok, g_pos, g_slot, g_ids, g_logits)
        return self

    @torch.no_grad()
    def graph_step(self, tokens: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor | None = None,
                   return_logits: bool = False):
        """Replay the graph captured for ``tokens.shape[0]`` rows. tokens/pos/slots:
        [rows] (slots default to row b -> slot b); positions must be < max_seq."""
        R = tokens.shape[0]
        graph, g_tok, g_pos, g_slot, g_ids, g_logits = self._graphs[R]
        g_tok.copy_(tokens, non_blocking=True)
        g_pos.copy_(pos, non_blocking=True)
        if g_slot is not None:
            if slots is None:
                slots = torch.arange(R, dtype=torch.int32).clamp_(max=self.scratch_slot)
            g_slot.copy_(slots, non_blocking=True)
        graph.replay()
        return (g_ids, g_logits) if return_logits else g_ids

    def cache_views_contiguous(self) -> bool:
        return all(self.k_cache[i, : self.max_batch].is_contiguous() for i in range(self.cfg.n_layers))

    # ------------------------------------------------------------------ fp32 reference
    @torch.no_grad()
    def reference_logits(self, seqs: torch.Tensor) -> torch.Tensor:
        """fp32 forward of full sequences [B, T]; returns logits of the last position [B, V]."""
        c = self.cfg
        B, T = seqs.shape
        f32 = lambda t: t.float()
        x = f32(self.embed)[seqs]  # [B, T, dim]

        def rms(v, wgt):
            return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + c.eps) * f32(wgt)

        def bf(v):  # mirror the bf16 storage points of the HIP path
            return v.to(torch.bfloat16).float()

        pos = torch.arange(T, device=seqs.device, dtype=torch.float32)
        inv_freq = torch.exp2(-math.log2(c.rope_theta) * torch.arange(0, c.head_dim // 2, device=seqs.device,
                                                                      dtype=torch.float32) * 2 / c.head_dim)
        ang = pos[:, None] * inv_freq[None, :]
        cos, sin = torch.cos(ang), torch.sin(ang)

        def rope(t):  # [B, T, nh, D]
            half = c.head_dim // 2
            t1, t2 = t[..., :half], t[..., half:]
            cc, ss = cos[None, :, None, :], sin[None, :, None, :]
            return torch.cat([t1 * cc - t2 * ss, t2 * cc + t1 * ss], -1)

        residual = x
        h = bf(rms(x, self.layers[0]["attn_norm"]))
        G = c.n_heads // c.n_kv_heads
        mask = torch.full((T, T), float("-inf"), device=seqs.device).triu(1)
        for i, L in enumerate(self.layers):
            qkv = bf(h @ f32(L["wqkv"]).T)
            q = qkv[..., : c.n_heads * c.head_dim].view(B, T, c.n_heads, c.head_dim)
            k = qkv[..., c.n_heads * c.head_dim: (c.n_heads + c.n_kv_heads) * c.head_dim].view(
                B, T, c.n_kv_heads, c.head_dim)
            v = qkv[..., (c.n_heads + c.n_kv_heads) * c.head_dim:].view(B, T, c.n_kv_heads, c.head_dim)
            q, k = bf(rope(q)), bf(rope(k))
            k = k.repeat_interleave(G, dim=2)
            v = v.repeat_interleave(G, dim=2)
            s = torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(c.head_dim) + mask
            a = bf(torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v).reshape(B, T, -1))
            o = bf(a @ f32(L["wo"]).T)
            residual = bf(residual + o)
            h = bf(rms(residual, L["ffn_norm"]))
            gu = bf(h @ f32(L["w_gate_up"]).T)
            g_, u_ = gu[..., : c.ffn], gu[..., c.ffn:]
            m = bf(bf(F.silu(g_) * u_) @ f32(L["w_down"]).T)
            residual = bf(residual + m)
            nxt = self.layers[i + 1]["attn_norm"] if i + 1 < len(self.layers) else self.final_norm
            h = bf(rms(residual, nxt))
        return (h[:, -1] @ f32(self.lm_head).T)

    @torch.no_grad()
    def generate(self, prompt: list[int], max_new: int) -> list[int]:
        """Greedy single-sequence generation on slot 0 (prefill = sequential decode steps)."""
        out = []
        tok = None
        for p, t in enumerate(prompt + [None] * max_new):
            if p >= self.cfg.max_seq:
                break
            cur = t if t is not None else tok
            ids = self.decode_step(torch.tensor([cur], device=self.device),
                                   torch.tensor([p], dtype=torch.int32, device=self.device), (p, p))
            tok = int(ids.item())
            if p >= len(prompt) - 1:
                out.append(tok)
                if len(out) >= max_new:
                    break
        return out
