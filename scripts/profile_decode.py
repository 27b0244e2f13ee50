"""Decode-step microbenchmark of the on-node inference upstream (for rocprofv3).

    python scripts/profile_decode.py --config tiny --batch 8 --ctx 1024 --steps 50 [--eager]

Fills the KV cache with random values up to `ctx`, then times `steps`
batched decode steps through the HIP kernels — replayed from a captured
hipGraph by default, or launched eagerly with --eager; the fused step
(decode_fused.hip) by default, the unfused kernels + hipBLASLt with
--unfused — and prints tokens/s.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2p_llm_tunnel_amd.models.tiny_llm import CONFIGS, TinyLlama  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--unfused", action="store_true", help="kernels.hip + hipBLASLt path instead of decode_fused.hip")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=INT",
                    help="override a field of --config (e.g. --set n_layers=2 --set vocab=8000)")
    ap.add_argument("--checkpoint", default=None, help="load this HF Llama checkpoint instead of a random --config")
    ap.add_argument("--loop", action="store_true",
                    help="device-side autoregression: one graph = the fused step (ids feed the next step's "
                         "tokens in place) + pos += 1, no host copies per step")
    a = ap.parse_args()
    if a.checkpoint:
        from p2p_llm_tunnel_amd.models.checkpoint import load_llama
        m = load_llama(a.checkpoint, device="cuda", max_batch=a.batch, fused=not a.unfused)
        a.config = os.path.basename(os.path.normpath(a.checkpoint))
    else:
        cfg = CONFIGS[a.config]
        if a.set:
            cfg = dataclasses.replace(cfg, **{k: int(v) for k, v in (x.split("=", 1) for x in a.set)})
            a.config += "[" + ",".join(a.set) + "]"
        m = TinyLlama(cfg, device="cuda", max_batch=a.batch, fused=not a.unfused)
    m.k_cache.normal_()
    m.v_cache.normal_()
    if a.loop:
        return loop(m, a)
    if not a.eager:
        m.capture_graph(rows=a.batch)
    B = a.batch
    tok = torch.randint(0, m.cfg.vocab, (B,), device="cuda")

    def step(q):
        p = torch.full((B,), q, dtype=torch.int32, device="cuda")
        return m.decode_step(tok, p, (q, q)) if a.eager else m.graph_step(tok, p)

    for i in range(a.warmup):
        tok = step(a.ctx + i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tok = step(a.ctx + a.warmup + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"config": a.config, "batch": B, "ctx": a.ctx, "steps": a.steps, "graph": not a.eager, "fused": not a.unfused,
                      "ms_per_step": dt * 1e3 / a.steps, "tokens_per_s": B * a.steps / dt}))


def loop(m, a):
    """The decode step as the only work in the graph: the step's ids buffer is
    the next step's token buffer and a pos += 1 kernel follows it, so a replay
    is the fused kernels plus one tiny elementwise kernel."""
    B, c = a.batch, m.cfg
    dec = m.fused_decoder()
    tok = torch.randint(0, c.vocab, (B,), device="cuda")
    pos = torch.full((B,), a.ctx, dtype=torch.int32, device="cuda")
    logits = torch.empty(B, c.vocab, dtype=torch.bfloat16, device="cuda")

    def body():
        dec.step(tok, pos, c.max_seq, logits, tok, None, 0)
        pos.add_(1)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    pos.fill_(a.ctx)
    for _ in range(a.warmup):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nbytes = sum(t.numel() * t.element_size() for t in dec.weights[2:]) + m.embed.shape[1] * 2 * B
    print(json.dumps({"config": a.config, "batch": B, "ctx": a.ctx, "steps": a.steps, "graph": True, "loop": True,
                      "ms_per_step": dt * 1e3 / a.steps, "tokens_per_s": B * a.steps / dt,
                      "weight_TBps": nbytes / (dt / a.steps) / 1e12}))


if __name__ == "__main__":
    main()
