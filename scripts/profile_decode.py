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
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--unfused", action="store_true", help="kernels.hip + hipBLASLt path instead of decode_fused.hip")
    a = ap.parse_args()
    m = TinyLlama(a.config, device="cuda", max_batch=a.batch, fused=not a.unfused)
    m.k_cache.normal_()
    m.v_cache.normal_()
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


if __name__ == "__main__":
    main()
