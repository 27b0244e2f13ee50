"""Decode-step microbenchmark of the on-node inference upstream (for rocprofv3).

    python scripts/profile_decode.py --config tiny --batch 8 --ctx 1024 --steps 50

Prefills `ctx` positions by writing random KV (fast path), then times
`steps` batched decode steps through the HIP kernels and prints tokens/s.
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
    a = ap.parse_args()
    m = TinyLlama(a.config, device="cuda", max_batch=a.batch)
    m.k_cache.normal_()
    m.v_cache.normal_()
    B = a.batch
    tok = torch.randint(0, m.cfg.vocab, (B,), device="cuda")
    pos0 = a.ctx
    for i in range(a.warmup):
        p = torch.full((B,), pos0 + i, dtype=torch.int32, device="cuda")
        tok = m.decode_step(tok, p, (pos0 + i, pos0 + i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        q = pos0 + a.warmup + i
        p = torch.full((B,), q, dtype=torch.int32, device="cuda")
        tok = m.decode_step(tok, p, (q, q))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"config": a.config, "batch": B, "ctx": a.ctx, "steps": a.steps,
                      "ms_per_step": dt * 1e3 / a.steps, "tokens_per_s": B * a.steps / dt}))


if __name__ == "__main__":
    main()
