#!/usr/bin/env python3
"""Write a random-weight Hugging Face Llama checkpoint of a real model's shape
(config.json + index-sharded model-*.safetensors), for loading and serving
tests at full size without downloading anything.

    python scripts/make_synthetic_checkpoint.py --shape tinyllama-1.1b --out /tmp/tl11 [--shards 2]

Weights are N(0, 0.02) bf16 (norms ~1), named and shaped as transformers'
LlamaForCausalLM saves them; there is no tokenizer (the endpoint then falls
back to byte-level prompts).
"""
from __future__ import annotations

import argparse
import json
import os

import torch
from safetensors.torch import save_file

SHAPES = {
    # TinyLlama/TinyLlama-1.1B-Chat-v1.0 config.json
    "tinyllama-1.1b": dict(vocab_size=32000, hidden_size=2048, intermediate_size=5632, num_hidden_layers=22,
                           num_attention_heads=32, num_key_value_heads=4, max_position_embeddings=2048,
                           rms_norm_eps=1e-5, rope_theta=10000.0, tie_word_embeddings=False),
    # meta-llama/Llama-3.2-1B shape with a 32000-entry vocabulary (the fused LM head
    # takes vocab % 32 == 0; 128256 also qualifies but makes the file 0.5 GB larger)
    "llama-1b": dict(vocab_size=32000, hidden_size=2048, intermediate_size=8192, num_hidden_layers=16,
                     num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=4096,
                     rms_norm_eps=1e-5, rope_theta=500000.0, tie_word_embeddings=True),
}


def tensors(cfg: dict, seed: int):
    g = torch.Generator().manual_seed(seed)
    d, f, H, Hkv = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_attention_heads"], cfg["num_key_value_heads"]
    D = d // H

    def w(*shape):
        return (torch.randn(*shape, generator=g) * 0.02).to(torch.bfloat16)

    def norm(n):
        return (1.0 + 0.05 * torch.randn(n, generator=g)).to(torch.bfloat16)

    yield "model.embed_tokens.weight", w(cfg["vocab_size"], d)
    for i in range(cfg["num_hidden_layers"]):
        p = f"model.layers.{i}."
        yield p + "input_layernorm.weight", norm(d)
        yield p + "self_attn.q_proj.weight", w(H * D, d)
        yield p + "self_attn.k_proj.weight", w(Hkv * D, d)
        yield p + "self_attn.v_proj.weight", w(Hkv * D, d)
        yield p + "self_attn.o_proj.weight", w(d, H * D)
        yield p + "post_attention_layernorm.weight", norm(d)
        yield p + "mlp.gate_proj.weight", w(f, d)
        yield p + "mlp.up_proj.weight", w(f, d)
        yield p + "mlp.down_proj.weight", w(d, f)
    yield "model.norm.weight", norm(d)
    if not cfg.get("tie_word_embeddings"):
        yield "lm_head.weight", w(cfg["vocab_size"], d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", choices=sorted(SHAPES), default="tinyllama-1.1b")
    ap.add_argument("--out", required=True)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    cfg = dict(SHAPES[a.shape], architectures=["LlamaForCausalLM"], model_type="llama", hidden_act="silu",
               torch_dtype="bfloat16", bos_token_id=1, eos_token_id=2)
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "config.json"), "w") as fh:
        json.dump(cfg, fh, indent=1)
    items = list(tensors(cfg, a.seed))
    total = sum(t.numel() * 2 for _, t in items)
    per = total / a.shards
    shards, cur, size = [], {}, 0
    for name, t in items:
        cur[name] = t
        size += t.numel() * 2
        if size >= per and len(shards) < a.shards - 1:
            shards.append(cur)
            cur, size = {}, 0
    shards.append(cur)
    wmap = {}
    for k, sh in enumerate(shards):
        fn = f"model-{k + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(a.out, fn), metadata={"format": "pt"})
        wmap.update({n: fn for n in sh})
    with open(os.path.join(a.out, "model.safetensors.index.json"), "w") as fh:
        json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, fh)
    print(json.dumps({"out": a.out, "shape": a.shape, "params": total // 2, "bytes": total, "shards": len(shards)}))


if __name__ == "__main__":
    main()
