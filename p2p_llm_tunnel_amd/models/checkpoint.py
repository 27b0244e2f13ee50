"""Weights-only loading of Llama-architecture checkpoints (Hugging Face
layout: ``config.json`` + ``model.safetensors`` or sharded
``model-0000k-of-0000n.safetensors`` with ``model.safetensors.index.json``)
into the endpoint's model (``TinyLlama``), plus the checkpoint's tokenizer.

Only safetensors is read — a flat tensor format with no code in it — through
``safetensors.safe_open`` (memory-mapped, one tensor at a time), so loading a
checkpoint executes nothing from the file and never holds the whole
checkpoint in host memory twice.

Name mapping (HF ``LlamaForCausalLM`` → ours, see ``tiny_llm.py``):

=====================================================  ===========================
``model.embed_tokens.weight``                            ``embed``
``model.layers.i.input_layernorm.weight``                ``layers[i]["attn_norm"]``
``...self_attn.{q,k,v}_proj.weight`` (concatenated)      ``layers[i]["wqkv"]``
``...self_attn.o_proj.weight``                           ``layers[i]["wo"]``
``...post_attention_layernorm.weight``                   ``layers[i]["ffn_norm"]``
``...mlp.{gate,up}_proj.weight`` (concatenated)          ``layers[i]["w_gate_up"]``
``...mlp.down_proj.weight``                              ``layers[i]["w_down"]``
``model.norm.weight``                                    ``final_norm``
``lm_head.weight`` (or the embedding when tied)          ``lm_head``
=====================================================  ===========================

HF Llama q/k projections are already laid out for the rotate-half RoPE
convention our kernels use (``reference_logits``), so no head permutation is
needed here; the fused decoder applies its own interleaving at setup.
"""
from __future__ import annotations

import json
import os

import torch

from p2p_llm_tunnel_amd.models.tiny_llm import LlamaConfig, TinyLlama

_SUPPORTED = {"LlamaForCausalLM", "MistralForCausalLM"}


def read_config(path: str, max_seq: int | None = None) -> tuple[LlamaConfig, dict]:
    """LlamaConfig from an HF ``config.json`` (file or checkpoint directory);
    also returns the raw dict (tokenizer ids, tie flag)."""
    f = os.path.join(path, "config.json") if os.path.isdir(path) else path
    with open(f) as fh:
        raw = json.load(fh)
    arch = (raw.get("architectures") or ["LlamaForCausalLM"])[0]
    if arch not in _SUPPORTED:
        raise ValueError(f"unsupported architecture {arch!r} (Llama-style decoders only: {sorted(_SUPPORTED)})")
    # transformers >= 5 writes rope_parameters {rope_theta, rope_type}; older
    # files carry rope_theta (+ rope_scaling) at the top level.
    rope = raw.get("rope_parameters") or raw.get("rope_scaling") or {}
    if rope.get("rope_type", rope.get("type", "default")) != "default":
        raise ValueError(f"rope type {rope.get('rope_type', rope.get('type'))!r} is not supported by the decode kernels")
    theta = rope.get("rope_theta", raw.get("rope_theta", 10000.0))
    if raw.get("hidden_act", "silu") != "silu":
        raise ValueError(f"hidden_act {raw['hidden_act']!r}: only SwiGLU (silu) decoders are supported")
    if raw.get("attention_bias") or raw.get("mlp_bias"):
        raise ValueError("projection biases are not supported by the decode kernels")
    sw = raw.get("sliding_window")
    if sw and raw.get("use_sliding_window", True):  # full attention == sliding attention up to the window
        max_seq = min(int(max_seq or sw), int(sw))
    heads = int(raw["num_attention_heads"])
    dim = int(raw["hidden_size"])
    cfg = LlamaConfig(
        vocab=int(raw["vocab_size"]), dim=dim, n_layers=int(raw["num_hidden_layers"]), n_heads=heads,
        n_kv_heads=int(raw.get("num_key_value_heads", heads)), head_dim=int(raw.get("head_dim") or dim // heads),
        ffn=int(raw["intermediate_size"]),
        max_seq=int(max_seq or min(int(raw.get("max_position_embeddings", 2048)), 8192)),
        eps=float(raw.get("rms_norm_eps", 1e-5)), rope_theta=float(theta))
    return cfg, raw


def _tensor_files(path: str) -> dict[str, str]:
    """tensor name -> safetensors file, for a single or an index-sharded checkpoint."""
    if os.path.isfile(path):
        files = [path]
    else:
        idx = os.path.join(path, "model.safetensors.index.json")
        if os.path.exists(idx):
            with open(idx) as fh:
                index = json.load(fh)["weight_map"]
            return {k: os.path.join(path, v) for k, v in index.items()}
        files = sorted(os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors"))
        if not files:
            raise FileNotFoundError(f"no .safetensors files in {path}")
    from safetensors import safe_open
    out = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as sf:
            for k in sf.keys():
                out[k] = f
    return out


class _Reader:
    """Tensors by name across the checkpoint's files, opened lazily."""

    def __init__(self, path: str):
        from safetensors import safe_open
        self._open = safe_open
        self.where = _tensor_files(path)
        self._handles = {}

    def has(self, name: str) -> bool:
        return name in self.where

    def get(self, name: str) -> torch.Tensor:
        f = self.where.get(name)
        if f is None:
            raise KeyError(f"checkpoint has no tensor {name!r}")
        h = self._handles.get(f)
        if h is None:
            h = self._handles[f] = self._open(f, framework="pt", device="cpu").__enter__()
        return h.get_tensor(name)

    def close(self):
        for h in self._handles.values():
            h.__exit__(None, None, None)
        self._handles.clear()


def load_llama(path: str, device="cuda", max_batch: int = 8, max_seq: int | None = None,
               fused: bool = True, prefix: str = "model.") -> TinyLlama:
    """A TinyLlama with the checkpoint's weights (bf16 on ``device``)."""
    cfg, raw = read_config(path, max_seq)
    c = cfg
    rd = _Reader(path)
    dev = torch.device(device)

    def t(name, shape):
        x = rd.get(name)
        if tuple(x.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(x.shape)} != expected {tuple(shape)}")
        return x.to(torch.bfloat16).to(dev)

    try:
        q_out, kv_out = c.n_heads * c.head_dim, c.n_kv_heads * c.head_dim
        w = {"embed": t(prefix + "embed_tokens.weight", (c.vocab, c.dim)),
             "final_norm": t(prefix + "norm.weight", (c.dim,)), "layers": []}
        if rd.has("lm_head.weight"):
            w["lm_head"] = t("lm_head.weight", (c.vocab, c.dim))
        elif raw.get("tie_word_embeddings", True):
            w["lm_head"] = w["embed"]
        else:
            raise KeyError("checkpoint has no lm_head.weight and does not tie embeddings")
        for i in range(c.n_layers):
            p = f"{prefix}layers.{i}."
            q = t(p + "self_attn.q_proj.weight", (q_out, c.dim))
            k = t(p + "self_attn.k_proj.weight", (kv_out, c.dim))
            v = t(p + "self_attn.v_proj.weight", (kv_out, c.dim))
            if rd.has(p + "self_attn.q_proj.bias"):
                raise ValueError("attention projection biases are not supported by the decode kernels")
            gate = t(p + "mlp.gate_proj.weight", (c.ffn, c.dim))
            up = t(p + "mlp.up_proj.weight", (c.ffn, c.dim))
            w["layers"].append({
                "attn_norm": t(p + "input_layernorm.weight", (c.dim,)),
                "wqkv": torch.cat([q, k, v], 0).contiguous(),
                "wo": t(p + "self_attn.o_proj.weight", (c.dim, q_out)),
                "ffn_norm": t(p + "post_attention_layernorm.weight", (c.dim,)),
                "w_gate_up": torch.cat([gate, up], 0).contiguous(),
                "w_down": t(p + "mlp.down_proj.weight", (c.dim, c.ffn)),
            })
            del q, k, v, gate, up
    finally:
        rd.close()
    return TinyLlama.from_weights(cfg, w, device=dev, max_batch=max_batch, fused=fused)


class Detokenizer:
    """Incremental detokenisation of one generated sequence: ``push(id)``
    returns the text that token adds. Decodes a short window (the tokens since
    the last emitted boundary) rather than the whole sequence, so a token costs
    O(window), and holds text back while it ends in an incomplete UTF-8
    sequence (byte-fallback tokens)."""

    __slots__ = ("tok", "ids", "prefix", "read")

    def __init__(self, tok, prompt_ids: list[int]):
        self.tok = tok
        self.ids = list(prompt_ids[-4:])  # a little context: leading-space rules depend on it
        self.prefix = 0
        self.read = len(self.ids)

    def push(self, tid: int) -> str:
        self.ids.append(tid)
        before = self.tok.decode(self.ids[self.prefix:self.read], skip_special_tokens=True)
        after = self.tok.decode(self.ids[self.prefix:], skip_special_tokens=True)
        if len(after) <= len(before) or after.endswith("\ufffd"):
            return ""
        self.prefix, self.read = self.read, len(self.ids)
        return after[len(before):]


class Tokenizer:
    """The checkpoint's ``tokenizer.json`` (Hugging Face ``tokenizers``: a
    Rust library; the file is data, no code from it runs), its special ids and
    its chat template (``tokenizer_config.json``), rendered in jinja2's
    immutable sandbox."""

    def __init__(self, path: str, eos_ids: list[int] | None = None):
        from tokenizers import Tokenizer as _T
        d = path if os.path.isdir(path) else os.path.dirname(path)
        f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
        self.tok = _T.from_file(f)
        self.eos_ids = set(eos_ids or [])
        self.bos = self.eos = ""
        self.template = None
        tc = os.path.join(d, "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as fh:
                conf = json.load(fh)

            def tokstr(v):
                return v.get("content", "") if isinstance(v, dict) else (v or "")
            self.bos, self.eos = tokstr(conf.get("bos_token")), tokstr(conf.get("eos_token"))
            t = conf.get("chat_template")
            if isinstance(t, list):  # [{name, template}, ...]
                t = next((x["template"] for x in t if x.get("name") == "default"), t[0]["template"] if t else None)
            if t:
                from jinja2.sandbox import ImmutableSandboxedEnvironment

                def fail(msg):
                    raise ValueError(msg)
                env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
                env.globals["raise_exception"] = fail
                self.template = env.from_string(t)
            if self.eos and not self.eos_ids:
                e = self.tok.token_to_id(self.eos)
                if e is not None:
                    self.eos_ids.add(e)

    @classmethod
    def for_checkpoint(cls, path: str) -> "Tokenizer | None":
        f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else None
        if not f or not os.path.exists(f):
            return None
        eos = []
        try:
            _, raw = read_config(path)
            e = raw.get("eos_token_id")
            eos = e if isinstance(e, list) else ([e] if e is not None else [])
        except (OSError, ValueError, KeyError):
            pass
        return cls(path, eos)

    def encode(self, text: str, special: bool = True) -> list[int]:
        return self.tok.encode(text, add_special_tokens=special).ids

    def decode(self, ids: list[int]) -> str:
        return self.tok.decode(ids, skip_special_tokens=True)

    def chat(self, messages: list[dict]) -> list[int]:
        """Prompt ids for a chat: the checkpoint's template with the generation
        prompt appended, or plain ``role: content`` lines without one."""
        msgs = [{"role": str(m.get("role", "user")), "content": str(m.get("content", ""))} for m in messages]
        if self.template is not None:
            text = self.template.render(messages=msgs, add_generation_prompt=True, bos_token=self.bos,
                                        eos_token=self.eos)
            return self.encode(text, special=False)
        return self.encode("".join(f"{m['role']}: {m['content']}\n" for m in msgs) + "assistant:")

    def detokenizer(self, prompt_ids: list[int]) -> Detokenizer:
        return Detokenizer(self.tok, prompt_ids)
