"""Weights-only checkpoint loading (models/checkpoint.py) and the endpoint's
tokenizer path, on synthetic checkpoints written here (no downloads).

The name mapping is pinned against an independent implementation:
transformers' ``LlamaForCausalLM`` (random-init, saved with
``save_pretrained``) computes logits on the CPU in fp32; our loader maps the
same safetensors file into ``TinyLlama`` and ``reference_logits`` (the fp32
mirror of the HIP path) must agree. The GPU test runs the fused decode
kernels on the loaded weights."""
import http.client
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from p2p_llm_tunnel_amd.models.checkpoint import Tokenizer, load_llama, read_config

MICRO = dict(vocab_size=4096, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
             num_key_value_heads=2, head_dim=64, max_position_embeddings=512, rms_norm_eps=1e-5, rope_theta=10000.0)


def _hf_checkpoint(path, tie=False, seed=0):
    """A random transformers Llama saved as safetensors, weights rounded to bf16
    (our storage dtype) so both sides compute with identical weights."""
    transformers = pytest.importorskip("transformers")
    cfg = transformers.LlamaConfig(**MICRO, tie_word_embeddings=tie)
    torch.manual_seed(seed)
    m = transformers.LlamaForCausalLM(cfg).eval()
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0, 0.05) if p.dim() > 1 else p.uniform_(0.8, 1.2)
            p.copy_(p.to(torch.bfloat16).float())
    m.save_pretrained(path, safe_serialization=True)
    return m


def _hf_logits(m, seqs):
    with torch.no_grad():
        return m(seqs).logits[:, -1].float()


@pytest.mark.parametrize("tie", [False, True])
def test_loader_matches_transformers_llama(tmp_path, tie):
    m = _hf_checkpoint(str(tmp_path), tie=tie)
    ours = load_llama(str(tmp_path), device="cpu", max_batch=2)
    c = ours.cfg
    assert (c.vocab, c.dim, c.n_layers, c.n_heads, c.n_kv_heads, c.head_dim, c.ffn) == (4096, 256, 2, 4, 2, 64, 512)
    assert c.max_seq == 512 and c.rope_theta == 10000.0
    if tie:
        assert ours.lm_head is ours.embed
    torch.manual_seed(3)
    seqs = torch.randint(0, c.vocab, (2, 29))
    ref = ours.reference_logits(seqs)
    hf = _hf_logits(m, seqs)
    scale = hf.abs().max().item()
    # reference_logits rounds activations to bf16 where the kernels store them;
    # transformers stays fp32: agreement to bf16 accuracy.
    assert (ref - hf).abs().max().item() < 0.03 * scale
    assert torch.nn.functional.cosine_similarity(ref, hf, dim=-1).min().item() > 0.999


def test_sharded_index_and_mapping(tmp_path):
    """Index-sharded checkpoint written by hand; tied embeddings; q/k/v and
    gate/up land in the fused row order; wrong shapes and unsupported configs
    are refused with a message."""
    H, Hkv, D, dim, ffn, V, L = 4, 2, 64, 256, 512, 512, 2
    g = torch.Generator().manual_seed(0)

    def r(*s):
        return torch.randn(*s, generator=g).to(torch.bfloat16)
    ts = {"model.embed_tokens.weight": r(V, dim), "model.norm.weight": r(dim)}
    for i in range(L):
        p = f"model.layers.{i}."
        ts.update({p + "input_layernorm.weight": r(dim), p + "post_attention_layernorm.weight": r(dim),
                   p + "self_attn.q_proj.weight": r(H * D, dim), p + "self_attn.k_proj.weight": r(Hkv * D, dim),
                   p + "self_attn.v_proj.weight": r(Hkv * D, dim), p + "self_attn.o_proj.weight": r(dim, H * D),
                   p + "mlp.gate_proj.weight": r(ffn, dim), p + "mlp.up_proj.weight": r(ffn, dim),
                   p + "mlp.down_proj.weight": r(dim, ffn)})
    names = sorted(ts)
    shards = [names[: len(names) // 2], names[len(names) // 2:]]
    wmap = {}
    for k, part in enumerate(shards):
        fn = f"model-{k + 1:05d}-of-00002.safetensors"
        save_file({n: ts[n] for n in part}, str(tmp_path / fn))
        wmap.update({n: fn for n in part})
    (tmp_path / "model.safetensors.index.json").write_text(json.dumps({"metadata": {}, "weight_map": wmap}))
    conf = {"architectures": ["LlamaForCausalLM"], "vocab_size": V, "hidden_size": dim, "intermediate_size": ffn,
            "num_hidden_layers": L, "num_attention_heads": H, "num_key_value_heads": Hkv,
            "max_position_embeddings": 4096, "rms_norm_eps": 1e-6, "rope_theta": 500000.0}
    (tmp_path / "config.json").write_text(json.dumps(conf))
    m = load_llama(str(tmp_path), device="cpu", max_batch=1, max_seq=128)
    assert m.cfg.max_seq == 128 and m.cfg.eps == 1e-6 and m.cfg.rope_theta == 500000.0 and m.cfg.head_dim == 64
    assert m.lm_head is m.embed  # tie_word_embeddings defaults to true
    L1 = m.layers[1]
    p = "model.layers.1."
    assert torch.equal(L1["wqkv"], torch.cat([ts[p + "self_attn.q_proj.weight"], ts[p + "self_attn.k_proj.weight"],
                                              ts[p + "self_attn.v_proj.weight"]]))
    assert torch.equal(L1["w_gate_up"], torch.cat([ts[p + "mlp.gate_proj.weight"], ts[p + "mlp.up_proj.weight"]]))
    assert torch.equal(L1["wo"], ts[p + "self_attn.o_proj.weight"])
    assert m.k_cache.shape == (2, 2, 128, Hkv, D)

    # refusals: tie off without lm_head, wrong shapes, unsupported rope / activation / arch
    def conf_with(**kw):
        (tmp_path / "config.json").write_text(json.dumps(dict(conf, **kw)))
    conf_with(tie_word_embeddings=False)
    with pytest.raises(KeyError, match="lm_head"):
        load_llama(str(tmp_path), device="cpu", max_seq=64)
    conf_with(intermediate_size=1024)
    with pytest.raises(ValueError, match="shape"):
        load_llama(str(tmp_path), device="cpu", max_seq=64)
    for bad, msg in ((dict(rope_scaling={"rope_type": "llama3", "factor": 8.0}), "rope"),
                     (dict(hidden_act="gelu"), "hidden_act"), (dict(architectures=["GPT2LMHeadModel"]), "architecture"),
                     (dict(attention_bias=True), "bias")):
        conf_with(**bad)
        with pytest.raises(ValueError, match=msg):
            read_config(str(tmp_path))
    conf_with(architectures=["MistralForCausalLM"], sliding_window=256)
    assert read_config(str(tmp_path))[0].max_seq == 256


def _tokenizer_dir(path, eos="</s>"):
    """A small byte-level BPE trained here, with a chat template."""
    from tokenizers import Tokenizer as T, decoders, models, pre_tokenizers, trainers
    tok = T(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    text = ["hello world, the tunnel streams tokens over a data channel",
            "ünïcödé text and emoji 🚀 should round-trip"] * 20
    tok.train_from_iterator(text, trainers.BpeTrainer(vocab_size=400, special_tokens=["<s>", eos],
                                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    tok.save(os.path.join(path, "tokenizer.json"))
    tmpl = ("{{ bos_token }}{% for m in messages %}<|{{ m['role'] }}|>{{ m['content'] }}{{ eos_token }}{% endfor %}"
            "{% if add_generation_prompt %}<|assistant|>{% endif %}")
    with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<s>", "eos_token": {"content": eos}, "chat_template": tmpl}, f)
    return tok


def test_tokenizer_template_and_incremental_decode(tmp_path):
    raw = _tokenizer_dir(str(tmp_path))
    t = Tokenizer(str(tmp_path))
    assert t.eos_ids == {raw.token_to_id("</s>")}
    ids = t.chat([{"role": "user", "content": "hello world"}])
    assert t.tok.decode(ids, skip_special_tokens=False) == "<s><|user|>hello world</s><|assistant|>"
    text = "ünïcödé text and emoji 🚀 should round-trip, the tunnel"
    gen = t.encode(text, special=False)
    d = t.detokenizer(t.encode("hello", special=False))
    pieces = [d.push(i) for i in gen]
    assert "".join(pieces) == text
    # a multi-byte character split over byte tokens is held back, not emitted as U+FFFD
    assert all("�" not in p for p in pieces)


class _FakeModel:
    """next = (31 * token + pos + 7) % vocab (as in test_inference_server)."""

    def __init__(self, vocab, max_seq=256):
        from types import SimpleNamespace
        self.cfg = SimpleNamespace(vocab=vocab, max_seq=max_seq)
        self.device = torch.device("cpu")
        self.scratch_slot = 4

    def decode_step(self, tokens, pos, pos_range, slots=None):
        return (tokens * 31 + pos.to(torch.int64) + 7) % self.cfg.vocab


def test_server_text_and_eos_stop(tmp_path):
    """With a tokenizer the endpoint encodes prompts through the chat template,
    streams detokenised text as JSON-escaped pieces and stops at EOS with
    finish_reason "stop"."""
    from p2p_llm_tunnel_amd.models.server import Engine, start_server
    _tokenizer_dir(str(tmp_path))
    tok = Tokenizer(str(tmp_path))
    V = tok.tok.get_vocab_size()
    msgs = [{"role": "user", "content": "hello world"}]
    prompt = tok.chat(msgs)
    # the fake model's greedy continuation of that prompt
    last, pos, cont = prompt[-1], len(prompt) - 1, []
    for _ in range(12):
        last = (last * 31 + pos + 7) % V
        cont.append(last)
        pos += 1
    stop_at = next(i for i in range(3, 12) if cont[i] not in cont[:i])
    tok.eos_ids = {cont[stop_at]}
    eng = Engine(max_batch=4, model=_FakeModel(V))
    srv, port, _ = start_server(port=0, engine=eng, model_name="ckpt", tokenizer=tok)
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=20)
        want = tok.decode(cont[:stop_at]).rstrip("\ufffd")  # a dangling partial character is never sent
        for stream in (True, False):
            c.request("POST", "/v1/chat/completions",
                      body=json.dumps({"stream": stream, "max_tokens": 12, "messages": msgs}))
            data = c.getresponse().read()
            if stream:
                objs = [json.loads(l[6:]) for l in data.split(b"\n") if l.startswith(b"data: {")]
                text = "".join(o["choices"][0]["delta"].get("content", "") for o in objs)
                reason = objs[-1]["choices"][0]["finish_reason"]
                assert data.rstrip().endswith(b"data: [DONE]")
            else:
                j = json.loads(data)
                text, reason = j["choices"][0]["message"]["content"], j["choices"][0]["finish_reason"]
            assert reason == "stop" and text == want, (stream, text, want)
        # without the EOS in reach: length-limited
        c.request("POST", "/v1/completions", body=json.dumps({"stream": False, "max_tokens": 2, "prompt": "hello"}))
        j = json.loads(c.getresponse().read())
        assert j["choices"][0]["finish_reason"] == "length"
    finally:
        srv.shutdown()
        eng.stop()


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_fused_decode_on_loaded_checkpoint(tmp_path):
    """The fused HIP decode on weights loaded from a transformers-written
    checkpoint agrees with transformers' fp32 forward; the endpoint serves it
    (hipGraph path) with the checkpoint's tokenizer."""
    m = _hf_checkpoint(str(tmp_path))
    _tokenizer_dir(str(tmp_path))
    ours = load_llama(str(tmp_path), device="cuda", max_batch=2, max_seq=256)
    torch.manual_seed(5)
    T = 33
    seqs = torch.randint(0, ours.cfg.vocab, (2, T))
    d = seqs.cuda()
    for p in range(T):
        _, logits = ours.decode_step(d[:, p], torch.full((2,), p, dtype=torch.int32, device="cuda"), (p, p),
                                     return_logits=True)
    hf = _hf_logits(m, seqs)
    scale = hf.abs().max().item()
    assert (logits.float().cpu() - hf).abs().max().item() < 0.05 * scale
    assert torch.nn.functional.cosine_similarity(logits.float().cpu(), hf, dim=-1).min().item() > 0.995

    from p2p_llm_tunnel_amd.models.server import start_server
    srv, port, eng = start_server(port=0, device="cuda:0", max_batch=2, checkpoint=str(tmp_path), max_seq=256)
    try:
        assert eng.use_graph and srv.tok is not None
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        c.request("POST", "/v1/chat/completions", body=json.dumps(
            {"stream": True, "max_tokens": 8, "messages": [{"role": "user", "content": "hello world"}]}))
        r = c.getresponse()
        data = r.read()
        assert r.status == 200 and data.rstrip().endswith(b"data: [DONE]")
        c.request("GET", "/v1/models")
        assert os.path.basename(str(tmp_path)).encode() in c.getresponse().read()
    finally:
        srv.shutdown()
        eng.stop()
