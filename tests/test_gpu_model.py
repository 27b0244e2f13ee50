"""The on-node inference upstream: HIP decode vs fp32 reference, and the
GPU endpoint streamed through a real tunnel."""
import http.client
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")


@cuda
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("cfg", ["micro", "tiny"])
def test_decode_matches_fp32_reference(cfg, fused):
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    m = TinyLlama(cfg, device="cuda", max_batch=3, seed=1, fused=fused)
    torch.manual_seed(0)
    T = 37
    seqs = torch.randint(0, m.cfg.vocab, (3, T), device="cuda")
    logits = None
    for p in range(T):
        _, logits = m.decode_step(seqs[:, p], torch.full((3,), p, dtype=torch.int32, device="cuda"), (p, p),
                                  return_logits=True)
    ref = m.reference_logits(seqs)
    err = (logits.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err < 0.05 * scale, (err, scale)
    # top-1 agreement where the reference margin is comfortable
    top2 = ref.topk(2, -1).values
    confident = (top2[:, 0] - top2[:, 1]) > 0.05 * scale
    assert torch.equal(logits.float().argmax(-1)[confident], ref.argmax(-1)[confident])


@cuda
@pytest.mark.parametrize("cfg,B", [("micro", 5), ("tiny", 8), ("small", 2)])
def test_fused_matches_unfused(cfg, B):
    # Same weights, same token stream: the fused 5-kernels-per-layer step and the
    # unfused kernels + hipBLASLt path agree on logits, caches and greedy ids.
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    mf = TinyLlama(cfg, device="cuda", max_batch=B, seed=4, fused=True)
    mu = TinyLlama(cfg, device="cuda", max_batch=B, seed=4, fused=False)
    torch.manual_seed(1)
    T = 70  # crosses a 64-token attention split
    seqs = torch.randint(0, mf.cfg.vocab, (B, T), device="cuda")
    for p in range(T):
        pos = torch.full((B,), p, dtype=torch.int32, device="cuda")
        idf, lf = mf.decode_step(seqs[:, p], pos, (p, p), return_logits=True)
        idu, lu = mu.decode_step(seqs[:, p], pos, (p, p), return_logits=True)
    scale = lu.float().abs().max().item()
    assert (lf.float() - lu.float()).abs().max().item() < 0.03 * scale
    top2 = lu.float().topk(2, -1).values
    confident = (top2[:, 0] - top2[:, 1]) > 0.03 * scale
    assert torch.equal(idf[confident], idu[confident])
    kdiff = (mf.k_cache[:, :B, :T].float() - mu.k_cache[:, :B, :T].float()).abs().max().item()
    assert kdiff < 0.05 * mu.k_cache[:, :B, :T].float().abs().max().item()


@cuda
@pytest.mark.parametrize("cfg,positions", [("micro", [0, 63, 64, 300]),
                                           # head_dim 128: 1024-token workgroup splits, merged across splits
                                           ("small", [3, 1023, 1024, 2500])])
def test_fused_ragged_positions(cfg, positions):
    # Slots at different positions in one step (continuous batching).
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    mf = TinyLlama(cfg, device="cuda", max_batch=4, seed=6, fused=True)
    mu = TinyLlama(cfg, device="cuda", max_batch=4, seed=6, fused=False)
    torch.manual_seed(2)
    mf.k_cache.normal_()
    mf.v_cache.normal_()
    mu.k_cache.copy_(mf.k_cache)
    mu.v_cache.copy_(mf.v_cache)
    toks = torch.randint(0, mf.cfg.vocab, (4,), device="cuda")
    pos = torch.tensor(positions, dtype=torch.int32, device="cuda")
    rng = (min(positions), max(positions))
    _, lf = mf.decode_step(toks, pos, rng, return_logits=True)
    _, lu = mu.decode_step(toks, pos, rng, return_logits=True)
    assert (lf.float() - lu.float()).abs().max().item() < 0.03 * lu.float().abs().max().item()
    # the graph path launches for cache capacity (idle splits exit early)
    mf.k_cache.copy_(mu.k_cache)
    mf.v_cache.copy_(mu.v_cache)
    mf.capture_graph(rows=4)
    mf.k_cache.copy_(mu.k_cache)
    mf.v_cache.copy_(mu.v_cache)
    _, lg = mf.graph_step(toks, pos, return_logits=True)
    assert (lg.float() - lu.float()).abs().max().item() < 0.03 * lu.float().abs().max().item()


@cuda
def test_chunked_prefill_matches_sequential():
    # A prompt fed as 16-row chunks (rows -> one cache slot, causal within the
    # step) next to another sequence's decode row gives the same final logits
    # as feeding it one token per step.
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    m1 = TinyLlama("micro", device="cuda", max_batch=2, seed=7)
    m2 = TinyLlama("micro", device="cuda", max_batch=2, seed=7)
    torch.manual_seed(4)
    T = 37
    prompt = torch.randint(0, m1.cfg.vocab, (T,), device="cuda")
    one = torch.ones(1, dtype=torch.int32, device="cuda")
    for p in range(T):
        _, l1 = m1.decode_step(prompt[p:p + 1], torch.full((1,), p, dtype=torch.int32, device="cuda"), (p, p),
                               return_logits=True, slots=one)
    other = 0
    for c0 in range(0, T, 15):
        c1 = min(c0 + 15, T)
        toks = torch.cat([prompt[c0:c1], torch.tensor([5], device="cuda")])
        pos = torch.tensor(list(range(c0, c1)) + [other], dtype=torch.int32, device="cuda")
        slots = torch.tensor([1] * (c1 - c0) + [0], dtype=torch.int32, device="cuda")
        _, l2 = m2.decode_step(toks, pos, (0, c1 - 1), return_logits=True, slots=slots)
        other += 1
    last = l2[c1 - c0 - 1].float()
    assert (last - l1[0].float()).abs().max().item() <= 1e-6 + 0.01 * l1.float().abs().max().item()
    assert int(last.argmax()) == int(l1[0].float().argmax())


@cuda
def test_engine_batching_is_invisible():
    # Rows are computed independently, so a request's greedy tokens are the
    # same alone and when batched with others (chunked prefill + decode rows).
    from p2p_llm_tunnel_amd.models.server import Engine, Request
    eng = Engine(device="cuda:0", config="micro", max_batch=4)
    try:
        prompts = [list(range(3, 40)), list(b"hello there"), list(range(100, 171)), [7]]
        alone = []
        for pr in prompts:
            r = eng.submit(Request(pr, 9))
            alone.append(list(iter(r.out.get, None)))
        reqs = [eng.submit(Request(pr, 9)) for pr in prompts]
        together = [list(iter(r.out.get, None)) for r in reqs]
        assert all(len(a) == 9 for a in alone)
        assert together == alone
    finally:
        eng.stop()


@cuda
def test_graph_replay_matches_eager():
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    torch.manual_seed(3)
    m = TinyLlama("micro", device="cuda", max_batch=4, seed=2)
    m.k_cache.normal_()
    m.v_cache.normal_()
    m.capture_graph(rows=4)
    toks = torch.randint(0, m.cfg.vocab, (4,), device="cuda")
    pos = torch.tensor([5, 130, 0, 300], dtype=torch.int32, device="cuda")
    kc, vc = m.k_cache.clone(), m.v_cache.clone()
    ids_g, logits_g = m.graph_step(toks, pos, return_logits=True)
    logits_g = logits_g.clone()
    m.k_cache.copy_(kc)
    m.v_cache.copy_(vc)
    ids_e, logits_e = m.decode_step(toks, pos, (0, 300), return_logits=True)
    assert torch.equal(ids_g, ids_e)
    assert (logits_g.float() - logits_e.float()).abs().max().item() < 1e-2


@cuda
def test_gpu_endpoint_through_tunnel():
    from p2p_llm_tunnel_amd.models.server import start_server
    from p2p_llm_tunnel_amd.utils.procs import Tunnel
    srv, port, engine = start_server(device="cuda:0", config="micro", max_batch=4)
    try:
        with Tunnel(f"http://127.0.0.1:{port}", transport=os.environ.get("P2PT_TRANSPORT", "webrtc")) as t:
            outs = []
            for stream in (True, False):
                c = http.client.HTTPConnection("127.0.0.1", t.proxy_port, timeout=60)
                c.request("POST", "/v1/chat/completions",
                          body=json.dumps({"stream": stream, "max_tokens": 6,
                                           "messages": [{"role": "user", "content": "hi there"}]}),
                          headers={"content-type": "application/json"})
                r = c.getresponse()
                assert r.status == 200
                outs.append(r.read())
            events = [l for l in outs[0].split(b"\n") if l.startswith(b"data: ")]
            assert len(events) == 6 + 2 and events[-1] == b"data: [DONE]"
            streamed = "".join(json.loads(e[6:])["choices"][0]["delta"].get("content", "") for e in events[:-1])
            assert streamed == json.loads(outs[1])["choices"][0]["message"]["content"]  # deterministic greedy
    finally:
        engine.stop()
        srv.shutdown()


@cuda
def test_64_row_prefill_chunk_matches_16_row_chunks():
    # One 64-row step (4 MFMA row tiles: a 57-token prompt chunk plus decode
    # rows of other slots) equals the same prompt fed as 16-row chunks; with
    # emit_rows the LM head covers only the leading rows and their ids match.
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    m1 = TinyLlama("micro", device="cuda", max_batch=3, seed=9)
    m2 = TinyLlama("micro", device="cuda", max_batch=3, seed=9)
    torch.manual_seed(5)
    T = 57
    prompt = torch.randint(0, m1.cfg.vocab, (T,), device="cuda")
    two = lambda n: torch.full((n,), 2, dtype=torch.int32, device="cuda")
    for c0 in range(0, T, 16):
        c1 = min(c0 + 16, T)
        ids1, l1 = m1.decode_step(prompt[c0:c1], torch.arange(c0, c1, dtype=torch.int32, device="cuda"), (c0, c1 - 1),
                                  return_logits=True, slots=two(c1 - c0))
    # 64 rows: two decode rows first (slots 0, 1 at position 0), then the chunk, then padding to the scratch slot
    toks = torch.cat([torch.tensor([11, 12], device="cuda"), prompt,
                      torch.zeros(64 - 2 - T, dtype=torch.int64, device="cuda")])
    pos = torch.cat([torch.zeros(2, dtype=torch.int32, device="cuda"), torch.arange(T, dtype=torch.int32, device="cuda"),
                     torch.zeros(64 - 2 - T, dtype=torch.int32, device="cuda")])
    slots = torch.cat([torch.tensor([0, 1], dtype=torch.int32, device="cuda"), two(T),
                       torch.full((64 - 2 - T,), m2.scratch_slot, dtype=torch.int32, device="cuda")])
    ids2, l2 = m2.decode_step(toks, pos, (0, T - 1), return_logits=True, slots=slots)
    ref = l1[-1].float()
    assert (l2[2 + T - 1].float() - ref).abs().max().item() <= 1e-6 + 0.01 * ref.abs().max().item()
    assert int(ids2[2 + T - 1]) == int(ids1[-1])
    # the KV cache written by the 64-row step matches the chunked one
    assert torch.equal(m1.k_cache[:, 2, :T], m2.k_cache[:, 2, :T])
    # emit_rows: LM head on the first rows only; same ids there
    m3 = TinyLlama("micro", device="cuda", max_batch=3, seed=9)
    order = torch.cat([torch.tensor([0, 1, 2 + T - 1], device="cuda"), torch.arange(2, 2 + T - 1, device="cuda"),
                       torch.arange(2 + T, 64, device="cuda")])
    ids3 = m3.decode_step(toks[order], pos[order], (0, T - 1), slots=slots[order], emit_rows=3)
    assert torch.equal(ids3[:3], ids2[order[:3]])
    # both graphs of the engine's pair replay correctly
    m3.capture_graph(rows=16)
    m3.capture_graph(rows=64, emit_rows=3)
    m3.k_cache.zero_()
    m3.v_cache.zero_()
    g = m3.graph_step(toks[order], pos[order], slots[order])
    assert torch.equal(g[:3], ids2[order[:3]])


@cuda
@pytest.mark.parametrize("cfg,B", [("micro", 64), ("small", 40)])
def test_fused_prefill_sized_steps_match_unfused(cfg, B):
    # Steps of more than 16 rows run every GEMM with four 16-row tiles per
    # workgroup sharing each weight fragment (decode_fused.hip RT = 4); they
    # must agree with the unfused kernels + hipBLASLt on the same rows.
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    mf = TinyLlama(cfg, device="cuda", max_batch=B, seed=9, fused=True)
    mu = TinyLlama(cfg, device="cuda", max_batch=B, seed=9, fused=False)
    torch.manual_seed(3)
    T = 6
    seqs = torch.randint(0, mf.cfg.vocab, (B, T), device="cuda")
    for p in range(T):
        pos = torch.full((B,), p, dtype=torch.int32, device="cuda")
        idf, lf = mf.decode_step(seqs[:, p], pos, (p, p), return_logits=True)
        idu, lu = mu.decode_step(seqs[:, p], pos, (p, p), return_logits=True)
    scale = lu.float().abs().max().item()
    assert (lf.float() - lu.float()).abs().max().item() < 0.03 * scale
    top2 = lu.float().topk(2, -1).values
    confident = (top2[:, 0] - top2[:, 1]) > 0.03 * scale
    assert torch.equal(idf[confident], idu[confident])
    kdiff = (mf.k_cache[:, :B, :T].float() - mu.k_cache[:, :B, :T].float()).abs().max().item()
    assert kdiff < 0.05 * mu.k_cache[:, :B, :T].float().abs().max().item()


@cuda
def test_64_row_prefill_chunk_matches_sequential():
    # A 60-token prompt fed as ONE chunk (rows -> one slot, causal within the
    # step) next to 4 other slots' decode rows: 64 rows, the four-tile path.
    from p2p_llm_tunnel_amd.models.tiny_llm import TinyLlama
    m1 = TinyLlama("micro", device="cuda", max_batch=5, seed=11)
    m2 = TinyLlama("micro", device="cuda", max_batch=5, seed=11)
    torch.manual_seed(5)
    T = 60
    prompt = torch.randint(0, m1.cfg.vocab, (T,), device="cuda")
    four = torch.full((1,), 4, dtype=torch.int32, device="cuda")
    for p in range(T):
        _, l1 = m1.decode_step(prompt[p:p + 1], torch.full((1,), p, dtype=torch.int32, device="cuda"), (p, p),
                               return_logits=True, slots=four)
    toks = torch.cat([prompt, torch.tensor([5, 6, 7, 8], device="cuda")])
    pos = torch.tensor(list(range(T)) + [0, 0, 0, 0], dtype=torch.int32, device="cuda")
    slots = torch.tensor([4] * T + [0, 1, 2, 3], dtype=torch.int32, device="cuda")
    _, l2 = m2.decode_step(toks, pos, (0, T - 1), return_logits=True, slots=slots)
    last = l2[T - 1].float()
    assert (last - l1[0].float()).abs().max().item() <= 1e-6 + 0.01 * l1.float().abs().max().item()
    assert int(last.argmax()) == int(l1[0].float().argmax())


@cuda
def test_engine_sampling_on_device():
    """Requests with sampling parameters draw on device inside the captured
    step (ops.sample_): a fixed seed replays the same completion, different
    seeds give different ones, temperature 0 and top_k 1 are the greedy
    tokens bit for bit, and greedy neighbours in the same step are unaffected."""
    from p2p_llm_tunnel_amd.models.server import Engine, Request, Sampling
    eng = Engine(device="cuda:0", config="micro", max_batch=4)
    try:
        pr = list(b"sampling prompt")

        def run(sampling, n=24):
            r = eng.submit(Request(pr, n, sampling=sampling))
            return list(iter(r.out.get, None))

        greedy = run(Sampling())
        assert run(Sampling(temperature=0.0, seed=1)) == greedy
        assert run(Sampling(temperature=1.3, top_k=1, seed=2)) == greedy
        a = run(Sampling(temperature=1.0, top_p=0.95, seed=42))
        assert run(Sampling(temperature=1.0, top_p=0.95, seed=42)) == a  # replayable
        b = run(Sampling(temperature=1.0, top_p=0.95, seed=43))
        assert a != b and a != greedy
        # batched together: a sampled request beside a greedy one
        rs = [eng.submit(Request(pr, 24, sampling=Sampling(temperature=1.0, top_p=0.95, seed=42))),
              eng.submit(Request(pr, 24))]
        both = [list(iter(r.out.get, None)) for r in rs]
        assert both == [a, greedy]
    finally:
        eng.stop()


@cuda
def test_endpoint_honours_and_validates_sampling_parameters():
    from p2p_llm_tunnel_amd.models.server import start_server
    srv, port, engine = start_server(device="cuda:0", config="micro", max_batch=4)
    try:
        def post(path, body):
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
            c.request("POST", path, body=json.dumps(body), headers={"content-type": "application/json"})
            r = c.getresponse()
            return r.status, r.read()

        chat = {"max_tokens": 12, "messages": [{"role": "user", "content": "hi"}]}
        st, greedy = post("/v1/chat/completions", chat)
        assert st == 200
        st, s1 = post("/v1/chat/completions", dict(chat, temperature=0.9, top_p=0.9, top_k=40, seed=7))
        st2, s2 = post("/v1/chat/completions", dict(chat, temperature=0.9, top_p=0.9, top_k=40, seed=7))
        txt = lambda b: json.loads(b)["choices"][0]["message"]["content"]  # noqa: E731
        assert st == st2 == 200 and txt(s1) == txt(s2)  # same seed, same text (ids differ per response)
        assert txt(s1) != txt(greedy)
        st, o1 = post("/api/generate", {"prompt": "hi", "stream": False, "num_predict": 12,
                                        "options": {"temperature": 0.9, "seed": 7}})
        assert st == 200 and json.loads(o1)["done"]
        for bad in ({"temperature": -1}, {"top_p": 0}, {"top_k": 2.5}, {"n": 2}, {"presence_penalty": 0.3},
                    {"logit_bias": {"5": 1}}, {"stop": [7]}):
            st, body = post("/v1/chat/completions", dict(chat, **bad))
            assert st == 400, (bad, body)
        # Stop sequences: every piece of the random-init model starts with " t",
        # so " t" ends a completion before its first token; a sequence that
        # never occurs leaves the completion as it was.
        st, o = post("/v1/chat/completions", dict(chat, stop=" t", stream=False))
        j = json.loads(o)
        assert st == 200 and j["choices"][0]["message"]["content"] == "" and j["choices"][0]["finish_reason"] == "stop"
        st, o = post("/v1/chat/completions", dict(chat, stop=["never-emitted"], stream=False))
        assert st == 200 and json.loads(o)["choices"][0]["finish_reason"] == "length"
        st, _ = post("/api/generate", {"prompt": "hi", "options": {"repeat_penalty": 1.1}})
        assert st == 400
    finally:
        engine.stop()
        srv.shutdown()
