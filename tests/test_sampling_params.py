"""Sampling parameters of the inference endpoint (models/server.py), CPU side:
OpenAI fields (temperature, top_p, seed, the top_k extension) and Ollama
"options" are parsed and range-checked; parameters that would change the
output but are not implemented are refused with 400 instead of being ignored.
Stop sequences (OpenAI "stop", Ollama "options.stop") end a completion at the
first match in its text, streamed or not.
The on-device sampler itself is tested on the GPU (tests/test_gpu_ops.py,
tests/test_gpu_model.py)."""
import http.client
import json

import pytest

from p2p_llm_tunnel_amd.models.server import (Engine, SamplingError, StopMatcher, sampling_params, start_server,
                                              stop_sequences)
from tests.test_inference_server import FakeModel, expected


def test_defaults_are_greedy():
    s = sampling_params({}, False)
    assert s.greedy and s.temperature == 0 and s.top_k == 0 and s.top_p == 1
    assert sampling_params({}, False, default_temperature=0.8).temperature == 0.8
    assert sampling_params({"options": None}, True).greedy


def test_openai_and_ollama_fields():
    s = sampling_params({"temperature": 0.7, "top_p": 0.9, "top_k": 40, "seed": 5}, False)
    assert (s.temperature, s.top_p, s.top_k, s.seed) == (0.7, 0.9, 40, 5) and not s.greedy
    o = sampling_params({"options": {"temperature": 1.2, "top_k": 10, "top_p": 0.5, "seed": 9, "num_ctx": 4096}}, True)
    assert (o.temperature, o.top_k, o.top_p, o.seed) == (1.2, 10, 0.5, 9)
    assert sampling_params({"temperature": 2, "top_k": 1}, False).greedy  # top-1 is argmax
    # the sampler's column: float32 bits of T, k, bits of p, seed, counter
    col = s.column(3)
    assert col[1] == 40 and col[3] == 5 and col[4] == 3
    # unseeded requests get distinct random seeds
    assert sampling_params({"temperature": 1}, False).seed != sampling_params({"temperature": 1}, False).seed


@pytest.mark.parametrize("body,ollama", [
    ({"temperature": -0.1}, False), ({"temperature": "hot"}, False), ({"top_p": 0}, False), ({"top_p": 1.5}, False),
    ({"top_k": -1}, False), ({"top_k": 3.5}, False), ({"seed": "x"}, False), ({"n": 2}, False),
    ({"best_of": 3}, False), ({"presence_penalty": 0.5}, False), ({"frequency_penalty": -1}, False),
    ({"logprobs": True}, False), ({"top_logprobs": 2}, False), ({"logit_bias": {"1": 5}}, False),
    ({"options": {"repeat_penalty": 1.1}}, True), ({"options": {"mirostat": 2}}, True),
    ({"options": {"min_p": 0.05}}, True), ({"options": "hot"}, True),
    ({"options": {"temperature": 500}}, True),
])
def test_unsupported_or_out_of_range_is_refused(body, ollama):
    with pytest.raises(SamplingError):
        sampling_params(body, ollama)


def test_neutral_values_pass():
    sampling_params({"n": 1, "presence_penalty": 0, "frequency_penalty": 0.0, "logprobs": False, "logit_bias": {},
                     "stop": [], "best_of": 1}, False)
    sampling_params({"options": {"repeat_penalty": 1.0, "mirostat": 0, "min_p": 0.0, "typical_p": 1.0}}, True)


def test_http_400_names_the_parameter():
    eng = Engine(max_batch=4, model=FakeModel())
    srv, port, _ = start_server(port=0, engine=eng, model_name="fake")
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        c.request("POST", "/v1/chat/completions", body=json.dumps({"messages": [], "presence_penalty": 0.4}))
        r = c.getresponse()
        body = json.loads(r.read())
        assert r.status == 400 and r.reason == "Bad Request" and "presence_penalty" in body["error"]["message"]
        c.request("POST", "/v1/chat/completions", body=json.dumps({"messages": [], "max_tokens": 2, "n": 1}))
        r = c.getresponse()
        assert r.status == 200 and r.read()  # the connection stays usable
    finally:
        srv.shutdown()
        eng.stop()


@pytest.mark.parametrize("body,ollama,want", [
    ({}, False, []), ({"stop": None}, False, []), ({"stop": "END"}, False, ["END"]),
    ({"stop": ["a", "", "bc"]}, False, ["a", "bc"]), ({"options": {"stop": ["\n", "x"]}}, True, ["\n", "x"]),
    ({"options": None}, True, []),
])
def test_stop_sequences_parsed(body, ollama, want):
    assert stop_sequences(body, ollama) == want


@pytest.mark.parametrize("body,ollama", [
    ({"stop": 5}, False), ({"stop": ["a", 3]}, False), ({"stop": ["a", "b", "c", "d", "e"]}, False),
    ({"options": {"stop": [1]}}, True), ({"stop": {"a": 1}}, False),
])
def test_bad_stop_sequences_refused(body, ollama):
    with pytest.raises(SamplingError):
        stop_sequences(body, ollama)


def test_stop_matcher_holds_back_only_a_possible_prefix():
    m = StopMatcher(["END", "\n\n"])
    assert m.push("hello E") == ("hello ", False)  # "E" could begin END
    assert m.push("N") == ("", False)
    assert m.push("X more") == ("ENX more", False)  # it did not
    assert m.push(" then\n") == (" then", False)
    assert m.push("\nrest") == ("", True)  # the match and what follows are dropped
    m = StopMatcher(["abc"])
    assert m.push("xxab") == ("xx", False) and m.flush() == "ab"
    m = StopMatcher(["t5", "zz"])
    assert m.push(" t1 t5") == (" t1 ", True)  # earliest match wins
    m = StopMatcher(["aa", "b"])
    assert m.push("xab") == ("xa", True)


def _stop_server():
    eng = Engine(max_batch=4, model=FakeModel())
    srv, port, _ = start_server(port=0, engine=eng, model_name="fake")
    return srv, port, eng


def _post(port, path, body):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=20)
    c.request("POST", path, body=json.dumps(body), headers={"content-type": "application/json"})
    r = c.getresponse()
    return r.status, r.read()


def test_stop_sequences_end_completions():
    """The FakeModel's pieces are " t<id>": stop on the third token's piece
    (split across two pieces), streamed and not, OpenAI and Ollama."""
    toks = expected(b"hello", 12)
    full = "".join(f" t{t}" for t in toks)
    stop = f"{toks[2]} t{toks[3]}"  # spans the 3rd and 4th pieces
    cut = full[:full.index(stop)]
    srv, port, eng = _stop_server()
    try:
        msgs = [{"role": "user", "content": "hello"}]
        st, data = _post(port, "/v1/chat/completions", {"messages": msgs, "max_tokens": 12, "stop": [stop, "nope"]})
        j = json.loads(data)
        assert st == 200 and j["choices"][0]["message"]["content"] == cut
        assert j["choices"][0]["finish_reason"] == "stop"
        st, data = _post(port, "/v1/chat/completions", {"messages": msgs, "max_tokens": 12, "stop": stop,
                                                         "stream": True})
        events = [l[6:] for l in data.split(b"\n") if l.startswith(b"data: ")]
        assert st == 200 and events[-1] == b"[DONE]"
        objs = [json.loads(e) for e in events[:-1]]
        assert "".join(o["choices"][0]["delta"].get("content", "") for o in objs) == cut
        assert objs[-1]["choices"][0]["finish_reason"] == "stop"
        st, data = _post(port, "/v1/completions", {"prompt": "hello", "max_tokens": 12, "stop": "zzz"})
        j = json.loads(data)  # no match: the whole text, held-back tails included
        assert j["choices"][0]["text"] == full and j["choices"][0]["finish_reason"] == "length"
        st, data = _post(port, "/api/generate", {"prompt": "hello", "num_predict": 12,
                                                  "options": {"stop": [stop]}})
        lines = [json.loads(l) for l in data.split(b"\n") if l.strip()]
        assert st == 200 and lines[-1]["done"] and "".join(x["response"] for x in lines) == cut
    finally:
        srv.shutdown()
        eng.stop()


def test_eos_flushes_a_held_back_tail():
    """EOS also ends with finish_reason "stop"; a tail the matcher
    held back because it could begin a stop sequence is real completion text
    then and must be emitted (streamed and not)."""
    toks = expected(b"hello", 12)
    srv, port, eng = _stop_server()
    srv.eos = frozenset({toks[3]})  # the 4th token is EOS
    try:
        text = "".join(f" t{t}" for t in toks[:3])
        stop = f" t{toks[2]}QQ"  # the 3rd piece is a prefix of it: held back until EOS
        msgs = [{"role": "user", "content": "hello"}]
        st, data = _post(port, "/v1/chat/completions", {"messages": msgs, "max_tokens": 12, "stop": stop})
        j = json.loads(data)
        assert st == 200 and j["choices"][0]["message"]["content"] == text
        assert j["choices"][0]["finish_reason"] == "stop"
        st, data = _post(port, "/v1/chat/completions", {"messages": msgs, "max_tokens": 12, "stop": stop,
                                                         "stream": True})
        events = [l[6:] for l in data.split(b"\n") if l.startswith(b"data: ")]
        objs = [json.loads(e) for e in events[:-1]]
        assert "".join(o["choices"][0]["delta"].get("content", "") for o in objs) == text
    finally:
        srv.shutdown()
        eng.stop()


def test_sampling_refused_on_an_eager_engine():
    """The eager step (CPU stand-ins) has no sampler: a sampled request is
    refused instead of silently answered greedily (advice r3)."""
    srv, port, eng = _stop_server()
    try:
        st, data = _post(port, "/v1/chat/completions", {"messages": [], "temperature": 0.8, "max_tokens": 2})
        assert st == 400 and b"graph-captured" in data
        st, data = _post(port, "/v1/chat/completions", {"messages": [], "temperature": 0, "max_tokens": 2})
        assert st == 200
        st, data = _post(port, "/v1/chat/completions", {"messages": [], "temperature": 1, "top_k": 1,
                                                         "max_tokens": 2})
        assert st == 200  # top-1 is the argmax
    finally:
        srv.shutdown()
        eng.stop()
