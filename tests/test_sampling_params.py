"""Sampling parameters of the inference endpoint (models/server.py), CPU side:
OpenAI fields (temperature, top_p, seed, the top_k extension) and Ollama
"options" are parsed and range-checked; parameters that would change the
output but are not implemented are refused with 400 instead of being ignored.
The on-device sampler itself is tested on the GPU (tests/test_gpu_ops.py,
tests/test_gpu_model.py)."""
import http.client
import json

import pytest

from p2p_llm_tunnel_amd.models.server import Engine, SamplingError, sampling_params, start_server
from tests.test_inference_server import FakeModel


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
    ({"stop": ["\n\n"]}, False), ({"stop": "END"}, False),
    ({"options": {"repeat_penalty": 1.1}}, True), ({"options": {"mirostat": 2}}, True),
    ({"options": {"min_p": 0.05}}, True), ({"options": {"stop": ["x"]}}, True), ({"options": "hot"}, True),
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
