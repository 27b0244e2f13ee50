"""Frame codec + handshake behaviour.

Re-expresses the reference's 24 protocol unit tests
(reference tunnel/src/protocol.rs:265-550) against the native codec, plus
property-based round-trips.
"""
import json

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

HELLO, AGREE, PING, PONG = 1, 2, 3, 4
REQ_HEADERS, REQ_BODY, REQ_END = 10, 11, 12
RES_HEADERS, RES_BODY, RES_END, ERROR = 20, 21, 22, 99


def rt(n, t, sid, payload=b""):
    return n.decode_frame(n.encode_frame(t, sid, payload))


# ---- round trips (protocol.rs:271-388)

def test_roundtrip_hello(native):
    t, sid, p = rt(native, HELLO, 0, native.hello_json().encode())
    assert (t, sid) == (HELLO, 0)
    h = json.loads(p)
    assert h["proto"] == native.PROTOCOL_NAME == "httptunnel"
    assert h["min_version"] == 1 and h["max_version"] == native.PROTOCOL_VERSION


def test_hello_wire_bytes(native):
    # Exact reference serialisation (serde field order): 73-byte payload.
    assert native.hello_json() == '{"proto":"httptunnel","min_version":1,"max_version":1,"features":["sse"]}'
    assert len(native.encode_frame(HELLO, 0, native.hello_json().encode())) == 78


def test_roundtrip_agree(native):
    payload = json.dumps({"version": 1, "features": ["sse"]}).encode()
    t, _, p = rt(native, AGREE, 0, payload)
    assert t == AGREE
    assert json.loads(p) == {"version": 1, "features": ["sse"]}


def test_roundtrip_req_headers(native):
    s = native.request_headers_json(42, "POST", "/v1/chat/completions", [("content-type", "application/json")])
    t, sid, p = rt(native, REQ_HEADERS, 42, s.encode())
    assert (t, sid) == (REQ_HEADERS, 42)
    stream_id, method, path, headers = native.parse_request_headers(p.decode())
    assert (stream_id, method, path) == (42, "POST", "/v1/chat/completions")
    assert dict(headers) == {"content-type": "application/json"}


def test_req_headers_field_order(native):
    s = native.request_headers_json(1, "GET", "/x", [("host", "h")])
    assert s == '{"stream_id":1,"method":"GET","path":"/x","headers":{"host":"h"}}'


def test_roundtrip_req_body(native):
    assert rt(native, REQ_BODY, 7, b"hello world") == (REQ_BODY, 7, b"hello world")


def test_roundtrip_req_end(native):
    assert rt(native, REQ_END, 7) == (REQ_END, 7, b"")


def test_roundtrip_res_headers(native):
    s = json.dumps({"stream_id": 99, "status": 200, "headers": {"content-type": "text/event-stream"}})
    t, sid, p = rt(native, RES_HEADERS, 99, s.encode())
    assert (t, sid) == (RES_HEADERS, 99)
    assert native.parse_response_headers(p.decode())[1] == 200


def test_roundtrip_res_body(native):
    data = b'data: {"token": "hello"}\n\n'
    assert rt(native, RES_BODY, 99, data) == (RES_BODY, 99, data)


def test_roundtrip_res_end(native):
    assert rt(native, RES_END, 99) == (RES_END, 99, b"")


def test_roundtrip_error(native):
    assert rt(native, ERROR, 5, b"upstream timeout") == (ERROR, 5, b"upstream timeout")


# ---- negatives (protocol.rs:392-422)

def test_decode_empty(native):
    with pytest.raises(ValueError, match="too short"):
        native.decode_frame(b"")


def test_decode_too_short(native):
    with pytest.raises(ValueError, match="too short: 3 bytes"):
        native.decode_frame(bytes([1, 0, 0]))


def test_decode_unknown_type(native):
    with pytest.raises(ValueError, match="unknown message type: 255"):
        native.decode_frame(bytes([255, 0, 0, 0, 0]))


def test_decode_exactly_header_no_payload(native):
    assert native.decode_frame(bytes([12, 0, 0, 0, 0])) == (REQ_END, 0, b"")


# ---- boundaries (protocol.rs:426-460)

def test_zero_stream_id(native):
    assert rt(native, REQ_END, 0)[1] == 0


def test_max_stream_id(native):
    assert rt(native, REQ_END, 2**32 - 1)[1] == 2**32 - 1


def test_stream_id_big_endian(native):
    assert native.encode_frame(REQ_END, 0x01020304, b"") == bytes([12, 1, 2, 3, 4])


def test_large_payload(native):
    data = b"\xab" * native.MAX_BODY_CHUNK
    enc = native.encode_frame(RES_BODY, 1, data)
    assert len(enc) == 5 + native.MAX_BODY_CHUNK == 65413
    assert native.decode_frame(enc)[2] == data


def test_constants(native):
    assert native.MAX_FRAME_SIZE == 65536 and native.MAX_BODY_CHUNK == 65408


def test_empty_payload_body(native):
    assert rt(native, RES_BODY, 1) == (RES_BODY, 1, b"")


# ---- negotiation (protocol.rs:464-549)

def hello(minv=1, maxv=1, features=("sse",), proto="httptunnel"):
    return json.dumps({"proto": proto, "min_version": minv, "max_version": maxv, "features": list(features)})


def test_version_negotiation_exact_match(native):
    assert json.loads(native.agree_from_hello(hello()))["version"] == 1


def test_version_negotiation_range_overlap(native):
    assert json.loads(native.agree_from_hello(hello(1, 3)))["version"] == 1


def test_version_negotiation_no_overlap(native):
    with pytest.raises(ValueError, match=r"no compatible version: peer=\[5,10\], ours=\[1,1\]"):
        native.agree_from_hello(hello(5, 10, ()))


def test_version_negotiation_wrong_protocol(native):
    with pytest.raises(ValueError, match="unknown protocol: wrongproto"):
        native.agree_from_hello(hello(proto="wrongproto", features=()))


def test_feature_intersection(native):
    a = json.loads(native.agree_from_hello(hello(features=("sse", "gzip", "unknown"))))
    assert a["features"] == ["sse"]


def test_feature_no_overlap(native):
    assert json.loads(native.agree_from_hello(hello(features=("gzip", "brotli"))))["features"] == []


def test_hello_default_values(native):
    h = json.loads(native.hello_json())
    assert h["proto"] == "httptunnel" and h["min_version"] == 1 and "sse" in h["features"]


def test_cancel_feature_only_when_both_sides(native):
    # Our build understands "cancel"; a reference peer (features ["sse"]) never gets it.
    both = json.loads(native.agree_from_hello(hello(features=("sse", "cancel")), ["sse", "cancel"]))
    assert both["features"] == ["sse", "cancel"]
    ref_peer = json.loads(native.agree_from_hello(hello(features=("sse",)), ["sse", "cancel"]))
    assert ref_peer["features"] == ["sse"]


def test_malformed_hello_rejected(native):
    with pytest.raises(ValueError, match="missing field"):
        native.agree_from_hello('{"proto":"httptunnel"}')


# ---- properties

@settings(max_examples=300, deadline=None)
@given(t=st.sampled_from([1, 2, 3, 4, 10, 11, 12, 20, 21, 22, 99]),
       sid=st.integers(0, 2**32 - 1), payload=st.binary(max_size=4096))
def test_roundtrip_property(native, t, sid, payload):
    assert rt(native, t, sid, payload) == (t, sid, payload)


@settings(max_examples=300, deadline=None)
@given(raw=st.binary(max_size=64))
def test_decode_never_crashes(native, raw):
    try:
        t, sid, p = native.decode_frame(raw)
    except ValueError as e:
        assert "too short" in str(e) or "unknown message type" in str(e)
    else:
        assert len(raw) >= 5 and p == raw[5:] and sid == int.from_bytes(raw[1:5], "big")
