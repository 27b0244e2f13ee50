// pybind11 bindings: expose the native codec and protocol helpers to the
// Python test-suite and harness (SURVEY §4.2 "Python unit via pybind11").
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core/crypto.h"
#include "core/json.h"
#include "http/http.h"
#include "proto/frame.h"
#include "tunnel/app.h"
#include "ws/ws.h"

namespace py = pybind11;
using namespace p2pt;

static py::bytes to_py(const Bytes& b) { return py::bytes(reinterpret_cast<const char*>(b.data()), b.size()); }

static std::string canonical_json(const std::string& s) {
  Json j;
  std::string err;
  if (!Json::parse(s, j, &err)) throw py::value_error(err);
  return j.dump();
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "p2p_llm_tunnel_amd native core";
  m.attr("MAX_FRAME_SIZE") = proto::kMaxFrameSize;
  m.attr("MAX_BODY_CHUNK") = proto::kMaxBodyChunk;
  m.attr("PROTOCOL_VERSION") = proto::kProtocolVersion;
  m.attr("PROTOCOL_NAME") = proto::kProtocolName;

  m.def("encode_frame", [](int type, uint32_t sid, py::bytes payload) {
    std::string p = payload;
    if (!proto::msg_type_from_u8(uint8_t(type))) throw py::value_error("unknown message type");
    proto::Frame f{proto::MsgType(type), sid, Bytes::copy(p)};
    return to_py(f.encode());
  });
  m.def("decode_frame", [](py::bytes raw) {
    std::string r = raw;
    proto::Frame f;
    std::string err;
    if (!proto::decode(Bytes::copy(r), f, &err)) throw py::value_error(err);
    return py::make_tuple(int(f.type), f.stream_id, to_py(f.payload));
  });
  m.def("msg_type_name", [](int t) {
    auto mt = proto::msg_type_from_u8(uint8_t(t));
    if (!mt) throw py::value_error("unknown message type");
    return std::string(proto::msg_type_name(*mt));
  });
  m.def("hello_json", [](std::vector<std::string> features) {
    proto::Hello h;
    if (!features.empty()) h.features = features;
    return h.to_json().dump();
  }, py::arg("features") = std::vector<std::string>{});
  m.def("agree_from_hello", [](const std::string& hello_json, std::vector<std::string> ours) {
    Json j;
    std::string err;
    proto::Hello h;
    if (!Json::parse(hello_json, j, &err) || !proto::Hello::from_json(j, h, &err)) throw py::value_error(err);
    proto::Agree a;
    if (ours.empty()) ours = {"sse"};
    if (!proto::agree_from_hello(h, a, &err, ours)) throw py::value_error(err);
    return a.to_json().dump();
  }, py::arg("hello_json"), py::arg("ours") = std::vector<std::string>{});
  m.def("request_headers_json", [](uint32_t sid, const std::string& method, const std::string& path,
                                   std::vector<std::pair<std::string, std::string>> headers) {
    proto::RequestHeaders h{sid, method, path, {}};
    for (auto& kv : headers) proto::header_set(h.headers, kv.first, kv.second);
    return h.to_json().dump();
  });
  m.def("parse_request_headers", [](const std::string& s) {
    Json j;
    std::string err;
    proto::RequestHeaders h;
    if (!Json::parse(s, j, &err) || !proto::RequestHeaders::from_json(j, h, &err)) throw py::value_error(err);
    return py::make_tuple(h.stream_id, h.method, h.path, h.headers);
  });
  m.def("parse_response_headers", [](const std::string& s) {
    Json j;
    std::string err;
    proto::ResponseHeaders h;
    if (!Json::parse(s, j, &err) || !proto::ResponseHeaders::from_json(j, h, &err)) throw py::value_error(err);
    return py::make_tuple(h.stream_id, h.status, h.headers);
  });
  m.def("build_upstream_url", &proto::build_upstream_url);
  m.def("canonical_json", &canonical_json);
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c(s.data(), s.size());
  });
  m.def("crc32", [](py::bytes b) {
    std::string s = b;
    return crc32_ieee(s.data(), s.size());
  });
  m.def("ws_accept_key", [](const std::string& k) { return ws::accept_key(k); });
  m.def("ws_encode_frame", [](int op, py::bytes payload, bool mask) {
    std::string p = payload;
    return py::bytes(ws::encode_frame(ws::Op(op), p, mask));
  });
  m.def("ws_decode_frames", [](py::bytes data, bool expect_masked) {
    std::string d = data;
    ws::FrameParser p(expect_masked);
    py::list out;
    bool ok = p.feed(reinterpret_cast<const uint8_t*>(d.data()), d.size(), [&](ws::Op op, bool fin, std::string&& pl) {
      out.append(py::make_tuple(int(op), fin, py::bytes(pl)));
    });
    if (!ok) throw py::value_error(p.error());
    return out;
  });
  m.def("backoff_secs", &backoff_secs);
  m.def("uuid4", &uuid4);
  m.def("parse_url", [](const std::string& u) {
    http::Url url;
    std::string err;
    if (!http::parse_url(u, url, &err)) throw py::value_error(err);
    return py::make_tuple(url.scheme, url.host, url.port, url.path);
  });
  m.def("decode_chunked", [](py::bytes data) {
    std::string d = data;
    http::BodyDecoder dec;
    dec.reset(http::BodyDecoder::Mode::Chunked);
    std::string out;
    size_t used = dec.feed(reinterpret_cast<const uint8_t*>(d.data()), d.size(),
                           [&](const uint8_t* p, size_t n) { out.append(reinterpret_cast<const char*>(p), n); });
    if (used == SIZE_MAX) throw py::value_error(dec.error());
    return py::make_tuple(py::bytes(out), dec.done(), used);
  });
}
