// `tunnel serve|proxy` CLI.
//
// Flags, env fallbacks and defaults match reference tunnel/src/cli.rs:
//   serve: --signal (TUNNEL_SIGNAL, wss://signal-server.fly.dev) --room (TUNNEL_ROOM, required)
//          --upstream (TUNNEL_UPSTREAM, required) --advertise (default "/", no env)
//          --turn/--turn-user/--turn-pass (TUNNEL_TURN, TUNNEL_TURN_USER, TUNNEL_TURN_PASS)
//   proxy: --signal --room --listen (TUNNEL_LISTEN, 127.0.0.1:8000) --turn...
// Logging filter from RUST_LOG (or TUNNEL_LOG), default info (main.rs:21-25).
// Extra opt-in flags (defaults keep reference behaviour) are listed in --help.
#include <malloc.h>
#include <sched.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "core/affinity.h"
#include "core/log.h"
#include "core/profiler.h"
#include "rtc/dtls.h"
#include "rtc/turn.h"
#include "tunnel/app.h"

using namespace p2pt;

static const char* kVersion = "0.2.0";

namespace {

// Value kinds checked after parsing (clap's value parsers, cli.rs:13-68, reject
// what does not parse; a bare strtoull would turn "x" into 0).
enum class Kind { Str, Flag, U64, U64OrAuto };

// Which subcommand accepts an extension (clap rejects a flag the subcommand
// does not define, so `tunnel proxy --max-request-body 1` is an error).
enum class Role { Both, Serve, Proxy };

struct Opt {
  const char* name;
  const char* env;
  const char* dflt;
  const char* help;
  Kind kind = Kind::Str;
  Role role = Role::Both;
  uint64_t lo = 0, hi = UINT64_MAX;  // accepted range of a numeric value
};

const std::vector<Opt>& serve_opts() {
  static const std::vector<Opt> o = {
      {"signal", "TUNNEL_SIGNAL", "wss://signal-server.fly.dev", "WebSocket URL of the signaling server"},
      {"room", "TUNNEL_ROOM", nullptr, "Room name to join"},
      {"upstream", "TUNNEL_UPSTREAM", nullptr, "Upstream HTTP URL to forward requests to (comma-separated: least-loaded across several)"},
      {"advertise", nullptr, "/", "Path prefix to advertise (e.g. /v1)"},
      {"turn", "TUNNEL_TURN", "", "TURN server URL (turn:host[:3478][?transport=udp|tcp], turns:host[:5349])"},
      {"turn-user", "TUNNEL_TURN_USER", "", "TURN server username"},
      {"turn-pass", "TUNNEL_TURN_PASS", "", "TURN server password"},
  };
  return o;
}

const std::vector<Opt>& proxy_opts() {
  static const std::vector<Opt> o = {
      {"signal", "TUNNEL_SIGNAL", "wss://signal-server.fly.dev", "WebSocket URL of the signaling server"},
      {"room", "TUNNEL_ROOM", nullptr, "Room name to join"},
      {"listen", "TUNNEL_LISTEN", "127.0.0.1:8000", "Local address to listen on"},
      {"turn", "TUNNEL_TURN", "", "TURN server URL (turn:host[:3478][?transport=udp|tcp], turns:host[:5349])"},
      {"turn-user", "TUNNEL_TURN_USER", "", "TURN server username"},
      {"turn-pass", "TUNNEL_TURN_PASS", "", "TURN server password"},
  };
  return o;
}

// Opt-in extensions shared by both subcommands (not in the reference).
const std::vector<Opt>& ext_opts() {
  static const std::vector<Opt> o = {
      {"transport", "TUNNEL_TRANSPORT", "webrtc", "webrtc | tcp-listen:HOST:PORT | tcp-connect:HOST:PORT"},
      {"stun", "TUNNEL_STUN", "stun:stun.l.google.com:19302", "STUN server(s), comma-separated; 'none' disables"},
      {"no-loopback-candidates", nullptr, nullptr, "Do not gather 127.0.0.1 host candidates", Kind::Flag},
      {"ipv6", nullptr, nullptr, "Gather IPv6 host candidates", Kind::Flag},
      {"ipv6-only", nullptr, nullptr, "Gather host candidates on IPv6 interfaces only", Kind::Flag},
      {"ice-relay-only", nullptr, nullptr, "Only use TURN-relayed candidates (iceTransportPolicy=relay)", Kind::Flag},
      {"gather-timeout-ms", "TUNNEL_GATHER_TIMEOUT_MS", "5000", "Max wait for ICE gathering before sending SDP", Kind::U64},
      {"ice-timeout-ms", "TUNNEL_ICE_TIMEOUT_MS", "30000", "No traffic for this long => connection failed", Kind::U64},
      {"sctp-mtu", "TUNNEL_SCTP_MTU", "1200", "SCTP packet size budget (bytes)", Kind::U64, Role::Both, 576, 65535},
      {"no-jumbo-loopback", nullptr, nullptr, "Disable large SCTP packets on loopback paths", Kind::Flag},
      {"max-retries", "TUNNEL_MAX_RETRIES", "4294967295", "Give up after this many failed attempts", Kind::U64},
      {"reset-backoff-after", "TUNNEL_RESET_BACKOFF_AFTER", "0", "Reset backoff after a session lasted N s (0=never)", Kind::U64},
      {"ping-interval-ms", "TUNNEL_PING_INTERVAL_MS", "10000", "Keepalive PING interval", Kind::U64},
      {"pong-timeout-ms", "TUNNEL_PONG_TIMEOUT_MS", "0", "Fail the session if no PONG for this long (0=off)", Kind::U64},
      {"header-timeout-ms", "TUNNEL_HEADER_TIMEOUT_MS", "60000", "Proxy wait for response headers (504 after)", Kind::U64},
      {"handshake-timeout-ms", "TUNNEL_HANDSHAKE_TIMEOUT_MS", "300000", "HELLO/AGREE timeout", Kind::U64},
      {"listen-early", nullptr, nullptr, "proxy: bind before the tunnel is up and answer 503 until ready", Kind::Flag,
       Role::Proxy},
      {"metrics-listen", "TUNNEL_METRICS_LISTEN", "", "Serve Prometheus metrics on HOST:PORT"},
      {"busy-poll-us", "TUNNEL_BUSY_POLL_US", "250",
       "Keep polling for N us after I/O instead of sleeping: a token's hop then costs no wake-up (0 = always sleep)",
       Kind::U64},
      {"workers", "TUNNEL_WORKERS", "auto",
       "HTTP worker threads beside the association thread (auto: half the usable CPUs less one, 1..4; 0: single thread)", Kind::U64OrAuto, Role::Both, 0, 256},
      {"inline-streams", "TUNNEL_INLINE_STREAMS", "16",
       "Concurrent streams handled on the association thread before new ones go to workers", Kind::U64},
      {"assoc", "TUNNEL_ASSOC", "3",
       "Parallel associations (PeerConnections, one thread each) when the peer agrees and the path is short (<= 10 ms): "
       "bulk requests spread over them, interactive ones stay on the first (1 = the reference's single data channel)",
       Kind::U64, Role::Both, 1, 8},
      {"max-request-body", "TUNNEL_MAX_REQUEST_BODY", "0",
       "serve: answer 413 to request bodies larger than this many bytes (0 = unlimited)", Kind::U64, Role::Serve},
      {"stream-body-threshold", "TUNNEL_STREAM_BODY_THRESHOLD", "8388608",
       "serve: request bodies this big stream to the upstream as they arrive instead of being buffered", Kind::U64, Role::Serve},
      {"upstream-prewarm", "TUNNEL_UPSTREAM_PREWARM", "4",
       "serve: spare pre-connected upstream sockets (follows peak concurrency; 0=off)", Kind::U64, Role::Serve},
      {"upstream-prewarm-ttl-ms", "TUNNEL_UPSTREAM_PREWARM_TTL_MS", "1000",
       "serve: close a spare upstream socket unused for this long", Kind::U64, Role::Serve},
      {"secret", "TUNNEL_SECRET", "",
       "Pre-shared secret both peers must prove (HMAC bound to the DTLS fingerprints); prefer the env var"},
      {"cpu-affinity", "TUNNEL_CPU_AFFINITY", "",
       "Pin the process to these CPUs, e.g. 0-3,64 (the NIC's NUMA node, away from inference threads)"},
      {"identity", "TUNNEL_IDENTITY", "",
       "PEM file with this peer's DTLS key + certificate (created if missing): a stable fingerprint to pin"},
      {"pin-peer", "TUNNEL_PIN_PEER", "",
       "Only accept a peer whose DTLS certificate SHA-256 is listed (comma-separated; see `tunnel fingerprint`)"},
  };
  return o;
}

void usage_main() {
  printf("P2P HTTP tunnel over WebRTC\n\nUsage: tunnel <COMMAND>\n\nCommands:\n"
         "  serve  Serve an upstream HTTP service through the tunnel\n"
         "  proxy  Create a local HTTP proxy that tunnels to a remote provider\n"
         "  fingerprint  Print the DTLS fingerprint of an --identity file (for --pin-peer)\n"
         "  help   Print this message or the help of the given subcommand(s)\n\n"
         "Options:\n  -h, --help     Print help\n  -V, --version  Print version\n");
}

bool for_role(const Opt& o, const char* cmd) {
  return o.role == Role::Both || (o.role == Role::Serve) == (strcmp(cmd, "serve") == 0);
}

void usage_sub(const char* cmd, const std::vector<Opt>& opts) {
  printf("Usage: tunnel %s [OPTIONS]\n\nOptions:\n", cmd);
  for (auto* list : {&opts, &ext_opts()}) {
    if (list == &ext_opts()) printf("\nExtensions (defaults keep reference behaviour):\n");
    for (auto& o : *list) {
      if (!for_role(o, cmd)) continue;
      std::string left = std::string("      --") + o.name + (o.kind == Kind::Flag ? "" : " <VALUE>");
      printf("%-36s %s", left.c_str(), o.help);
      if (o.env) printf(" [env: %s=]", o.env);
      if (o.dflt && *o.dflt) printf(" [default: %s]", o.dflt);
      printf("\n");
    }
  }
  printf("  -h, --help                           Print help\n");
}

// A whole unsigned decimal within [lo, hi] (clap's u64 parser: no sign, no
// trailing text, no overflow).
bool parse_u64(const std::string& v, uint64_t lo, uint64_t hi, uint64_t* out, std::string* why) {
  if (v.empty()) {
    *why = "cannot parse integer from empty string";
    return false;
  }
  uint64_t x = 0;
  for (char c : v) {
    if (c < '0' || c > '9') {
      *why = "invalid digit found in string";
      return false;
    }
    if (x > (UINT64_MAX - uint64_t(c - '0')) / 10) {
      *why = "number too large to fit in target type";
      return false;
    }
    x = x * 10 + uint64_t(c - '0');
  }
  if (x < lo || x > hi) {
    *why = std::to_string(x) + " is not in " + std::to_string(lo) + ".." + std::to_string(hi);
    return false;
  }
  *out = x;
  return true;
}

bool parse_sub(int argc, char** argv, const char* cmd, const std::vector<Opt>& opts,
               std::map<std::string, std::string>& out) {
  std::vector<Opt> all = opts;
  for (auto& o : ext_opts())
    if (for_role(o, cmd)) all.push_back(o);
  for (int i = 2; i < argc; i++) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help") {
      usage_sub(cmd, opts);
      exit(0);
    }
    if (a.rfind("--", 0) != 0) {
      fprintf(stderr, "error: unexpected argument '%s' found\n", a.c_str());
      return false;
    }
    std::string name = a.substr(2), val;
    bool has_eq = false;
    size_t eq = name.find('=');
    if (eq != std::string::npos) {
      val = name.substr(eq + 1);
      name = name.substr(0, eq);
      has_eq = true;
    }
    const Opt* found = nullptr;
    for (auto& o : all)
      if (name == o.name) found = &o;
    if (!found) {
      fprintf(stderr, "error: unexpected argument '--%s' found\n\nUsage: tunnel %s [OPTIONS]\n", name.c_str(), cmd);
      return false;
    }
    if (found->kind == Kind::Flag) {
      if (has_eq) {
        fprintf(stderr, "error: unexpected value '%s' for '--%s' found; no more were expected\n", val.c_str(),
                name.c_str());
        return false;
      }
      out[name] = "1";
      continue;
    }
    if (!has_eq) {
      if (i + 1 >= argc) {
        fprintf(stderr, "error: a value is required for '--%s <VALUE>' but none was supplied\n", name.c_str());
        return false;
      }
      val = argv[++i];
    }
    out[name] = val;
  }
  for (auto& o : all) {
    if (out.count(o.name)) continue;
    const char* e = o.env ? getenv(o.env) : nullptr;
    if (e && o.kind != Kind::Flag) out[o.name] = e;
    else if (o.dflt) out[o.name] = o.dflt;
  }
  for (auto& o : opts) {
    if (!o.dflt && o.kind != Kind::Flag && !out.count(o.name)) {
      fprintf(stderr, "error: the following required arguments were not provided:\n  --%s <%s>\n\nUsage: tunnel %s --%s <VALUE>\n",
              o.name, o.name, cmd, o.name);
      return false;
    }
  }
  // Numeric values, from the command line or the environment alike.
  for (auto& o : all) {
    if (o.kind != Kind::U64 && o.kind != Kind::U64OrAuto) continue;
    auto it = out.find(o.name);
    if (it == out.end() || (o.kind == Kind::U64OrAuto && it->second == "auto")) continue;
    uint64_t v;
    std::string why;
    if (!parse_u64(it->second, o.lo, o.hi, &v, &why)) {
      fprintf(stderr, "error: invalid value '%s' for '--%s <VALUE>': %s\n\nFor more information, try '--help'.\n",
              it->second.c_str(), o.name, why.c_str());
      return false;
    }
  }
  return true;
}

// "0-3,8,10-11" -> sched_setaffinity. The tunnel is one reactor thread: pin it
// next to the NIC (same NUMA node) and away from the inference server's cores.
bool pin_cpus(const std::string& list, std::string* err) {
  cpu_set_t set;
  CPU_ZERO(&set);
  size_t a = 0;
  while (a < list.size()) {
    size_t c = list.find(',', a);
    if (c == std::string::npos) c = list.size();
    std::string part = list.substr(a, c - a);
    char* end = nullptr;
    long lo = strtol(part.c_str(), &end, 10), hi = lo;
    if (end == part.c_str()) {
      *err = "expected a CPU number in '" + part + "'";
      return false;
    }
    if (*end == '-') {
      const char* h = end + 1;
      hi = strtol(h, &end, 10);
      if (end == h) {
        *err = "expected a range end in '" + part + "'";
        return false;
      }
    }
    if (*end || lo < 0 || hi < lo || hi >= CPU_SETSIZE) {
      *err = "bad CPU range '" + part + "'";
      return false;
    }
    for (long i = lo; i <= hi; i++) CPU_SET(i, &set);
    a = c + 1;
  }
  if (sched_setaffinity(0, sizeof set, &set) != 0) {
    *err = strerror(errno);
    return false;
  }
  return true;
}

// Validated by parse_sub; absent (an option of the other subcommand) reads 0.
uint64_t num(const std::map<std::string, std::string>& m, const char* k) {
  auto it = m.find(k);
  return it == m.end() ? 0 : strtoull(it->second.c_str(), nullptr, 10);
}

}  // namespace

// TUNNEL_* variables this build reads besides the flags' own (README,
// "Environment switches"), and the retired ones with what replaced them: a
// setting nobody reads is reported instead of silently doing nothing.
const char* const kSwitches[] = {"TUNNEL_LOG",       "TUNNEL_TRACE",    "TUNNEL_PROFILE",     "TUNNEL_THREAD_TIMELINE",
                                 "TUNNEL_FAULT",     "TUNNEL_NAT",      "TUNNEL_UDP_OFFLOAD", "TUNNEL_UDP_BUF_KB",
                                 "TUNNEL_RX_READER", "TUNNEL_COALESCE_US", "TUNNEL_SCTP_CC",  "TUNNEL_DTLS_RECORDS",
                                 "TUNNEL_FEATURES",  "TUNNEL_PIN_THREADS", "TUNNEL_TLS_INSECURE"};

const char* retired_hint(const std::string& name) {
  if (name.rfind("TUNNEL_FAULT_", 0) == 0) return "use TUNNEL_FAULT=key=value,... (drop, dup, delay_ms, blackhole, rtt_ms, rate_mbps, queue_kb)";
  if (name.rfind("TUNNEL_SCTP_", 0) == 0) return "congestion knobs are folded into TUNNEL_SCTP_CC=reno|beta=NN";
  if (name == "TUNNEL_GSO" || name == "TUNNEL_GRO") return "use TUNNEL_UDP_OFFLOAD=gso,gro|none";
  if (name.rfind("TUNNEL_DTLS_", 0) == 0) return "use TUNNEL_DTLS_RECORDS=evp|openssl";
  return "removed (README lists the switches this build reads)";
}

void warn_unused_env(const std::vector<Opt>& a, const std::vector<Opt>& b) {
  for (char** e = environ; e && *e; e++) {
    std::string kv = *e;
    if (kv.rfind("TUNNEL_", 0) != 0) continue;
    std::string name = kv.substr(0, kv.find('='));
    bool known = false;
    for (auto* s : kSwitches) known |= name == s;
    for (auto* v : {&a, &b})
      for (auto& o : *v) known |= o.env && name == o.env;
    if (!known) LOG_WARN("tunnel", "%s is not read by this build and is ignored: %s", name.c_str(), retired_hint(name));
  }
}

int main(int argc, char** argv) {
  // Receive/datagram buffers come and go in 64 KiB units: keep freed heap
  // instead of trimming it back to the kernel after every burst (brk/sbrk
  // showed up at ~10 % of the serve process under 256-stream bursts).
  mallopt(M_TRIM_THRESHOLD, 64 << 20);
  mallopt(M_TOP_PAD, 16 << 20);
  log::init_from_env();
  if (argc < 2) {
    usage_main();
    return 2;
  }
  std::string cmd = argv[1];
  if (cmd == "-V" || cmd == "--version") {
    printf("tunnel %s\n", kVersion);
    return 0;
  }
  if (cmd == "-h" || cmd == "--help" || cmd == "help") {
    if (argc > 2 && std::string(argv[2]) == "serve") usage_sub("serve", serve_opts());
    else if (argc > 2 && std::string(argv[2]) == "proxy") usage_sub("proxy", proxy_opts());
    else usage_main();
    return 0;
  }
  if (cmd == "fingerprint") {  // print (creating if needed) the identity's fingerprint for --pin-peer
    std::string path = argc > 3 && std::string(argv[2]) == "--identity" ? argv[3] : "";
    if (path.empty() && getenv("TUNNEL_IDENTITY")) path = getenv("TUNNEL_IDENTITY");
    if (path.empty()) {
      fprintf(stderr, "Usage: tunnel fingerprint --identity <PEM FILE>  [env: TUNNEL_IDENTITY=]\n");
      return 2;
    }
    std::string err;
    if (!rtc::set_identity_file(path, &err)) {
      fprintf(stderr, "error: --identity %s: %s\n", path.c_str(), err.c_str());
      return 2;
    }
    printf("%s\n", rtc::DtlsTransport::local_fingerprint().c_str());
    return 0;
  }
  if (cmd != "serve" && cmd != "proxy") {
    fprintf(stderr, "error: unrecognized subcommand '%s'\n\n", cmd.c_str());
    usage_main();
    return 2;
  }
  std::map<std::string, std::string> m;
  if (!parse_sub(argc, argv, cmd.c_str(), cmd == "serve" ? serve_opts() : proxy_opts(), m)) return 2;
  warn_unused_env(serve_opts(), proxy_opts());

  AppConfig cfg;
  cfg.mode = cmd;
  cfg.signal = m["signal"];
  cfg.room = m["room"];
  if (cmd == "serve") {
    cfg.upstream = m["upstream"];
    cfg.advertise = m["advertise"];
  } else {
    cfg.listen = m["listen"];
  }
  cfg.rtc.turn.url = m["turn"];
  if (!cfg.rtc.turn.url.empty()) {
    rtc::TurnUrl tu;
    std::string err;
    if (!rtc::TurnClient::parse_url(cfg.rtc.turn.url, tu, &err)) {
      fprintf(stderr, "error: --turn: %s\n", err.c_str());
      return 2;
    }
  }
  cfg.rtc.turn.username = m["turn-user"];
  cfg.rtc.turn.password = m["turn-pass"];
  cfg.transport = m["transport"];
  cfg.rtc.stun_servers.clear();
  if (m["stun"] != "none") {
    std::string s = m["stun"];
    size_t start = 0;
    while (start < s.size()) {
      size_t c = s.find(',', start);
      if (c == std::string::npos) c = s.size();
      if (c > start) cfg.rtc.stun_servers.push_back(s.substr(start, c - start));
      start = c + 1;
    }
  }
  cfg.rtc.include_loopback = !m.count("no-loopback-candidates");
  cfg.rtc.include_ipv6 = m.count("ipv6") > 0 || m.count("ipv6-only") > 0;
  cfg.rtc.ipv6_only = m.count("ipv6-only") > 0;
  cfg.rtc.relay_only = m.count("ice-relay-only") > 0;
  cfg.rtc.gather_timeout_ms = num(m, "gather-timeout-ms");
  cfg.rtc.ice_failed_timeout_ms = num(m, "ice-timeout-ms");
  cfg.rtc.sctp_mtu = num(m, "sctp-mtu");
  cfg.rtc.allow_jumbo_loopback = !m.count("no-jumbo-loopback");
  cfg.max_retries = num(m, "max-retries");
  cfg.reset_backoff_after_s = num(m, "reset-backoff-after");
  cfg.ping_interval_ms = num(m, "ping-interval-ms");
  cfg.pong_timeout_ms = num(m, "pong-timeout-ms");
  cfg.header_timeout_ms = num(m, "header-timeout-ms");
  cfg.handshake_timeout_ms = num(m, "handshake-timeout-ms");
  cfg.listen_early = m.count("listen-early") > 0;
  cfg.metrics_listen = m["metrics-listen"];
  cfg.busy_poll_us = num(m, "busy-poll-us");
  cfg.workers = m["workers"] == "auto" ? -1 : int(num(m, "workers"));
  cfg.inline_streams = num(m, "inline-streams");
  cfg.assoc = uint32_t(num(m, "assoc"));
  if (cmd == "serve") {
    cfg.upstream_prewarm = num(m, "upstream-prewarm");
    cfg.upstream_prewarm_ttl_ms = num(m, "upstream-prewarm-ttl-ms");
    cfg.max_request_body = num(m, "max-request-body");
    cfg.stream_body_threshold = num(m, "stream-body-threshold");
  }
  cfg.secret = m["secret"];
  if (!m["cpu-affinity"].empty()) {
    std::string err;
    if (!pin_cpus(m["cpu-affinity"], &err)) {
      fprintf(stderr, "error: --cpu-affinity %s: %s\n", m["cpu-affinity"].c_str(), err.c_str());
      return 2;
    }
    LOG_INFO("tunnel", "pinned to CPUs %s", m["cpu-affinity"].c_str());
    affinity::set_default(true);  // given its CPUs: one per thread (TUNNEL_PIN_THREADS=0: off)
  }
  affinity::pin_this_thread(0);

  if (!m["identity"].empty()) {
    std::string err;
    if (!rtc::set_identity_file(m["identity"], &err)) {
      fprintf(stderr, "error: --identity %s: %s\n", m["identity"].c_str(), err.c_str());
      return 2;
    }
    LOG_INFO("tunnel", "DTLS identity %s: %s", m["identity"].c_str(), rtc::DtlsTransport::local_fingerprint().c_str());
  }
  if (!m["pin-peer"].empty()) {
    std::vector<std::string> pins;
    const std::string& s = m["pin-peer"];
    for (size_t a = 0; a < s.size();) {
      size_t c = s.find(',', a);
      if (c == std::string::npos) c = s.size();
      if (c > a) pins.push_back(s.substr(a, c - a));
      a = c + 1;
    }
    std::string bad;
    if (pins.empty() || !rtc::set_pinned_fingerprints(pins, &bad)) {
      fprintf(stderr, "error: --pin-peer: '%s' is not a SHA-256 fingerprint\n", bad.c_str());
      return 2;
    }
    LOG_INFO("tunnel", "accepting only %zu pinned peer certificate(s)", pins.size());
  }

  if (cmd == "serve") {
    LOG_INFO("tunnel", "starting serve mode: signal=%s, room=%s, upstream=%s, advertise=%s", cfg.signal.c_str(),
             cfg.room.c_str(), cfg.upstream.c_str(), cfg.advertise.c_str());
  } else {
    LOG_INFO("tunnel", "starting proxy mode: signal=%s, room=%s, listen=%s", cfg.signal.c_str(), cfg.room.c_str(),
             cfg.listen.c_str());
  }
  if (cfg.rtc.turn.set()) LOG_INFO("tunnel", "TURN server configured: %s", cfg.rtc.turn.url.c_str());
  profiler::start_from_env();
  profiler::start_timeline_from_env();
  return run_app(cfg);
}
