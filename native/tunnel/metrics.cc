#include "tunnel/metrics.h"

#include <sys/socket.h>
#include <time.h>

#include <cstring>
#include <vector>

#include <algorithm>

#include <unistd.h>

#include <fcntl.h>

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <string_view>

#include "http/http.h"
#include "proto/frame.h"

namespace p2pt::metrics {
namespace {
// Frame counters are bumped on the association thread; named counters and
// gauges may also come from worker threads (tunnel/workers.h): a mutex guards
// the maps, relaxed atomics the per-type arrays.
struct Registry {
  std::mutex mu;
  std::map<std::string, double> counters;
  std::map<std::string, double> gauges;
  std::map<std::string, std::function<double()>> gauge_fns;
  std::atomic<uint64_t> frames_sent[256] = {};
  std::atomic<uint64_t> bytes_sent[256] = {};
  std::atomic<uint64_t> frames_recv[256] = {};
  std::atomic<uint64_t> bytes_recv[256] = {};
};
Registry& reg() {
  static Registry r;
  return r;
}

std::string type_label(int t) {
  auto mt = proto::msg_type_from_u8(uint8_t(t));
  return mt ? proto::msg_type_name(*mt) : std::to_string(t);
}
}  // namespace

void frame_sent(uint8_t type, size_t bytes) {
  reg().frames_sent[type].fetch_add(1, std::memory_order_relaxed);
  reg().bytes_sent[type].fetch_add(bytes, std::memory_order_relaxed);
}
void frame_recv(uint8_t type, size_t bytes) {
  reg().frames_recv[type].fetch_add(1, std::memory_order_relaxed);
  reg().bytes_recv[type].fetch_add(bytes, std::memory_order_relaxed);
}
void counter_add(const std::string& name, double v) {
  std::lock_guard<std::mutex> lk(reg().mu);
  reg().counters[name] += v;
}
void gauge_set(const std::string& name, double v) {
  std::lock_guard<std::mutex> lk(reg().mu);
  reg().gauges[name] = v;
}
void gauge_fn(const std::string& name, std::function<double()> fn) {
  std::lock_guard<std::mutex> lk(reg().mu);
  reg().gauge_fns[name] = std::move(fn);
}
void gauge_fn_remove(const std::string& name) {
  std::lock_guard<std::mutex> lk(reg().mu);
  reg().gauge_fns.erase(name);
}
double counter_get(const std::string& name) {
  std::lock_guard<std::mutex> lk(reg().mu);
  auto it = reg().counters.find(name);
  return it == reg().counters.end() ? 0 : it->second;
}

std::string render_prometheus() {
  auto& r = reg();
  std::lock_guard<std::mutex> lk(r.mu);
  std::string out;
  char buf[256];
  auto line = [&](const std::string& name, const std::string& labels, double v) {
    snprintf(buf, sizeof buf, " %.17g\n", v);
    out += name;
    if (!labels.empty()) out += "{" + labels + "}";
    out += buf;
  };
  out += "# TYPE tunnel_frames_sent_total counter\n";
  for (int t = 0; t < 256; t++)
    if (r.frames_sent[t]) line("tunnel_frames_sent_total", "type=\"" + type_label(t) + "\"", double(r.frames_sent[t]));
  out += "# TYPE tunnel_frame_bytes_sent_total counter\n";
  for (int t = 0; t < 256; t++)
    if (r.bytes_sent[t]) line("tunnel_frame_bytes_sent_total", "type=\"" + type_label(t) + "\"", double(r.bytes_sent[t]));
  out += "# TYPE tunnel_frames_received_total counter\n";
  for (int t = 0; t < 256; t++)
    if (r.frames_recv[t]) line("tunnel_frames_received_total", "type=\"" + type_label(t) + "\"", double(r.frames_recv[t]));
  out += "# TYPE tunnel_frame_bytes_received_total counter\n";
  for (int t = 0; t < 256; t++)
    if (r.bytes_recv[t]) line("tunnel_frame_bytes_received_total", "type=\"" + type_label(t) + "\"", double(r.bytes_recv[t]));
  for (auto& kv : r.counters) {
    out += "# TYPE " + kv.first + " counter\n";
    line(kv.first, "", kv.second);
  }
  for (auto& kv : r.gauges) {
    out += "# TYPE " + kv.first + " gauge\n";
    line(kv.first, "", kv.second);
  }
  for (auto& kv : r.gauge_fns) {
    out += "# TYPE " + kv.first + " gauge\n";
    line(kv.first, "", kv.second());
  }
  return out;
}

namespace {
struct MetricsServer {
  std::unique_ptr<TcpListener> listener;
  std::map<int, std::shared_ptr<TcpConn>> conns;
  int next = 0;
};
}  // namespace

std::shared_ptr<void> serve(Reactor& r, const std::string& addr, std::string* err) {
  auto srv = std::make_shared<MetricsServer>();
  std::weak_ptr<MetricsServer> w = srv;
  Reactor* rp = &r;
  srv->listener = TcpListener::bind(
      r, addr,
      [w, rp](int fd, SockAddr) {
        auto s = w.lock();
        if (!s) return;
        auto c = TcpConn::adopt(*rp, fd);
        int id = s->next++;
        s->conns[id] = c;
        auto buf = std::make_shared<std::string>();
        std::weak_ptr<TcpConn> wc = c;
        c->on_data([buf, wc](const uint8_t* p, size_t n) {
          buf->append(reinterpret_cast<const char*>(p), n);
          http::Head h;
          size_t used = 0;
          auto res = http::parse_request_head(*buf, h, used, nullptr);
          auto conn = wc.lock();
          if (!conn || res == http::ParseResult::Incomplete) return;
          std::string body, status = "200 OK";
          if (res == http::ParseResult::Error) {
            status = "400 Bad Request";
          } else if (h.target == "/metrics" || h.target == "/") {
            body = render_prometheus();
          } else {
            status = "404 Not Found";
            body = "not found\n";
          }
          conn->write("HTTP/1.1 " + status + "\r\ncontent-type: text/plain; version=0.0.4\r\ncontent-length: " +
                      std::to_string(body.size()) + "\r\nconnection: close\r\n\r\n" + body);
          conn->close_after_flush();
        });
        c->on_close([w, id](const std::string&) {
          if (auto s2 = w.lock()) s2->conns.erase(id);
        });
      },
      err);
  if (!srv->listener) return nullptr;
  return srv;
}

}  // namespace p2pt::metrics

namespace p2pt::trace {
namespace {
// Events collect in memory and go out in whole-line write()s of up to 512
// KiB (and at exit): a waterfall stamps ~10 events per request, and a write
// per event cost a syscall each on the measured path. Several processes
// append to one file (O_APPEND), so a write never ends inside a line.
struct Sink {
  int fd = -1;
  std::mutex mu;
  std::string buf;
  void drain() {  // mu held
    size_t off = 0;
    while (off < buf.size()) {
      ssize_t n = ::write(fd, buf.data() + off, buf.size() - off);
      if (n <= 0) break;
      off += size_t(n);
    }
    buf.clear();
  }
};

Sink* sink() {
  static Sink* s = [] () -> Sink* {
    const char* p = getenv("TUNNEL_TRACE");
    if (!p || !*p) return nullptr;
    int fd = ::open(p, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd < 0) return nullptr;
    auto* k = new Sink;
    k->fd = fd;
    k->buf.reserve(1 << 20);
    std::atexit([] { flush(); });
    return k;
  }();
  return s;
}
}  // namespace

bool enabled() { return sink() != nullptr; }

void event(const char* role, uint32_t sid, const char* ev) {
  if (sink()) event_at(role, sid, ev, Reactor::now_us());
}

void event_at(const char* role, uint32_t sid, const char* ev, uint64_t t_us) {
  Sink* k = sink();
  if (!k) return;
  char line[160];
  int n = snprintf(line, sizeof line, "{\"t_us\":%llu,\"role\":\"%s\",\"sid\":%u,\"ev\":\"%s\"}\n",
                   static_cast<unsigned long long>(t_us), role, sid, ev);
  if (n <= 0) return;
  n = std::min(n, int(sizeof line) - 1);
  std::lock_guard<std::mutex> lk(k->mu);
  k->buf.append(line, size_t(n));
  if (k->buf.size() >= (512u << 10)) k->drain();
}

void flush() {
  Sink* k = sink();
  if (!k) return;
  std::lock_guard<std::mutex> lk(k->mu);
  k->drain();
}

namespace {
thread_local uint64_t t_rx_kernel = 0, t_rx_read = 0, t_rx_assoc = 0;
thread_local std::vector<std::pair<const char*, uint32_t>> t_tx_pending;
}  // namespace

void set_rx(uint64_t kernel_us, uint64_t read_us, uint64_t assoc_us) {
  t_rx_kernel = kernel_us;
  t_rx_read = read_us;
  t_rx_assoc = assoc_us;
}

void rx_stamps(const char* role, uint32_t sid) {
  if (!sink() || !t_rx_read) return;
  if (t_rx_kernel) event_at(role, sid, "udp_kernel", t_rx_kernel);
  event_at(role, sid, "udp_read", t_rx_read);
  event_at(role, sid, "rx_assoc", t_rx_assoc);
}

void mark_tx(const char* role, uint32_t sid) {
  if (sink() && t_tx_pending.size() < 4096) t_tx_pending.emplace_back(role, sid);
}

void tx_done() {
  if (t_tx_pending.empty()) return;
  const uint64_t now = Reactor::now_us();
  for (auto& p : t_tx_pending) event_at(p.first, p.second, "udp_tx", now);
  t_tx_pending.clear();
}

uint64_t kernel_rx_us(const void* mh_) {
  const msghdr* mh = static_cast<const msghdr*>(mh_);
  for (cmsghdr* c = CMSG_FIRSTHDR(const_cast<msghdr*>(mh)); c; c = CMSG_NXTHDR(const_cast<msghdr*>(mh), c)) {
    if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_TIMESTAMPNS) {
      timespec ts;
      memcpy(&ts, CMSG_DATA(c), sizeof ts);
      timespec rt, mt;
      clock_gettime(CLOCK_REALTIME, &rt);
      clock_gettime(CLOCK_MONOTONIC, &mt);
      const int64_t real_ns = int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec;
      const int64_t off = (int64_t(mt.tv_sec) - int64_t(rt.tv_sec)) * 1000000000 + (mt.tv_nsec - rt.tv_nsec);
      const int64_t mono_ns = real_ns + off;
      return mono_ns > 0 ? uint64_t(mono_ns / 1000) : 0;
    }
  }
  return 0;
}
}  // namespace p2pt::trace
