#include "rtc/datapath.h"

#include <netinet/in.h>
#include <netinet/udp.h>
#include <poll.h>
#include <pthread.h>
#include <sys/eventfd.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "core/affinity.h"
#include "core/log.h"
#include "core/profiler.h"
#include "core/reactor.h"
#include "tunnel/metrics.h"

#ifndef UDP_SEGMENT
#define UDP_SEGMENT 103
#endif
#ifndef UDP_GRO
#define UDP_GRO 104
#endif

namespace p2pt::rtc {

static const char* kT = "tunnel::datapath";

// ------------------------------------------------------------------ Lane

Lane::Lane(const char* name) {
  th_ = std::thread([this, n = std::string(name)] {
    // Signals belong to the main reactor's signalfd (as on the HTTP workers).
    sigset_t mask;
    sigemptyset(&mask);
    for (int sig : {SIGINT, SIGTERM, SIGHUP, SIGQUIT, SIGUSR1, SIGUSR2, SIGPIPE}) sigaddset(&mask, sig);
    pthread_sigmask(SIG_BLOCK, &mask, nullptr);
    pthread_setname_np(pthread_self(), n.c_str());
    // T90 seal / T93 send / T91 rx / T95-96 open lanes in profiles and timelines
    profiler::register_thread(n.find("-txsend") != std::string::npos  ? 93
                              : n.find("-tx") != std::string::npos    ? 90
                              : n.find("-open1") != std::string::npos ? 96
                              : n.find("-open") != std::string::npos  ? 95
                                                                      : 91);
    run();
  });
}

Lane::~Lane() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_one();
  th_.join();
}

void Lane::submit(std::function<void()> job) {
  pending_.fetch_add(1, std::memory_order_relaxed);
  bool wake;
  {
    std::lock_guard<std::mutex> lk(mu_);
    wake = q_.empty();
    q_.push_back(std::move(job));
  }
  if (wake) cv_.notify_one();
}

void Lane::run() {
  std::vector<std::function<void()>> jobs;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ and drained
      jobs.swap(q_);
    }
    for (auto& j : jobs) {
      j();
      j = nullptr;  // release what the job held before counting it done
      pending_.fetch_sub(1, std::memory_order_release);
    }
    jobs.clear();
  }
}

LaneFd::LaneFd(int source, uint64_t generation) : fd(::dup(source)), src(source), gen(generation) {}
LaneFd::~LaneFd() {
  if (fd >= 0) ::close(fd);
}

// ------------------------------------------------------------------ batches

void TxBatch::clear() {
  arena.clear();
  pieces.clear();
  recs.clear();
  keep.clear();
  bytes = 0;
  last_owner = nullptr;
}

void TxBatch::add(uint64_t seq, uint8_t type, const iovec* iov, const Bytes* const* owners, int cnt) {
  Rec r{seq, type, uint32_t(pieces.size()), 0, 0};
  for (int i = 0; i < cnt; i++) {
    const size_t n = iov[i].iov_len;
    if (!n) continue;
    const Bytes* o = owners ? owners[i] : nullptr;
    if (o && o->owner()) {
      // One reference per run of pieces from the same buffer (a body frame
      // spans many packets): the count is touched once per frame, not per
      // packet, on both threads.
      if (o->owner().get() != last_owner) {
        keep.push_back(o->owner());
        last_owner = o->owner().get();
      }
      pieces.push_back(Piece{static_cast<const uint8_t*>(iov[i].iov_base), 0, uint32_t(n)});
    } else {
      pieces.push_back(Piece{nullptr, uint32_t(arena.size()), uint32_t(n)});
      arena.insert(arena.end(), static_cast<const uint8_t*>(iov[i].iov_base),
                   static_cast<const uint8_t*>(iov[i].iov_base) + n);
    }
    r.count++;
    r.total += uint32_t(n);
  }
  bytes += r.total;
  recs.push_back(r);
}

int TxBatch::gather(const Rec& r, iovec* out, int max) const {
  int k = 0;
  for (uint32_t i = 0; i < r.count && k < max; i++) {
    const Piece& p = pieces[r.first + i];
    out[k].iov_base = const_cast<uint8_t*>(p.p ? p.p : arena.data() + p.off);
    out[k].iov_len = p.n;
    k++;
  }
  return k;
}

// ------------------------------------------------------------------ records

namespace {
void wr48(uint8_t* p, uint64_t v) {
  for (int i = 5; i >= 0; i--) {
    p[i] = uint8_t(v);
    v >>= 8;
  }
}
}  // namespace

void seal_record(const AesGcm& g, const uint8_t iv[4], uint8_t* out, uint8_t type, uint64_t seq, const iovec* iov,
                 int cnt, size_t total) {
  out[0] = type;
  out[1] = 0xFE;  // DTLS 1.2
  out[2] = 0xFD;
  wr16(out + 3, 1);  // epoch
  wr48(out + 5, seq);
  wr16(out + 11, uint16_t(kExplicit + total + kTag));
  memcpy(out + kRecHdr, out + 3, 8);  // explicit nonce = epoch || seq (as OpenSSL does)
  uint8_t nonce[12], aad[13];
  memcpy(nonce, iv, 4);
  memcpy(nonce + 4, out + 3, 8);
  memcpy(aad, out + 3, 8);
  aad[8] = type;
  aad[9] = 0xFE;
  aad[10] = 0xFD;
  wr16(aad + 11, uint16_t(total));
  uint8_t* o = out + kRecHdr + kExplicit;
  g.seal_gather(nonce, aad, 13, iov, cnt, o, total, o + total);
}

bool open_record(const AesGcm& g, const uint8_t iv[4], uint8_t* rec, size_t len, uint8_t** pt, size_t* ptl) {
  if (len < kRecHdr + kExplicit + kTag) return false;
  const size_t ctlen = len - kRecHdr - kExplicit - kTag;
  uint8_t* ct = rec + kRecHdr + kExplicit;
  uint8_t nonce[12], aad[13];
  memcpy(nonce, iv, 4);
  memcpy(nonce + 4, rec + kRecHdr, 8);
  memcpy(aad, rec + 3, 8);
  aad[8] = rec[0];
  aad[9] = rec[1];
  aad[10] = rec[2];
  wr16(aad + 11, uint16_t(ctlen));
  if (!g.open(nonce, aad, 13, ct, ct, ctlen, ct + ctlen)) return false;
  *pt = ct;
  *ptl = ctlen;
  return true;
}

// ------------------------------------------------------------------ TX lane

std::shared_ptr<SealedBatch> TxLaneState::get_sealed() {
  std::lock_guard<std::mutex> lk(mu_);
  if (free_.empty()) return std::make_shared<SealedBatch>();
  auto s = std::move(free_.back());
  free_.pop_back();
  return s;
}

void TxLaneState::put_sealed(std::shared_ptr<SealedBatch> s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (free_.size() < 16) free_.push_back(std::move(s));
}

void TxLaneState::run(const TxBatch& b, const RecordKeys& k, int fd, const SockAddr& to, size_t coalesce) {
  seal(b, k, coalesce, one_);
  send(one_, fd, to);
}

TxLaneState::TxLaneState() = default;

void TxLaneState::seal(const TxBatch& b, const RecordKeys& k, size_t coalesce, SealedBatch& sb) {
  // Seal every record into one contiguous buffer; datagram boundaries are
  // kept aside (several records per datagram on same-host jumbo paths).
  std::vector<uint8_t>& out_ = sb.out;
  auto& dgs_ = sb.dgs;
  const size_t n = b.recs.size();
  offs_.resize(n);
  dgs_.clear();
  size_t off = 0;
  for (size_t i = 0; i < n; i++) {
    const size_t sz = record_size(b.recs[i].total);
    if (coalesce && !dgs_.empty() && dgs_.back().second + sz <= coalesce) dgs_.back().second += sz;
    else dgs_.emplace_back(off, sz);
    offs_[i] = off;
    off += sz;
  }
  if (out_.size() < off) out_.resize(off);
  iovec iov[64];
  for (size_t i = 0; i < n; i++) {
    const auto& r = b.recs[i];
    const int cnt = b.gather(r, iov, 64);
    seal_record(*k.w, k.wiv, out_.data() + offs_[i], r.type, r.seq, iov, cnt, r.total);
  }
  records.fetch_add(b.recs.size(), std::memory_order_relaxed);
  batches.fetch_add(1, std::memory_order_relaxed);
  datagrams.fetch_add(dgs_.size(), std::memory_order_relaxed);
}

void TxLaneState::send(SealedBatch& sb, int fd, const SockAddr& to) {
  std::vector<uint8_t>& out_ = sb.out;
  auto& dgs_ = sb.dgs;
  // 2. sendmmsg: runs of equal-size datagrams leave as one UDP GSO message
  // (contiguous in out_, so one iovec each); a shorter datagram ends a run.
  constexpr int kBatch = 64;
  constexpr size_t kGsoMaxSegs = 64, kGsoMaxBytes = 60000;
  mmsghdr msgs[kBatch];
  iovec iovs[kBatch];
  size_t first_dg[kBatch];  // index in dgs_ of each message's first datagram
  alignas(cmsghdr) char ctrl[kBatch][CMSG_SPACE(sizeof(uint16_t))];
  size_t i = 0;
  while (i < dgs_.size()) {
    int cnt = 0;
    while (i < dgs_.size() && cnt < kBatch) {
      const size_t seg = dgs_[i].second;
      size_t j = i + 1, total = seg;
      if (gso_ok_)
        while (j < dgs_.size() && j - i < kGsoMaxSegs && dgs_[j].second <= seg && total + dgs_[j].second <= kGsoMaxBytes) {
          total += dgs_[j].second;
          if (dgs_[j++].second < seg) break;
        }
      mmsghdr& m = msgs[cnt];
      memset(&m, 0, sizeof m);
      first_dg[cnt] = i;
      iovs[cnt].iov_base = out_.data() + dgs_[i].first;
      iovs[cnt].iov_len = total;
      m.msg_hdr.msg_iov = &iovs[cnt];
      m.msg_hdr.msg_iovlen = 1;
      m.msg_hdr.msg_name = const_cast<sockaddr*>(to.sa());
      m.msg_hdr.msg_namelen = to.len;
      if (j - i > 1) {
        m.msg_hdr.msg_control = ctrl[cnt];
        m.msg_hdr.msg_controllen = sizeof ctrl[cnt];
        cmsghdr* c = CMSG_FIRSTHDR(&m.msg_hdr);
        c->cmsg_level = SOL_UDP;
        c->cmsg_type = UDP_SEGMENT;
        c->cmsg_len = CMSG_LEN(sizeof(uint16_t));
        uint16_t gs = uint16_t(seg);
        memcpy(CMSG_DATA(c), &gs, sizeof gs);
      }
      cnt++;
      i = j;
    }
    int sent = 0;
    int waited_ms = 0;
    while (sent < cnt) {
      int rc = sendmmsg(fd, msgs + sent, unsigned(cnt - sent), 0);
      if (rc < 0) {
        if (errno == EINTR) continue;
        if ((errno == EIO || errno == EINVAL || errno == ENOPROTOOPT) && gso_ok_ && msgs[sent].msg_hdr.msg_controllen) {
          // No UDP GSO on this path: rebuild the rest of the batch datagram by
          // datagram (its later messages were built with UDP_SEGMENT too and
          // would fail the same way).
          LOG_DEBUG(kT, "UDP GSO unavailable (%s); sending datagrams individually", strerror(errno));
          gso_ok_ = false;
          i = first_dg[sent];
          break;
        }
        if ((errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOBUFS) && waited_ms < kSendWaitMs) {
          // Socket buffer full: wait (bounded) for room instead of dropping
          // packets SCTP would have to recover by retransmission.
          pollfd pf{fd, POLLOUT, 0};
          send_waits.fetch_add(1, std::memory_order_relaxed);
          const int rcp = poll(&pf, 1, 1);
          waited_ms += 1;
          (void)rcp;
          continue;
        }
        // Still full after the bound, or unreachable: drop; SCTP retransmits.
        for (int k = sent; k < cnt; k++) {
          const size_t end = k + 1 < cnt ? first_dg[k + 1] : i;
          send_drops.fetch_add(uint64_t(end - first_dg[k]), std::memory_order_relaxed);
        }
        break;
      }
      for (int k = sent; k < sent + rc; k++)
        if (msgs[k].msg_hdr.msg_controllen) gso_msgs.fetch_add(1, std::memory_order_relaxed);
      sent += rc;
    }
  }
}

// ------------------------------------------------------------------ RX reader

RxReader::RxReader(int fd, const SockAddr& remote, std::shared_ptr<const RecordKeys> keys, Deliver deliver, uint64_t id,
                   size_t slot, bool adaptive, uint64_t idle_us, size_t idle_bytes)
    : fd_(fd), stop_fd_(eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC)), remote_(remote), keys_(std::move(keys)),
      deliver_(std::move(deliver)), id_(id), slot_(slot), pool_(slot), adaptive_(adaptive), idle_us_(idle_us),
      idle_bytes_(idle_bytes), active_(!adaptive) {
  // One lane per CPU it can have: pinned on a set too small to give the open
  // lanes CPUs of their own (affinity::open_lane_count), a second lane would
  // only preempt the first.
  n_open_ = affinity::open_lane_count(kOpenLanes);
  for (int k = 0; k < n_open_; k++) open_[k] = std::make_unique<Lane>(k == 0 ? "p2pt-udp-open0" : "p2pt-udp-open1");
  th_ = std::thread([this] {
    sigset_t mask;
    sigemptyset(&mask);
    for (int sig : {SIGINT, SIGTERM, SIGHUP, SIGQUIT, SIGUSR1, SIGUSR2, SIGPIPE}) sigaddset(&mask, sig);
    pthread_sigmask(SIG_BLOCK, &mask, nullptr);
    pthread_setname_np(pthread_self(), "p2pt-udp-rx");
    profiler::register_thread(92);  // T92 in profiles
    run();
  });
}

RxReader::~RxReader() {
  stop_.store(true, std::memory_order_release);
  uint64_t one = 1;
  if (stop_fd_ >= 0 && ::write(stop_fd_, &one, sizeof one) < 0) {
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
  }
  cv_.notify_all();
  th_.join();
  for (auto& l : open_) l.reset();  // runs (and delivers) what is queued, then joins
  if (stop_fd_ >= 0) ::close(stop_fd_);
}

void RxReader::engage() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    active_.store(true, std::memory_order_release);
  }
  engages.fetch_add(1, std::memory_order_relaxed);
  cv_.notify_all();
}

void RxReader::done() {
  if (outstanding_.fetch_sub(1, std::memory_order_acq_rel) == kMaxOutstanding) {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_one();
  }
}

namespace {
// The GRO segment size, and the socket's drop count when SO_RXQ_OVFL reports
// one (the kernel attaches it once drops have happened).
size_t gro_seg(const msghdr* mh, uint32_t* ovfl) {
  size_t seg = 0;
  for (cmsghdr* c = CMSG_FIRSTHDR(const_cast<msghdr*>(mh)); c; c = CMSG_NXTHDR(const_cast<msghdr*>(mh), c)) {
    if (c->cmsg_level == SOL_UDP && c->cmsg_type == UDP_GRO) {
      int v = 0;
      memcpy(&v, CMSG_DATA(c), sizeof v);
      seg = size_t(v);
    } else if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SO_RXQ_OVFL) {
      memcpy(ovfl, CMSG_DATA(c), sizeof *ovfl);
    }
  }
  return seg;
}
}  // namespace

// One datagram: all-application-data from the selected remote is opened here;
// anything else goes to the association thread as it came.
void RxReader::segment(const RawBufPtr& buf, uint32_t off, uint32_t len, const SockAddr& from, Burst& b) {
  datagrams.fetch_add(1, std::memory_order_relaxed);
  uint8_t* p = buf->data.get() + off;
  bool fast = from == remote_ && len >= kRecHdr;
  if (fast) {  // every record epoch-1 application data and whole
    for (size_t o = 0; o < len;) {
      if (o + kRecHdr > len || p[o] != 23 || rd16(p + o + 3) != 1) {
        fast = false;
        break;
      }
      const size_t rl = kRecHdr + rd16(p + o + 11);
      if (o + rl > len) {
        fast = false;
        break;
      }
      o += rl;
    }
  }
  if (!fast) {
    raw_datagrams.fetch_add(1, std::memory_order_relaxed);
    b.raw.push_back(Raw{buf, off, len, from});
    return;
  }
  for (size_t o = 0; o < len;) {
    uint8_t* rec = p + o;
    const size_t rl = kRecHdr + rd16(rec + 11);
    o += rl;
    RxBatch::Rec r;
    r.rec = rec;
    r.len = uint32_t(rl);
    r.type = rec[0];
    uint64_t seq = 0;
    for (int i = 0; i < 6; i++) seq = (seq << 8) | rec[5 + i];
    r.seq = seq;
    r.owner = buf;
    b.opened.bytes += rl;
    b.opened.recs.push_back(std::move(r));
    records.fetch_add(1, std::memory_order_relaxed);
  }
}

// Authenticates and decrypts a burst's records in place (a lane or the reader).
void RxReader::open_burst(Burst& b) const {
  for (auto& r : b.opened.recs) {
    size_t ptl = 0;
    r.ok = open_record(*keys_->r, keys_->riv, r.rec, r.len, &r.pt, &ptl);
    r.ptl = uint32_t(ptl);
  }
}

void RxReader::complete(uint64_t seq, std::unique_ptr<Burst> b) {
  std::lock_guard<std::mutex> lk(ord_mu_);
  ready_.emplace_back(seq, std::move(b));
  for (bool more = true; more;) {
    more = false;
    for (size_t i = 0; i < ready_.size(); i++) {
      if (ready_[i].first != seq_deliver_) continue;
      std::unique_ptr<Burst> next = std::move(ready_[i].second);
      ready_.erase(ready_.begin() + long(i));
      seq_deliver_++;
      deliver_(std::move(next));
      more = true;
      break;
    }
  }
}

void RxReader::run() {
  constexpr int kBatch = 32;
  mmsghdr msgs[kBatch];
  iovec iovs[kBatch];
  sockaddr_storage from[kBatch];
  alignas(cmsghdr) char ctrl[kBatch][CMSG_SPACE(sizeof(int)) + CMSG_SPACE(sizeof(uint32_t)) +
                                      CMSG_SPACE(sizeof(timespec))];
  RawBufPtr slots[kBatch];
  const bool traced = trace::enabled();
  pollfd pf[2] = {{fd_.fd, POLLIN, 0}, {stop_fd_, POLLIN, 0}};
  uint64_t win_start = 0, win_bytes = 0;  // adaptive: what was read since win_start
  while (!stop_.load(std::memory_order_acquire)) {
    if (!active_.load(std::memory_order_acquire)) {
      // Paused (adaptive): the association thread reads the socket.
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] {
        return stop_.load(std::memory_order_acquire) || active_.load(std::memory_order_acquire);
      });
      win_start = Reactor::now_us();
      win_bytes = 0;
      continue;
    }
    if (adaptive_) {
      const uint64_t now = Reactor::now_us();
      if (now - win_start >= idle_us_) {
        if (win_bytes < idle_bytes_) {
          // Interactive again: pause, and give the socket back behind every
          // burst already delivered (the association thread reads on in order).
          active_.store(false, std::memory_order_release);
          handbacks.fetch_add(1, std::memory_order_relaxed);
          auto hb = std::make_unique<Burst>();
          hb->reader = id_;
          hb->handback = true;
          outstanding_.fetch_add(1, std::memory_order_acq_rel);
          complete(seq_next_++, std::move(hb));  // after every burst still on a lane
          continue;
        }
        win_start = now;
        win_bytes = 0;
      }
    }
    if (outstanding_.load(std::memory_order_acquire) >= kMaxOutstanding) {
      // Back-pressure: the association thread is kMaxOutstanding bursts
      // behind, so the socket buffer holds what arrives meanwhile. Escape
      // before that buffer overflows (the kernel would drop what SCTP then
      // has to retransmit, and nothing in the stack would see why): past half
      // of it, read on. The sender's windows still bound what can pile up.
      size_t alloc = 0, limit = 0;
      if (escape_ && udp_socket_rmem(fd_.fd, &alloc, &limit) && limit && alloc * 2 >= limit) {
        escapes.fetch_add(1, std::memory_order_relaxed);
      } else {
        waits.fetch_add(1, std::memory_order_relaxed);
        std::unique_lock<std::mutex> lk(mu_);
        // Short waits: without UDP GRO every datagram is its own skb (about
        // twice its size in buffer accounting), and a 1 ms pause let a 512 KiB
        // buffer go from under half to overflowing (TUNNEL_UDP_OFFLOAD=none).
        // wait_until on the system clock: libstdc++ 11's steady-clock wait_for
        // goes through pthread_cond_clockwait, which GCC 11's ThreadSanitizer
        // does not intercept (it then reports the mutex as locked twice).
        cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(100), [this] {
          return stop_.load(std::memory_order_acquire) || outstanding_.load(std::memory_order_acquire) < kMaxOutstanding;
        });
        continue;
      }
    }
    // Adaptive: wake by the end of the window even when nothing arrives.
    int wait_ms = 100;
    if (adaptive_) {
      const uint64_t end = win_start + idle_us_, now = Reactor::now_us();
      wait_ms = now >= end ? 1 : int((end - now + 999) / 1000);
    }
    if (poll(pf, 2, wait_ms) <= 0 || (pf[1].revents & POLLIN)) continue;  // the loop head sees stop_ / the window
    auto burst = std::make_unique<Burst>();
    burst->reader = id_;
    const size_t slot = slot_.load(std::memory_order_relaxed);
    for (int round = 0; round < 8; round++) {
      for (int i = 0; i < kBatch; i++) {
        slots[i] = pool_.get();
        memset(&msgs[i], 0, sizeof msgs[i]);
        iovs[i].iov_base = slots[i]->data.get();
        iovs[i].iov_len = slot;
        msgs[i].msg_hdr.msg_iov = &iovs[i];
        msgs[i].msg_hdr.msg_iovlen = 1;
        msgs[i].msg_hdr.msg_name = &from[i];
        msgs[i].msg_hdr.msg_namelen = sizeof from[i];
        msgs[i].msg_hdr.msg_control = ctrl[i];
        msgs[i].msg_hdr.msg_controllen = sizeof ctrl[i];
      }
      const int n = recvmmsg(fd_.fd, msgs, kBatch, MSG_DONTWAIT, nullptr);
      if (n <= 0) break;
      if (traced) {
        // A burst's frames are stamped with its latest datagram's kernel time
        // (the first datagram's made a frame from a later one read as queued
        // before it was sent); the read time is the first read's.
        if (round == 0) burst->t_read = Reactor::now_us();
        for (int i = 0; i < n; i++) burst->t_kernel = std::max(burst->t_kernel, trace::kernel_rx_us(&msgs[i].msg_hdr));
      }
      for (int i = 0; i < n; i++) {
        SockAddr a;
        memcpy(&a.ss, &from[i], msgs[i].msg_hdr.msg_namelen);
        a.len = msgs[i].msg_hdr.msg_namelen;
        const uint32_t total = msgs[i].msg_len;
        if (msgs[i].msg_hdr.msg_flags & MSG_TRUNC) {
          // Larger than a slot: the peer sends bigger packets than this side's
          // path settings predicted. This one is lost (counted, SCTP resends
          // it); later reads use 64 KiB slots so the resend gets through.
          if (truncated.fetch_add(1, std::memory_order_relaxed) == 0)
            LOG_WARN(kT, "UDP datagram larger than the %zu-byte receive slot; reading with 64 KiB slots from now on",
                     slot);
          if (slot_.load(std::memory_order_relaxed) < 65536) {
            slot_.store(65536, std::memory_order_relaxed);
            pool_ = BufPool(65536);
          }
          continue;
        }
        uint32_t ovfl = 0;
        const uint32_t seg = uint32_t(gro_seg(&msgs[i].msg_hdr, &ovfl));
        if (ovfl > rxq_ovfl.load(std::memory_order_relaxed)) rxq_ovfl.store(ovfl, std::memory_order_relaxed);
        if (!seg || seg >= total) {
          segment(slots[i], 0, total, a, *burst);
        } else {
          gro_batches.fetch_add(1, std::memory_order_relaxed);
          for (uint32_t o = 0; o < total; o += seg) segment(slots[i], o, std::min(seg, total - o), a, *burst);
        }
      }
      for (auto& sl : slots) sl.reset();  // the burst holds what it uses
      if (n < kBatch || slot_.load(std::memory_order_relaxed) != slot) break;
    }
    if (burst->opened.recs.empty() && burst->raw.empty()) continue;
    win_bytes += burst->opened.bytes;
    for (auto& r : burst->raw) win_bytes += r.len;
    bursts.fetch_add(1, std::memory_order_relaxed);
    outstanding_.fetch_add(1, std::memory_order_acq_rel);
    const uint64_t seq = seq_next_++;
    if (burst->opened.bytes >= kLaneBytes && open_[0]) {
      lane_bursts.fetch_add(1, std::memory_order_relaxed);
      Burst* raw = burst.release();
      open_[next_lane_]->submit([this, seq, raw] {
        std::unique_ptr<Burst> b(raw);
        open_burst(*b);
        complete(seq, std::move(b));
      });
      next_lane_ = (next_lane_ + 1) % n_open_;
    } else {
      open_burst(*burst);
      complete(seq, std::move(burst));
    }
  }
}


namespace {
std::atomic<int> g_rx_reader{-1};  // -1: from the environment
std::atomic<bool> g_rx_escape{true};
}

bool rx_escape_enabled() { return g_rx_escape.load(std::memory_order_relaxed); }
void set_rx_escape_enabled(bool on) { g_rx_escape.store(on, std::memory_order_relaxed); }

int rx_reader_mode() {
  int v = g_rx_reader.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("TUNNEL_RX_READER");
    v = !(e && *e) ? kRxReaderAdaptive : *e == '0' ? kRxReaderOff : *e == '1' ? kRxReaderAlways : kRxReaderAdaptive;
    g_rx_reader.store(v, std::memory_order_relaxed);
  }
  return v;
}

void set_rx_reader_mode(int mode) { g_rx_reader.store(mode, std::memory_order_relaxed); }


}  // namespace p2pt::rtc
