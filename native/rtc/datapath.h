// Crypto/IO lanes for the DTLS record layer: AES-GCM sealing + UDP sends and
// AES-GCM opening run beside the association thread instead of on it.
//
// The reference runs webrtc-rs on tokio's multi-threaded runtime
// (tunnel/src/main.rs:18, Cargo.toml:11), so its record encryption and socket
// I/O for a bulk body (serve.rs:263-286, proxy.rs:318-330) spread over cores.
// Here one association thread owns everything that must stay ordered — the
// SCTP state machine, DTLS epoch/sequence numbers, the replay window — and in
// a 64 x 1 MB echo it spent three quarters of its time on the bytes instead:
// sealing 21-25 %, sendmmsg 12-27 %, opening 12-16 % (profiles/r02/bulk_prof).
//
//   TX: SCTP packets (gather lists of headers + zero-copy body slices) become
//       records with their sequence numbers assigned on the association
//       thread; a flush's records go to the TX lane as one batch holding
//       references to the body buffers. The lane seals them into one
//       contiguous buffer and sends it with sendmmsg + UDP GSO on its own
//       dup of the socket.
//   RX: a reader thread owns the selected pair's socket (RxReader): recvmmsg
//       with GRO, application records authenticated and decrypted in place
//       there; the replay check and hand-off to SCTP run on the association
//       thread, in order. Without a reader (relay, emulation, before the pair
//       is direct) the association thread reads the socket and a burst's
//       records go to the RX lane instead.
//
// Small batches never cross threads: a flush (or receive burst) below
// kInlineBytes whose lane has nothing outstanding is processed inline, so an
// SSE token keeps the single-thread latency and only bulk pays a hand-off.
// Lanes are used only with the vector AES-GCM (its contexts are immutable
// after key setup, so both threads may use them) and on a direct UDP path
// (no TURN relay, NAT or WAN emulation, which live in the ICE agent's send
// path).
#pragma once

#include <sys/uio.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "core/aesgcm.h"
#include "core/buf.h"
#include "core/net.h"

namespace p2pt::rtc {

// One thread that runs submitted jobs in submission order.
class Lane {
 public:
  explicit Lane(const char* name);
  ~Lane();  // runs what is queued, then joins
  Lane(const Lane&) = delete;
  Lane& operator=(const Lane&) = delete;
  void submit(std::function<void()> job);
  // Nothing queued or running (the last job's effects are visible).
  bool idle() const { return pending_.load(std::memory_order_acquire) == 0; }

 private:
  void run();
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::function<void()>> q_;
  bool stop_ = false;
  std::atomic<int> pending_{0};
  std::thread th_;
};

// A dup() of the ICE agent's socket for the TX lane: the lane sends on its
// own descriptor, so the agent closing (or the kernel reusing) its fd number
// never points a queued batch at another socket.
struct LaneFd {
  int fd = -1;
  int src = -1;      // the agent's descriptor it duplicates
  uint64_t gen = 0;  // the ICE path generation it was taken for (an fd number can be reused)
  explicit LaneFd(int source, uint64_t generation = 0);
  ~LaneFd();
};

// Where the TX lane sends: the selected pair's socket and remote address, and
// how many bytes of records may share one datagram (same-host jumbo paths).
struct TxTarget {
  int fd = -1;
  SockAddr to;
  size_t coalesce = 0;
  uint64_t gen = 0;  // IceAgent::path_generation() of this target
};

// One flush's records: inline bytes (SCTP headers, small chunks) copied into
// `arena`, large body slices referenced in place and kept alive by `keep`.
struct TxBatch {
  struct Piece {
    const uint8_t* p;   // nullptr: arena[off, off + n)
    uint32_t off;
    uint32_t n;
  };
  struct Rec {
    uint64_t seq;
    uint8_t type;
    uint32_t first, count;  // pieces
    uint32_t total;         // plaintext bytes
  };
  std::vector<uint8_t> arena;
  std::vector<Piece> pieces;
  std::vector<Rec> recs;
  std::vector<std::shared_ptr<const void>> keep;
  size_t bytes = 0;  // plaintext bytes of all records
  const void* last_owner = nullptr;
  void clear();
  // Appends one record; `owners[i]` (may be null) keeps iov[i] alive, or the
  // piece is copied into the arena.
  void add(uint64_t seq, uint8_t type, const iovec* iov, const Bytes* const* owners, int cnt);
  // The gather list of record r (arena pieces resolved; arena must be final).
  int gather(const Rec& r, iovec* out, int max) const;
};

// Finished TX batches travel back to the association thread for reuse, so
// their buffers are allocated once and never freed across threads.
class TxBatchPool {
 public:
  std::shared_ptr<TxBatch> get() {
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.empty()) return std::make_shared<TxBatch>();
    auto b = std::move(free_.back());
    free_.pop_back();
    return b;
  }
  void put(std::shared_ptr<TxBatch> b) {  // any thread; b already cleared
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.size() < 64) free_.push_back(std::move(b));
  }

 private:
  std::mutex mu_;
  std::vector<std::shared_ptr<TxBatch>> free_;
};

// Application records of one receive burst, decrypted in place by the lane.
struct RxBatch {
  struct Rec {
    uint8_t* rec;
    uint32_t len;
    uint8_t type;
    bool ok = false;
    uint64_t seq;
    uint8_t* pt = nullptr;
    uint32_t ptl = 0;
    std::shared_ptr<const void> owner;
  };
  std::vector<Rec> recs;
  size_t bytes = 0;
};

// Record crypto shared by the association thread and the lanes (the keys are
// immutable once derived).
struct RecordKeys {
  std::shared_ptr<const AesGcm> w, r;
  uint8_t wiv[4] = {}, riv[4] = {};
};
constexpr size_t kRecHdr = 13;    // type, version(2), epoch(2), seq(6), length(2)
constexpr size_t kExplicit = 8;   // GCM explicit nonce
constexpr size_t kTag = 16;
inline size_t record_size(size_t plaintext) { return kRecHdr + kExplicit + plaintext + kTag; }
// DTLS 1.2 epoch-1 AEAD record of `type`/`seq` from the gather list, into out.
void seal_record(const AesGcm& g, const uint8_t iv[4], uint8_t* out, uint8_t type, uint64_t seq, const iovec* iov,
                 int cnt, size_t total);
// Authenticates and decrypts one record in place; false if it fails.
bool open_record(const AesGcm& g, const uint8_t iv[4], uint8_t* rec, size_t len, uint8_t** pt, size_t* ptl);

// One TX batch after sealing: the records back to back in `out`, datagram
// boundaries aside (several records per datagram on same-host jumbo paths).
struct SealedBatch {
  std::vector<uint8_t> out;
  std::vector<std::pair<size_t, size_t>> dgs;  // (offset, length) in out
};

// TX lane state. The lane is a two-stage pipeline: the seal stage encrypts a
// batch into a SealedBatch, the send stage (a thread of its own) hands it to
// the kernel with sendmmsg + UDP GSO, in batch order, while the seal stage
// works on the next batch. On the MI355X host the single TX lane that did
// both was the saturated stage of the 64 x 1 MB echo (>= 90 % CPU in 54-82 %
// of its active 2 ms intervals at 1200-byte MTU, the association thread
// under 10 %; profiles/r04/flow_ab), its time split about evenly between
// AES-GCM and sendmmsg.
class TxLaneState {
 public:
  TxLaneState();
  // Seal stage: encrypts the batch (runs on the seal lane).
  void seal(const TxBatch& b, const RecordKeys& k, size_t coalesce, SealedBatch& out);
  // Send stage: sends a sealed batch to target (runs on the send lane).
  void send(SealedBatch& s, int fd, const SockAddr& to);
  // Both stages in a row (tests).
  void run(const TxBatch& b, const RecordKeys& k, int fd, const SockAddr& to, size_t coalesce);
  // Sealed batches are recycled between the stages (buffers allocated once).
  std::shared_ptr<SealedBatch> get_sealed();
  void put_sealed(std::shared_ptr<SealedBatch> s);
  // send_drops: datagrams dropped (socket buffer still full after kSendWaitMs
  // of POLLOUT waits, or unreachable); send_waits: POLLOUT waits taken.
  std::atomic<uint64_t> batches{0}, records{0}, datagrams{0}, gso_msgs{0}, send_drops{0}, send_waits{0};
  static constexpr int kSendWaitMs = 20;

 private:
  SealedBatch one_;  // run()'s buffer
  std::vector<size_t> offs_;    // record offsets in out (seal stage only)
  bool gso_ok_ = true;  // send stage only
  std::mutex mu_;
  std::vector<std::shared_ptr<SealedBatch>> free_;
};

// Tests: a paused reader's escape (it reads on once the socket buffer is half
// full) on or off for readers created afterwards (default on).
bool rx_escape_enabled();
void set_rx_escape_enabled(bool on);

// Socket reader: the selected pair's UDP socket read on a thread of its own
// (recvmmsg + GRO), application records from the selected remote opened
// there, everything else (STUN, handshake or alert records, other senders)
// passed on untouched. A burst goes to the association thread through
// `deliver`, which must post it (it runs on the reader); the association
// thread calls done() once it has processed one, and the reader stops
// reading (the socket buffer holds, then drops) while kMaxOutstanding bursts
// wait, so a slow association thread never piles up pinned buffers.
//
// Engaged only under bulk (adaptive, the default): every datagram the reader
// reads reaches the association thread through a second wake-up, and on the
// MI355X host that hop put the headline's added p50 TTFT at 0.244 ms against
// 0.162 ms with the association thread reading the socket itself (3
// interleaved runs each, profiles/r05/b01). So an adaptive reader starts
// paused: the association thread reads the socket (one thread per hop for
// tokens and requests) until its receive rate is bulk-like, then hands the
// socket over (engage()); the reader hands it back — a Burst with `handback`
// set, after everything it read — once it has read less than kIdleBytes in
// kIdleUs.
class RxReader {
 public:
  struct Raw {
    RawBufPtr buf;
    uint32_t off, len;
    SockAddr from;
  };
  struct Burst {
    RxBatch opened;         // application records, authenticated (ok) or not
    std::vector<Raw> raw;   // datagrams for the ICE agent / DTLS state machine
    uint64_t reader = 0;    // id of the RxReader that read it (done() goes to that one only)
    int si = -1;            // the ICE socket index it was read from (set by the deliver hook)
    bool handback = false;  // adaptive reader: paused; the socket is the association thread's again
    uint64_t t_read = 0, t_kernel = 0;  // traced runs: when it was read / queued by the kernel (us)
  };
  using Deliver = std::function<void(std::unique_ptr<Burst>)>;
  static constexpr int kMaxOutstanding = 4;
  static constexpr uint64_t kIdleUs = 20000;         // adaptive: hand back after this long ...
  static constexpr size_t kIdleBytes = 256 * 1024;   // ... with less than this read in it (12.8 MB/s)

  // `slot`: receive buffer per datagram — 64 KiB when the socket coalesces
  // (UDP GRO), else the largest datagram the path carries (a 1200-byte
  // datagram in a 64 KiB slot pinned ~50x its size per burst); a datagram
  // larger than the slot (a peer with larger packets) grows it to 64 KiB.
  // `adaptive`: start paused, run only between engage() and a handback.
  // `idle_us` / `idle_bytes`: the adaptive reader's handback window.
  RxReader(int fd, const SockAddr& remote, std::shared_ptr<const RecordKeys> keys, Deliver deliver, uint64_t id = 0,
           size_t slot = 65536, bool adaptive = false, uint64_t idle_us = kIdleUs, size_t idle_bytes = kIdleBytes);
  uint64_t id() const { return id_; }
  size_t slot() const { return slot_.load(std::memory_order_relaxed); }
  ~RxReader();  // stops and joins; bursts already delivered stay valid
  RxReader(const RxReader&) = delete;
  RxReader& operator=(const RxReader&) = delete;
  void done();  // association thread: one delivered burst processed
  // Association thread, adaptive reader: it has detached the socket from its
  // reactor (everything it read is processed); the reader reads from now on.
  void engage();
  bool engaged() const { return active_.load(std::memory_order_acquire); }
  std::atomic<uint64_t> engages{0}, handbacks{0};

  // waits: back-pressure pauses (the association thread kMaxOutstanding
  // bursts behind); escapes: reads taken anyway because the socket buffer was
  // past half full (a pause there would end in kernel drops).
  std::atomic<uint64_t> bursts{0}, datagrams{0}, records{0}, raw_datagrams{0}, waits{0}, escapes{0}, gro_batches{0};
  // The socket's drop count as last reported by SO_RXQ_OVFL (cumulative).
  std::atomic<uint32_t> rxq_ovfl{0};
  std::atomic<uint64_t> truncated{0};  // datagrams larger than a slot (MSG_TRUNC): lost
  std::atomic<uint64_t> lane_bursts{0};  // bursts whose records the open lanes decrypted

  // Bursts of at least this many bytes of records are decrypted on the open
  // lanes (kOpenLanes threads, bursts alternating between them) while this
  // thread reads on; smaller ones here. The 1200-MTU download next to SSE had
  // the reader at >= 90 % CPU in 94 % of its active intervals, opening every
  // record itself (profiles/r05/b13/mixed_tl.json).
  static constexpr int kOpenLanes = 2;
  static constexpr size_t kLaneBytes = 64 * 1024;

 private:
  void run();
  void segment(const RawBufPtr& buf, uint32_t off, uint32_t len, const SockAddr& from, Burst& b);
  void open_burst(Burst& b) const;
  // Bursts go up in read order whichever thread opened them (`seq`).
  void complete(uint64_t seq, std::unique_ptr<Burst> b);
  LaneFd fd_;
  int stop_fd_ = -1;
  SockAddr remote_;
  std::shared_ptr<const RecordKeys> keys_;
  Deliver deliver_;
  uint64_t id_ = 0;
  bool escape_ = rx_escape_enabled();
  std::atomic<size_t> slot_{65536};
  BufPool pool_{65536};
  bool adaptive_ = false;
  uint64_t idle_us_ = kIdleUs;
  size_t idle_bytes_ = kIdleBytes;
  std::atomic<bool> active_{true};
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<int> outstanding_{0};
  std::atomic<bool> stop_{false};
  uint64_t seq_next_ = 0;  // reader thread
  std::mutex ord_mu_;
  uint64_t seq_deliver_ = 0;                                // ord_mu_
  std::vector<std::pair<uint64_t, std::unique_ptr<Burst>>> ready_;  // ord_mu_: opened, waiting for an earlier one
  std::unique_ptr<Lane> open_[kOpenLanes];
  int n_open_ = kOpenLanes;  // lanes started (affinity::open_lane_count)
  int next_lane_ = 0;
  std::thread th_;  // last: started after everything above exists
};

// Flushes and receive bursts below this are sealed / opened on the association
// thread itself (no hand-off on a token's path).
constexpr size_t kInlineBytes = 32 * 1024;
inline size_t datapath_inline_bytes() { return kInlineBytes; }
// TUNNEL_RX_READER: 0 = the association thread always reads the socket, 1 =
// a reader always does (round 4), unset = adaptive (engaged under bulk).
enum RxReaderMode { kRxReaderOff = 0, kRxReaderAlways = 1, kRxReaderAdaptive = 2 };
int rx_reader_mode();
void set_rx_reader_mode(int mode);  // tests: every receive path in one process
inline bool rx_reader_enabled() { return rx_reader_mode() != kRxReaderOff; }
inline void set_rx_reader_enabled(bool on) { set_rx_reader_mode(on ? kRxReaderAlways : kRxReaderOff); }

}  // namespace p2pt::rtc
