// Refcounted immutable byte slices + a growable write buffer.
//
// Equivalent of the `bytes` crate usage in the reference (zero-copy decode of
// tunnel frames, reference tunnel/src/protocol.rs:157-172). A Bytes is a view
// into a shared, immutable allocation: slicing never copies.
#pragma once

#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace p2pt {

class Bytes {
 public:
  Bytes() = default;

  static Bytes copy(const void* p, size_t n) {
    auto v = std::make_shared<std::vector<uint8_t>>(static_cast<const uint8_t*>(p),
                                                    static_cast<const uint8_t*>(p) + n);
    return Bytes(std::move(v));
  }
  static Bytes copy(std::string_view s) { return copy(s.data(), s.size()); }
  static Bytes take(std::vector<uint8_t>&& v) {
    return Bytes(std::make_shared<std::vector<uint8_t>>(std::move(v)));
  }
  static Bytes take(std::string&& s) { return copy(s.data(), s.size()); }
  // View of memory kept alive by an arbitrary owner (e.g. a pooled receive
  // buffer that received datagrams are decrypted in place into).
  static Bytes adopt(std::shared_ptr<const void> owner, const uint8_t* p, size_t n) {
    Bytes b;
    b.owner_ = std::move(owner);
    b.ptr_ = p;
    b.len_ = n;
    return b;
  }

  const uint8_t* data() const { return ptr_; }
  size_t size() const { return len_; }
  bool empty() const { return len_ == 0; }
  uint8_t operator[](size_t i) const { return ptr_[i]; }
  const uint8_t* begin() const { return ptr_; }
  const uint8_t* end() const { return ptr_ + len_; }

  // Zero-copy sub-view sharing the same owner.
  Bytes slice(size_t off, size_t n = SIZE_MAX) const {
    Bytes b;
    if (off > len_) off = len_;
    if (n > len_ - off) n = len_ - off;
    b.owner_ = owner_;
    b.ptr_ = ptr_ + off;
    b.len_ = n;
    return b;
  }
  std::string_view view() const { return {reinterpret_cast<const char*>(ptr_), len_}; }
  // What keeps the bytes alive (null for views of unowned memory).
  const std::shared_ptr<const void>& owner() const { return owner_; }
  std::string str() const { return std::string(view()); }
  bool operator==(const Bytes& o) const {
    return len_ == o.len_ && (len_ == 0 || std::memcmp(ptr_, o.ptr_, len_) == 0);
  }

 private:
  explicit Bytes(std::shared_ptr<std::vector<uint8_t>> v) : ptr_(v->data()), len_(v->size()) { owner_ = std::move(v); }
  std::shared_ptr<const void> owner_;
  const uint8_t* ptr_ = nullptr;
  size_t len_ = 0;
};

// Fixed-size, uninitialised, refcounted buffer (datagram receive/send pools).
// A pool hands one out again once use_count() drops back to 1, i.e. once no
// Bytes view into it is alive. Cache-line aligned so that make_shared puts
// every buffer's reference counts on a line of their own: buffers handed out
// one after another (token slabs, pipe arenas) are filled by one thread while
// another drops the views of the previous one, and counts sharing a line made
// each update a cross-core miss (the proxy's association thread spent 12 % of
// its time copying a buffer reference in ProxySession::route at 1024 streams,
// profiles/r05/b20/nodeprof).
struct alignas(64) RawBuf {
  explicit RawBuf(size_t n) : data(new uint8_t[n]), cap(n) {}
  std::unique_ptr<uint8_t[]> data;
  size_t cap;
};
using RawBufPtr = std::shared_ptr<RawBuf>;
// Call after seeing use_count() == 1 and before writing into the buffer again:
// views may live on worker threads (tunnel/workers.h), and use_count() is a
// relaxed load, so this orders the reuse after their last reads.
inline void reuse_fence() { std::atomic_thread_fence(std::memory_order_acquire); }

// Recycling pool of fixed-size receive buffers whose contents are handed up
// the stack as zero-copy views (datagram receive: DTLS decrypts in place and
// SCTP messages are views of the datagram). A buffer goes back into service
// once no view of it is alive (use_count() == 1: only the pool holds it),
// wherever the last view was dropped — on a worker thread, typically. Without
// it every receive slot whose previous datagram is still being written to a
// client would need a fresh 64 KiB allocation (and a cross-thread free later).
class BufPool {
 public:
  explicit BufPool(size_t buf_size, size_t max_keep = 512) : size_(buf_size), max_keep_(max_keep) {}
  RawBufPtr get() {
    // Buffers come back roughly in the order they went out, so a short scan
    // from the rotating cursor finds a free one; when it does not, the pool
    // grows (up to max_keep) rather than scanning every pinned buffer.
    size_t n = bufs_.size();
    for (size_t k = 0; k < n && k < kScan; k++) {
      size_t i = next_ + k < n ? next_ + k : next_ + k - n;
      if (bufs_[i].use_count() == 1) {
        reuse_fence();
        next_ = i + 1 < n ? i + 1 : 0;
        return bufs_[i];
      }
    }
    auto b = std::make_shared<RawBuf>(size_);
    if (n < max_keep_) {
      bufs_.insert(bufs_.begin() + long(next_ < n ? next_ : n), b);  // scanned last next time round
      next_ = next_ < n ? next_ + 1 : 0;
    }
    return b;
  }
  size_t size() const { return bufs_.size(); }

 private:
  static constexpr size_t kScan = 16;
  size_t size_, max_keep_;
  std::vector<RawBufPtr> bufs_;
  size_t next_ = 0;
};

// Copies of small byte ranges (SSE tokens read from an upstream socket, chunk
// headers) packed into per-thread 64 KiB blocks instead of one heap
// allocation each: the block is shared by the views and recycled once they
// are all gone. Frames cross threads (tunnel/workers.h), so per-piece mallocs
// would be freed on another thread's arena — the contention this avoids.
inline Bytes slab_copy(const void* p, size_t n) {
  constexpr size_t kBlock = 64 * 1024, kMax = 2048;
  if (n == 0 || n > kMax) return Bytes::copy(p, n);
  struct Slab {
    BufPool pool{kBlock, 64};
    RawBufPtr cur;
    size_t off = kBlock;
  };
  thread_local Slab s;
  if (s.off + n > kBlock) {
    s.cur.reset();  // a block in use stays alive through its views, then returns to the pool
    s.cur = s.pool.get();
    s.off = 0;
  }
  uint8_t* d = s.cur->data.get() + s.off;
  memcpy(d, p, n);
  s.off += (n + 15) & ~size_t(15);
  return Bytes::adopt(s.cur, d, n);
}

// Append-only big-endian writer over a std::vector.
class ByteWriter {
 public:
  explicit ByteWriter(std::vector<uint8_t>& out) : out_(out) {}
  void u8(uint8_t v) { out_.push_back(v); }
  void u16(uint16_t v) {
    out_.push_back(uint8_t(v >> 8));
    out_.push_back(uint8_t(v));
  }
  void u32(uint32_t v) {
    out_.push_back(uint8_t(v >> 24));
    out_.push_back(uint8_t(v >> 16));
    out_.push_back(uint8_t(v >> 8));
    out_.push_back(uint8_t(v));
  }
  void u64(uint64_t v) {
    u32(uint32_t(v >> 32));
    u32(uint32_t(v));
  }
  void bytes(const void* p, size_t n) {
    out_.insert(out_.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n);
  }
  void bytes(std::string_view s) { bytes(s.data(), s.size()); }
  void zeros(size_t n) { out_.insert(out_.end(), n, 0); }
  size_t size() const { return out_.size(); }
  std::vector<uint8_t>& vec() { return out_; }

 private:
  std::vector<uint8_t>& out_;
};

inline uint16_t rd16(const uint8_t* p) { return uint16_t(p[0] << 8 | p[1]); }
inline uint32_t rd32(const uint8_t* p) {
  return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | uint32_t(p[3]);
}
inline uint64_t rd64(const uint8_t* p) { return uint64_t(rd32(p)) << 32 | rd32(p + 4); }
inline void wr16(uint8_t* p, uint16_t v) {
  p[0] = uint8_t(v >> 8);
  p[1] = uint8_t(v);
}
inline void wr32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24);
  p[1] = uint8_t(v >> 16);
  p[2] = uint8_t(v >> 8);
  p[3] = uint8_t(v);
}

// Bounds-checked big-endian reader.
class ByteReader {
 public:
  ByteReader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  bool has(size_t k) const { return n_ - off_ >= k; }
  size_t remaining() const { return n_ - off_; }
  size_t offset() const { return off_; }
  const uint8_t* cur() const { return p_ + off_; }
  bool u8(uint8_t& v) {
    if (!has(1)) return false;
    v = p_[off_++];
    return true;
  }
  bool u16(uint16_t& v) {
    if (!has(2)) return false;
    v = rd16(p_ + off_);
    off_ += 2;
    return true;
  }
  bool u32(uint32_t& v) {
    if (!has(4)) return false;
    v = rd32(p_ + off_);
    off_ += 4;
    return true;
  }
  bool skip(size_t k) {
    if (!has(k)) return false;
    off_ += k;
    return true;
  }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t off_ = 0;
};

}  // namespace p2pt
