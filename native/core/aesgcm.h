// AES-GCM (NIST SP 800-38D, 96-bit IVs, 128-bit tags) for the DTLS record
// layer, on VAES + VPCLMULQDQ (AVX-512): 32 counter blocks per round of
// 512-bit AES instructions stitched with a 32-block aggregated GHASH (one
// reduction per 512 bytes). OpenSSL 3.0's AES-NI/AVX code ran ~7 GB/s per
// core on the MI355X hosts' EPYC 9575F and was ~40 % of a tunnel process in
// the 64 x 1 MB body benchmark (profiles/bulk_profile_*).
//
// Falls back to nothing by itself: init() returns false on a CPU without
// AVX-512F/BW/VL + VAES + VPCLMULQDQ, and the caller keeps OpenSSL's EVP path.
// Verified against EVP and the GCM specification's test vectors
// (native/tests/test_core.cc aesgcm_*), and at every DTLS session start
// against a record OpenSSL itself encrypted (native/rtc/dtls.cc).
#pragma once

#include <sys/uio.h>

#include <cstddef>
#include <cstdint>

namespace p2pt {

class AesGcm {
 public:
  AesGcm() = default;
  AesGcm(const AesGcm&) = delete;
  AesGcm& operator=(const AesGcm&) = delete;
  ~AesGcm();

  static bool supported();
  // 16- or 32-byte key. False (and unusable) on a CPU without the extensions.
  bool init(const uint8_t* key, size_t key_len);
  bool ready() const { return rounds_ != 0; }

  // in == out is allowed.
  void seal(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const uint8_t* in, uint8_t* out, size_t n,
            uint8_t tag[16]) const;
  // Same, reading the plaintext from a gather list totalling n bytes (no
  // gather copy); out must not overlap the pieces.
  void seal_gather(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const iovec* iov, int cnt, uint8_t* out,
                   size_t n, uint8_t tag[16]) const;
  // Decrypts in -> out (in == out allowed) and checks the tag; on failure
  // returns false with out zeroed.
  bool open(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const uint8_t* in, uint8_t* out, size_t n,
            const uint8_t tag[16]) const;

 private:
  alignas(64) uint8_t rk_[15][64];    // round keys, each broadcast to 4 lanes
  alignas(64) uint8_t hpow_[32][16];  // H^32 .. H^1, bit-reflected (GHASH domain)
  int rounds_ = 0;
};

}  // namespace p2pt
