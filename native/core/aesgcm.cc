// AES-GCM on VAES + VPCLMULQDQ. See aesgcm.h.
//
// GHASH runs in the bit-reflected domain of Gueron & Kounavis ("Intel
// Carry-Less Multiplication Instruction and its Usage for Computing the GCM
// Mode"): blocks are byte-reversed, multiplied with four PCLMULQDQs, the
// 256-bit product shifted left by one and reduced modulo
// x^128 + x^7 + x^2 + x + 1. Shift and reduction are linear, so 16 products
// (X_i * H^(33-i) for 512-byte chunks) are summed unreduced and reduced once.
#include "core/aesgcm.h"

#include <immintrin.h>
#include <openssl/crypto.h>

#include <cstring>

namespace p2pt {

namespace {

#pragma GCC push_options
#pragma GCC target("aes,pclmul,ssse3,sse4.1,avx2,avx512f,avx512bw,avx512vl,vaes,vpclmulqdq")

inline __m128i bswap128(__m128i x) {
  return _mm_shuffle_epi8(x, _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
}

inline __m512i bswap_mask512() {
  return _mm512_broadcast_i32x4(_mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
}

// ---------------------------------------------------------------- key schedule
inline __m128i kx_mix(__m128i k, __m128i a) {
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
  return _mm_xor_si128(k, a);
}
// First word of a new 4-word group: SubWord(RotWord(w)) ^ rcon (dword 3).
#define P2PT_KX_A(prev, last, rc) kx_mix(prev, _mm_shuffle_epi32(_mm_aeskeygenassist_si128(last, rc), 0xff))
// AES-256 middle group: SubWord(w) (dword 2), no rotation or rcon.
#define P2PT_KX_B(prev, last) kx_mix(prev, _mm_shuffle_epi32(_mm_aeskeygenassist_si128(last, 0), 0xaa))

void expand128(const uint8_t* key, __m128i* rk) {
  rk[0] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key));
  rk[1] = P2PT_KX_A(rk[0], rk[0], 0x01);
  rk[2] = P2PT_KX_A(rk[1], rk[1], 0x02);
  rk[3] = P2PT_KX_A(rk[2], rk[2], 0x04);
  rk[4] = P2PT_KX_A(rk[3], rk[3], 0x08);
  rk[5] = P2PT_KX_A(rk[4], rk[4], 0x10);
  rk[6] = P2PT_KX_A(rk[5], rk[5], 0x20);
  rk[7] = P2PT_KX_A(rk[6], rk[6], 0x40);
  rk[8] = P2PT_KX_A(rk[7], rk[7], 0x80);
  rk[9] = P2PT_KX_A(rk[8], rk[8], 0x1b);
  rk[10] = P2PT_KX_A(rk[9], rk[9], 0x36);
}

void expand256(const uint8_t* key, __m128i* rk) {
  rk[0] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key));
  rk[1] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key + 16));
  rk[2] = P2PT_KX_A(rk[0], rk[1], 0x01);
  rk[3] = P2PT_KX_B(rk[1], rk[2]);
  rk[4] = P2PT_KX_A(rk[2], rk[3], 0x02);
  rk[5] = P2PT_KX_B(rk[3], rk[4]);
  rk[6] = P2PT_KX_A(rk[4], rk[5], 0x04);
  rk[7] = P2PT_KX_B(rk[5], rk[6]);
  rk[8] = P2PT_KX_A(rk[6], rk[7], 0x08);
  rk[9] = P2PT_KX_B(rk[7], rk[8]);
  rk[10] = P2PT_KX_A(rk[8], rk[9], 0x10);
  rk[11] = P2PT_KX_B(rk[9], rk[10]);
  rk[12] = P2PT_KX_A(rk[10], rk[11], 0x20);
  rk[13] = P2PT_KX_B(rk[11], rk[12]);
  rk[14] = P2PT_KX_A(rk[12], rk[13], 0x40);
}
#undef P2PT_KX_A
#undef P2PT_KX_B

inline __m128i rk128(const uint8_t (*rk)[64], int r) { return _mm_load_si128(reinterpret_cast<const __m128i*>(rk[r])); }
inline __m512i rk512(const uint8_t (*rk)[64], int r) { return _mm512_load_si512(rk[r]); }

inline __m128i enc_block(const uint8_t (*rk)[64], int nr, __m128i x) {
  x = _mm_xor_si128(x, rk128(rk, 0));
  for (int r = 1; r < nr; r++) x = _mm_aesenc_si128(x, rk128(rk, r));
  return _mm_aesenclast_si128(x, rk128(rk, nr));
}

// ---------------------------------------------------------------- GHASH
#define P2PT_CLMUL(a, b, s) _mm_clmulepi64_si128(a, b, s)

// (hi:mid:lo) unreduced product in the reflected domain -> reduced product.
inline __m128i gf_reduce(__m128i lo, __m128i mid, __m128i hi) {
  __m128i t3 = _mm_xor_si128(lo, _mm_slli_si128(mid, 8));
  __m128i t6 = _mm_xor_si128(hi, _mm_srli_si128(mid, 8));
  // 256-bit shift left by one (bit reflection)
  __m128i t7 = _mm_srli_epi32(t3, 31);
  __m128i t8 = _mm_srli_epi32(t6, 31);
  t3 = _mm_slli_epi32(t3, 1);
  t6 = _mm_slli_epi32(t6, 1);
  __m128i t9 = _mm_srli_si128(t7, 12);
  t8 = _mm_slli_si128(t8, 4);
  t7 = _mm_slli_si128(t7, 4);
  t3 = _mm_or_si128(t3, t7);
  t6 = _mm_or_si128(_mm_or_si128(t6, t8), t9);
  // reduction
  t7 = _mm_xor_si128(_mm_xor_si128(_mm_slli_epi32(t3, 31), _mm_slli_epi32(t3, 30)), _mm_slli_epi32(t3, 25));
  t8 = _mm_srli_si128(t7, 4);
  t7 = _mm_slli_si128(t7, 12);
  t3 = _mm_xor_si128(t3, t7);
  __m128i t2 = _mm_xor_si128(_mm_xor_si128(_mm_srli_epi32(t3, 1), _mm_srli_epi32(t3, 2)), _mm_srli_epi32(t3, 7));
  t2 = _mm_xor_si128(t2, t8);
  t3 = _mm_xor_si128(t3, t2);
  return _mm_xor_si128(t6, t3);
}

inline __m128i gf_mul(__m128i a, __m128i b) {
  __m128i lo = P2PT_CLMUL(a, b, 0x00);
  __m128i hi = P2PT_CLMUL(a, b, 0x11);
  __m128i mid = _mm_xor_si128(P2PT_CLMUL(a, b, 0x01), P2PT_CLMUL(a, b, 0x10));
  return gf_reduce(lo, mid, hi);
}

inline __m128i fold4(__m512i v) {
  __m256i a = _mm256_xor_si256(_mm512_castsi512_si256(v), _mm512_extracti64x4_epi64(v, 1));
  return _mm_xor_si128(_mm256_castsi256_si128(a), _mm256_extracti128_si256(a, 1));
}

// y <- GHASH_H(y, data zero-padded to a block multiple). hp = H^16..H^1.
// (Also the tail after the stitched 512-byte chunks.)
__m128i ghash(const uint8_t (*hp)[16], __m128i y, const uint8_t* p, size_t n) {
  const __m512i bsw = bswap_mask512();
  if (n >= 256) {
    const __m512i h0 = _mm512_loadu_si512(hp[0]), h1 = _mm512_loadu_si512(hp[4]);
    const __m512i h2 = _mm512_loadu_si512(hp[8]), h3 = _mm512_loadu_si512(hp[12]);
    do {
      __m512i x0 = _mm512_shuffle_epi8(_mm512_loadu_si512(p), bsw);
      __m512i x1 = _mm512_shuffle_epi8(_mm512_loadu_si512(p + 64), bsw);
      __m512i x2 = _mm512_shuffle_epi8(_mm512_loadu_si512(p + 128), bsw);
      __m512i x3 = _mm512_shuffle_epi8(_mm512_loadu_si512(p + 192), bsw);
      x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(y));
      __m512i lo = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x0, h0, 0x00),
                                             _mm512_clmulepi64_epi128(x1, h1, 0x00),
                                             _mm512_clmulepi64_epi128(x2, h2, 0x00), 0x96);
      lo = _mm512_xor_si512(lo, _mm512_clmulepi64_epi128(x3, h3, 0x00));
      __m512i hi = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x0, h0, 0x11),
                                             _mm512_clmulepi64_epi128(x1, h1, 0x11),
                                             _mm512_clmulepi64_epi128(x2, h2, 0x11), 0x96);
      hi = _mm512_xor_si512(hi, _mm512_clmulepi64_epi128(x3, h3, 0x11));
      __m512i mid = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x0, h0, 0x01),
                                              _mm512_clmulepi64_epi128(x0, h0, 0x10),
                                              _mm512_clmulepi64_epi128(x1, h1, 0x01), 0x96);
      mid = _mm512_ternarylogic_epi64(mid, _mm512_clmulepi64_epi128(x1, h1, 0x10),
                                      _mm512_clmulepi64_epi128(x2, h2, 0x01), 0x96);
      mid = _mm512_ternarylogic_epi64(mid, _mm512_clmulepi64_epi128(x2, h2, 0x10),
                                      _mm512_clmulepi64_epi128(x3, h3, 0x01), 0x96);
      mid = _mm512_xor_si512(mid, _mm512_clmulepi64_epi128(x3, h3, 0x10));
      y = gf_reduce(fold4(lo), fold4(mid), fold4(hi));
      p += 256;
      n -= 256;
    } while (n >= 256);
  }
  if (n >= 64) {
    const __m512i h = _mm512_loadu_si512(hp[12]);  // H^4..H^1
    do {
      __m512i x = _mm512_shuffle_epi8(_mm512_loadu_si512(p), bsw);
      x = _mm512_xor_si512(x, _mm512_zextsi128_si512(y));
      __m512i lo = _mm512_clmulepi64_epi128(x, h, 0x00);
      __m512i hi = _mm512_clmulepi64_epi128(x, h, 0x11);
      __m512i mid = _mm512_xor_si512(_mm512_clmulepi64_epi128(x, h, 0x01), _mm512_clmulepi64_epi128(x, h, 0x10));
      y = gf_reduce(fold4(lo), fold4(mid), fold4(hi));
      p += 64;
      n -= 64;
    } while (n >= 64);
  }
  if (n) {
    const __m128i h1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(hp[15]));
    while (n >= 16) {
      y = gf_mul(_mm_xor_si128(y, bswap128(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p)))), h1);
      p += 16;
      n -= 16;
    }
    if (n) {
      __m128i x = _mm_maskz_loadu_epi8(__mmask16((1u << n) - 1), p);  // zero padding
      y = gf_mul(_mm_xor_si128(y, bswap128(x)), h1);
    }
  }
  return y;
}

// ---------------------------------------------------------------- CTR
// Plaintext/ciphertext sources for the CTR passes: a flat buffer, or the
// gather list of an outgoing record (SCTP headers inline, payload slices
// referenced), read 64 bytes at a time so sealing needs no gather copy.
struct FlatSrc {
  const uint8_t* p;
  __m512i next64() {
    const __m512i v = _mm512_loadu_si512(p);
    p += 64;
    return v;
  }
  __m512i last(size_t n) { return _mm512_maskz_loadu_epi8(~0ULL >> (64 - n), p); }  // 0 < n < 64
};

struct GatherSrc {
  const iovec* iov;
  int cnt;
  int i = 0;
  size_t pos = 0;
  __m512i next64() {
    while (i < cnt && pos == iov[i].iov_len) {
      i++;
      pos = 0;
    }
    if (i < cnt && iov[i].iov_len - pos >= 64) {  // common case: inside one piece
      const __m512i v = _mm512_loadu_si512(static_cast<const uint8_t*>(iov[i].iov_base) + pos);
      pos += 64;
      return v;
    }
    return assemble(64);
  }
  __m512i last(size_t n) { return assemble(n); }
  __m512i assemble(size_t want) {  // across piece boundaries (a few times per record)
    alignas(64) uint8_t t[64] = {};
    size_t got = 0;
    while (got < want && i < cnt) {
      const size_t avail = iov[i].iov_len - pos;
      if (!avail) {
        i++;
        pos = 0;
        continue;
      }
      const size_t take = avail < want - got ? avail : want - got;
      memcpy(t + got, static_cast<const uint8_t*>(iov[i].iov_base) + pos, take);
      got += take;
      pos += take;
    }
    return _mm512_load_si512(t);
  }
};

struct CtrState {
  __m512i c, cmask, inc4, k0, klast;
  CtrState(const uint8_t (*rk)[64], int nr, const uint8_t iv[12], uint32_t ctr) {
    alignas(16) uint8_t b[16];
    memcpy(b, iv, 12);
    memcpy(b + 12, &ctr, 4);  // native (little-endian) counter word; byte-swapped per block
    const __m512i base = _mm512_broadcast_i32x4(_mm_load_si128(reinterpret_cast<const __m128i*>(b)));
    cmask = _mm512_broadcast_i32x4(_mm_set_epi8(12, 13, 14, 15, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0));
    inc4 = _mm512_set_epi32(4, 0, 0, 0, 4, 0, 0, 0, 4, 0, 0, 0, 4, 0, 0, 0);
    c = _mm512_add_epi32(base, _mm512_set_epi32(3, 0, 0, 0, 2, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0));
    k0 = rk512(rk, 0);
    klast = rk512(rk, nr);
  }
  __m512i next_block4() {  // 4 counter blocks, whitened with round key 0
    const __m512i b = _mm512_xor_si512(_mm512_shuffle_epi8(c, cmask), k0);
    c = _mm512_add_epi32(c, inc4);
    return b;
  }
};

// out = src ^ E(IV || ctr), E(IV || ctr+1), ... (32-bit big-endian counter),
// for the sub-512-byte tail.
template <class Src>
void ctr_xor(const uint8_t (*rk)[64], int nr, CtrState& st, Src& src, uint8_t* out, size_t n) {
  while (n) {
    __m512i b0 = st.next_block4();
    for (int r = 1; r < nr; r++) b0 = _mm512_aesenc_epi128(b0, rk512(rk, r));
    b0 = _mm512_aesenclast_epi128(b0, st.klast);
    if (n >= 64) {
      _mm512_storeu_si512(out, _mm512_xor_si512(b0, src.next64()));
      out += 64;
      n -= 64;
    } else {
      _mm512_mask_storeu_epi8(out, ~0ULL >> (64 - n), _mm512_xor_si512(b0, src.last(n)));
      n = 0;
    }
  }
}

// One 512-byte chunk (32 blocks) of GHASH, unreduced, against H^32..H^1; y
// is folded into the first block.
inline void gh_chunk512(const uint8_t (*hp)[16], const uint8_t* p, __m128i y, __m512i bsw, __m512i& lo,
                        __m512i& mid, __m512i& hi) {
  lo = mid = hi = _mm512_setzero_si512();
#pragma GCC unroll 8
  for (int j = 0; j < 8; j++) {
    __m512i x = _mm512_shuffle_epi8(_mm512_loadu_si512(p + 64 * j), bsw);
    if (j == 0) x = _mm512_xor_si512(x, _mm512_zextsi128_si512(y));
    const __m512i h = _mm512_loadu_si512(hp[4 * j]);
    lo = _mm512_xor_si512(lo, _mm512_clmulepi64_epi128(x, h, 0x00));
    hi = _mm512_xor_si512(hi, _mm512_clmulepi64_epi128(x, h, 0x11));
    mid = _mm512_ternarylogic_epi64(mid, _mm512_clmulepi64_epi128(x, h, 0x01), _mm512_clmulepi64_epi128(x, h, 0x10),
                                    0x96);
  }
}

// CTR over n (a multiple of 512) bytes stitched with GHASH so the AES
// (VAES) and carry-less multiply (VPCLMULQDQ) streams overlap. Decryption
// hashes the chunk it decrypts (its loads precede the stores, so in == out
// works); encryption hashes the ciphertext one chunk behind. hp = H^32..H^1.
template <bool ENC, class Src>
__m128i ctr_ghash512(const uint8_t (*rk)[64], int nr, const uint8_t (*hp)[16], CtrState& st, Src& src,
                     const uint8_t* in, uint8_t* out, size_t n, __m128i y) {
  const __m512i bsw = bswap_mask512();
  for (size_t off = 0; off < n; off += 512) {
    const uint8_t* gp = ENC ? (off ? out + off - 512 : nullptr) : in + off;
    __m512i blk[8];
#pragma GCC unroll 8
    for (int j = 0; j < 8; j++) blk[j] = st.next_block4();
    __m512i lo, mid, hi;
    if (gp) gh_chunk512(hp, gp, y, bsw, lo, mid, hi);
    for (int r = 1; r < nr; r++) {
      const __m512i k = rk512(rk, r);
#pragma GCC unroll 8
      for (int j = 0; j < 8; j++) blk[j] = _mm512_aesenc_epi128(blk[j], k);
    }
#pragma GCC unroll 8
    for (int j = 0; j < 8; j++)
      _mm512_storeu_si512(out + off + 64 * j, _mm512_xor_si512(_mm512_aesenclast_epi128(blk[j], st.klast),
                                                               src.next64()));
    if (gp) y = gf_reduce(fold4(lo), fold4(mid), fold4(hi));
  }
  if (ENC) {
    __m512i lo, mid, hi;
    gh_chunk512(hp, out + n - 512, y, bsw, lo, mid, hi);
    y = gf_reduce(fold4(lo), fold4(mid), fold4(hi));
  }
  return y;
}

__m128i ghash_len(const uint8_t (*hp16)[16], __m128i y, size_t aad_len, size_t n) {
  alignas(16) uint8_t lb[16];
  const uint64_t abits = uint64_t(aad_len) * 8, cbits = uint64_t(n) * 8;
  for (int i = 0; i < 8; i++) {
    lb[i] = uint8_t(abits >> (56 - 8 * i));
    lb[8 + i] = uint8_t(cbits >> (56 - 8 * i));
  }
  return ghash(hp16, y, lb, 16);
}

__m128i j0_block(const uint8_t iv[12]) {
  alignas(16) uint8_t b[16];
  memcpy(b, iv, 12);
  b[12] = b[13] = b[14] = 0;
  b[15] = 1;
  return _mm_load_si128(reinterpret_cast<const __m128i*>(b));
}

void setup(const uint8_t* key, size_t key_len, uint8_t (*rk)[64], uint8_t (*hp)[16], int* rounds) {
  __m128i k[15];
  int nr;
  if (key_len == 16) {
    expand128(key, k);
    nr = 10;
  } else {
    expand256(key, k);
    nr = 14;
  }
  for (int r = 0; r <= nr; r++) _mm512_store_si512(rk[r], _mm512_broadcast_i32x4(k[r]));
  const __m128i h = bswap128(enc_block(rk, nr, _mm_setzero_si128()));
  __m128i p = h;  // H^1
  for (int i = 31; i >= 0; i--) {  // hp[31] = H^1 ... hp[0] = H^32
    _mm_storeu_si128(reinterpret_cast<__m128i*>(hp[i]), p);
    p = gf_mul(p, h);
  }
  *rounds = nr;
  volatile __m128i* vk = k;  // do not leave the schedule on the stack
  for (int r = 0; r < 15; r++) vk[r] = _mm_setzero_si128();
}

template <class Src>
void seal_impl(const uint8_t (*rk)[64], const uint8_t (*hp)[16], int nr, const uint8_t iv[12], const uint8_t* aad,
               size_t aad_len, Src& src, uint8_t* out, size_t n, uint8_t tag[16]) {
  const uint8_t (*hp16)[16] = hp + 16;
  const __m128i ej0 = enc_block(rk, nr, j0_block(iv));
  __m128i y = ghash(hp16, _mm_setzero_si128(), aad, aad_len);
  CtrState st(rk, nr, iv, 2);
  const size_t big = n & ~size_t(511);
  if (big) y = ctr_ghash512<true>(rk, nr, hp, st, src, nullptr, out, big, y);
  ctr_xor(rk, nr, st, src, out + big, n - big);
  y = ghash_len(hp16, ghash(hp16, y, out + big, n - big), aad_len, n);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(tag), _mm_xor_si128(bswap128(y), ej0));
}

bool open_impl(const uint8_t (*rk)[64], const uint8_t (*hp)[16], int nr, const uint8_t iv[12], const uint8_t* aad,
               size_t aad_len, const uint8_t* in, uint8_t* out, size_t n, const uint8_t tag[16]) {
  const uint8_t (*hp16)[16] = hp + 16;
  const __m128i ej0 = enc_block(rk, nr, j0_block(iv));
  __m128i y = ghash(hp16, _mm_setzero_si128(), aad, aad_len);
  CtrState st(rk, nr, iv, 2);
  FlatSrc src{in};
  const size_t big = n & ~size_t(511);
  if (big) y = ctr_ghash512<false>(rk, nr, hp, st, src, in, out, big, y);
  y = ghash_len(hp16, ghash(hp16, y, in + big, n - big), aad_len, n);  // hash the tail before decrypting it
  ctr_xor(rk, nr, st, src, out + big, n - big);
  alignas(16) uint8_t want[16];
  _mm_store_si128(reinterpret_cast<__m128i*>(want), _mm_xor_si128(bswap128(y), ej0));
  if (CRYPTO_memcmp(want, tag, 16) == 0) return true;
  OPENSSL_cleanse(out, n);  // release no unauthenticated plaintext
  return false;
}

#undef P2PT_CLMUL
#pragma GCC pop_options

}  // namespace

bool AesGcm::supported() {
  static const bool ok = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("vaes") &&
           __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("aes") &&
           __builtin_cpu_supports("pclmul");
  }();
  return ok;
}

AesGcm::~AesGcm() {
  OPENSSL_cleanse(rk_, sizeof rk_);
  OPENSSL_cleanse(hpow_, sizeof hpow_);
}

bool AesGcm::init(const uint8_t* key, size_t key_len) {
  rounds_ = 0;
  if ((key_len != 16 && key_len != 32) || !supported()) return false;
  setup(key, key_len, rk_, hpow_, &rounds_);
  return true;
}

void AesGcm::seal(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const uint8_t* in, uint8_t* out, size_t n,
                  uint8_t tag[16]) const {
  FlatSrc src{in};
  seal_impl(rk_, hpow_, rounds_, iv, aad, aad_len, src, out, n, tag);
}

void AesGcm::seal_gather(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const iovec* iov, int cnt,
                         uint8_t* out, size_t n, uint8_t tag[16]) const {
  GatherSrc src{iov, cnt};
  seal_impl(rk_, hpow_, rounds_, iv, aad, aad_len, src, out, n, tag);
}

bool AesGcm::open(const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const uint8_t* in, uint8_t* out, size_t n,
                  const uint8_t tag[16]) const {
  return open_impl(rk_, hpow_, rounds_, iv, aad, aad_len, in, out, n, tag);
}

}  // namespace p2pt
