// bf16 helpers shared by the gfx950 kernels: raw uint16 storage, fp32 math,
// round-to-nearest-even packing, 16-byte (8 x bf16) vector unpack/pack, and
// LDS-free cross-lane reductions (DPP + gfx950 permlane swaps).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2pt_gpu {

constexpr int kWave = 64;

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(uint32_t(v) << 16); }

__device__ __forceinline__ uint32_t f2bf_bits(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);                       // round to nearest even
  return u >> 16;
}
// Value of f after a round trip through bf16.
__device__ __forceinline__ float bf_round(float f) { return __uint_as_float(f2bf_bits(f) << 16); }
__device__ __forceinline__ uint32_t pack2(float a, float b) { return f2bf_bits(a) | (f2bf_bits(b) << 16); }

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf_lo(v.x); f[1] = bf_hi(v.x);
  f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
  f[4] = bf_lo(v.z); f[5] = bf_hi(v.z);
  f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// Cross-lane reductions without LDS. __shfl_xor lowers to ds_bpermute (an
// LDS round trip, ~50+ cycles each, serialised by its waitcnt); these use
// DPP row operations inside 16-lane rows (fused into v_add/v_max) and the
// gfx950 half-swaps v_permlane16_swap / v_permlane32_swap across rows.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i <- 7-i within 8
constexpr int kDppMirror = 0x140;      // lane i <- 15-i within 16
constexpr int kDppXor8 = 0x128;        // row_ror:8 == lane i <- i^8 within 16

// All-reduce over 8-lane groups (only for values every lane of the group
// reduces fully: mirrors pair lanes i and 7-i, not i^4).
__device__ __forceinline__ float row8_sum(float v) {
  v += dpp<kDppXor1>(v);
  v += dpp<kDppXor2>(v);
  return v + dpp<kDppHalfMirror>(v);
}
__device__ __forceinline__ float row16_sum(float v) { v = row8_sum(v); return v + dpp<kDppMirror>(v); }
__device__ __forceinline__ float row8_max(float v) {
  v = fmaxf(v, dpp<kDppXor1>(v));
  v = fmaxf(v, dpp<kDppXor2>(v));
  return fmaxf(v, dpp<kDppHalfMirror>(v));
}
__device__ __forceinline__ float row16_max(float v) { v = row8_max(v); return fmaxf(v, dpp<kDppMirror>(v)); }
// Exact lane pairings i <-> i^8, i^16, i^32 (element-wise data may differ per lane).
__device__ __forceinline__ float xor8_sum(float v) { return v + dpp<kDppXor8>(v); }
__device__ __forceinline__ float xor8_max(float v) { return fmaxf(v, dpp<kDppXor8>(v)); }
__device__ __forceinline__ float xor16_sum(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor16_max(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// (value, index) argmax step, first index on ties.
__device__ __forceinline__ void am_take(float& b, int& i, float ob, int oi) {
  if (ob > b || (ob == b && oi < i)) {
    b = ob;
    i = oi;
  }
}
template <int CTRL>
__device__ __forceinline__ void am_dpp(float& b, int& i) {
  am_take(b, i, dpp<CTRL>(b), dpp_i<CTRL>(i));
}
// Argmax over each 16-lane row; every lane of the row ends with the winner.
__device__ __forceinline__ void row16_argmax(float& b, int& i) {
  am_dpp<kDppXor1>(b, i);
  am_dpp<kDppXor2>(b, i);
  am_dpp<kDppHalfMirror>(b, i);
  am_dpp<kDppMirror>(b, i);
}
__device__ __forceinline__ void wave_argmax(float& b, int& i) {
  row16_argmax(b, i);
  auto rb = __builtin_amdgcn_permlane16_swap(__float_as_uint(b), __float_as_uint(b), false, false);
  auto ri = __builtin_amdgcn_permlane16_swap(uint32_t(i), uint32_t(i), false, false);
  b = __uint_as_float(rb[0]); i = int(ri[0]);
  am_take(b, i, __uint_as_float(rb[1]), int(ri[1]));
  rb = __builtin_amdgcn_permlane32_swap(__float_as_uint(b), __float_as_uint(b), false, false);
  ri = __builtin_amdgcn_permlane32_swap(uint32_t(i), uint32_t(i), false, false);
  b = __uint_as_float(rb[0]); i = int(ri[0]);
  am_take(b, i, __uint_as_float(rb[1]), int(ri[1]));
}

__device__ __forceinline__ float wave_sum(float v) { return xor32_sum(xor16_sum(row16_sum(v))); }
__device__ __forceinline__ float wave_max(float v) { return xor32_max(xor16_max(row16_max(v))); }

}  // namespace p2pt_gpu
