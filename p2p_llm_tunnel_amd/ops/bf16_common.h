// bf16 helpers shared by the gfx950 kernels: raw uint16 storage, fp32 math,
// round-to-nearest-even packing, 16-byte (8 x bf16) vector unpack/pack, and
// 64-lane wave reductions.
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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

}  // namespace p2pt_gpu
