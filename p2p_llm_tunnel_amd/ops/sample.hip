// Stochastic sampling for the on-node inference endpoint (gfx950 / CDNA4):
// temperature, top-k and top-p (nucleus) over a bf16 logits row, on device,
// inside the captured decode step.
//
//   p2pt_sample   one 1024-thread workgroup (16 waves of 64) per row:
//     z_i = logit_i / T                                   (fp32)
//     top-k: the k-th largest z by radix select on order-preserving keys
//            (4 passes of 8 bits, LDS histograms)         -> keep z >= z_(k)
//     top-p: the smallest set of the largest kept z whose softmax mass
//            reaches p, by the same radix select over mass (LDS fp32
//            histograms of exp(z - max))                  -> keep z >= z_(p)
//     draw:  Gumbel-max over the kept set: argmax_i z_i - log(-log u_i), u_i
//            from a counter-based hash of (seed, counter, i), i.e. an exact
//            draw from softmax(z) restricted to the kept set (HF / vLLM
//            order: temperature, then top-k, then top-p; ties at a cut are
//            kept, as HF's `logits < kth` filter does).
//   Rows with T <= 0 keep the greedy id already in `ids` (the fused LM head's
//   argmax): greedy decoding stays bit-exact and costs one early-exit wave.
//
// params: int64 [5, ld] — float32 bits of T, top_k (<= 0: off), float32 bits
// of top_p (>= 1: off), seed, counter (the request's token index, so each
// draw of a request uses fresh noise and a fixed seed replays the same text).
#include "bf16_common.h"

namespace {

using namespace p2pt_gpu;

constexpr int kThreads = 1024, kWaves = kThreads / 64;

__device__ __forceinline__ uint32_t okey(float f) {  // order-preserving float -> uint32
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // SplitMix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Gumbel(0, 1) noise for element i of draw (seed, ctr). In double: the
// winners of a Gumbel-max come from u near 1, where -log(u) ~ 1 - u is tiny
// and the fast single-precision log's absolute error is of its own size (a
// measurable bias in the 12,800-draw chi-square test).
__device__ __forceinline__ float gumbel(uint64_t seed, uint64_t ctr, uint32_t i) {
  uint64_t h = mix64(seed + mix64(ctr * 0x9E3779B97F4A7C15ull + i + 1));
  double u = (double(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);  // (0, 1), 53 bits
  return float(-log(-log(u)));
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int w = 1; w < kWaves; w++) m = fmaxf(m, red[w]);
  return m;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kWaves; w++) s += red[w];
  return s;
}

// Among 256 buckets (descending digit order), the digit where the running sum
// from the top first reaches `need`; *above = the sum of the buckets above it.
// One wave: lane j holds digits 255-4j .. 252-4j.
template <class T>
__device__ __forceinline__ void find_bucket(const T* hist, T need, int* digit_out, T* above_out) {
  const int lane = threadIdx.x & 63;
  T v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    v[q] = hist[255 - 4 * lane - q];
    s += v[q];
  }
  T incl = s;  // inclusive prefix over lanes
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  const T excl = incl - s;
  const bool hit = excl < need && incl >= need;
  const uint64_t b = __ballot(hit);
  const int first = b ? __ffsll((unsigned long long)b) - 1 : 63;
  if (lane == first) {
    T run = excl;
    int dg = 255 - 4 * lane - 3;
    T ab = run;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (run + v[q] >= need || q == 3) {
        dg = 255 - 4 * lane - q;
        ab = run;
        break;
      }
      run += v[q];
    }
    *digit_out = dg;
    *above_out = ab;
  }
}

__global__ __launch_bounds__(kThreads) void k_sample(const uint16_t* __restrict__ logits, int64_t* __restrict__ ids,
                                                     const int64_t* __restrict__ params, int ld, int V) {
  const int row = blockIdx.x;
  const int B = ld;  // params rows are `ld` long (a view of the engine's staging block)
  const float T = __uint_as_float(uint32_t(params[row]));
  if (!(T >= 1e-4f)) return;  // greedy row (or T -> 0, whose limit is greedy): the fused argmax stands
  int64_t k = params[B + row];
  float p = __uint_as_float(uint32_t(params[2 * B + row]));
  const uint64_t seed = uint64_t(params[3 * B + row]), ctr = uint64_t(params[4 * B + row]);
  if (k <= 0 || k > V) k = V;
  if (!(p > 0.f && p < 1.f)) p = 1.f;
  const float invT = 1.0f / T;
  const uint16_t* lr = logits + size_t(row) * V;

  __shared__ float red[kWaves];
  __shared__ uint32_t hist_u[256];
  __shared__ float hist_f[256];
  __shared__ int s_digit;
  __shared__ uint32_t s_above_u;
  __shared__ float s_above_f;
  __shared__ float s_best[kWaves];
  __shared__ int s_bi[kWaves];

  float m = -INFINITY;
  for (int i = threadIdx.x; i < V; i += kThreads) m = fmaxf(m, bf2f(lr[i]) * invT);
  m = block_max(m, red);

  // ---- top-k: the k-th largest key
  uint32_t kth = 0;  // keep key >= kth (0: everything)
  if (k < V) {
    uint32_t prefix = 0, mask = 0, need = uint32_t(k);
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int d = threadIdx.x; d < 256; d += kThreads) hist_u[d] = 0;
      __syncthreads();
      for (int i = threadIdx.x; i < V; i += kThreads) {
        const uint32_t key = okey(bf2f(lr[i]) * invT);
        if ((key & mask) == prefix) atomicAdd(&hist_u[(key >> shift) & 0xFF], 1u);
      }
      __syncthreads();
      if (threadIdx.x < 64) find_bucket<uint32_t>(hist_u, need, &s_digit, &s_above_u);
      __syncthreads();
      need -= s_above_u;
      prefix |= uint32_t(s_digit) << shift;
      mask |= 0xFFu << shift;
      __syncthreads();
    }
    kth = prefix;
  }

  // ---- top-p over the kept set: mass radix select
  uint32_t pth = 0;
  if (p < 1.f) {
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float zi = bf2f(lr[i]) * invT;
      if (okey(zi) >= kth) z += __expf(zi - m);
    }
    float need = p * block_sum(z, red);
    uint32_t prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int d = threadIdx.x; d < 256; d += kThreads) hist_f[d] = 0.f;
      __syncthreads();
      for (int i = threadIdx.x; i < V; i += kThreads) {
        const float zi = bf2f(lr[i]) * invT;
        const uint32_t key = okey(zi);
        if (key >= kth && (key & mask) == prefix) atomicAdd(&hist_f[(key >> shift) & 0xFF], __expf(zi - m));
      }
      __syncthreads();
      if (threadIdx.x < 64) find_bucket<float>(hist_f, need, &s_digit, &s_above_f);
      __syncthreads();
      need -= s_above_f;
      prefix |= uint32_t(s_digit) << shift;
      mask |= 0xFFu << shift;
      __syncthreads();
    }
    pth = prefix;
  }
  const uint32_t cut = kth > pth ? kth : pth;

  // ---- Gumbel-max over the kept set
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += kThreads) {
    const float zi = bf2f(lr[i]) * invT;
    if (okey(zi) < cut) continue;
    am_take(best, bi, zi + gumbel(seed, ctr, uint32_t(i)), i);
  }
  wave_argmax(best, bi);
  if ((threadIdx.x & 63) == 0) {
    s_best[threadIdx.x >> 6] = best;
    s_bi[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kWaves; w++) am_take(best, bi, s_best[w], s_bi[w]);
    if (bi != 0x7fffffff) ids[row] = bi;
  }
}

}  // namespace

extern "C" {

// ids: int64 [B] (in: greedy ids; out: samples for rows with T > 0);
// params: int64 [5, ld] (ld >= B, row k of parameter p at params[p * ld + k]);
// logits: bf16 [B, V] rows contiguous.
int p2pt_sample(const void* logits, int64_t* ids, const int64_t* params, int B, int ld, int V, void* stream) {
  if (B <= 0 || V <= 0 || ld < B) return int(hipErrorInvalidValue);
  hipLaunchKernelGGL(k_sample, dim3(B), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t*>(logits), ids, params, ld, V);
  return int(hipGetLastError());
}

}  // extern "C"
