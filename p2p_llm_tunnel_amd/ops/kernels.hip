// HIP kernels (gfx950 / CDNA4) for the on-node inference upstream that
// `tunnel serve` fronts (BASELINE.json north star: "the serve side runs on the
// 8xMI355X node and fronts a local OpenAI/Ollama-compatible inference
// endpoint"). The reference has no GPU code; these kernels are
// the hot decode-step ops of that endpoint, written directly for CDNA4:
//
//   p2pt_rmsnorm           fused residual-add + RMSNorm (one pass, row in VGPRs)
//   p2pt_silu_mul          SwiGLU activation, 16-byte vector I/O
//   p2pt_rope_qkv_cache    RoPE on q/k of the new token + KV-cache append, fused
//   p2pt_decode_attention  GQA flash-decoding: split-K over the sequence, K/V
//                          tiles staged in LDS once per workgroup and shared by
//                          the group's query heads (one wave per head)
//   p2pt_argmax            greedy sampling: per-row argmax over the vocabulary
//
// All tensors are bf16 (raw uint16 storage) with fp32 accumulation. Waves are
// 64 lanes; every block is a multiple of 64 threads. Launchers are extern "C"
// (loaded with ctypes, no torch headers) and return the hipError_t of the launch.
#include "bf16_common.h"

namespace {

using namespace p2pt_gpu;

// ------------------------------------------------------------ RMSNorm
// One 256-thread block per row; the row stays in registers between the
// sum-of-squares and the scaling pass (one HBM read, one write).
template <int MAXV>
__global__ __launch_bounds__(256) void k_rmsnorm(const uint4* __restrict__ x, const uint4* __restrict__ res,
                                                 uint4* __restrict__ res_out, const uint4* __restrict__ w,
                                                 uint4* __restrict__ out, int hv, float inv_h, float eps) {
  const size_t row = blockIdx.x;
  const uint4* xr = x + row * hv;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    int idx = threadIdx.x + i * 256;
    if (idx < hv) {
      unpack8(xr[idx], v[i]);
      if (res) {
        float r[8];
        unpack8(res[row * hv + idx], r);
#pragma unroll
        for (int k = 0; k < 8; k++) v[i][k] += r[k];
        uint4 packed = pack8(v[i]);
        res_out[row * hv + idx] = packed;
        // Normalise the bf16-rounded sum, exactly what the next layer reads.
        unpack8(packed, v[i]);
      }
#pragma unroll
      for (int k = 0; k < 8; k++) ss += v[i][k] * v[i][k];
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float rs = rsqrtf(ss * inv_h + eps);
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    int idx = threadIdx.x + i * 256;
    if (idx < hv) {
      float g[8];
      unpack8(w[idx], g);
#pragma unroll
      for (int k = 0; k < 8; k++) v[i][k] = v[i][k] * rs * g[k];
      out[row * hv + idx] = pack8(v[i]);
    }
  }
}

// ------------------------------------------------------------ SwiGLU
__global__ __launch_bounds__(256) void k_silu_mul(const uint4* __restrict__ in, uint4* __restrict__ out, int rows,
                                                  int fv) {
  size_t n = size_t(rows) * fv;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    size_t r = i / fv, c = i % fv;
    float g[8], u[8], o[8];
    unpack8(in[r * 2 * fv + c], g);
    unpack8(in[r * 2 * fv + fv + c], u);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = g[k] / (1.f + __expf(-g[k])) * u[k];
    out[i] = pack8(o);
  }
}

// ------------------------------------------------------------ RoPE + KV append
// qkv: [B, (H + 2*Hkv) * D]; q_out: [B, H, D]; caches: [B, Smax, Hkv, D].
// NeoX rotate-half convention, inv_freq_i = theta^(-2i/D).
__global__ __launch_bounds__(256) void k_rope_qkv_cache(const uint16_t* __restrict__ qkv, const int* __restrict__ pos,
                                                        uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc,
                                                        uint16_t* __restrict__ vc, int H, int Hkv, int D, int Smax,
                                                        float log2_theta) {
  const int b = blockIdx.x;
  const int p = pos[b];
  const int half = D / 2;
  const uint16_t* src = qkv + size_t(b) * (H + 2 * Hkv) * D;
  const size_t cache_row = (size_t(b) * Smax + p) * Hkv * D;
  const int pairs = (H + Hkv) * half;
  for (int j = threadIdx.x; j < pairs; j += blockDim.x) {
    int head = j / half, i = j % half;
    float inv_freq = exp2f(-log2_theta * (2.f * i) / D);
    float s, c;
    sincosf(float(p) * inv_freq, &s, &c);
    const uint16_t* x = src + head * D;
    float x1 = bf2f(x[i]), x2 = bf2f(x[i + half]);
    uint16_t o1 = uint16_t(f2bf_bits(x1 * c - x2 * s));
    uint16_t o2 = uint16_t(f2bf_bits(x2 * c + x1 * s));
    if (head < H) {
      uint16_t* q = q_out + (size_t(b) * H + head) * D;
      q[i] = o1;
      q[i + half] = o2;
    } else {
      uint16_t* k = kc + cache_row + size_t(head - H) * D;
      k[i] = o1;
      k[i + half] = o2;
    }
  }
  const uint16_t* v = src + size_t(H + Hkv) * D;
  for (int j = threadIdx.x; j < Hkv * D; j += blockDim.x) vc[cache_row + j] = v[j];
}

// ------------------------------------------------------------ decode attention
// Grid: (n_splits, B*Hkv). Block: G waves (one per query head of the GQA
// group, G = H/Hkv <= 8). A workgroup owns one KV head and a CHUNK of the
// sequence; K/V tiles of 64 tokens are staged in LDS once and read by every
// query head of the group. Lane t of a wave scores token t of the tile (full
// dot product from a padded LDS row: the 144/272-byte stride keeps
// ds_read_b128 conflict-free), then lanes switch to the head dimension for
// P·V. Online softmax across tiles; partials (unnormalised acc, running max,
// running sum) go to a workspace merged by k_attn_reduce.
template <int D>
__global__ __launch_bounds__(512) void k_decode_attn(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                     const uint16_t* __restrict__ vc, const int* __restrict__ lens,
                                                     float* __restrict__ part_o, float* __restrict__ part_ml, int H,
                                                     int Hkv, int Smax, int chunk, int nsplit, float scale) {
  constexpr int TILE = 64;
  constexpr int ROWB = D * 2 + 16;  // padded row stride in bytes
  constexpr int DPL = D / kWave;    // head dims per lane in the P·V phase
  __shared__ __attribute__((aligned(16))) uint8_t ks[TILE * ROWB];
  __shared__ __attribute__((aligned(16))) uint8_t vs[TILE * ROWB];
  __shared__ __attribute__((aligned(16))) float ps[8][TILE];  // softmax weights, one row per wave

  const int split = blockIdx.x;
  const int b = blockIdx.y / Hkv, kvh = blockIdx.y % Hkv;
  const int G = H / Hkv;
  const int len = lens[b];
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int start = split * chunk;
  const int stop = min(start + chunk, len);
  const int nthr = blockDim.x;
  // Splits past this sequence's length do nothing (k_attn_reduce only reads
  // the first ceil(len/chunk) partials), so graphs can launch for capacity.
  if (start >= len) return;

  float qf[D];
  {
    const uint16_t* qp = q + (size_t(b) * H + kvh * G + g) * D;
#pragma unroll
    for (int d = 0; d < D; d += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qp + d), f);
#pragma unroll
      for (int k = 0; k < 8; k++) qf[d + k] = f[k] * scale;
    }
  }
  float m = -INFINITY, l = 0.f, acc[DPL];
#pragma unroll
  for (int k = 0; k < DPL; k++) acc[k] = 0.f;

  const size_t tok_stride = size_t(Hkv) * D;  // elements between consecutive tokens
  const uint16_t* kbase = kc + (size_t(b) * Smax) * tok_stride + size_t(kvh) * D;
  const uint16_t* vbase = vc + (size_t(b) * Smax) * tok_stride + size_t(kvh) * D;

  for (int t0 = start; t0 < stop; t0 += TILE) {
    const int nt = min(TILE, stop - t0);
    // Cooperative 16-byte loads of the K and V tiles into LDS.
    constexpr int VPR = D / 8;  // uint4 per row
    for (int e = threadIdx.x; e < TILE * VPR; e += nthr) {
      int t = e / VPR, c = e % VPR;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (t < nt) {
        kv = *reinterpret_cast<const uint4*>(kbase + size_t(t0 + t) * tok_stride + c * 8);
        vv = *reinterpret_cast<const uint4*>(vbase + size_t(t0 + t) * tok_stride + c * 8);
      }
      *reinterpret_cast<uint4*>(ks + t * ROWB + c * 16) = kv;
      *reinterpret_cast<uint4*>(vs + t * ROWB + c * 16) = vv;
    }
    __syncthreads();
    // Scores: lane = token.
    float s = -INFINITY;
    if (lane < nt) {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < D; d += 8) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(ks + lane * ROWB + d * 2), f);
#pragma unroll
        for (int k = 0; k < 8; k++) dot += qf[d + k] * f[k];
      }
      s = dot;
    }
    const float mnew = fmaxf(m, wave_max(s));
    const float p = (lane < nt) ? __expf(s - mnew) : 0.f;
    const float corr = __expf(m - mnew);
    l = l * corr + wave_sum(p);
    m = mnew;
#pragma unroll
    for (int k = 0; k < DPL; k++) acc[k] *= corr;
    // P·V: lane = head dim. p goes through this wave's LDS row and is read back
    // as broadcast float4s over the full (zero-filled) tile, so the loop unrolls
    // into independent LDS reads instead of a shuffle-per-token chain.
    ps[g][lane] = p;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 2
    for (int t = 0; t < TILE; t += 8) {
      const float4 pa = *reinterpret_cast<const float4*>(&ps[g][t]);
      const float4 pb = *reinterpret_cast<const float4*>(&ps[g][t + 4]);
      const float pt[8] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint16_t* vrow = reinterpret_cast<const uint16_t*>(vs + (t + j) * ROWB);
#pragma unroll
        for (int k = 0; k < DPL; k++) acc[k] += pt[j] * bf2f(vrow[lane + k * kWave]);
      }
    }
    __syncthreads();
  }
  const size_t hb = size_t(b) * H + kvh * G + g;
  float* po = part_o + (hb * nsplit + split) * D;
#pragma unroll
  for (int k = 0; k < DPL; k++) po[lane + k * kWave] = acc[k];
  if (lane == 0) {
    part_ml[(hb * nsplit + split) * 2 + 0] = m;
    part_ml[(hb * nsplit + split) * 2 + 1] = l;
  }
}

// One 64-thread block per (b, head): merge split partials.
template <int D>
__global__ __launch_bounds__(64) void k_attn_reduce(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                                    uint16_t* __restrict__ out, int nsplit, const int* __restrict__ lens,
                                                    int H, int chunk) {
  constexpr int DPL = D / kWave;
  const size_t hb = blockIdx.x;
  const int b = int(hb / H);
  const int used = min(nsplit, (lens[b] + chunk - 1) / chunk);
  float M = -INFINITY;
  for (int s = 0; s < used; s++) M = fmaxf(M, part_ml[(hb * nsplit + s) * 2]);
  float L = 0.f, o[DPL];
#pragma unroll
  for (int k = 0; k < DPL; k++) o[k] = 0.f;
  for (int s = 0; s < used; s++) {
    float w = __expf(part_ml[(hb * nsplit + s) * 2] - M);
    L += part_ml[(hb * nsplit + s) * 2 + 1] * w;
#pragma unroll
    for (int k = 0; k < DPL; k++) o[k] += part_o[(hb * nsplit + s) * D + threadIdx.x + k * kWave] * w;
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int k = 0; k < DPL; k++) out[hb * D + threadIdx.x + k * kWave] = uint16_t(f2bf_bits(o[k] * inv));
}

// ------------------------------------------------------------ argmax
__global__ __launch_bounds__(256) void k_argmax(const uint16_t* __restrict__ logits, int64_t* __restrict__ out, int V) {
  const size_t row = blockIdx.x;
  const uint16_t* x = logits + row * V;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int vv = V / 8;
  const uint4* x4 = reinterpret_cast<const uint4*>(x);
  for (int i = threadIdx.x; i < vv; i += 256) {
    float f[8];
    unpack8(x4[i], f);
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (f[k] > best) {  // strict: keeps the first index within a thread
        best = f[k];
        bi = i * 8 + k;
      }
  }
  for (int i = vv * 8 + threadIdx.x; i < V; i += 256) {
    float f = bf2f(x[i]);
    if (f > best || (f == best && i < bi)) {
      best = f;
      bi = i;
    }
  }
  wave_argmax(best, bi);
  __shared__ float sb[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = best;
    si[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++)
      if (sb[w] > best || (sb[w] == best && si[w] < bi)) {
        best = sb[w];
        bi = si[w];
      }
    out[row] = bi;
  }
}

}  // namespace

// ------------------------------------------------------------ launchers
extern "C" {

int p2pt_rmsnorm(const void* x, const void* res, void* res_out, const void* w, void* out, int rows, int hidden,
                 float eps, void* stream) {
  if (hidden % 8 || rows <= 0) return int(hipErrorInvalidValue);
  int hv = hidden / 8;
  auto s = static_cast<hipStream_t>(stream);
  float inv_h = 1.f / float(hidden);
  auto X = static_cast<const uint4*>(x);
  auto R = static_cast<const uint4*>(res);
  auto RO = static_cast<uint4*>(res_out);
  auto W = static_cast<const uint4*>(w);
  auto O = static_cast<uint4*>(out);
  if (hv <= 256) hipLaunchKernelGGL(k_rmsnorm<1>, dim3(rows), dim3(256), 0, s, X, R, RO, W, O, hv, inv_h, eps);
  else if (hv <= 512) hipLaunchKernelGGL(k_rmsnorm<2>, dim3(rows), dim3(256), 0, s, X, R, RO, W, O, hv, inv_h, eps);
  else if (hv <= 1024) hipLaunchKernelGGL(k_rmsnorm<4>, dim3(rows), dim3(256), 0, s, X, R, RO, W, O, hv, inv_h, eps);
  else if (hv <= 2048) hipLaunchKernelGGL(k_rmsnorm<8>, dim3(rows), dim3(256), 0, s, X, R, RO, W, O, hv, inv_h, eps);
  else return int(hipErrorInvalidValue);
  return int(hipGetLastError());
}

int p2pt_silu_mul(const void* in, void* out, int rows, int F, void* stream) {
  if (F % 8 || rows <= 0) return int(hipErrorInvalidValue);
  int fv = F / 8;
  size_t n = size_t(rows) * fv;
  int blocks = int((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_silu_mul, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(in), static_cast<uint4*>(out), rows, fv);
  return int(hipGetLastError());
}

int p2pt_rope_qkv_cache(const void* qkv, const int* pos, void* q_out, void* kc, void* vc, int B, int H, int Hkv, int D,
                        int Smax, float theta, void* stream) {
  if (D % 2 || B <= 0 || H % Hkv) return int(hipErrorInvalidValue);
  hipLaunchKernelGGL(k_rope_qkv_cache, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t*>(qkv), pos, static_cast<uint16_t*>(q_out), static_cast<uint16_t*>(kc),
                     static_cast<uint16_t*>(vc), H, Hkv, D, Smax, log2f(theta));
  return int(hipGetLastError());
}

// Workspace: part_o [B*H*nsplit*D] f32 followed by part_ml [B*H*nsplit*2] f32.
int p2pt_decode_attention(const void* q, const void* kc, const void* vc, const int* lens, void* out, float* ws, int B,
                          int H, int Hkv, int D, int Smax, int nsplit, int chunk, float scale, void* stream) {
  if (H % Hkv || H / Hkv > 8 || B <= 0 || nsplit <= 0 || chunk <= 0) return int(hipErrorInvalidValue);
  auto s = static_cast<hipStream_t>(stream);
  float* part_o = ws;
  float* part_ml = ws + size_t(B) * H * nsplit * D;
  dim3 grid(nsplit, B * Hkv);
  auto Q = static_cast<const uint16_t*>(q);
  auto K = static_cast<const uint16_t*>(kc);
  auto V = static_cast<const uint16_t*>(vc);
  auto O = static_cast<uint16_t*>(out);
  if (D == 64) {
    hipLaunchKernelGGL(k_decode_attn<64>, grid, dim3(64 * (H / Hkv)), 0, s, Q, K, V, lens, part_o, part_ml, H, Hkv, Smax, chunk,
                       nsplit, scale);
    hipLaunchKernelGGL(k_attn_reduce<64>, dim3(B * H), dim3(64), 0, s, part_o, part_ml, O, nsplit, lens, H, chunk);
  } else if (D == 128) {
    hipLaunchKernelGGL(k_decode_attn<128>, grid, dim3(64 * (H / Hkv)), 0, s, Q, K, V, lens, part_o, part_ml, H, Hkv, Smax, chunk,
                       nsplit, scale);
    hipLaunchKernelGGL(k_attn_reduce<128>, dim3(B * H), dim3(64), 0, s, part_o, part_ml, O, nsplit, lens, H, chunk);
  } else {
    return int(hipErrorInvalidValue);
  }
  return int(hipGetLastError());
}

int p2pt_argmax(const void* logits, int64_t* out, int B, int V, void* stream) {
  if (B <= 0 || V <= 0) return int(hipErrorInvalidValue);
  hipLaunchKernelGGL(k_argmax, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t*>(logits), out, V);
  return int(hipGetLastError());
}

}  // extern "C"
