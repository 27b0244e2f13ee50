// Fused Llama decode step for gfx950 (CDNA4 / MI355X).
//
// The unfused step (kernels.hip + hipBLASLt) is ~50 kernels per token for a
// 4-layer model; at decode batch sizes every one of them is a few-µs latency
// chain (dispatch, one HBM round trip, write back) and the step is bound by
// kernel count, not bytes. This file rebuilds the step as 5 kernels per layer
// plus 2, each a weight-streaming MFMA GEMM with its neighbours fused in:
//
//   k_embed              token gather -> residual stream, per-row sum of squares
//   per layer:
//     k_skinny<ROPE>     RMSNorm (attn_norm) -> QKV GEMM -> RoPE on q/k,
//                        q to the attention buffer, k/v appended to the cache
//     k_attn             GQA flash-decoding split-K; the last split to finish
//                        for a (sequence, KV head) merges the partials in-kernel
//     k_skinny<RESID>    O projection -> residual add -> per-row sum-of-squares
//                        partials for the next norm
//     k_skinny<SILU>     RMSNorm (ffn_norm) -> gate/up GEMM -> SwiGLU
//     k_skinny<RESID>    down projection -> residual add -> sum-of-squares
//   k_skinny<ARGMAX>     RMSNorm (final norm) -> LM head -> logits and
//                        per-block greedy winners
//   k_argmax_merge       one block per row merges the winners
//
// Skinny GEMM (M <= 64 tokens): Y[M,N] = A[M,K] * W[N,K]^T on
// v_mfma_f32_16x16x32_bf16. A workgroup owns 16*TN output columns of one
// 16-row tile (blockIdx.y; prefill-heavy steps carry up to 4) and splits K
// over its NW waves; each lane streams its weight rows with 16-byte loads
// straight into MFMA B fragments (no LDS staging: every weight byte is used
// exactly once, by exactly one lane), the K-split partials are summed through
// LDS and wave 0 runs the epilogue. RMSNorm is folded away: its weight g is
// multiplied into the columns of the following projection once at load time
// (W'[n][k] = W[n][k] g[k]), and the per-row 1/rms factors out of the dot
// product, so the GEMM streams the raw residual and the epilogue scales the
// accumulator. 1/rms comes from per-block partial sums of squares written by
// the residual producer (deterministic: fixed order, no float atomics).
// The attention splits merge in-kernel through write-through stores and an
// arrival ticket, never an L2 write-back fence. QKV and gate/up weights have
// their rows interleaved in pairs (RoPE partners; gate_j/up_j) so that one
// 16-column tile holds both members of every pair (lanes c, c^1).
//
// Numerics: GEMM outputs, the residual and the attention output are rounded
// to bf16 where the unfused path rounds them; the normed activation is not
// materialised (rounding differs at the bf16-ulp level); fp32 accumulation.
#include "bf16_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

using namespace p2pt_gpu;

constexpr int kMaxM = 64;  // token rows per step: up to 4 MFMA row tiles (blockIdx.y)

typedef short frag8 __attribute__((ext_vector_type(8)));
typedef float frag4 __attribute__((ext_vector_type(4)));

enum Epi : int { EPI_STORE = 0, EPI_ROPE = 1, EPI_SILU = 2, EPI_RESID = 3, EPI_ARGMAX = 4 };

struct GemmArgs {
  const uint16_t* x;  // A [M][K]
  const uint16_t* w;  // W [N][K]; for a normed input, W[n][k] * g[k] folded in
  int M, N, K;
  // RMSNorm of A's rows (ss_part == nullptr: A used as is). The norm weight g
  // is folded into W offline, so only the per-row 1/rms remains, and that
  // factors out of the dot product: it scales the accumulator in the epilogue.
  const float* ss_part;  // [ss_parts][16] partial row sums of squares
  int ss_parts;
  float eps;
  // epilogue
  uint16_t* out;   // STORE/ARGMAX: [M][N] logits; SILU: [M][N/2]; RESID: residual [M][N], in place
  float* ss_out;   // RESID: [gridDim.x][16]
  const int* pos;   // ROPE: cache position of each row
  const int* slot;  // ROPE: cache slot of each row (nullptr: row m -> slot m)
  int nslots;
  uint16_t* q_out;
  uint16_t* kc;
  uint16_t* vc;
  int H, Hkv, D, Smax;
  float log2_theta;
  float* am_val;  // ARGMAX: [gridDim.x][16]
  int* am_idx;
  // Split-K over workgroups (ks > 1): the ks workgroups of a column tile each
  // reduce a K range, publish a 16 x 16*TN fp32 slab write-through, and the
  // last to arrive sums the slabs in fixed order (deterministic) and runs the
  // epilogue. Small-N projections (N = d_model) otherwise leave CUs idle.
  int ks;
  float* kpart;     // [tiles][ks][TN][4][64]
  unsigned* kctr;   // [tiles] arrival tickets (self-resetting)
  // Column-tile width 2^cwl (16, 8 or 4 output columns per 16-lane MFMA
  // subtile). Narrower tiles put a small-N projection on more workgroups, so
  // its weight stream spreads over every CU (one CU streams ~10 B/cycle, a
  // 2048-wide projection in 16-column tiles reached only 128 of the 256 CUs).
  // Lanes c and c + 2^cwl load the same weight row in the same instruction
  // (one fetch); their duplicate MFMA columns are dropped in the epilogue.
  int cwl;
  // K parts (kpl = log2 P, 0: off; P = 16 >> cwl, TN = 1, M * P <= 16): lanes
  // past the tile width take the other K parts of the same columns instead of
  // repeating them, and MFMA rows m * P + p carry activation row m's K part p,
  // so every lane streams unique weight bytes. The diagonal blocks of the
  // 16 x 16 accumulator are summed in the epilogue. With spare MFMA rows (a
  // decode step of <= 16 / P tokens) a 2048-wide projection then spreads
  // over every CU without the duplicate fetches of narrow tiles.
  int kpl;
};

__device__ __forceinline__ frag8 as_frag(const uint4& v) { return __builtin_bit_cast(frag8, v); }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// v_dot2_f32_bf16: c + a.lo * b.lo + a.hi * b.hi, products and sum in fp32.
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}

// Weights use the default cache policy on purpose: a decode step replays the
// same weights back to back, and models up to the 256 MB MALL keep them
// resident between steps (non-temporal loads measured 1.75x slower on the
// 4-layer config in round 1; with buffer loads, nt (aux 2) on the weights was
// 5 % slower on the 0.85 GB config too: profiles/r02/decode/decode_sweep_s9.log).

// Cross-workgroup hand-off without L2 write-back/invalidate fences: payload
// stores are agent-scope relaxed atomics (write-through, `sc1`), drained with
// s_waitcnt before the arrival ticket; the last arriver reads them back with
// agent-scope loads that bypass stale cache lines (MI355X_MICROARCH handoff-flag).
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_wt(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ unsigned arrive(unsigned* ctr) {
  return __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Output column of lane column c (0..15) in subtile t of block bx, for
// subtiles of 2^cwl distinct columns (lanes past 2^cwl repeat them).
template <int TN>
__device__ __forceinline__ int tile_col(int bx, int t, int c, int cwl) {
  return ((bx * TN + t) << cwl) + (c & ((1 << cwl) - 1));
}

// Operand loads go through buffer descriptors (wave-uniform base and size
// from the kernel arguments): a lane whose byte offset lies past the buffer
// gets zeros from the range check without a memory access. Rows past M and
// k-steps past a wave's share use that (kOob), so a batch is branch-free and a
// decode step at batch 1 fetches its one activation row once per k-step
// instead of for all 16 MFMA rows.
constexpr uint32_t kOob = 0x80000000u;  // host keeps every operand below 2 GiB

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// One batch of up to UM consecutive 32-wide k-steps [s, min(s + UM, s1)):
// every load of the batch is issued before any of it is used.
template <int UM, int TN>
struct Batch {
  uint4 b[UM][TN];
  uint4 a[UM];
};

template <int UM, int TN>
__device__ __forceinline__ void load_batch(Batch<UM, TN>& bt, __amdgpu_buffer_rsrc_t ra, uint32_t xoff,
                                           __amdgpu_buffer_rsrc_t rw, const uint32_t (&woff)[TN], int s, int s1) {
#pragma unroll
  for (int u = 0; u < UM; u++) {
    const bool in = s + u < s1;
    const uint32_t su = uint32_t(s + u) * 64u;  // bytes per 32-wide k-step
#pragma unroll
    for (int t = 0; t < TN; t++) bt.b[u][t] = buf_ld16(rw, in ? woff[t] + su : kOob);
    bt.a[u] = buf_ld16(ra, in ? xoff + su : kOob);
  }
}

template <int UM, int TN>
__device__ __forceinline__ void mma_apply(frag4 (&acc)[TN], const Batch<UM, TN>& bt) {
#pragma unroll
  for (int u = 0; u < UM; u++)
#pragma unroll
    for (int t = 0; t < TN; t++)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(bt.a[u]), as_frag(bt.b[u][t]), acc[t], 0, 0, 0);
}

// The wave's k-steps [s0, s1), one batch at a time. Measured slower on
// MI355X and dropped (profiles/r02/decode/decode_sweep_s6..s8.log): a
// two-deep batch pipeline (every projection +0.5-1.8 us, LM head +0.5-2.4),
// 16 waves on the K = 5632 down projection (9.4 -> 10.5 us), and one
// workgroup per CU forced through padded LDS with 8-column tiles (down
// unchanged at 9.4 us, QKV 5.9 -> 9.9): the down projection is not bound by
// per-CU bandwidth or by its serial batches.
template <int UM, int TN>
__device__ __forceinline__ void mma_stream(frag4 (&acc)[TN], __amdgpu_buffer_rsrc_t ra, uint32_t xoff,
                                           __amdgpu_buffer_rsrc_t rw, const uint32_t (&woff)[TN], int s0, int s1) {
  for (int s = s0; s < s1; s += UM) {
    Batch<UM, TN> p;
    load_batch<UM, TN>(p, ra, xoff, rw, woff, s, s1);
    // Keep every load of the batch ahead of the first MFMA: left alone, the
    // scheduler interleaves them and the batch pays several memory latencies.
    __builtin_amdgcn_sched_barrier(0);
    mma_apply<UM, TN>(acc, p);
  }
}

// Skinny GEMM + fused epilogue. NW waves split K; TN subtiles of 2^cwl
// columns per block; UM k-steps per load batch (host: >= each wave's share
// when possible). Steps of more than 16 rows put each 16-row tile on its own
// workgroup (blockIdx.y). Sharing each weight fragment across the four tiles
// of a 64-row step in one workgroup was measured slower (small config, 64
// rows: 1.19 -> 1.26 ms; 1.1B-shaped checkpoint served at 16 streams 3.0 K ->
// 2.7 K tok/s, profiles/r02/decode/decode_sweep_s10_rowtiles.log): the extra
// tiles' weight reads hit the MALL, and a quarter of the workgroups each
// issuing five times the loads leaves the load path, not HBM, as the limit. ROPE and SILU take weights whose rows are interleaved in
// pairs (RoPE partners d, d + D/2 of a head; gate_j, up_j), so a pair sits in
// lanes c, c^1.
template <int NW, int TN, int EPI, int UM>
__global__ __launch_bounds__(NW * 64) void k_skinny(GemmArgs a) {
  __shared__ float red[NW][TN][4][kWave];
  __shared__ float red_ss[NW][kWave];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m0 = blockIdx.y << 4;    // first row of this workgroup's 16-row tile
  const int bx = blockIdx.x / a.ks;  // column tile
  const int kslice = blockIdx.x % a.ks;
  const bool norm = a.ss_part != nullptr;

  // Row sums of squares for the folded RMSNorm, spread over every wave (lane:
  // row lane & 15, partials (lane >> 4) + 4 * wave + 4 * NW * i): up to 8
  // loads per lane issued ahead of the weight stream and summed only after
  // it, so they never stall it; combined through LDS before the epilogue.
  constexpr int kSsRegs = 8;
  float ssv[kSsRegs];
  const int ss_p0 = (lane >> 4) + 4 * wv;
  if (norm) {
#pragma unroll
    for (int i = 0; i < kSsRegs; i++) {
      const int p = ss_p0 + 4 * NW * i;
      ssv[i] = p < a.ss_parts ? a.ss_part[p * kMaxM + m0 + (lane & 15)] : 0.f;
    }
  }

  // A fragment: row lane & 15, k = 32*s + 8*(lane>>4) + j; B fragment: W row n, same k.
  // The K steps are split evenly over the NW waves.
  const int kparts = 1 << a.kpl, Kp = a.K >> a.kpl;  // Kp: K elements per part
  const int m_a = (lane & 15) >> a.kpl;              // activation row of this lane's MFMA row
  const int p_a = (lane & 15) & (kparts - 1);        // ... and the K part it carries
  const bool a_ok = m0 + m_a < a.M;
  const int kq = (lane >> 4) << 3;
  const int S = Kp >> 5;
  const int b0 = kslice * S / a.ks, bs = (kslice + 1) * S / a.ks - b0;  // this workgroup's k-steps
  const int s0 = b0 + wv * bs / NW, s1 = b0 + (wv + 1) * bs / NW;
  // Byte offsets of this lane's A row and weight rows at k-step 0; rows past
  // M read as zeros (kOob).
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.x, uint32_t(a.M) * uint32_t(a.K) * 2u);
  const __amdgpu_buffer_rsrc_t rw = rsrc(a.w, uint32_t(a.N) * uint32_t(a.K) * 2u);
  const uint32_t xoff = a_ok ? (uint32_t(m0 + m_a) * uint32_t(a.K) + uint32_t(p_a * Kp + kq)) * 2u : kOob;
  const int p_b = a.kpl ? (lane & 15) >> a.cwl : 0;  // K part of this lane's weight column
  uint32_t woff[TN];
#pragma unroll
  for (int t = 0; t < TN; t++)
    woff[t] = (uint32_t(tile_col<TN>(bx, t, lane & 15, a.cwl)) * uint32_t(a.K) + uint32_t(p_b * Kp + kq)) * 2u;

  // C layout: row m = m0 + 4*(lane>>4) + r, column = tile_col(.., lane & 15).
  const int lrow0 = (lane >> 4) << 2, mrow0 = m0 + lrow0;
  const int c = lane & 15;
  const bool col_ok = c < (1 << a.cwl);  // lanes past the tile width repeat its columns

  // RESID: the residual values this lane's epilogue updates, loaded by wave 0
  // ahead of the weight stream (they do not depend on it) instead of after
  // the reduction, which would add a dependent memory round trip.
  float rprev[EPI == EPI_RESID ? TN : 1][4];
  if constexpr (EPI == EPI_RESID) {
    if (wv == 0) {
#pragma unroll
      for (int t = 0; t < TN; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int m = min(mrow0 + r, a.M - 1);
          rprev[t][r] = bf2f(a.out[size_t(m) * a.N + tile_col<TN>(bx, t, c, a.cwl)]);
        }
    }
  }

  frag4 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; t++) acc[t] = frag4{0.f, 0.f, 0.f, 0.f};
  mma_stream<UM, TN>(acc, ra, xoff, rw, woff, s0, s1);

  if (norm) {
    float ssum = 0.f;
#pragma unroll
    for (int i = 0; i < kSsRegs; i++) ssum += ssv[i];
    for (int p = ss_p0 + 4 * NW * kSsRegs; p < a.ss_parts; p += 4 * NW) ssum += a.ss_part[p * kMaxM + m0 + (lane & 15)];
    red_ss[wv][lane] = ssum;
  }
  // K-split reduction through LDS (lane-contiguous: conflict-free).
#pragma unroll
  for (int t = 0; t < TN; t++)
#pragma unroll
    for (int r = 0; r < 4; r++) red[wv][t][r][lane] = acc[t][r];
  __syncthreads();
  if (wv != 0) return;
  float v[TN][4];
#pragma unroll
  for (int t = 0; t < TN; t++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; w++) sum += red[w][t][r][lane];
      v[t][r] = sum;
    }
  if (a.ks > 1) {
    float* slab = a.kpart + size_t(bx) * a.ks * (TN * 4 * kWave);
#pragma unroll
    for (int t = 0; t < TN; t++)
#pragma unroll
      for (int r = 0; r < 4; r++) st_wt(slab + size_t(kslice) * (TN * 4 * kWave) + (t * 4 + r) * kWave + lane, v[t][r]);
    drain_stores();
    unsigned tk = 0;
    if (lane == 0) tk = arrive(&a.kctr[bx]);
    tk = __shfl(tk, 0, kWave);
    if (tk != unsigned(a.ks - 1)) return;
#pragma unroll
    for (int t = 0; t < TN; t++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float sum = 0.f;
        for (int j = 0; j < a.ks; j++) sum += ld_wt(slab + size_t(j) * (TN * 4 * kWave) + (t * 4 + r) * kWave + lane);
        v[t][r] = sum;
      }
    if (lane == 0) st_wt(&a.kctr[bx], 0u);
  }

  if (a.kpl) {
    // Sum the diagonal blocks: output (row m, column c < 2^cwl) is
    // sum_p C[m * P + p][c + p * 2^cwl]. Wave 0 alone from here on: the
    // reduction buffer (its own reads are done) holds C [16][17].
    float* cbuf = &red[0][0][0][0];
#pragma unroll
    for (int r = 0; r < 4; r++) cbuf[(lrow0 + r) * 17 + c] = v[0][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = lrow0 + r;
      float sum = 0.f;
      if (row < (16 >> a.kpl) && col_ok)
        for (int p = 0; p < kparts; p++) sum += cbuf[(row * kparts + p) * 17 + c + (p << a.cwl)];
      v[0][r] = sum;
    }
  }

  if (norm) {
    float ssum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; w++) ssum += red_ss[w][lane];
    ssum = xor32_sum(xor16_sum(ssum));
    const float rs_row = rsqrtf(ssum * (1.f / float(a.K)) + a.eps);  // for row m0 + (lane & 15)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const float rs = __shfl(rs_row, lrow0 + r, kWave);
#pragma unroll
      for (int t = 0; t < TN; t++) v[t][r] *= rs;
    }
  }

  if constexpr (EPI == EPI_STORE || EPI == EPI_ARGMAX) {
    // Logits (bf16) and, for ARGMAX, this block's per-row winner (first index on ties).
    float best[4];
    int bi[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      best[r] = -INFINITY;
      bi[r] = 0x7fffffff;
    }
#pragma unroll
    for (int t = 0; t < TN; t++) {
      const int n = tile_col<TN>(bx, t, c, a.cwl);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int m = mrow0 + r;
        const float lv = bf_round(v[t][r]);
        if (m < a.M && col_ok) a.out[size_t(m) * a.N + n] = uint16_t(f2bf_bits(lv));
        if (lv > best[r] || (lv == best[r] && n < bi[r])) {
          best[r] = lv;
          bi[r] = n;
        }
      }
    }
    if constexpr (EPI == EPI_ARGMAX) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        row16_argmax(best[r], bi[r]);
        if (c == 0) {
          a.am_val[bx * kMaxM + mrow0 + r] = best[r];
          a.am_idx[bx * kMaxM + mrow0 + r] = bi[r];
        }
      }
    }
  } else if constexpr (EPI == EPI_SILU) {
    // Interleaved rows: even lane = gate_j, odd lane = up_j, j = column / 2.
    const int n = tile_col<TN>(bx, 0, c, a.cwl);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const float mine = bf_round(v[0][r]);
      const float other = dpp<kDppXor1>(mine);
      if ((c & 1) || !col_ok || mrow0 + r >= a.M) continue;
      a.out[size_t(mrow0 + r) * (a.N >> 1) + (n >> 1)] = uint16_t(f2bf_bits(mine / (1.f + __expf(-mine)) * other));
    }
  } else if constexpr (EPI == EPI_ROPE) {
    // Interleaved rows within each head: column 2i = dim i, 2i+1 = dim i + D/2.
    const int half = a.D >> 1;
    const int col = tile_col<TN>(bx, 0, c, a.cwl);
    const int head = col / a.D, i = (col % a.D) >> 1;
    const bool second = c & 1;
    const float inv_freq = exp2f(-a.log2_theta * (2.f * i) / a.D);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = mrow0 + r;
      const float mine = bf_round(v[0][r]);
      const float other = dpp<kDppXor1>(mine);
      if (m >= a.M || !col_ok) continue;
      // Host validates; clamped anyway so a bad index can never write outside the cache.
      const int p = min(max(a.pos[m], 0), a.Smax - 1);
      const int sl = a.slot ? min(max(a.slot[m], 0), a.nslots - 1) : m;
      const int d = i + (second ? half : 0);
      if (head < a.H + a.Hkv) {
        float sn, cs;
        sincosf(float(p) * inv_freq, &sn, &cs);
        const float x1 = second ? other : mine, x2 = second ? mine : other;
        const float o = second ? x2 * cs + x1 * sn : x1 * cs - x2 * sn;
        uint16_t* dst = head < a.H ? a.q_out + (size_t(m) * a.H + head) * a.D
                                   : a.kc + ((size_t(sl) * a.Smax + p) * a.Hkv + (head - a.H)) * a.D;
        dst[d] = uint16_t(f2bf_bits(o));
      } else {
        a.vc[((size_t(sl) * a.Smax + p) * a.Hkv + (head - a.H - a.Hkv)) * a.D + d] = uint16_t(f2bf_bits(mine));
      }
    }
  } else if constexpr (EPI == EPI_RESID) {
    float sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TN; t++) {
      const int n = tile_col<TN>(bx, t, c, a.cwl);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int m = mrow0 + r;
        if (m >= a.M || !col_ok) continue;
        const float nv = bf_round(rprev[t][r] + bf_round(v[t][r]));
        a.out[size_t(m) * a.N + n] = uint16_t(f2bf_bits(nv));
        sq[r] += nv * nv;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      sq[r] = row16_sum(sq[r]);
      if (c == 0) a.ss_out[bx * kMaxM + mrow0 + r] = sq[r];
    }
  }
}

// Greedy sampling, second stage: one block per row merges the LM-head blocks'
// winners (first index on ties).
__global__ __launch_bounds__(256) void k_argmax_merge(const float* __restrict__ am_val, const int* __restrict__ am_idx,
                                                      int parts, int64_t* __restrict__ ids) {
  const int m = blockIdx.x;
  float b = -INFINITY;
  int i = 0x7fffffff;
  for (int p0 = threadIdx.x; p0 < parts; p0 += 8 * 256) {
    float pv[8];
    int pi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {  // 8 loads in flight per thread
      const int p = p0 + j * 256;
      pv[j] = p < parts ? am_val[p * kMaxM + m] : -INFINITY;
      pi[j] = p < parts ? am_idx[p * kMaxM + m] : 0x7fffffff;
    }
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (pv[j] > b || (pv[j] == b && pi[j] < i)) {
        b = pv[j];
        i = pi[j];
      }
  }
  wave_argmax(b, i);
  __shared__ float sb[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = b;
    si[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++)
      if (sb[w] > b || (sb[w] == b && si[w] < i)) {
        b = sb[w];
        i = si[w];
      }
    ids[m] = i;
  }
}

// ------------------------------------------------------------ embedding gather
// One block per token: residual row = embed[token]; ss_out[0][b] = sum of squares.
__global__ __launch_bounds__(256) void k_embed(const uint16_t* __restrict__ embed, const int64_t* __restrict__ tok,
                                               uint16_t* __restrict__ resid, float* __restrict__ ss_out, int dim,
                                               int vocab) {
  const int b = blockIdx.x;
  int64_t t = tok[b];
  t = t < 0 ? 0 : (t >= vocab ? vocab - 1 : t);
  const uint4* src = reinterpret_cast<const uint4*>(embed + size_t(t) * dim);
  uint4* dst = reinterpret_cast<uint4*>(resid + size_t(b) * dim);
  float ss = 0.f;
  for (int i = threadIdx.x; i < dim / 8; i += 256) {
    const uint4 v = src[i];
    dst[i] = v;
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; j++) ss += f[j] * f[j];
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ss_out[b] = red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------ attention
// GQA flash-decoding with a fixed grid of (span slot, row b, KV head)
// workgroups: graph-captured steps launch the same grid whatever the context
// length, so the grid is sized by the batch (about one round of workgroups on
// the chip), not by the cache capacity — idle workgroups were a third of the
// kernel at 1k tokens. Each slot covers a span of >= 256 tokens of row b; its
// 8 waves walk the span in 32-token pieces with an online softmax.
// A piece is loaded straight into registers with 16-byte loads whose lanes
// tile whole K/V rows (D/8 lanes per row: every instruction reads full cache
// lines); nothing is staged through LDS. A lane keeps one 8-dim group of every
// query head of the KV head (K/V are read once per GQA group), computes its
// dot products with v_dot2_f32_bf16 and finishes them with in-row DPP sums,
// and ends up holding the softmax weights of exactly the tokens whose V it
// loaded: P.V needs no data exchange until the final cross-row sum. Scores and
// P.V are fp32 VALU: with G <= 8 query rows an MFMA tile would be >= half
// padding; the kernel is bound by the K/V stream and latency.
// The 8 waves of a slot merge through LDS; only spans split over several
// slots publish a partial (write-through + arrival ticket) that the last slot
// to finish merges, its waves taking different heads.
// Row b reads cache slot slot[b] (rows may share a slot: chunked prefill) and
// attends to positions 0..pos[b]; the output is bf16 [B][H*D].
template <int D, int G, int TOK = 32>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(TOK == 16 ? 4 : 1))) void k_attn(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                              const uint16_t* __restrict__ vc, const int* __restrict__ pos,
                                              const int* __restrict__ slot, int nslots, float* __restrict__ part_o,
                                              float* __restrict__ part_ml, unsigned* __restrict__ counters,
                                              uint16_t* __restrict__ out, int H, int Hkv, int Smax, int nsplit,
                                              float scale, int min_span) {
  constexpr int NWV = 8;
  constexpr int DPL = D / kWave;  // merges: dims per lane
  constexpr int MAXC = 16;        // partials merged per load batch
  constexpr int LPR = D / 8, RPI = kWave / LPR, NI = TOK / RPI;
  __shared__ __attribute__((aligned(16))) float pacc[NWV][G][D];
  __shared__ float pml[NWV][G][2];
  __shared__ unsigned s_ticket;

  const int b = blockIdx.y / Hkv, kvh = blockIdx.y % Hkv;
  const int len = min(max(pos[b], 0), Smax - 1) + 1;
  int span = (len + gridDim.x - 1) / gridDim.x;
  span = max(min_span, (span + TOK - 1) / TOK * TOK);
  const int nact = (len + span - 1) / span;  // slots with tokens
  const int sl = blockIdx.x;
  if (sl >= nact) return;
  const int s0 = sl * span, s1 = min(len, s0 + span);
  const int sb = slot ? min(max(slot[b], 0), nslots - 1) : b;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int dg = lane % LPR, ri = lane / LPR;

  const size_t tok_stride = size_t(Hkv) * D;
  const uint16_t* kbase = kc + size_t(sb) * Smax * tok_stride + size_t(kvh) * D + 8 * dg;
  const uint16_t* vbase = vc + size_t(sb) * Smax * tok_stride + size_t(kvh) * D + 8 * dg;
  // This lane's 8 query dims of every head as bf16 pairs (v_dot2 operands).
  uint4 qpk[G];
  {
    const uint16_t* qp = q + (size_t(b) * H + size_t(kvh) * G) * D + 8 * dg;
#pragma unroll
    for (int g = 0; g < G; g++) qpk[g] = *reinterpret_cast<const uint4*>(qp + size_t(g) * D);
  }

  // Running state over this wave's pieces. m is wave-uniform per head; l and
  // acc hold this lane's tokens only and are summed across rows at the end.
  float mg[G], lg[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; g++) {
    mg[g] = -INFINITY;
    lg[g] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) acc[g][k] = 0.f;
  }
  for (int p0 = s0 + wv * TOK; p0 < s1; p0 += NWV * TOK) {
    const int ntok = min(TOK, s1 - p0);
    // Issue the piece (lanes past the end re-read the last valid row).
    uint4 kr[NI], vr[NI];
#pragma unroll
    for (int j = 0; j < NI; j++)
      kr[j] = *reinterpret_cast<const uint4*>(kbase + size_t(p0 + min(j * RPI + ri, ntok - 1)) * tok_stride);
#pragma unroll
    for (int j = 0; j < NI; j++)
      vr[j] = *reinterpret_cast<const uint4*>(vbase + size_t(p0 + min(j * RPI + ri, ntok - 1)) * tok_stride);
    // Scores: lane (ri, dg) ends with token j*RPI + ri's score for every head.
    float sc[G][NI];
#pragma unroll
    for (int j = 0; j < NI; j++) {
#pragma unroll
      for (int g = 0; g < G; g++) {
        float d = 0.f;
        d = dot2_bf16(qpk[g].x, kr[j].x, d);
        d = dot2_bf16(qpk[g].y, kr[j].y, d);
        d = dot2_bf16(qpk[g].z, kr[j].z, d);
        d = dot2_bf16(qpk[g].w, kr[j].w, d);
        d = (LPR == 16 ? row16_sum(d) : row8_sum(d)) * scale;
        sc[g][j] = (j * RPI + ri < ntok) ? d : -INFINITY;
      }
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      float pm = -INFINITY;
#pragma unroll
      for (int j = 0; j < NI; j++) pm = fmaxf(pm, sc[g][j]);
      if constexpr (LPR == 8) pm = xor8_max(pm);
      pm = xor32_max(xor16_max(pm));
      const float mnew = fmaxf(mg[g], pm);
      const float corr = __expf(mg[g] - mnew);  // 0 on the first piece (mg = -inf)
      mg[g] = mnew;
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < NI; j++) {
        sc[g][j] = __expf(sc[g][j] - mnew);  // now p (0 for masked tokens)
        ls += sc[g][j];
      }
      lg[g] = lg[g] * corr + ls;
#pragma unroll
      for (int k = 0; k < 8; k++) acc[g][k] *= corr;
    }
    // P.V: the lane's own tokens times its 8 dims.
#pragma unroll
    for (int j = 0; j < NI; j++) {
      float f[8];
      unpack8(vr[j], f);
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int k = 0; k < 8; k++) acc[g][k] += sc[g][j] * f[k];
    }
  }
  // Sum across rows (lanes with the same dim group).
#pragma unroll
  for (int g = 0; g < G; g++) {
    float l = lg[g];
    if constexpr (LPR == 8) l = xor8_sum(l);
    lg[g] = xor32_sum(xor16_sum(l));
#pragma unroll
    for (int k = 0; k < 8; k++) {
      float v = acc[g][k];
      if constexpr (LPR == 8) v = xor8_sum(v);
      acc[g][k] = xor32_sum(xor16_sum(v));
    }
  }
  // Publish this wave to the workgroup (waves without pieces: m = -inf, l = 0).
  if (ri == 0) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      *reinterpret_cast<float4*>(&pacc[wv][g][8 * dg]) = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      *reinterpret_cast<float4*>(&pacc[wv][g][8 * dg + 4]) = make_float4(acc[g][4], acc[g][5], acc[g][6], acc[g][7]);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      pml[wv][g][0] = mg[g];
      pml[wv][g][1] = lg[g];
    }
  }
  __syncthreads();

  // Slot merge through LDS: wave w takes heads w, w + 8, ...
  const size_t hb0 = size_t(b) * H + size_t(kvh) * G;
  for (int g = wv; g < G; g += NWV) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; w++) M = fmaxf(M, pml[w][g][0]);
    float L = 0.f, o[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) o[k] = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; w++) {
      const float ww = pml[w][g][1] > 0.f ? __expf(pml[w][g][0] - M) : 0.f;
      L += pml[w][g][1] * ww;
#pragma unroll
      for (int k = 0; k < DPL; k++) o[k] += ww * pacc[w][g][lane + k * kWave];
    }
    const size_t hb = hb0 + g;
    if (nact == 1) {
      const float inv = 1.f / L;
#pragma unroll
      for (int k = 0; k < DPL; k++) out[hb * D + lane + k * kWave] = uint16_t(f2bf_bits(o[k] * inv));
    } else {
      float* po = part_o + (hb * nsplit + sl) * D;
#pragma unroll
      for (int k = 0; k < DPL; k++) st_wt(po + lane + k * kWave, o[k]);
      if (lane == 0) {
        st_wt(part_ml + (hb * nsplit + sl) * 2 + 0, M);
        st_wt(part_ml + (hb * nsplit + sl) * 2 + 1, L);
      }
    }
  }
  if (nact == 1) return;
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) s_ticket = arrive(&counters[blockIdx.y]);
  __syncthreads();
  if (s_ticket != unsigned(nact - 1)) return;

  // Last slot: merge the slot partials, heads spread over the waves. Each
  // batch of up to MAXC partials (maxima, sums and vectors together) is loaded
  // before any of it is used and folded in with a running maximum, so a merge
  // of <= MAXC slots is one memory round trip (a separate pass for the global
  // maximum first cost a second one).
  for (int g = wv; g < G; g += NWV) {
    const size_t hb = hb0 + g;
    const float* ml = part_ml + hb * nsplit * 2;
    float M = -INFINITY;
    float L = 0.f, o[DPL];
#pragma unroll
    for (int k = 0; k < DPL; k++) o[k] = 0.f;
    for (int c0 = 0; c0 < nact; c0 += MAXC) {
      float pv[MAXC][DPL], wl[MAXC], ll[MAXC];
#pragma unroll
      for (int j = 0; j < MAXC; j++) {
        const bool ok = c0 + j < nact;
        const int c = min(c0 + j, nact - 1);
        wl[j] = ld_wt(ml + 2 * c);
        ll[j] = ok ? ld_wt(ml + 2 * c + 1) : 0.f;
#pragma unroll
        for (int k = 0; k < DPL; k++) pv[j][k] = ld_wt(part_o + (hb * nsplit + c) * D + lane + k * kWave);
      }
      float Mb = M;
#pragma unroll
      for (int j = 0; j < MAXC; j++)
        if (ll[j] > 0.f) Mb = fmaxf(Mb, wl[j]);
      const float rs = M == -INFINITY ? 0.f : __expf(M - Mb);  // rescale what is folded in so far
      L *= rs;
#pragma unroll
      for (int k = 0; k < DPL; k++) o[k] *= rs;
      M = Mb;
#pragma unroll
      for (int j = 0; j < MAXC; j++) {
        const float ww = ll[j] > 0.f ? __expf(wl[j] - M) : 0.f;
        L += ll[j] * ww;
#pragma unroll
        for (int k = 0; k < DPL; k++) o[k] += ww * pv[j][k];
      }
    }
    const float inv = 1.f / L;
#pragma unroll
    for (int k = 0; k < DPL; k++) out[hb * D + lane + k * kWave] = uint16_t(f2bf_bits(o[k] * inv));
  }
  if (threadIdx.x == 0) st_wt(&counters[blockIdx.y], 0u);
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}

// Span slots per (row, KV head): about one round of workgroups on the chip,
// at most the workspace's partial slots.
int attn_slots(int B, int Hkv, int nsplit_ws) {
  static const int cap = env_int("P2PT_ATTN_SLOTS", 16);
  // Target workgroups of the launch: 256 (one 512-thread, 234-VGPR workgroup
  // per CU). More slots per row are slower: b16 0.522 / 0.567 / 0.597 /
  // 0.645 ms at 256 / 512 / 768 / 1024 (profiles/r03/decode/attn_grid_sweep_head.log).
  static const int wgs = std::max(1, env_int("P2PT_ATTN_WGS", 256));
  int sl = wgs / std::max(1, B * Hkv);
  return std::max(1, std::min({sl, cap, nsplit_ws}));
}

// Smallest token span of one attention workgroup (a multiple of its 32-token
// wave piece). 64 (two busy waves per workgroup) puts a short context on 4x
// the workgroups of 256 (one piece per wave): at batch 1 and 1k tokens the
// decode step went 396 -> 380 us on MI355X, unchanged at batch 16
// (profiles/r02/decode/decode_sweep_s4.log). P2PT_ATTN_MINSPAN overrides.
// Tokens per wave piece: 32, or 16 (half the K/V registers: 128 instead of
// 234 VGPRs, so two 8-wave workgroups fit a CU). Occupancy is not what bounds
// the kernel: 16 measured slower at every batch on MI355X (small, ctx 1024:
// b1 0.358 -> 0.365 ms, b16 0.522 -> 0.531, b64 1.125 -> 1.134;
// profiles/r03/decode/attn_tok_ab_head.log). P2PT_ATTN_TOK=16 opts in.
int attn_tok() {
  static const int v = env_int("P2PT_ATTN_TOK", 32) == 16 ? 16 : 32;
  return v;
}

int attn_min_span() {
  static const int v = std::max(32, env_int("P2PT_ATTN_MINSPAN", 64) / 32 * 32);
  return v;
}

// ------------------------------------------------------------ host side
struct LlamaDims {
  int vocab, dim, n_layers, H, Hkv, D, ffn, max_seq, max_batch;
  float eps, theta;
};

constexpr int kChunk = 64;  // tokens per attention workgroup = workspace granularity of its partials
constexpr int kTnResid = 1, kTnStore = 2;  // LM head: two 16-column subtiles per block
constexpr int kMaxKs = 8;    // split-K ways over workgroups
// O / down projections: 16-column tiles too. Narrowing them to one workgroup
// per CU (256) measured 1-4 % slower end to end once operands went through
// buffer loads (profiles/r02/decode/decode_sweep_*.log, "min256" vs "cw16").
constexpr int kResidMinTiles = 0;
constexpr int kCUs = 256;  // MI355X compute units: K-parts tiling aims at one workgroup per CU

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Workspace {
  uint16_t *resid, *q, *attn, *h;
  float *ss, *part_o, *part_ml, *am_val;
  int* am_idx;
  unsigned* counters;  // [kMaxM * H] attention split tickets (self-resetting)
  float* kpart;        // split-K slabs of the widest split GEMM
  unsigned* kctr;      // split-K tickets per column tile (self-resetting)
  size_t bytes;
};

Workspace carve(const LlamaDims& d, uint8_t* base) {
  Workspace w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    uint8_t* p = base ? base + off : nullptr;
    off += align256(n);
    return p;
  };
  const int nsplit = (d.max_seq + kChunk - 1) / kChunk;
  const int ss_parts = d.dim / (16 * kTnResid);
  const int am_parts = d.vocab / (16 * kTnStore);
  w.resid = reinterpret_cast<uint16_t*>(take(size_t(kMaxM) * d.dim * 2));
  w.q = reinterpret_cast<uint16_t*>(take(size_t(kMaxM) * d.H * d.D * 2));
  w.attn = reinterpret_cast<uint16_t*>(take(size_t(kMaxM) * d.H * d.D * 2));
  w.h = reinterpret_cast<uint16_t*>(take(size_t(kMaxM) * d.ffn * 2));
  w.ss = reinterpret_cast<float*>(take(size_t(ss_parts > 1 ? ss_parts : 1) * kMaxM * 4 * 4));  // up to 4-column tiles
  w.part_o = reinterpret_cast<float*>(take(size_t(kMaxM) * d.H * nsplit * d.D * 4));
  w.part_ml = reinterpret_cast<float*>(take(size_t(kMaxM) * d.H * nsplit * 2 * 4));
  w.am_val = reinterpret_cast<float*>(take(size_t(am_parts) * kMaxM * 4));
  w.am_idx = reinterpret_cast<int*>(take(size_t(am_parts) * kMaxM * 4));
  w.counters = reinterpret_cast<unsigned*>(take(size_t(kMaxM * d.H) * 4));
  const int qkv_n = (d.H + 2 * d.Hkv) * d.D;
  const int max_n = std::max(std::max(qkv_n, d.dim), 2 * d.ffn);
  w.kpart = reinterpret_cast<float*>(take(size_t(max_n / 16) * kMaxKs * 4 * kWave * 4));
  w.kctr = reinterpret_cast<unsigned*>(take(size_t(max_n / 16) * 4));
  w.bytes = off;
  return w;
}

// Waves per workgroup for `steps` 32-wide k-steps per workgroup. Measured on
// MI355X (scripts/bench_skinny.py, M = 8): 4 and 8 waves tie up to K = 2048,
// 8 beats 16 by 20-30 % at K = 5632 (a 16-wave block's reduction and barrier
// cost more than its extra loads in flight win back).
int pick_nw(int steps) {
  if (steps <= 0) return 0;
  return steps <= 16 ? 4 : 8;
}

// Split-K ways. Off by default: on MI355X the seam (write-through slabs,
// drain, arrival ticket, slab reads by the last arriver) costs more latency
// than the extra workgroups win back at d_model <= 2048 (QKV 8.7 -> 13.5 us,
// O 7.4 -> 12.0 us, down 17.3 -> 17.3 us on the 2048-wide config, batch 8).
// P2PT_DECODE_SPLITK=1 enables it (grid grown toward 512 workgroups while
// every workgroup keeps >= 8 k-steps) for wider models / experiments.
int pick_ks(int tiles, int K) {
  static const bool on = [] {
    const char* e = getenv("P2PT_DECODE_SPLITK");
    return e && *e == '1';
  }();
  if (!on) return 1;
  const int S = K >> 5;
  int ks = 1;
  while (ks < kMaxKs && tiles * ks < 512 && S / (ks * 2) >= 8) ks *= 2;
  return ks;
}

template <int NW, int TN, int EPI>
hipError_t launch_nw(const GemmArgs& a, int grid, hipStream_t s) {
  // Load batch: each wave's share of k-steps, rounded up to a power of two,
  // capped by the VGPR budget (8, or 4 for 1024-thread two-subtile blocks).
  // Batches of at most 4 k-steps: fewer registers, more resident waves (batch
  // 1: 396 -> 389 us per step, batch 16 unchanged; P2PT_DECODE_UMCAP=8 restores
  // 8-step batches).
  static const int ucap = env_int("P2PT_DECODE_UMCAP", 4);
  const int kCap = ((NW >= 16 && TN >= 2) || ucap <= 4) ? 4 : 8;
  const int per_wave = (((a.K >> a.kpl) >> 5) / a.ks + NW - 1) / NW;
  const dim3 g(grid * a.ks, (a.M + 15) >> 4), b(NW * 64);
  if (per_wave <= 1)
    hipLaunchKernelGGL((k_skinny<NW, TN, EPI, 1>), g, b, 0, s, a);
  else if (per_wave <= 2)
    hipLaunchKernelGGL((k_skinny<NW, TN, EPI, 2>), g, b, 0, s, a);
  else if (per_wave <= 4 || kCap == 4)
    hipLaunchKernelGGL((k_skinny<NW, TN, EPI, 4>), g, b, 0, s, a);
  else
    hipLaunchKernelGGL((k_skinny<NW, TN, EPI, 8>), g, b, 0, s, a);
  return hipGetLastError();
}

// Column-tile width (log2) for an N-column projection with TN subtiles per
// workgroup: the widest tile (16) that still gives >= min_tiles workgroups,
// down to 4 columns (P2PT_DECODE_MIN_TILES overrides the threshold; 0: always
// 16). Measured on MI355X (profiles/r02/decode/): narrower tiles win a
// little on the O projection alone (5.8 -> 5.5 us at batch 1) and lose on QKV
// (6.1 -> 7.8 us), where the repeated activation loads cost more than the
// extra CUs win; 16 everywhere is fastest end to end.
int pick_cwl(int N, int TN, int dflt_min_tiles) {
  static const int env = env_int("P2PT_DECODE_MIN_TILES", -1);
  const int min_tiles = env >= 0 ? env : dflt_min_tiles;
  int cwl = 4;
  while (cwl > 2 && (N >> cwl) / TN < min_tiles) cwl--;
  return cwl;
}

// K-parts tiling (GemmArgs::kpl) for an N-column, TN = 1 projection of M rows:
// the tile width 2^cwl whose N >> cwl column tiles first reach `min_tiles`
// workgroups (one per CU), if the spare MFMA rows allow it (M * P <= 16,
// P = 16 >> cwl) and K splits into P parts of whole k-steps; false otherwise.
bool pick_kparts(int N, int M, int K, int min_tiles, int* cwl, int* kpl) {
  for (int c = 4; c >= 2; c--) {
    if ((N >> c) < min_tiles && c > 2) continue;
    const int P = 16 >> c;
    if (P == 1 || M * P > 16 || K % (P * 32)) return false;
    *cwl = c;
    *kpl = 4 - c;
    return true;
  }
  return false;
}

// K parts for the 2048-wide O and down projections (one workgroup per CU):
// small config, batch 1, 0.372 -> 0.359 ms per step (profiles/r03/decode/
// decode_ab_kparts.log). On QKV (3072 columns: 384 workgroups of 8) it cost
// 3-4 us per step, so that stays opt-in (P2PT_DECODE_QKV_KPARTS=1).
// P2PT_DECODE_KPARTS=0 turns it off.
// K parts at a given tile width (2^cwl columns, P = 16 >> cwl parts); false
// where the rows or K do not allow it.
bool kparts_at(int M, int K, int cwl, int* out_cwl, int* kpl) {
  if (cwl < 2 || cwl > 3) return false;
  const int P = 16 >> cwl;
  if (M * P > 16 || K % (P * 32)) return false;
  *out_cwl = cwl;
  *kpl = 4 - cwl;
  return true;
}

bool kparts_on() {
  static const bool v = env_int("P2PT_DECODE_KPARTS", 1) != 0;
  return v;
}

// grid = column tiles of the chosen width; the launch has grid * a.ks workgroups (a.ks == 0: pick).
template <int EPI, int TN>
hipError_t launch_gemm(GemmArgs a, hipStream_t s, int nw_override = 0) {
  if (a.cwl <= 0) a.cwl = pick_cwl(a.N, TN, 0);
  if (a.kpl && (TN != 1 || a.M * (16 >> a.cwl) > 16 || (16 >> a.cwl) != (1 << a.kpl) || a.K % (32 << a.kpl)))
    return hipErrorInvalidValue;
  const int grid = a.N / (TN << a.cwl);
  if (a.ks <= 0) a.ks = (a.kpart && a.kctr && a.cwl == 4) ? pick_ks(grid, a.K) : 1;
  if (a.M > 16 || a.cwl != 4 || a.kpl) a.ks = 1;  // split-K slabs and tickets: one row tile of 16-column tiles only
  const int nw = nw_override ? nw_override : pick_nw(((a.K >> a.kpl) >> 5) / a.ks);
  if (nw == 16) return launch_nw<16, TN, EPI>(a, grid, s);
  if (nw == 8) return launch_nw<8, TN, EPI>(a, grid, s);
  if (nw == 4) return launch_nw<4, TN, EPI>(a, grid, s);
  return hipErrorInvalidValue;
}

bool dims_ok(const LlamaDims& d) {
  if (d.D != 64 && d.D != 128) return false;
  // GEMM operands are addressed with 32-bit byte offsets below kOob (2 GiB):
  // each weight's own N x K bf16 extent (LM head vocab x dim, QKV, gate/up,
  // O, down), not the widest N times the largest K of different GEMMs.
  const size_t dim = size_t(d.dim), ffn = size_t(d.ffn), hd = size_t(d.H) * d.D;
  const size_t gemm_bytes[] = {size_t(d.vocab) * dim * 2, size_t(d.H + 2 * d.Hkv) * d.D * dim * 2,
                               2 * ffn * dim * 2, dim * hd * 2, dim * ffn * 2};
  for (size_t b : gemm_bytes)
    if (b >= kOob) return false;
  if (d.H % d.Hkv || (d.H / d.Hkv != 1 && d.H / d.Hkv != 2 && d.H / d.Hkv != 4 && d.H / d.Hkv != 8)) return false;
  if (d.dim % 32 || (d.H * d.D) % 32 || d.ffn % 32) return false;
  if (d.dim % (16 * kTnResid) || d.vocab % (16 * kTnStore) || d.ffn % 16) return false;
  if (d.max_batch <= 0 || d.max_seq <= 0 || d.n_layers <= 0) return false;
  return true;
}

}  // namespace

extern "C" {

// Workspace bytes for p2pt_llama_decode; it must be zero-filled once before first use
// (the in-kernel arrival counters reset themselves afterwards).
size_t p2pt_llama_ws_bytes(const LlamaDims* d) {
  if (!dims_ok(*d)) return 0;
  return carve(*d, nullptr).bytes;
}

// One decode step for B <= 16 sequences (slots 0..B-1 of the caches).
//   w: embed, final_norm, lm_head, then per layer
//      attn_norm, wqkv [(H+2Hkv)*D, dim], wo [dim, H*D], ffn_norm, w_gate_up [2*ffn, dim], w_down [dim, ffn]
//      where wqkv, w_gate_up and lm_head carry the preceding RMSNorm weight folded
//      into their columns (W[n][k] * g[k]); the norm-weight slots are not read.
//      wqkv rows are interleaved per head (dim i, dim i + D/2, ...) and w_gate_up
//      rows per pair (gate_j, up_j, ...).
//   k_cache/v_cache: [n_layers][max_batch][max_seq][Hkv][D]
//   tokens int64 [B <= 64], pos int32 [B] (< max_seq), logits bf16 [B][vocab], ids int64 [B]
//   emit_rows: only rows [0, emit_rows) get logits and ids (the LM head runs on
//     them alone: prefill rows that sample nothing go last); <= 0 means B
//   slots int32 [B] or nullptr: cache slot of each row (< max_batch). Rows of one
//     slot at consecutive positions form a prefill chunk: every row's K/V is
//     appended before attention runs, and each row attends up to its own position.
//   max_len: host bound on max(pos) + 1 (sizes the attention grid; use max_seq under graph capture)
int p2pt_llama_decode(const LlamaDims* dp, const void* const* w, void* k_cache, void* v_cache, const int64_t* tokens,
                      const int* pos, const int* slots, int B, int emit_rows, int max_len, void* ws, size_t ws_bytes,
                      void* logits, int64_t* ids, void* stream) {
  const LlamaDims d = *dp;
  if (!dims_ok(d) || B <= 0 || B > kMaxM || (!slots && B > d.max_batch) || max_len <= 0 || max_len > d.max_seq)
    return int(hipErrorInvalidValue);
  if (emit_rows <= 0 || emit_rows > B) emit_rows = B;
  Workspace W = carve(d, static_cast<uint8_t*>(ws));
  if (ws_bytes < W.bytes) return int(hipErrorInvalidValue);
  auto s = static_cast<hipStream_t>(stream);
  auto bf = [&](int i) { return static_cast<const uint16_t*>(w[i]); };
  const int qkv_n = (d.H + 2 * d.Hkv) * d.D;
  const size_t layer_cache = size_t(d.max_batch) * d.max_seq * d.Hkv * d.D;
  const int nsplit_ws = (d.max_seq + kChunk - 1) / kChunk;
  const float log2_theta = log2f(d.theta);

  hipLaunchKernelGGL(k_embed, dim3(B), dim3(256), 0, s, bf(0), tokens, W.resid, W.ss, d.dim, d.vocab);
  int ss_parts = 1;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return int(e);

  for (int L = 0; L < d.n_layers; L++) {
    const uint16_t* wqkv = bf(4 + 6 * L);
    const uint16_t* wo = bf(5 + 6 * L);
    const uint16_t* wgu = bf(7 + 6 * L);
    const uint16_t* wdown = bf(8 + 6 * L);
    uint16_t* kc = static_cast<uint16_t*>(k_cache) + L * layer_cache;
    uint16_t* vc = static_cast<uint16_t*>(v_cache) + L * layer_cache;

    GemmArgs a{};
    a.M = B;
    a.eps = d.eps;
    // QKV + RoPE + cache append
    a.x = W.resid; a.w = wqkv; a.N = qkv_n; a.K = d.dim;
    a.ss_part = W.ss; a.ss_parts = ss_parts;
    a.pos = pos; a.slot = slots; a.nslots = d.max_batch; a.q_out = W.q; a.kc = kc; a.vc = vc;
    a.H = d.H; a.Hkv = d.Hkv; a.D = d.D; a.Smax = d.max_seq; a.log2_theta = log2_theta;
    a.kpart = W.kpart; a.kctr = W.kctr;
    static const bool qkv_kparts = env_int("P2PT_DECODE_QKV_KPARTS", 0) != 0;
    // Experiments: K parts at a given width. Slower than 16-column tiles on
    // QKV (batch 1: 4 columns 0.360 -> 0.373 ms per step) and gate/up (8
    // columns 0.368, 4 columns 0.391 ms): more, smaller workgroups do not
    // stream faster once the grid already covers the chip
    // (profiles/r03/decode/decode_ab_cwl.log).
    static const int qkv_cwl = env_int("P2PT_DECODE_QKV_CWL", 0);
    if (!(kparts_on() && ((qkv_cwl && kparts_at(B, d.dim, qkv_cwl, &a.cwl, &a.kpl)) ||
                          (qkv_kparts && pick_kparts(qkv_n, B, d.dim, kCUs, &a.cwl, &a.kpl)))))
      a.kpl = 0;
    if (a.kpl == 0) a.cwl = 0;
    if ((e = launch_gemm<EPI_ROPE, 1>(a, s)) != hipSuccess) return int(e);

    // attention: (span slot, row, KV head) workgroups of 8 waves
    {
      (void)max_len;  // the grid no longer depends on the context length
      dim3 grid(attn_slots(B, d.Hkv, nsplit_ws), B * d.Hkv);
      const float scale = 1.f / sqrtf(float(d.D));
      const int G = d.H / d.Hkv;
#define P2PT_ATTN(DD, GG)                                                                                          \
  do {                                                                                                             \
    if (attn_tok() == 16)                                                                                          \
      hipLaunchKernelGGL((k_attn<DD, GG, 16>), grid, dim3(512), 0, s, W.q, kc, vc, pos, slots, d.max_batch,      \
                         W.part_o, W.part_ml, W.counters, W.attn, d.H, d.Hkv, d.max_seq, nsplit_ws, scale,        \
                         attn_min_span());                                                                         \
    else                                                                                                           \
      hipLaunchKernelGGL((k_attn<DD, GG>), grid, dim3(512), 0, s, W.q, kc, vc, pos, slots, d.max_batch, W.part_o, \
                         W.part_ml, W.counters, W.attn, d.H, d.Hkv, d.max_seq, nsplit_ws, scale, attn_min_span());\
  } while (0)
      if (d.D == 64) {
        if (G == 1) P2PT_ATTN(64, 1); else if (G == 2) P2PT_ATTN(64, 2); else if (G == 4) P2PT_ATTN(64, 4); else P2PT_ATTN(64, 8);
      } else {
        if (G == 1) P2PT_ATTN(128, 1); else if (G == 2) P2PT_ATTN(128, 2); else if (G == 4) P2PT_ATTN(128, 4); else P2PT_ATTN(128, 8);
      }
#undef P2PT_ATTN
      if ((e = hipGetLastError()) != hipSuccess) return int(e);
    }

    // O projection + residual
    GemmArgs o{};
    o.M = B; o.x = W.attn; o.w = wo; o.N = d.dim; o.K = d.H * d.D;
    o.out = W.resid; o.ss_out = W.ss; o.kpart = W.kpart; o.kctr = W.kctr;
    if (!(kparts_on() && pick_kparts(d.dim, B, d.H * d.D, kCUs, &o.cwl, &o.kpl))) {
      o.kpl = 0;
      o.cwl = pick_cwl(d.dim, kTnResid, kResidMinTiles);
    }
    // Three launches: a persistent O -> gate/up -> down kernel (one launch, an
    // in-order tile queue with write-through hand-offs) was built in round 3
    // and measured slower in every variant (small b1 0.358 -> 0.61-1.09 ms,
    // profiles/r03/decode_block/), then removed.
    if ((e = launch_gemm<EPI_RESID, kTnResid>(o, s)) != hipSuccess) return int(e);
    ss_parts = d.dim / (kTnResid << o.cwl);

    // gate/up + SwiGLU
    GemmArgs g{};
    g.M = B; g.eps = d.eps; g.x = W.resid; g.w = wgu; g.N = 2 * d.ffn; g.K = d.dim;
    g.ss_part = W.ss; g.ss_parts = ss_parts; g.out = W.h; g.kpart = W.kpart; g.kctr = W.kctr;
    static const int gu_cwl = env_int("P2PT_DECODE_GU_CWL", 0);  // experiments (see QKV above)
    if (!(kparts_on() && gu_cwl && kparts_at(B, d.dim, gu_cwl, &g.cwl, &g.kpl))) {
      g.kpl = 0;
      g.cwl = 0;
    }
    if ((e = launch_gemm<EPI_SILU, 1>(g, s)) != hipSuccess) return int(e);

    // down + residual
    GemmArgs dn{};
    dn.M = B; dn.x = W.h; dn.w = wdown; dn.N = d.dim; dn.K = d.ffn; dn.out = W.resid; dn.ss_out = W.ss;
    dn.kpart = W.kpart; dn.kctr = W.kctr;
    if (!(kparts_on() && pick_kparts(d.dim, B, d.ffn, kCUs, &dn.cwl, &dn.kpl))) {
      dn.kpl = 0;
      dn.cwl = pick_cwl(d.dim, kTnResid, kResidMinTiles);
    }
    if ((e = launch_gemm<EPI_RESID, kTnResid>(dn, s)) != hipSuccess) return int(e);
    ss_parts = d.dim / (kTnResid << dn.cwl);
  }

  // final norm + LM head + argmax
  GemmArgs h{};
  h.M = emit_rows; h.eps = d.eps; h.x = W.resid; h.w = bf(2); h.N = d.vocab; h.K = d.dim;
  h.ss_part = W.ss; h.ss_parts = ss_parts;
  h.out = static_cast<uint16_t*>(logits);
  h.am_val = W.am_val; h.am_idx = W.am_idx;
  h.cwl = 4;  // the argmax partials are sized for 16-column tiles
  const int parts = d.vocab / (16 * kTnStore);
  // 4 waves x 2 subtiles: the fastest LM-head shape measured (vocab 32000, K 2048: 22.6 vs 29.6 us).
  // The merge stays a launch of its own: folded into the LM head's last block
  // (write-through partials + arrival ticket) the step took 0.359 -> 0.366 ms
  // at batch 1 and 0.522 -> 0.554 ms at 16, the 1,000 blocks' arrivals on one
  // counter costing more than the launch (profiles/r03/decode/decode_ab_kparts.log).
  if ((e = launch_gemm<EPI_ARGMAX, kTnStore>(h, s, 4)) != hipSuccess) return int(e);
  hipLaunchKernelGGL(k_argmax_merge, dim3(emit_rows), dim3(256), 0, s, W.am_val, W.am_idx, parts, ids);
  return int(hipGetLastError());
}

// Standalone skinny GEMM (tests/benchmarks): out[M][N] = bf16(x[M][K] @ w[N][K]^T), M <= 64.
int p2pt_skinny_gemm(const void* x, const void* w, void* out, int M, int N, int K, void* stream) {
  if (M <= 0 || M > kMaxM || N % 32 || K <= 0 || K % 32) return int(hipErrorInvalidValue);
  GemmArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w);
  a.out = static_cast<uint16_t*>(out);
  a.M = M; a.N = N; a.K = K; a.ks = 1; a.cwl = 4;
  return int(launch_gemm<EPI_STORE, 2>(a, static_cast<hipStream_t>(stream)));
}

// Microbenchmark hook (scripts/bench_skinny.py --attn): `reps` back-to-back
// launches of the decode attention kernel. part_o / part_ml / counters as in
// the workspace (counters zeroed); q [B][H*D], caches [B][Smax][Hkv][D].
int p2pt_attn_bench(const void* q, const void* kc, const void* vc, const int* pos, int B, int H, int Hkv, int D,
                    int Smax, int max_len, float* part_o, float* part_ml, unsigned* counters, void* out, int reps,
                    void* stream) {
  const int G = Hkv > 0 ? H / Hkv : 0;
  if (B <= 0 || B > kMaxM || (D != 64 && D != 128) || G != 4 || max_len <= 0 || max_len > Smax || reps <= 0)
    return int(hipErrorInvalidValue);
  auto st = static_cast<hipStream_t>(stream);
  const int nsplit_ws = (Smax + kChunk - 1) / kChunk;
  const float scale = 1.f / sqrtf(float(D));
  for (int r = 0; r < reps; r++) {
    dim3 grid(attn_slots(B, Hkv, nsplit_ws), B * Hkv);
    auto qq = static_cast<const uint16_t*>(q);
    auto kk = static_cast<const uint16_t*>(kc);
    auto vv = static_cast<const uint16_t*>(vc);
    auto oo = static_cast<uint16_t*>(out);
    if (D == 64)
      hipLaunchKernelGGL((k_attn<64, 4>), grid, dim3(512), 0, st, qq, kk, vv, pos, nullptr, B, part_o, part_ml,
                         counters, oo, H, Hkv, Smax, nsplit_ws, scale, attn_min_span());
    else
      hipLaunchKernelGGL((k_attn<128, 4>), grid, dim3(512), 0, st, qq, kk, vv, pos, nullptr, B, part_o, part_ml,
                         counters, oo, H, Hkv, Smax, nsplit_ws, scale, attn_min_span());
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return int(e);
  }
  return 0;
}

// Microbenchmark hook (scripts/bench_skinny.py): `reps` back-to-back launches
// of the skinny GEMM with an explicit waves-per-block / subtile choice.
int p2pt_skinny_bench(const void* x, const void* w, void* out, int M, int N, int K, int nw, int tn, int reps,
                      void* stream) {
  if (M <= 0 || M > kMaxM || N % (16 * tn) || K <= 0 || K % 32 || reps <= 0) return int(hipErrorInvalidValue);
  GemmArgs a{};
  a.x = static_cast<const uint16_t*>(x);
  a.w = static_cast<const uint16_t*>(w);
  a.out = static_cast<uint16_t*>(out);
  a.M = M; a.N = N; a.K = K; a.ks = 1; a.cwl = 4;
  auto st = static_cast<hipStream_t>(stream);
  for (int r = 0; r < reps; r++) {
    hipError_t e;
    const int grid = N / (16 * tn);
    if (tn == 1)
      e = nw == 4 ? launch_nw<4, 1, EPI_STORE>(a, grid, st) : nw == 8 ? launch_nw<8, 1, EPI_STORE>(a, grid, st)
                                                          : launch_nw<16, 1, EPI_STORE>(a, grid, st);
    else
      e = nw == 4 ? launch_nw<4, 2, EPI_STORE>(a, grid, st) : nw == 8 ? launch_nw<8, 2, EPI_STORE>(a, grid, st)
                                                          : launch_nw<16, 2, EPI_STORE>(a, grid, st);
    if (e != hipSuccess) return int(e);
  }
  return 0;
}

}  // extern "C"
