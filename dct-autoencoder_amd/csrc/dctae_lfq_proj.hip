// LFQ with projections (lfq.py:54-62: dim != codebook_dim * num_codebooks puts
// nn.Linear project_in / project_out around the quantiser; conf/patch14-l.json:
// 196-element tokens -> 16 codebooks x 13 bits = 208).  Both directions are one
// fused kernel each on v_mfma_f32_16x16x4_f32 (f32 operands, f32 accumulate):
//
//  mode 0, encode (lfq.py:164 project_in, :175-187 sign + index packing):
//    h = x W_in^T + b_in; bit = h > 0 (NaN -> 0); index of codebook c =
//    sum_b bit[c cd + b] 2^(cd - 1 - b) (mask = 2^arange(cd-1..0), lfq.py:70).
//    h never leaves the CU: four 16-bit sign ballots per 16x16 tile go to LDS
//    and each lane assembles (token, codebook) indices from them.
//  mode 1, decode (lfq.py:105-127 indices_to_codes + project_out):
//    codes = +-scale from the index bits (bits * 2 scale - scale, lfq.py:117-124),
//    built straight into the LDS A tile; out = codes W_out^T + b_out.
//
// Tile: 128 tokens per 512-thread block (16 per wave), all N <= 256 outputs per
// wave (NT tiles of 16: NT x 4 accumulators), K in chunks of 16 (double-buffered in LDS, one barrier per chunk) with the
// next chunk's global loads in flight during the current chunk's MFMAs.  Lane
// (r = l & 15, q = l >> 4) reads float4 k = 4q .. 4q + 3 of its A row (token)
// and B row (output feature); MFMA step s pairs k = 4q + s on both sides, so
// the 16 k of a chunk are covered once (the order of the f32 sum differs from
// torch's: results are not bit-equal to nn.Linear, see tests/test_gpu_lfq_proj.py).
#include "dctae_device.h"
#include "dctae_launch.h"

#include <cmath>

namespace dctae {

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// optional inverse PatchNorm fused into mode 1's epilogue (patchnorm.py:167-177:
// y * (b sqrt 2 + eps) + median at the token's (channel, h, w) table row)
struct InvNorm {
  const int64_t* ch;    // (n) channels of the tokens, or null: no inverse
  const int64_t* pos;   // (n, 2)
  const float* med;     // (3, maxph, maxpw, D)
  const float* b;
  float eps;
  int maxph, maxpw;
  int* err;             // bit 1: a table index out of range (the reference raises IndexError)
};

constexpr int kTokW = 16;    // tokens per wave and M tile
constexpr int kKc = 32;      // k chunk (one v_mfma_f32_16x16x32_bf16 step)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 hv8 __attribute__((ext_vector_type(8)));

// LDS image of a 32-k chunk: bf16 pieces of R rows, 64-byte rows, 16-byte k
// group kq of row r at slot kq ^ swz(r) (conflict-free for the fragment reads
// and the staging writes, as k_gemm_x3)
__device__ __forceinline__ int pswz(int r) { return ((r >> 1) ^ (r >> 2)) & 3; }
__device__ __forceinline__ int poff(int r, int kq) { return r * kKc + 8 * (kq ^ pswz(r)); }

// split 8 floats into NPC bf16 pieces (v = p0 + p1 + p2 to fp32 precision)
// and write them to the piece planes at offset o
template <int NPC>
__device__ __forceinline__ void split8(uint16_t* planes, int plane, int o, f32x8 v) {
  const bfv8 h0 = __builtin_convertvector(v, bfv8);
  *reinterpret_cast<bfv8*>(planes + o) = h0;
  if constexpr (NPC > 1) {
    const f32x8 r1 = v - __builtin_convertvector(h0, f32x8);
    const bfv8 h1 = __builtin_convertvector(r1, bfv8);
    const f32x8 r2 = r1 - __builtin_convertvector(h1, f32x8);
    *reinterpret_cast<bfv8*>(planes + plane + o) = h1;
    *reinterpret_cast<bfv8*>(planes + 2 * plane + o) = __builtin_convertvector(r2, bfv8);
  }
}

// the fp16 form (H2): v scaled by the power of two `sc` into [2^13, 2^14) at
// most, NPC pieces (2: v = p0 + p1 to 22 bits; 1: exact, e.g. +-scale codes)
template <int NPC>
__device__ __forceinline__ void split8h(uint16_t* planes, int plane, int o, f32x8 v, float sc) {
  const f32x8 vs = v * sc;
  const hv8 h0 = __builtin_convertvector(vs, hv8);
  *reinterpret_cast<hv8*>(planes + o) = h0;
  if constexpr (NPC > 1)
    *reinterpret_cast<hv8*>(planes + plane + o) = __builtin_convertvector(vs - __builtin_convertvector(h0, f32x8), hv8);
}

// Split-precision GEMM on the bf16 MFMA: A (tokens or +-scale codes) and W are
// split into three bf16 pieces each and the product keeps the six terms of
// piece order <= 2 (a0 b0 + a0 b1 + a1 b0 + a1 b1 + a0 b2 + a2 b0, fp32
// accumulation; the dropped terms are ~2^-24 |a b|: fp32-level accuracy, as
// k_gemm_x3).  A1: A is exact in bf16 (mode 1 with a bf16-exact scale: +-scale
// codes), one piece, three products.
// H2: the fp16 form -- A and W scaled by powers of two into the fp16 range
// (A by a_scale from the caller's bound on |A|, W by 2^w_exp[0] from
// k_split_w_h2), two pieces each (A1: one), three products (A1: two) on
// v_mfma_f32_16x16x32_f16; the dropped terms are <= 3 x 2^-22 |a w|, the
// accumulator is unscaled exactly before the bias
template <int NT, int MODE, int WB, bool A1, bool H2>
__device__ __forceinline__ void lfq_proj_body(const float* __restrict__ x, const int64_t* __restrict__ idx_in,
                                                 int64_t n, int K, int N, const float* __restrict__ w,
                                                 const float* __restrict__ bias, int cd, int ncb, float scale,
                                                 int64_t* __restrict__ idx_out, float* __restrict__ out,
                                                 uint16_t* __restrict__ idx16, InvNorm inv,
                                                 const uint16_t* __restrict__ wsp, int Kp, float a_scale,
                                                 const int* __restrict__ w_exp) {
  constexpr int MT = 1;                            // 16-token M tiles per wave
  constexpr int kThr = 64 * WB;                    // WB waves per block
  constexpr int kTok = kTokW * WB * MT;            // tokens per block
  constexpr int NP = NT * 16;                      // padded output features
  constexpr int NPA = A1 ? 1 : (H2 ? 2 : 3);       // A pieces
  constexpr int NPW = H2 ? 2 : 3;                  // W pieces
  constexpr int kPA = kTok * kKc, kPW = NP * kKc;  // plane sizes (16-bit elements)
  static_assert(kThr == 4 * kTok, "A staging: one 8-k group per thread");
  __shared__ __attribute__((aligned(16))) uint16_t As[NPA * kPA];
  __shared__ __attribute__((aligned(16))) uint16_t Ws[NPW * kPW];
  const float unscale = H2 ? ldexpf(1.0f / a_scale, -w_exp[0]) : 1.0f;
  __shared__ int64_t Tb[MODE == 1 ? 32 : 1];   // mode 1 + inverse: table rows of a round's 32 tokens
  __shared__ int32_t Ix[MODE == 1 ? kTok * 32 : 1];   // mode 1: the block's indices (ncb <= 32)
  __shared__ uint32_t Msk[MODE == 0 ? WB * 16 * MT * (NT + 3) : 1];  // mode 0: sign pieces [wave][token][tile]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int64_t tok0 = (int64_t)blockIdx.x * kTok;
  const int nt = n - tok0 < kTok ? (int)(n - tok0) : kTok;

  if (MODE == 1) {
    for (int e = tid; e < kTok * ncb; e += kThr) {
      const int t = e / ncb;
      Ix[e] = t < nt ? (int32_t)idx_in[tok0 * ncb + e] : 0;   // lfq.py:117 indices.int()
    }
    __syncthreads();
  }

  floatx4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // A staging: thread tid owns k group tid & 3 (8 k) of token tid >> 2
  const int at = tid >> 2, aq = tid & 3;
  // W: the three pre-split bf16 planes [3][NP][Kp] (k_split_w), 16-byte pieces
  constexpr int WG = (NP * 4 + kThr - 1) / kThr;   // W 8-k groups per thread and chunk
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(wsp), 0, NPW * NP * Kp * 2, 0x00020000);
  f32x8 ra;
  u32x4 rw[WG][NPW];
  auto load = [&](int k0) {
    const int k = k0 + 8 * aq;
    if (MODE == 0) {
      const bool ok = at < nt;
      const float* xr = x + (tok0 + (ok ? at : 0)) * K + k;
      const float4 lo = ok && k < K ? *reinterpret_cast<const float4*>(xr) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 hi = ok && k + 4 < K ? *reinterpret_cast<const float4*>(xr + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      ra = (f32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kk = k + e;
        const int c = kk / cd, b = kk - c * cd;
        const bool bit = kk < K && ((Ix[at * ncb + (kk < K ? c : 0)] >> (cd - 1 - b)) & 1);
        ra[e] = kk < K ? (bit ? scale : -scale) : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < WG; ++i) {
      const int g = tid + kThr * i;
      const int o = g < NP * 4 ? ((g >> 2) * Kp + k0 + 8 * (g & 3)) * 2 : 0x7ffffff0;
#pragma unroll
      for (int pc = 0; pc < NPW; ++pc)
        rw[i][pc] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, o + pc * NP * Kp * 2, 0, 0));
    }
  };
  auto store = [&]() {
    if constexpr (H2)
      split8h<NPA>(As, kPA, poff(at, aq), ra, a_scale);
    else
      split8<NPA>(As, kPA, poff(at, aq), ra);
#pragma unroll
    for (int i = 0; i < WG; ++i) {
      const int g = tid + kThr * i;
      if (g < NP * 4) {
#pragma unroll
        for (int pc = 0; pc < NPW; ++pc) *reinterpret_cast<u32x4*>(&Ws[pc * kPW + poff(g >> 2, g & 3)]) = rw[i][pc];
      }
    }
  };

  // wave w owns tokens [16 w, + 16) of the block; one 32-k MFMA step per chunk
  load(0);
  store();
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += kKc) {
    const bool more = k0 + kKc < K;
    if (more) load(k0 + kKc);
    bf16x8 a[NPA];
#pragma unroll
    for (int pc = 0; pc < NPA; ++pc) a[pc] = *reinterpret_cast<const bf16x8*>(&As[pc * kPA + poff(wave * kTokW + r, q)]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      bf16x8 b[NPW];
#pragma unroll
      for (int pc = 0; pc < NPW; ++pc) b[pc] = *reinterpret_cast<const bf16x8*>(&Ws[pc * kPW + poff(16 * t + r, q)]);
      floatx4& c = acc[0][t];
      if constexpr (H2) {
        const hv8 a0 = __builtin_bit_cast(hv8, a[0]), b0 = __builtin_bit_cast(hv8, b[0]), b1 = __builtin_bit_cast(hv8, b[1]);
        if constexpr (!A1) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hv8, a[NPA - 1]), b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, c, 0, 0, 0);
      } else {
        if constexpr (!A1) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[NPA - 1], b[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
        }
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[NPW - 1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }

  // C/D map: lane l, register v -> token 4 (l >> 4) + v of the M tile, feature 16 t + (l & 15)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int64_t wt0 = tok0 + (wave + WB * m) * kTokW;   // first token of this M tile
    if (MODE == 0) {
      uint32_t* msk = Msk + (wave * MT + m) * 16 * (NT + 3);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = 16 * t + r;
        const float bb = (bias && col < N) ? bias[col] : 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float h = acc[m][t][v] * unscale + bb;
          const uint64_t mk = __ballot(col < N && h > 0.0f);   // lfq.py:175 (NaN -> False)
          if (lane < 4) msk[(4 * lane + v) * (NT + 3) + t] = (uint32_t)(mk >> (16 * lane)) & 0xffffu;
        }
      }
      if (lane < 16 * 3) msk[(lane / 3) * (NT + 3) + NT + lane % 3] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // (token i, codebook c) pairs of the tile, token-major: contiguous int64 stores
      const int wn = n - wt0 <= 0 ? 0 : n - wt0 < kTokW ? (int)(n - wt0) : kTokW;
      for (int p = lane; p < wn * ncb; p += 64) {
        const int i = p / ncb, c = p - i * ncb;
        const int o0 = c * cd, pc = o0 >> 4, sh = o0 & 15;
        const uint32_t* mi = msk + i * (NT + 3);
        const uint64_t win = (uint64_t)mi[pc] | ((uint64_t)mi[pc + 1] << 16) | ((uint64_t)mi[pc + 2] << 32) |
                             ((uint64_t)mi[pc + 3] << 48);
        const uint32_t bits = (uint32_t)(win >> sh) & ((1u << cd) - 1u);   // bit b = feature o0 + b
        const uint32_t code = __builtin_bitreverse32(bits) >> (32 - cd);
        if (idx16)
          idx16[wt0 * ncb + p] = (uint16_t)code;   // encode staging (cd <= 16), gathered by k_sort_pack2
        else   // lfq.py:187: the bit of the quantized value (the staging above keeps the raw sign bits)
          idx_out[wt0 * ncb + p] = (int64_t)lfq_index_bits(code, scale > 0.0f ? ~0ull : 0ull, -scale > 0.0f ? ~0ull : 0ull) &
                                   ((1ll << cd) - 1);
      }
    } else {
      if (inv.ch) {
        // inverse PatchNorm: the output tiles go through the freed W buffers, 2
        // waves per round, so the table gathers and the stores run as 16-byte
        // pieces along each token's 196 contiguous floats (same fp32 ops as
        // dctae_norm_inverse on the stored projection: bit-equal)
        constexpr int WPR = 2;
        float* stg = reinterpret_cast<float*>(Ws);   // 6 NP kKc bytes >= WPR x 16 x N floats
        const int N4 = N >> 2;
        for (int rd = 0; rd < WB / WPR; ++rd) {
          __syncthreads();   // the previous round's (or the K loop's) LDS reads are done
          const int wl = wave - rd * WPR;
          if (wl >= 0 && wl < WPR) {
            float* tl = stg + wl * kTokW * N;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const int col = 16 * t + r;
              if (col >= N) continue;
              const float bb = bias ? bias[col] : 0.f;
#pragma unroll
              for (int v = 0; v < 4; ++v) tl[(4 * q + v) * N + col] = acc[m][t][v] * unscale + bb;
            }
          }
          const int64_t rt0 = tok0 + (int64_t)rd * WPR * kTokW;   // first token of the round
          if (tid < WPR * kTokW) {
            const int64_t row = rt0 + tid;
            int64_t tb = -2;   // -2: past n, -1: out-of-range table index
            if (row < n) {
              const int64_t c = inv.ch[row], h = inv.pos[2 * row], w = inv.pos[2 * row + 1];
              const bool ok = c >= 0 && c < 3 && h >= 0 && h < inv.maxph && w >= 0 && w < inv.maxpw;
              if (!ok) atomicOr(inv.err, 1);
              tb = ok ? ((c * inv.maxph + h) * inv.maxpw + w) * N : -1;
            }
            Tb[tid] = tb;
          }
          __syncthreads();
          for (int e = tid; e < WPR * kTokW * N4; e += kThr) {
            const int i = e / N4, c4 = e - i * N4;
            const int64_t tb = Tb[i];
            if (tb == -2) continue;
            float4 y = *reinterpret_cast<const float4*>(stg + i * N + 4 * c4);
            if (tb >= 0) {
              const float4 md = *reinterpret_cast<const float4*>(inv.med + tb + 4 * c4);
              const float4 bd = *reinterpret_cast<const float4*>(inv.b + tb + 4 * c4);
              y = make_float4(pn_inverse(y.x, md.x, bd.x, inv.eps), pn_inverse(y.y, md.y, bd.y, inv.eps),
                              pn_inverse(y.z, md.z, bd.z, inv.eps), pn_inverse(y.w, md.w, bd.w, inv.eps));
            } else {
              const float qn = __int_as_float(0x7fc00000);
              y = make_float4(qn, qn, qn, qn);
            }
            *reinterpret_cast<float4*>(out + (rt0 + i) * N + 4 * c4) = y;
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int col = 16 * t + r;
          if (col >= N) continue;
          const float bb = bias ? bias[col] : 0.f;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int64_t row = wt0 + 4 * q + v;
            if (row < n) out[row * N + col] = acc[m][t][v] * unscale + bb;
          }
        }
      }
    }
  }
}

#define DCTAE_LFQP_PARAMS                                                                                         \
  const float *__restrict__ x, const int64_t *__restrict__ idx_in, int64_t n, int K, int N, const float *__restrict__ w, \
      const float *__restrict__ bias, int cd, int ncb, float scale, int64_t *__restrict__ idx_out,                    \
      float *__restrict__ out, uint16_t *__restrict__ idx16, InvNorm inv, const uint16_t *__restrict__ wsp, int Kp,     \
      float a_scale, const int *__restrict__ w_exp
#define DCTAE_LFQP_ARGS x, idx_in, n, K, N, w, bias, cd, ncb, scale, idx_out, out, idx16, inv, wsp, Kp, a_scale, w_exp

template <int NT, int MODE, int WB, bool A1>
__global__ __launch_bounds__(64 * WB) void k_lfq_proj(DCTAE_LFQP_PARAMS) {
  lfq_proj_body<NT, MODE, WB, A1, false>(DCTAE_LFQP_ARGS);
}

// the fp16 form at 4 waves per SIMD (two 512-thread blocks per CU): its
// projection-out body compiled to 130 VGPRs, one block per CU, 1.5x slower
template <int NT, int MODE, int WB, bool A1>
__global__ __launch_bounds__(64 * WB) __attribute__((amdgpu_waves_per_eu(4))) void k_lfq_proj_h2(DCTAE_LFQP_PARAMS) {
  lfq_proj_body<NT, MODE, WB, A1, true>(DCTAE_LFQP_ARGS);
}

// W (N x K fp32, row-major) -> three bf16 planes [3][NP][Kp], zero padded
// (rows N .. NP, k K .. Kp): the same round-to-nearest-even split as split8
__global__ void k_split_w(const float* __restrict__ w, int N, int K, int NP, int Kp, uint16_t* __restrict__ ws) {
  const int64_t plane = (int64_t)NP * Kp;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < plane; e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / Kp), k = (int)(e - (int64_t)row * Kp);
    const float v = row < N && k < K ? w[(int64_t)row * K + k] : 0.f;
    const __bf16 h0 = (__bf16)v;
    const float r1 = v - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;
    ws[e] = __builtin_bit_cast(uint16_t, h0);
    ws[plane + e] = __builtin_bit_cast(uint16_t, h1);
    ws[2 * plane + e] = __builtin_bit_cast(uint16_t, (__bf16)r2);
  }
}

// W (N x K fp32) -> two fp16 planes [2][NP][Kp] of W 2^e, e from |max W| so
// the largest piece lies in [2^13, 2^14) (0 for an all-zero or non-finite W),
// e stored after the planes: one 1024-thread block (N x K <= 256 x 256)
__global__ __launch_bounds__(1024) void k_split_w_h2(const float* __restrict__ w, int N, int K, int NP, int Kp,
                                                     uint16_t* __restrict__ ws) {
  __shared__ uint32_t part[16];
  __shared__ int ex;
  uint32_t m = 0;
  for (int e = threadIdx.x; e < N * K; e += 1024) m = max(m, __float_as_uint(w[e]) & 0x7fffffffu);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 16; ++i) m = max(m, part[i]);
    int e = 0;
    if (m != 0u && m < 0x7f800000u) {
      frexpf(__uint_as_float(m), &e);
      e = 14 - e;
    }
    ex = e;
  }
  __syncthreads();
  const float sc = ldexpf(1.0f, ex);
  const int64_t plane = (int64_t)NP * Kp;
  for (int64_t e = threadIdx.x; e < plane; e += 1024) {
    const int row = (int)(e / Kp), k = (int)(e - (int64_t)row * Kp);
    const float v = (row < N && k < K ? w[(int64_t)row * K + k] : 0.f) * sc;
    const _Float16 h0 = (_Float16)v;
    ws[e] = __builtin_bit_cast(uint16_t, h0);
    ws[plane + e] = __builtin_bit_cast(uint16_t, (_Float16)(v - (float)h0));
  }
  if (threadIdx.x == 0) *reinterpret_cast<int*>(ws + 2 * plane) = ex;
}

template <int MODE, int WB, bool A1, bool H2>
void launch_nt(int nt, dim3 g, hipStream_t s, const float* x, const int64_t* idx_in, int64_t n, int K, int N,
               const float* w, const float* b, int cd, int ncb, float scale, int64_t* idx_out, float* out,
               uint16_t* idx16, InvNorm inv, const uint16_t* wsp, int Kp, float a_scale, const int* w_exp) {
#define DCTAE_LFQP(T) \
  case T: if (H2) hipLaunchKernelGGL((k_lfq_proj_h2<T, MODE, WB, A1>), g, dim3(64 * WB), 0, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv, wsp, Kp, a_scale, w_exp); \
          else hipLaunchKernelGGL((k_lfq_proj<T, MODE, WB, A1>), g, dim3(64 * WB), 0, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv, wsp, Kp, a_scale, w_exp); break;
  switch (nt) {
    DCTAE_LFQP(1) DCTAE_LFQP(2) DCTAE_LFQP(3) DCTAE_LFQP(4) DCTAE_LFQP(5) DCTAE_LFQP(6) DCTAE_LFQP(7)
    DCTAE_LFQP(8) DCTAE_LFQP(9) DCTAE_LFQP(10) DCTAE_LFQP(11) DCTAE_LFQP(12) DCTAE_LFQP(13)
    DCTAE_LFQP(14) DCTAE_LFQP(15) DCTAE_LFQP(16)
    default: break;
  }
#undef DCTAE_LFQP
}

}  // namespace

size_t lfq_proj_scratch_bytes(int N, int K) {
  const size_t NP = (size_t)(N + 15) / 16 * 16, Kp = (size_t)(K + 31) / 32 * 32;
  return 3 * NP * Kp * sizeof(uint16_t);
}

// fp16 form (H2) for mode 0 when the caller bounds |x| (a_bound > 0, e.g.
// the PatchNorm clamp of the fused encode), for mode 1 when +-scale is exact
// in fp16; otherwise the split-bf16 form
template <int MODE>
static void launch_mode(int nt, hipStream_t s, const float* x, const int64_t* idx_in, int64_t n, int K, int N,
                        const float* w, const float* b, int cd, int ncb, float scale, int64_t* idx_out, float* out,
                        uint16_t* wsp, uint16_t* idx16 = nullptr, InvNorm inv = InvNorm{}, float a_bound = 0.f,
                        bool ws = false) {
  const int NP = nt * 16, Kp = (K + 31) / 32 * 32;
  const dim3 g((unsigned)((n + 127) / 128));
  bool h2 = false;
  float a_scale = 1.0f;
  if (MODE == 0 && a_bound > 0.0f && std::isfinite(a_bound)) {
    int e;
    std::frexp(a_bound, &e);
    a_scale = std::ldexp(1.0f, 14 - e);
    h2 = true;
  }
  if (MODE == 1 && a_bound > 0.0f) {   // a_bound: the caller allows the fp16 form
    const float sh = (float)(_Float16)scale;
    h2 = sh == scale && std::fabs(scale) >= 6.103515625e-05f && std::fabs(scale) <= 16384.0f;
  }
  if (h2 && ws && lfq_ws_fits(MODE, K, N, cd, ncb)) {   // the W-stationary kernel (dctae_lfq_ws.hip)
    const int NPw = (N + 31) / 32 * 32;
    hipLaunchKernelGGL(k_split_w_h2, dim3(1), dim3(1024), 0, s, w, N, K, NPw, Kp, wsp);
    launch_lfq_ws(MODE, s, x, idx_in, n, K, N, b, cd, ncb, scale, idx_out, out, idx16, inv.ch, inv.pos, inv.med, inv.b,
                  inv.eps, inv.maxph, inv.maxpw, inv.err, wsp, NPw, Kp, MODE == 0 ? a_scale : 1.0f);
    return;
  }
  if (h2) {
    const int* w_exp = reinterpret_cast<const int*>(wsp + 2 * (size_t)NP * Kp);
    hipLaunchKernelGGL(k_split_w_h2, dim3(1), dim3(1024), 0, s, w, N, K, NP, Kp, wsp);
    if constexpr (MODE == 1)
      launch_nt<MODE, 8, true, true>(nt, g, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv, wsp,
                                     Kp, 1.0f, w_exp);
    else
      launch_nt<MODE, 8, false, true>(nt, g, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv,
                                      wsp, Kp, a_scale, w_exp);
    return;
  }
  // W pre-split once per call (a few microseconds: N x K <= 256 x 256)
  hipLaunchKernelGGL(k_split_w, dim3((NP * Kp + 255) / 256), dim3(256), 0, s, w, N, K, NP, Kp, wsp);
  // 8 waves x 16 tokens per block (the W chunk in LDS shared by 128 tokens).
  // Measured with the fp32 MFMA (v_mfma_f32_16x16x4_f32) on 3,145,728 tokens
  // (196 -> 208): project_in 2.45 ms / project_out 2.80 ms; 4 waves per block
  // 2.73 / 3.05; 16 waves 2.51 / 3.23; 32 tokens per wave 3.91 / 5.37.  Now on
  // the split bf16 MFMA.
  // Mode 1's A (+-scale) is exact in bf16 when scale is: one A piece
  uint32_t sb;
  memcpy(&sb, &scale, 4);
  if constexpr (MODE == 1) {
    if ((sb & 0xffffu) == 0) {
      launch_nt<MODE, 8, true, false>(nt, g, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv, wsp,
                                      Kp, 1.0f, nullptr);
      return;
    }
  }
  launch_nt<MODE, 8, false, false>(nt, g, s, x, idx_in, n, K, N, w, b, cd, ncb, scale, idx_out, out, idx16, inv, wsp,
                                   Kp, 1.0f, nullptr);
}

// x (n, D) fp32, w_in (ncb cd, D), b_in (ncb cd) or null -> indices (n, ncb)
// x_bound > 0: |x| <= x_bound (NaN aside), the fp16 forms
void launch_lfq_project_in(const float* x, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                           float scale, int64_t* idx, uint16_t* wsp, hipStream_t s, float x_bound, bool ws) {
  if (n <= 0) return;
  launch_mode<0>((cd * ncb + 15) / 16, s, x, nullptr, n, D, cd * ncb, w, b, cd, ncb, scale, idx, nullptr, wsp, nullptr,
                 InvNorm{}, x_bound, ws);
}

// the same into the encode's u16 token staging (cd <= 16)
// x_bound > 0: |x| <= x_bound (NaN aside), the fp16 form
void launch_lfq_project_in16(const float* x, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                             uint16_t* idx, uint16_t* wsp, hipStream_t s, float x_bound, bool ws) {
  if (n <= 0) return;
  launch_mode<0>((cd * ncb + 15) / 16, s, x, nullptr, n, D, cd * ncb, w, b, cd, ncb, 0.f, nullptr, nullptr, wsp, idx,
                 InvNorm{}, x_bound, ws);
}

// indices (n, ncb) -> codes (+-scale, n x ncb cd) -> out (n, D) = codes w_out^T + b_out; w_out (D, ncb cd)
void launch_lfq_project_out(const int64_t* idx, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                            float scale, float* out, uint16_t* wsp, hipStream_t s, const int64_t* ch, const int64_t* pos,
                            const float* med, const float* nb, float eps, int maxph, int maxpw, int* err, bool h2,
                            bool ws) {
  if (n <= 0) return;
  launch_mode<1>((D + 15) / 16, s, nullptr, idx, n, cd * ncb, D, w, b, cd, ncb, scale, nullptr, out, wsp, nullptr,
                 InvNorm{ch, pos, med, nb, eps, maxph, maxpw, err}, h2 ? 1.0f : 0.0f, ws);
}

}  // namespace dctae
