// W-stationary LFQ projections for the conf/patch14-l.json shapes (lfq.py:54-62:
// project_in 196 -> 16 x 13 = 208 fused with sign + index packing, lfq.py:164,
// :175-187; indices -> +-scale codes -> project_out 208 -> 196, lfq.py:105-127,
// optionally followed by the inverse PatchNorm, patchnorm.py:167-177).
//
// k_lfq_proj (dctae_lfq_proj.hip) stages a 32-k chunk of W in LDS for 128
// tokens and every wave reads all of it: per chunk 8 waves x 26 KB of W
// fragments out of LDS for 39 MFMAs each, the LDS port, not the MFMA pipe,
// sets its pace (1.38 ms for 3.1 M tokens).  Here each of the 7 waves of a
// block owns one 32-feature output tile and keeps that tile's W fragments in
// registers for the block's whole life (13 k steps x 2 fp16 planes x 8 halves
// = 104 VGPRs); only the tokens go through LDS (32 per tile, split once into
// fp16 planes and shared by the 7 waves).  One block per CU (the W registers
// allow no second), persistent over a contiguous run of 32-token tiles, the
// next tile's global loads in flight during the current tile's MFMAs, one
// barrier per tile.
//
// Arithmetic as k_lfq_proj_h2: A scaled by a power of two into the fp16
// range (mode 0: a_scale from the caller's bound |x| <= x_bound, two pieces;
// mode 1: +-scale exact in fp16, one piece), W scaled by 2^w_exp (k_split_w_h2,
// two pieces), the products of piece order <= 1 on v_mfma_f32_32x32x16_f16
// with fp32 accumulation, unscaled exactly before the bias.
#include "dctae_device.h"
#include "dctae_launch.h"



namespace dctae {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 hv8 __attribute__((ext_vector_type(8)));
typedef _Float16 hv4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kKS = 13;              // 16-k MFMA steps: 192 < K <= 208
constexpr int kNW = 7;               // waves = 32-feature output tiles: 192 < N <= 224
constexpr int kKp = 16 * kKS;        // k per LDS row
constexpr int kRow = kKp + 8;        // LDS row stride in halves (108 dwords: the 16 rows of a
                                     // b128 fragment read phase start on 16 distinct bank quads)
constexpr int kMw = 8;               // mask words per token (256 features)
constexpr int kK4 = 49;              // mode 0: float4 per token row (K = 196, conf/patch14-l.json's dim)

// mode 1's inverse-PatchNorm table pieces of a tile: 1 = loaded at the top of
// the tile's iteration (in flight during its MFMAs), 0 = after its staging
#ifndef DCTAE_LFQWS_TAB_EARLY
#define DCTAE_LFQWS_TAB_EARLY 1
#endif

struct WsInv {
  const int64_t* ch;    // (n) channels of the tokens, or null: no inverse
  const int64_t* pos;   // (n, 2)
  const float* med;     // (3, maxph, maxpw, N)
  const float* b;
  float eps;
  int maxph, maxpw;
  int* err;             // bit 1: a table index out of range (the reference raises IndexError)
};

// at most 256 registers per wave: two waves per SIMD (mode 0's 7-wave block;
// mode 1's two 4-wave blocks per CU)
template <int MODE, int MT, int NWB>
__global__ __launch_bounds__(64 * NWB) __attribute__((amdgpu_waves_per_eu(2))) void k_lfq_ws(const float* __restrict__ x, const int64_t* __restrict__ idx_in,
                                                 int64_t n, int K, int N, const float* __restrict__ bias, int cd,
                                                 int ncb, float scale, int64_t* __restrict__ idx_out,
                                                 float* __restrict__ out, uint16_t* __restrict__ idx16, WsInv inv,
                                                 const uint16_t* __restrict__ wsp, int NPw, int Kp, float a_scale,
                                                 int64_t tiles_per_block) {
  constexpr int kThr = 64 * NWB;           // NWB waves = output tiles per block
  constexpr int NSPLIT = (kNW + NWB - 1) / NWB;   // blocks sharing a token range, one output slice each
  constexpr int kYsB = 32 * NWB + 8;       // mode 1's output tile row stride (4 x stride = 32 mod 64 banks)
  static_assert(MODE == 1 || NSPLIT == 1, "project_in needs every feature of a token in one block");
  constexpr int TOK = 32 * MT;             // tokens per tile: MT 32-row M blocks
  constexpr int NPA = MODE == 0 ? 2 : 1;   // A pieces
  constexpr int SU0 = TOK * kK4 / kThr;                    // mode 0: float4 units per thread
  static_assert(MODE == 1 || TOK * kK4 % kThr == 0, "mode 0: whole float4 units per thread");
  constexpr int SU1 = (TOK * kKp / 8 + kThr - 1) / kThr;   // mode 1: 8-k units per thread
  constexpr int U1 = (TOK * 32 * NWB / 4 + kThr - 1) / kThr;   // mode 1: float4 output units per thread
  __shared__ __attribute__((aligned(16))) _Float16 As[2][NPA][TOK * kRow];
  __shared__ uint32_t Msk[MODE == 0 ? 2 * TOK * kMw : 1];   // sign bits [buf][token][32-feature word]
  __shared__ int64_t Tb[MODE == 1 ? 2 * TOK : 1];           // inverse PatchNorm table rows [buf][token]
  // mode 1: the tile's outputs [buf][token][kYs], re-read as float4 along each token's N floats
  __shared__ __attribute__((aligned(16))) float Ys[MODE == 1 ? 2 * TOK * kYsB : 1];
  __shared__ hv8 Lut[MODE == 1 ? 256 : 1];   // mode 1: the 8 codes of each byte of index bits
  __shared__ int32_t Ix[MODE == 1 ? 2 * TOK * 32 : 1];   // mode 1: the tiles' indices [buf][token][codebook]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5;
  // NSPLIT > 1: blocks 2 i, 2 i + 1 (..) run the same tokens, block 2 i + q the
  // output tiles q NWB .. q NWB + NWB - 1 (two blocks per CU: each one's waits
  // overlap the other's MFMAs)
  const int slice = NSPLIT > 1 ? (int)(blockIdx.x % NSPLIT) : 0;
  const int tw = slice * NWB + wave;           // this wave's 32-feature output tile
  const bool mf = 32 * tw < N;                 // wave-uniform: a tile past N does no MFMA
  const int fbase = 32 * NWB * slice;          // the block's first output feature
  const int64_t ntiles = (n + TOK - 1) / TOK;
  const int64_t t0 = (int64_t)(NSPLIT > 1 ? blockIdx.x / NSPLIT : blockIdx.x) * tiles_per_block;
  const int64_t t1 = t0 + tiles_per_block < ntiles ? t0 + tiles_per_block : ntiles;
  if (t0 >= t1) return;   // whole block

  // zero both A buffers (the k >= K tail stays zero) and the mask words
  for (int e = tid; e < 2 * NPA * TOK * kRow / 8; e += kThr)
    reinterpret_cast<f32x4v*>(&As[0][0][0])[e] = f32x4v{0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 0)
    for (int e = tid; e < 2 * TOK * kMw; e += kThr) Msk[e] = 0u;

  // this wave's W fragments: row 32 wave + l32 of the [2][NPw][Kp] fp16 planes,
  // k 16 s + 8 half .. + 7 (the B operand layout of v_mfma_f32_32x32x16_f16)
  const int* w_exp = reinterpret_cast<const int*>(wsp + 2 * (size_t)NPw * Kp);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(wsp), 0, 2 * NPw * Kp * 2, 0x00020000);
  hv8 wb[2][kKS];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int s = 0; s < kKS; ++s)
      wb[p][s] = __builtin_bit_cast(
          hv8, __builtin_amdgcn_raw_buffer_load_b128(wrs, ((32 * tw + l32) * Kp + 16 * s + 8 * half) * 2 + p * NPw * Kp * 2,
                                                     0, 0));
  const float unscale = ldexpf(1.0f / a_scale, -w_exp[0]);
  const int col = 32 * tw + l32;   // this lane's output feature
  const float bb = (bias && col < N) ? bias[col] : 0.f;
  // mode 0: h = acc unscale + bb > 0  <=>  acc > -bb / unscale (unscale a power
  // of two: the product and the quotient are exact); +inf past N: never set
  const float thr = col < N ? -bb / unscale : __int_as_float(0x7f800000);
  // mode 0: the (token, codebook) pairs p = tid + kThr j this thread assembles
  // each tile: token, mask word offset and shift are tile-invariant
  constexpr int NPJ = MODE == 0 ? (TOK * 32 + kThr - 1) / kThr : 1;   // ncb <= 32
  int pi[NPJ], pw[NPJ], psh[NPJ];
  const uint32_t cmask = cd >= 32 ? ~0u : (1u << cd) - 1u;
  if constexpr (MODE == 0) {
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int p = tid + kThr * j, i = p / ncb, o0 = (p - i * ncb) * cd;
      pi[j] = i;
      pw[j] = i * kMw + (o0 >> 5);
      psh[j] = o0 & 31;
    }
  }

  // staging, one tile ahead: mode 0 the tile's TOK token rows of fp32 (one
  // contiguous TOK K floats run) as float4 units, mode 1 the int64 indices of
  // the codebooks an 8-k unit touches.  Loads are unconditional (pieces past
  // the tile or past n re-read the last valid one and are zeroed at the
  // store): no VALU write to a register with a load in flight, no control
  // flow around the issue, so the wait before the store is exact
  f32x4v ra[MODE == 0 ? SU0 : 1];
  // mode 1: the tile's TOK x ncb int64 indices are one contiguous run; their low
  // dwords (lfq.py:117 indices.int()) go through registers (two tiles ahead)
  // into the LDS index buffers Ix (one tile ahead), where the staging reads them
  constexpr int RX = (TOK * 32 + kThr - 1) / kThr;   // ncb <= 32
  int32_t rx[MODE == 1 ? RX : 1];
  // mode 1: unit (row, k0 .. k0 + 7)'s codebooks c0 = k0 / cd, c1 and the shift of
  // its 8 bits in (i0 << cd | i1): k0 / cd = (k0 rc) >> 16 with rc = ceil(2^16 / cd)
  // (exact for k0 < 2^10), the rest from it
  const uint32_t rc = (65536u + (uint32_t)cd - 1u) / (uint32_t)cd;
  auto unit_cb = [&](int k0, int& c0, int& c1, int& sh) {
    c0 = (int)(((uint32_t)k0 * rc) >> 16);
    c1 = min((int)(((uint32_t)(k0 + 7) * rc) >> 16), ncb - 1);
    sh = 2 * cd - 8 - (k0 - c0 * cd);
  };
  if constexpr (MODE == 1) {
    // +-scale of the 8 bits of a byte, MSB first (lfq.py:117-124)
    for (int e = tid; e < 256; e += kThr) {
      hv8 v;
#pragma unroll
      for (int b = 0; b < 8; ++b) v[b] = (_Float16)(((e >> (7 - b)) & 1) ? scale : -scale);
      Lut[e] = v;
    }
  }
  auto load = [&](int64_t t) {
    if constexpr (MODE == 0) {
      const f32x4v* xt = reinterpret_cast<const f32x4v*>(x) + t * TOK * kK4;   // the tile's contiguous run
      if ((t + 1) * TOK <= n) {
#pragma unroll
        for (int i = 0; i < SU0; ++i) ra[i] = __builtin_nontemporal_load(xt + tid + kThr * i);
      } else {   // the last tile (or past t1): re-read the last valid piece
        const int64_t last = n * kK4 - 1 - t * TOK * kK4;
#pragma unroll
        for (int i = 0; i < SU0; ++i) {
          const int64_t u = tid + kThr * i;
          ra[i] = __builtin_nontemporal_load(xt + (u < last ? u : last));
        }
      }
    } else {
      const int64_t last = n * ncb - 1;   // unconditional, clamped (past n: unused)
#pragma unroll
      for (int i = 0; i < RX; ++i) {
        const int64_t f = t * TOK * ncb + tid + kThr * i;
        rx[i] = reinterpret_cast<const int32_t*>(idx_in)[2 * (f < last ? f : last)];
      }
    }
  };
  auto put_idx = [&](int b) {   // mode 1: the loaded indices -> Ix[b]
#pragma unroll
    for (int i = 0; i < RX; ++i)
      if (tid + kThr * i < TOK * ncb) Ix[b * TOK * 32 + tid + kThr * i] = rx[i];
  };
  auto store = [&](int64_t t, int buf) {
    const int64_t tok0 = t * TOK;
    if constexpr (MODE == 0) {
      const bool full = tok0 + TOK <= n;
#pragma unroll
      for (int i = 0; i < SU0; ++i) {
        const int u = tid + kThr * i;
        const int row = u / kK4, k4 = u - row * kK4;
        f32x4v v = ra[i] * a_scale;
        if (!full && tok0 + row >= n) v = f32x4v{0.f, 0.f, 0.f, 0.f};
        const hv4 h = __builtin_convertvector(v, hv4);
        const hv4 l = __builtin_convertvector(v - __builtin_convertvector(h, f32x4v), hv4);
        *reinterpret_cast<hv4*>(&As[buf][0][row * kRow + 4 * k4]) = h;
        *reinterpret_cast<hv4*>(&As[buf][NPA - 1][row * kRow + 4 * k4]) = l;
      }
    } else {
#pragma unroll 1
      for (int i = 0; i < SU1; ++i) {
        const int u = tid + kThr * i;
        if (u < TOK * (kKp / 8)) {
          const int row = u / (kKp / 8), k0 = 8 * (u - row * (kKp / 8));
          const bool live = tok0 + row < n;
          int c0, c1, sh;
          unit_cb(min(k0, K - 1), c0, c1, sh);
          const int i0 = Ix[buf * TOK * 32 + row * ncb + c0], i1 = Ix[buf * TOK * 32 + row * ncb + c1];
          hv8 a;
          if (live && k0 + 8 <= K) {
            // the unit's 8 code bits (MSB first, lfq.py:117-124 mask 2^(cd-1..0))
            // out of codebooks c0 / c1's low cd bits, then one LUT read
            const uint32_t cm = (1u << cd) - 1u;
            const uint32_t comb = ((uint32_t)i0 & cm) << cd | ((uint32_t)i1 & cm);
            a = Lut[(comb >> sh) & 0xffu];
          } else {
            const int c0 = k0 / cd;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int k = k0 + e, c = k / cd, b = k - c * cd;
              const int id = c == c0 ? i0 : i1;
              const bool bit = (id >> (cd - 1 - b)) & 1;
              a[e] = (_Float16)(live && k < K ? (bit ? scale : -scale) : 0.f);   // lfq.py:117-124
            }
          }
          *reinterpret_cast<hv8*>(&As[buf][0][row * kRow + k0]) = a;
        }
      }
      if (inv.ch && tid < TOK) {
        const int64_t row = tok0 + tid;
        int64_t tb = -2;   // -2: past n, -1: out-of-range table index
        if (row < n) {
          const int64_t c = inv.ch[row], h = inv.pos[2 * row], w = inv.pos[2 * row + 1];
          const bool ok = c >= 0 && c < 3 && h >= 0 && h < inv.maxph && w >= 0 && w < inv.maxpw;
          if (!ok) atomicOr(inv.err, 1);
          tb = ok ? ((c * inv.maxph + h) * inv.maxpw + w) * N : -1;
        }
        Tb[buf * TOK + tid] = tb;
      }
    }
  };

  __syncthreads();   // the zero fill before the first tile's stores
  load(t0);
  if constexpr (MODE == 1) {
    put_idx(0);
    load(t0 + 1);
    __syncthreads();   // Ix[0]
  }
  store(t0, 0);
  if constexpr (MODE == 1) put_idx(1);
  __syncthreads();
  const int N4 = (N - fbase < 32 * NWB ? N - fbase : 32 * NWB) >> 2;   // the block's float4 outputs per token
  for (int64_t t = t0; t < t1; ++t) {
    const int buf = (int)((t - t0) & 1);
    const int64_t tok0 = t * TOK;
    load(MODE == 1 ? t + 2 : t + 1);   // past t1: clamped, unused
    f32x4v tm[MODE == 1 ? U1 : 1], tbv[MODE == 1 ? U1 : 1];
#if DCTAE_LFQWS_TAB_EARLY
    // mode 1: this tile's table pieces (Tb[buf]: staged last iteration), in
    // flight during the MFMAs and the next tile's staging
    if (MODE == 1 && inv.ch) {
#pragma unroll
      for (int i = 0; i < U1; ++i) {
        const int u = tid + kThr * i, row = u / N4, c4 = u - row * N4;
        const int64_t tb = u < TOK * N4 ? Tb[buf * TOK + row] : -2;
        const int64_t o = tb >= 0 ? tb + fbase + 4 * c4 : 0;   // unconditional loads
        tm[i] = *reinterpret_cast<const f32x4v*>(inv.med + o);
        tbv[i] = *reinterpret_cast<const f32x4v*>(inv.b + o);
      }
    }
#endif
    floatx16 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[m][v] = 0.f;
#pragma unroll
    for (int s = 0; s < kKS; ++s) {
      if (!mf) break;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const _Float16* ap = &As[buf][0][(32 * m + l32) * kRow + 8 * half + 16 * s];
        const hv8 a0 = *reinterpret_cast<const hv8*>(ap);
        if constexpr (MODE == 0) {
          const hv8 a1 = *reinterpret_cast<const hv8*>(ap + TOK * kRow);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, wb[0][s], acc[m], 0, 0, 0);
        }
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[1][s], acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[0][s], acc[m], 0, 0, 0);
      }
    }
    // mode 1: keep the next tile's staging out of the MFMA chain's registers
    if constexpr (MODE == 1) __builtin_amdgcn_sched_barrier(0);
    // C/D map: feature = col (lane & 31), token row = 32 m + (v & 3) + 8 (v >> 2) + 4 half
    if constexpr (MODE == 0) {
      // ballot v = rows (v & 3) + 8 (v >> 2) (bits 0-31) and + 4 (bits 32-63) of
      // this wave's 32 features; lane v collects both words, lanes 0-15 store
      uint32_t* msk = Msk + buf * TOK * kMw;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        // (v_cndmask on the ballot's SGPRs: the compiler inserts the wait states
        // a VALU read of a VALU-written SGPR needs; an inline-asm v_writelane
        // right behind the v_cmp read stale SGPRs -- wrong words for most rows)
        uint32_t wlo = 0, whi = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const uint64_t mk = __ballot(acc[m][v] > thr);   // h > 0, lfq.py:175 (NaN -> False)
          const bool mine = lane == v;
          wlo = mine ? (uint32_t)mk : wlo;
          whi = mine ? (uint32_t)(mk >> 32) : whi;
        }
        if (lane < 16) {
          const int row = 32 * m + (lane & 3) + 8 * (lane >> 2);
          msk[row * kMw + wave] = wlo;
          msk[(row + 4) * kMw + wave] = whi;
        }
      }
    } else {
      float* ys = Ys + buf * TOK * kYsB;
      if (col < N) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int v = 0; v < 16; ++v)
            ys[(32 * m + (v & 3) + 8 * (v >> 2) + 4 * half) * kYsB + col - fbase] = acc[m][v] * unscale + bb;
      }
    }
    if (t + 1 < t1) store(t + 1, buf ^ 1);
    if constexpr (MODE == 1) {
      put_idx(buf);   // Ix[buf] held tile t's indices, read by the staging before the last barrier
      // this tile's table pieces, in flight during the barrier
      if (!DCTAE_LFQWS_TAB_EARLY && inv.ch) {
#pragma unroll
        for (int i = 0; i < U1; ++i) {
          const int u = tid + kThr * i, row = u / N4, c4 = u - row * N4;
          const int64_t tb = u < TOK * N4 ? Tb[buf * TOK + row] : -2;
          tm[i] = tbv[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
          if (tb >= 0) {
            tm[i] = *reinterpret_cast<const f32x4v*>(inv.med + tb + fbase + 4 * c4);
            tbv[i] = *reinterpret_cast<const f32x4v*>(inv.b + tb + fbase + 4 * c4);
          }
        }
      }
    }
    __syncthreads();
    if constexpr (MODE == 0) {
      // (token i, codebook c) pairs of the tile, token-major: contiguous stores
      const uint32_t* msk = Msk + buf * TOK * kMw;
#pragma unroll
      for (int j = 0; j < NPJ; ++j) {
        const int p = tid + kThr * j;
        if (p >= TOK * ncb || tok0 + pi[j] >= n) break;
        const uint64_t win = (uint64_t)msk[pw[j]] | ((uint64_t)msk[pw[j] + 1] << 32);
        const uint32_t bits = (uint32_t)(win >> psh[j]) & cmask;   // bit b = feature c cd + b
        const uint32_t code = __builtin_bitreverse32(bits) >> (32 - cd);
        if (idx16)
          idx16[tok0 * ncb + p] = (uint16_t)code;   // encode staging (cd <= 16), gathered by k_sort_pack2
        else   // lfq.py:187: the bit of the quantized value
          idx_out[tok0 * ncb + p] = (int64_t)lfq_index_bits(code, scale > 0.0f ? ~0ull : 0ull,
                                                            -scale > 0.0f ? ~0ull : 0ull) & ((1ll << cd) - 1);
      }
    } else {
      // outputs as float4 pieces along each token's N floats, the inverse
      // PatchNorm on the prefetched table pieces (same fp32 ops as dctae_norm_inverse)
      const float* ys = Ys + buf * TOK * kYsB;
#pragma unroll
      for (int i = 0; i < U1; ++i) {
        const int u = tid + kThr * i, row = u / N4, c4 = u - row * N4;
        if (u >= TOK * N4 || tok0 + row >= n) continue;
        f32x4v y = *reinterpret_cast<const f32x4v*>(ys + row * kYsB + 4 * c4);
        if (inv.ch) {
          const int64_t tb = Tb[buf * TOK + row];
          if (tb >= 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = pn_inverse(y[e], tm[i][e], tbv[i][e], inv.eps);
          } else {
            y = f32x4v{1.f, 1.f, 1.f, 1.f} * __int_as_float(0x7fc00000);
          }
        }
        __builtin_nontemporal_store(y, reinterpret_cast<f32x4v*>(out + (tok0 + row) * N + fbase) + c4);
      }
    }
  }
}

#ifndef DCTAE_LFQWS_OUT_NWB
#define DCTAE_LFQWS_OUT_NWB 4   // project_out: waves per block (4: two blocks per token range; 7: one)
#endif

int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

}  // namespace

bool lfq_ws_fits(int mode, int K, int N, int cd, int ncb) {
  const bool k_ok = mode == 0 ? K == 4 * kK4 : (K > 16 * (kKS - 1) && K <= kKp);
  const bool n_ok = N > 32 * (kNW - 1) && N <= 32 * kNW;
  // mode 1: an 8-k unit touches at most two codebooks (cd >= 8) whose low cd
  // bits are combined in 32 bits (cd <= 16); mode 0: u16 codes
  const bool cd_ok = cd <= 16 && (mode == 1 ? cd >= 8 : cd >= 1);
  return k_ok && n_ok && cd_ok && ncb >= 1 && (int64_t)cd * ncb == (mode == 0 ? N : K);
}

void launch_lfq_ws(int mode, hipStream_t s, const float* x, const int64_t* idx_in, int64_t n, int K, int N,
                   const float* bias, int cd, int ncb, float scale, int64_t* idx_out, float* out, uint16_t* idx16,
                   const int64_t* ch, const int64_t* pos, const float* med, const float* nb, float eps, int maxph,
                   int maxpw, int* err, const uint16_t* wsp, int NPw, int Kp, float a_scale) {
  // mode 0: 64-token tiles (two 32-row MFMA chains per wave), 7-wave blocks,
  // one per CU; mode 1: 32-token tiles, the 7 output tiles split over two
  // 4-wave blocks per token range, two blocks per CU
  const int tok = mode == 0 ? 64 : 32;
  const int64_t ntiles = (n + tok - 1) / tok;
  if (ntiles <= 0) return;
  const int64_t nb_ = ntiles < cu_count() ? ntiles : cu_count();
  const int64_t per = (ntiles + nb_ - 1) / nb_;
  const int64_t ranges = (ntiles + per - 1) / per;
  const WsInv inv{ch, pos, med, nb, eps, maxph, maxpw, err};
  if (mode == 0)
    hipLaunchKernelGGL((k_lfq_ws<0, 2, kNW>), dim3((unsigned)ranges), dim3(64 * kNW), 0, s, x, idx_in, n, K, N, bias,
                       cd, ncb, scale, idx_out, out, idx16, inv, wsp, NPw, Kp, a_scale, per);
  else if (DCTAE_LFQWS_OUT_NWB == kNW)
    hipLaunchKernelGGL((k_lfq_ws<1, 1, kNW>), dim3((unsigned)ranges), dim3(64 * kNW), 0, s, x, idx_in, n, K, N, bias,
                       cd, ncb, scale, idx_out, out, idx16, inv, wsp, NPw, Kp, a_scale, per);
  else
    hipLaunchKernelGGL((k_lfq_ws<1, 1, 4>), dim3((unsigned)(2 * ranges)), dim3(256), 0, s, x, idx_in, n, K, N, bias,
                       cd, ncb, scale, idx_out, out, idx16, inv, wsp, NPw, Kp, a_scale, per);
}

}  // namespace dctae
