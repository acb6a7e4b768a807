// Device pieces of the 512-point column kernel k_fft_cols7 (dctae_fft2.hip):
// T slice loads, the pass-2 butterfly map, LFQ thresholds and the token
// epilogue.
#pragma once
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_rows512.h"

namespace dctae {

// threadIdx.x through a volatile asm: not loop-invariant to the compiler, so
// the lane-derived LDS addresses of an item body are rebuilt per item instead
// of being hoisted out of a multi-image loop (and kept live in VGPRs)
__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

// ---------------------------------------------------------------------------
// Column pieces of N = 512 (P = 14) used by k_fft_cols7: the LFQ thresholds of
// a thread's epilogue rows and the token epilogue.
// ---------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

// Thresholds of this thread's epilogue rows: tiles h = g16 + 16 r, row jl;
// sbias (nullable): the score's -(h + strip) / ci[c] per tile row h (FE:411-416)
template <bool THR>
__device__ __forceinline__ void cols_thresholds(const ImgDesc& d, int c, int strip, const EncParams& ep,
                                                 float2 (&thr_r)[2][7], float* sbias) {
  constexpr int KS = 14, EPR = 2;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = tid & 15;
#if defined(DCTAE_PROFILING) && defined(DCTAE_C7_ABL)
  if (DCTAE_C7_ABL & 4) {   // profiling ablation: constant thresholds, no table loads (wrong codes)
#pragma unroll
    for (int r = 0; r < EPR; ++r)
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) thr_r[r][p] = make_float2(0.001f * (p + r), -0.002f * (p + jl));
    if (sbias && tid < 32) sbias[tid] = 0.0f;
    return;
  }
#endif
  if (THR) {
    const int jlc = min(jl, KS - 1);   // lanes 14 / 15 hold row 13's thresholds (cols512b_epilogue)
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int h = g16 + 16 * r;
      if (h < d.qh) {
        const float2* t2 = reinterpret_cast<const float2*>(
            ep.thr + ((((int64_t)c * ep.maxph + h) * ep.maxpw) + strip) * (KS * KS) + (int64_t)jlc * KS);
#pragma unroll
        for (int p = 0; p < KS / 2; ++p) thr_r[r][p] = t2[p];
      }
    }
  }
  if (THR && sbias && tid < 32) sbias[tid] = __fdiv_rn(-(float)(tid + strip), ep.ci[c]);
}

// staging index of tile (h, strip) of channel c: flat (h, strip, c) or
// item-major (c, strip, h) order (stage_pos, dctae_internal.h)
__device__ __forceinline__ int64_t cols_tok(const ImgDesc& d, int c, int strip, int h, int C) {
  return d.tok_off + ((d.tband & 2) ? (c * d.qw + strip) * d.qh + h : (h * d.qw + strip) * C + c);
}

// token outputs (raw DCT / PatchNorm) leave through LDS: tile h's 14 rows of
// 14 are the 196 contiguous floats Xf[196 h ..], the token's staged layout, so
// the whole block stores them as 16-byte pieces (49 per token) instead of 14
// scattered 4-byte stores per lane
#ifndef DCTAE_TOK_ST_NT
#define DCTAE_TOK_ST_NT 1
#endif
typedef float tok4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void cols_store_tokens(const ImgDesc& d, int c, int strip, const float* Xf, float* dst,
                                                  int C) {
  constexpr int KS = 14;
  for (int e = opaque_tid(); e < d.qh * 49; e += 256) {
    const int h = e / 49, q = e - h * 49;
    // write-once staging (the projection kernel reads it later, 196 floats a
    // token): nontemporal, as T'
#if DCTAE_TOK_ST_NT
    __builtin_nontemporal_store(reinterpret_cast<const tok4v*>(Xf + KS * KS * h)[q],
                                reinterpret_cast<tok4v*>(dst + cols_tok(d, c, strip, h, C) * (KS * KS)) + q);
#else
    reinterpret_cast<float4*>(dst + cols_tok(d, c, strip, h, C) * (KS * KS))[q] =
        reinterpret_cast<const float4*>(Xf + KS * KS * h)[q];
#endif
  }
}

// token epilogue of one (channel, tile column) item: X2 = the 448 x 14 kept
// coefficients (float index k * 14 + col) in LDS; tile (h, strip) per 16-lane
// group g16 (+16 r), tile row jl; codes from the thresholds held in registers;
// sb[r]: the score bias of tile row h = g16 + 16 r
template <bool THR>
__device__ __forceinline__ void cols_epilogue(const ImgDesc& d, int c, int strip, const f2v* X2, const float (&sb)[2],
                                               const float2 (&thr_r)[2][7], const EncParams& ep,
                                               const TokenSinks& sk) {
  constexpr int KS = 14, EPR = 2;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = tid & 15;
  auto tok_of = [&](int h) -> int64_t { return cols_tok(d, c, strip, h, ep.C); };
  float* Xf = reinterpret_cast<float*>(const_cast<f2v*>(X2));
  auto store_tokens = [&](float* dst) { cols_store_tokens(d, c, strip, Xf, dst, ep.C); };
  if (THR) {
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int h = g16 + 16 * r;
      if (h < d.qh) {
        const f2v* row = X2 + (KS * h + (jl < KS ? jl : 0)) * (KS / 2);
        uint32_t am = 0, code = 0;
#pragma unroll
        for (int p = 0; p < KS / 2; ++p) {
          const f2v v2 = row[p];
          am = max(am, max(__float_as_uint(v2.x) & 0x7fffffffu, __float_as_uint(v2.y) & 0x7fffffffu));
          // MSB-first (lfq.py:187): code = 2 code + bit (v_cmp + v_addc with the compare's carry)
          code = 2 * code + (v2.x >= thr_r[r][p].x ? 1u : 0u);
          code = 2 * code + (v2.y >= thr_r[r][p].y ? 1u : 0u);
        }
        am = jl < KS ? am : 0u;
        // max over the 16-lane row: DPP row rotations by 8, 4, 2, 1 (no LDS permutes)
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x128, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x124, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x122, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x121, 0xf, 0xf, false));
        const int64_t tok = tok_of(h);
        if (jl == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(__uint_as_float(am), ep.mw), sb[r]);
        if (jl < KS && sk.codes) sk.codes[tok * KS + jl] = (uint16_t)code;
      }
    }
    if (sk.raw) store_tokens(sk.raw);
  } else {
    const bool norm = sk.norm && ep.median;
    if (sk.raw) {
      store_tokens(sk.raw);
      if (norm) __syncthreads();   // raw reads before the in-place PatchNorm below
    }
    TokenSinks sc = sk;
    sc.raw = nullptr;
    sc.norm = nullptr;
    for (int h = g16; h < d.qh; h += 16) {
      float vals[KS];
      f2v* row = reinterpret_cast<f2v*>(Xf) + (KS * h + (jl < KS ? jl : 0)) * (KS / 2);
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) {
        const f2v v2 = row[p];
        vals[2 * p] = v2.x;
        vals[2 * p + 1] = v2.y;
      }
      const int64_t tok = tok_of(h);
      if (norm) {   // scores, codes and the PatchNorm values (patchnorm.py:157-165), written back in place
        float y[KS];
        token_epilogue_p<KS>(ep, c, h, strip, jl, vals, tok, sc, y);
        if (jl < KS) {
#pragma unroll
          for (int p = 0; p < KS / 2; ++p) row[p] = (f2v){y[2 * p], y[2 * p + 1]};
        }
      } else {
        token_epilogue_p<KS>(ep, c, h, strip, jl, vals, tok, sc);   // scores, codes
      }
    }
    if (norm) {
      __syncthreads();
      store_tokens(sk.norm);
    }
  }
}

// Threshold (codes-only) epilogue of k_cols512b: the same outputs as
// cols_epilogue<true> for its images (qh = qw = 32, so tiles h = g16 and
// g16 + 16 both exist) in about half the instructions:
//  * |x| max as a NaN-propagating v_maximum3_f32 (abs modifiers, two elements
//    per instruction; NaN scores as the reference's amax);
//  * each code bit is a v_cmp_ge_f32 into an SGPR pair plus a v_addc_co_u32
//    (code + code + carry): MSB first (lfq.py:187), two tile rows interleaved so
//    every carry read is >= 3 instructions after its compare (the VALU-SGPR
//    hazard) with no s_nop;
//  * lanes 14 / 15 repeat row 13 (its values and thresholds, cols_thresholds)
//    and store row 13's code and the row's score to the same addresses:
//    no divergent branches;
//  * stores through buffer descriptors on the item's first token: 32-bit lane
//    offsets, no 64-bit address math.
__device__ __forceinline__ void code_bits4(uint32_t& c0, uint32_t& c1, float& a0, float& a1, f2v x, f2v y,
                                           float2 tx, float2 ty) {
  uint64_t m0, m1, m2, m3;
  asm("v_cmp_ge_f32_e64 %[m0], %[x0], %[t0]\n\t"
      "v_cmp_ge_f32_e64 %[m1], %[x1], %[t1]\n\t"
      "v_cmp_ge_f32_e64 %[m2], %[y0], %[u0]\n\t"
      "v_cmp_ge_f32_e64 %[m3], %[y1], %[u1]\n\t"
      "v_maximum3_f32 %[a0], |%[x0]|, |%[x1]|, %[a0]\n\t"
      "v_maximum3_f32 %[a1], |%[y0]|, |%[y1]|, %[a1]\n\t"
      "v_addc_co_u32_e64 %[c0], %[m0], %[c0], %[c0], %[m0]\n\t"
      "v_addc_co_u32_e64 %[c0], %[m1], %[c0], %[c0], %[m1]\n\t"
      "v_addc_co_u32_e64 %[c1], %[m2], %[c1], %[c1], %[m2]\n\t"
      "v_addc_co_u32_e64 %[c1], %[m3], %[c1], %[c1], %[m3]"
      : [c0] "+v"(c0), [c1] "+v"(c1), [a0] "+v"(a0), [a1] "+v"(a1), [m0] "=&s"(m0), [m1] "=&s"(m1),
        [m2] "=&s"(m2), [m3] "=&s"(m3)
      : [x0] "v"(x.x), [x1] "v"(x.y), [y0] "v"(y.x), [y1] "v"(y.y), [t0] "v"(tx.x), [t1] "v"(tx.y),
        [u0] "v"(ty.x), [u1] "v"(ty.y));
}

__device__ __forceinline__ void cols512b_epilogue(const ImgDesc& d, int c, int strip, const f2v* X2,
                                                  const float (&sb)[2], const float2 (&thr_r)[2][7],
                                                  const EncParams& ep, const TokenSinks& sk) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = min(tid & 15, KS - 1);
  // token of tile h = tok0 + h * hs (cols_tok)
  const bool im = (d.tband & 2) != 0;
  const int64_t tok0 = d.tok_off + (im ? (int64_t)(c * d.qw + strip) * d.qh : (int64_t)strip * ep.C + c);
  const uint32_t hs = im ? 1u : (uint32_t)(d.qw * ep.C);
  const f2v* row0 = X2 + (KS * g16 + jl) * (KS / 2);   // tile g16, row jl
  const f2v* row1 = row0 + 16 * KS * (KS / 2);          // tile g16 + 16
  uint32_t code0 = 0, code1 = 0;
  float am0 = 0.0f, am1 = 0.0f;
#pragma unroll
  for (int p = 0; p < KS / 2; ++p) code_bits4(code0, code1, am0, am1, row0[p], row1[p], thr_r[0][p], thr_r[1][p]);
  // max over the 16-lane row (non-negative floats and +NaN: integer order)
  uint32_t u0 = __float_as_uint(am0), u1 = __float_as_uint(am1);
#define DCTAE_ROR_MAX(ctl)                                                        \
  u0 = max(u0, (uint32_t)__builtin_amdgcn_mov_dpp((int)u0, ctl, 0xf, 0xf, false)); \
  u1 = max(u1, (uint32_t)__builtin_amdgcn_mov_dpp((int)u1, ctl, 0xf, 0xf, false));
  DCTAE_ROR_MAX(0x128) DCTAE_ROR_MAX(0x124) DCTAE_ROR_MAX(0x122) DCTAE_ROR_MAX(0x121)
#undef DCTAE_ROR_MAX
  const uint32_t span = 31 * hs + 1;   // tokens from tok0 to tile 31's
  const uint32_t o0 = (uint32_t)g16 * hs, o1 = o0 + 16 * hs;
  const auto srs = __builtin_amdgcn_make_buffer_rsrc(sk.scores + tok0, 0, (int)(span * 4), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(__fadd_rn(__fmul_rn(__uint_as_float(u0), ep.mw), sb[0])),
                                        srs, o0 * 4, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(__fadd_rn(__fmul_rn(__uint_as_float(u1), ep.mw), sb[1])),
                                        srs, o1 * 4, 0, 0);
  if (sk.codes) {
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(sk.codes + tok0 * KS, 0, (int)(span * KS * 2), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)code0, crs, (o0 * KS + jl) * 2, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)code1, crs, (o1 * KS + jl) * 2, 0, 0);
  }
  if (sk.raw) cols_store_tokens(d, c, strip, reinterpret_cast<const float*>(X2), sk.raw, ep.C);
}

__device__ __forceinline__ constexpr int z7addr(int m) { return 16 * (m ^ ((m >> 3) & 1)); }

__device__ __forceinline__ int cols7_j2(int w, int g) {
  // wave 0: 0, 8, 1, 15;  wave w > 0: 2w, 16 - 2w, 2w + 1, 15 - 2w
  const int a = (g & 2) ? 2 * w + 1 : 2 * w;
  const int base = (w == 0 && g < 2) ? (g ? 8 : 0) : ((g & 1) ? (g & 2 ? 15 - 2 * w : 16 - 2 * w) : a);
  return base;
}

__device__ __forceinline__ void cols7_load(const ImgDesc& d, int c, int strip, const float* __restrict__ T,
                                           float (&va)[16], float (&vb)[16]) {
  constexpr int N = 512;
  const int tid = opaque_tid();
  const int j1 = tid >> 4, col = min(tid & 15, 13);
  const int rs = d.Kw;
  // buffer descriptor on the (channel, tile column) slice: 32-bit lane offsets, uniform row steps
  const float* cb = T + (int64_t)c * N * rs + strip * 14;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(cb), 0, N * rs * 4, 0x00020000);
  // m = j1 + 16 r: rows 4m (+2) for r < 8, 2N - 1 - 4m (-2) above; 64-row steps
  const int lo = (4 * j1 * rs + col) * 4;
  const int hi = ((2 * N - 1 - 4 * j1 - 64 * 15) * rs + col) * 4;   // r = 15: lowest row of the upper half
  const int step = 64 * rs * 4, two = 2 * rs * 4;
  constexpr int aux = 0;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    va[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, lo, r * step, aux));
    vb[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, lo + two, r * step, aux));
  }
#pragma unroll
  for (int r = 8; r < 16; ++r) {
    va[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, hi, (15 - r) * step, aux));
    vb[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, hi - two, (15 - r) * step, aux));
  }
}

// ---------------------------------------------------------------------------
// cols7 (N = 512): the column FFT with ONE LDS exchange.  Lane (w, g, col) =
// (wave, 16-lane row, column of the strip; col 14, 15 idle).
//  * pass 1: butterfly j1 = 4w + g reads z[j1 + 16 r] straight from T in
//    global memory (Makhoul pairs (x[4m], x[4m+2]) / (x[2N-1-4m], x[2N-3-4m]),
//    14 consecutive floats of a T row per 16-lane row), DFT16 in registers,
//    writes z[16 j1 + r] to LDS;
//  * pass 2: butterfly j2 (wave w owns the pairs j2 / 16 - j2) reads
//    z[j2 + 16 r], twiddles, DFT16: Z[j2 + 16 r] in registers;
//  * Makhoul post needs Z[M - k] = the partner row's Z[(16 - j2) + 16 (15 - i)]:
//    a v_permlane16_swap between rows g and g ^ 1 (j2 = 0 and 8 pair with
//    themselves), no LDS;
//  * X (448 x 14 kept coefficients) -> LDS -> the cols5 token epilogue.
// LDS slot of complex element m, column col: 16 m' + col, m' = m ^ bit3(m)
// (a permutation): the two 16-lane rows of a ds_read_b64 half-wave
// (j2 = a, 16 - a: bit 3 differs) fall on opposite 32-bank halves.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float partner_row(float x, bool even_row) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(even_row ? r[1] : r[0]);
}

// X aliases z (one more barrier, 37 KB instead of 62 KB: 4 workgroups per CU)
union Cols7Lds {
  float2 z[256 * 16];
  float X[449 * 14];   // 448 kept rows + a spare row (the post's unconditional X[448] store)
};

// Makhoul post of cols7 for one lane: v = Z[j2 + 16 i]; writes X[k], X[N - k]
// (Kh = 448: X[N - k] kept for k > 64) and X[M] (j2 = 0).  W0: wave 0, whose
// rows 0 and 1 (j2 = 0, 8) pair with themselves.
template <bool W0>
__device__ __forceinline__ void cols7_post(const cf (&v)[16], int j2, int g, int col, const float4* post4,
                                           float* Xs) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14;
  // lanes 14 / 15 loaded column 13 (cols7_load clamps) and hold its values:
  // they store the same values to the same slots (no divergent branches)
  const int colc = col < KS ? col : KS - 1;
  const bool self = W0 && g < 2;
  float* xa = Xs + j2 * KS + colc;                       // X[j2 + 16 i] at + 224 i
  float* xb = Xs + (N - j2 - 16 * 15) * KS + colc;       // X[N - j2 - 16 i] at + 224 (15 - i)
  const float4* ps = post4 + j2;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    cf P;
    P.x = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v[15 - i].x), 0x401f));   // lane ^ 16
    P.y = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v[15 - i].y), 0x401f));
    if (W0) P = self ? ((j2 == 0) ? v[(16 - i) & 15] : v[15 - i]) : P;
    const cf A = v[i];
    const float4 ab = ps[16 * i];
    const cf al = (cf){ab.x, ab.y}, be = (cf){ab.z, ab.w};
    const cf s1 = add_conj(A, P), d1 = sub_conj(A, P);
    const cf W = fma_iw(d1, be, fma_x(d1, be, fma_iw(s1, al, mul_x(s1, al))));
    xa[224 * i] = W.x;
    // i = 4, j2 = 0: k = 64, X[N - k] = X[448] is past Kh: the spare row
    if (i >= 4) xb[224 * (15 - i)] = -W.y;
  }
  if (W0 && j2 == 0) {   // k = M (< Kh): A = B = Z[0]
    const cf A = v[0];
    const float4 ab = post4[M];
    const cf s1 = add_conj(A, A), d1 = sub_conj(A, A);
    const cf W = fma_iw(d1, (cf){ab.z, ab.w}, fma_x(d1, (cf){ab.z, ab.w}, cmul_pk(s1, (cf){ab.x, ab.y})));
    Xs[M * KS + colc] = W.x;
  }
}

template <bool THR>
__device__ __forceinline__ void cols7_compute(const ImgDesc& d, int c, int strip, Cols7Lds& L, const float (&va)[16],
                                              const float (&vb)[16], const float4* post4, const float2* tw_s,
                                              const float* sbias, const float2 (&thr_r)[2][7], const EncParams& ep,
                                              const TokenSinks& sk) {
#pragma clang fp contract(fast)
  const int tid = opaque_tid();
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), g = (tid >> 4) & 3, col = tid & 15;
  cf* z = reinterpret_cast<cf*>(L.z);
  (void)d;
  // ---- pass 1 (Ns = 1): j1 = tid >> 4
  {
    const int j1 = tid >> 4;
    cf v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = (cf){va[r], vb[r]};
    DFTV<16>::run(v);
    // lanes 14 / 15 (duplicates of column 13) fill z's own columns 14 / 15
    cf* zw = z + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) zw[z7addr(16 * j1 + r)] = v[r];
  }
  __syncthreads();
  // ---- pass 2 (Ns = 16): z[j2 + 16 r] * W_M^{r j2} -> DFT16 -> Z[j2 + 16 r]
  const int j2 = cols7_j2(w, g);
  cf v[16];
  {
    const cf* zr = z + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = zr[z7addr(j2 + 16 * r)];
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      const float2 tw = tw_s[r * j2];
      v[r] = cmul_pk(v[r], (cf){tw.x, tw.y});
    }
    DFTV<16>::run(v);
  }
  // X aliases z: every wave's pass-2 reads of z must be done before any post writes X
  __syncthreads();
  // ---- Makhoul post: k = j2 + 16 i; A = Z[k], B = conj Z[M - k]
  //      j2 >= 1: Z[M - k] = partner row's v[15 - i] (lane ^ 16, ds_swizzle);
  //      j2 = 0: own v[(16 - i) & 15];  j2 = 8: own v[15 - i]  (wave 0, rows 0 and 1)
  //      kept rows: Kh = 448 (H = 512): X[k] always, X[N - k] for k > 64
#if defined(DCTAE_PROFILING) && defined(DCTAE_C7_ABL)
  // profiling ablations (wrong outputs): bit 0 no token epilogue, bit 1 no
  // Makhoul post either (pass-2 results summed into one LDS word per lane)
  if (DCTAE_C7_ABL & 2) {
    cf acc = v[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) acc += v[i];
    L.X[tid] = acc.x + acc.y;
    __syncthreads();
    return;
  }
#endif
  if (w == 0) cols7_post<true>(v, j2, g, col, post4, L.X);
  else cols7_post<false>(v, j2, g, col, post4, L.X);
  __syncthreads();
#if defined(DCTAE_PROFILING) && defined(DCTAE_C7_ABL)
  if (DCTAE_C7_ABL & 1) return;
#endif
  const int g16 = tid >> 4;
  const float sb[2] = {sbias[g16], sbias[g16 + 16]};
  cols_epilogue<THR>(d, c, strip, reinterpret_cast<const f2v*>(L.X), sb, thr_r, ep, sk);
}


// ---------------------------------------------------------------------------
// k_cols512b (N = 512 columns of 512 x 512 images whose row pass wrote the band
// layout: band16 T'[c][y / 16][kx][16 rows] by default, t4_index in
// dctae_rows512.h; float4 = 4 rows of one column): the column transform runs
// exactly like the row kernel's, one 16-lane group per column.  Block = 4 waves
// = 16 groups over the 14 columns of one tile strip (groups 14 / 15 repeat
// column 13 and store the same values to the same slots).
//  * lane j of column kx loads float4 T'[c][16 b + j][kx] = rows 64 b + 4 j +
//    (0, 2, 3, 1) (b < 8): the Makhoul pairs z[j + 16 b] = (x0, x2), mirror lane (x3, x1) --
//    8 16-byte loads per lane and image against k_fft_cols7's 32 4-byte loads;
//  * fft256_group (pass 1, one LDS transpose in the group's region, pass 2),
//    Makhoul post (makhoul_step) into the strip's 448 x 14 coefficients in LDS
//    (aliasing the transpose regions), then the token epilogue (cols_epilogue).
// ---------------------------------------------------------------------------
struct Cols512bLds {
  union {
    cf xch[16][kXchStridePk];   // per group transpose region (34,816 B)
    float X[449 * 14];          // 448 kept rows + the spare row of the k = 64 store
  } u;
  float2 tw2[16][16];
  float4 pc[256];               // c1..c4 of the Makhoul post, k < M (k = M in registers)
};                              // 40,960 B: 4 blocks per CU

// the band T' of one column as loaded (float4 of 4 rows, or with DCTAE_T23 the
// 12-byte record quarter, decoded by t_decode when the transform starts)
#if DCTAE_T23
typedef v3u TPiece;
#else
typedef float4 TPiece;
#endif
__device__ __forceinline__ void t_decode(const TPiece (&q)[8], float4 (&f)[8]) {
#if DCTAE_T23
  const int j = opaque_tid() & 15;
#pragma unroll
  for (int b = 0; b < 8; ++b) f[b] = t23_unpack(q[b], j & 3);
#else
#pragma unroll
  for (int b = 0; b < 8; ++b) f[b] = q[b];
#endif
}
__device__ __forceinline__ void t_opaque(TPiece (&q)[8]) {   // the loads become opaque values here
#pragma unroll
  for (int r = 0; r < 8; ++r) {
#if DCTAE_T23
    asm volatile("" : "+v"(q[r].x), "+v"(q[r].y), "+v"(q[r].z));
#else
    asm volatile("" : "+v"(q[r].x), "+v"(q[r].y), "+v"(q[r].z), "+v"(q[r].w));
#endif
  }
}
// lane j of column kx loads band4 = 16 b + j: record (band16 4 b + j / 4, kx), slot j % 4
__device__ __forceinline__ void t_load_column(int c, int kx, int j, const float* __restrict__ T, TPiece (&q)[8]) {
  constexpr int KW = 448;
#if DCTAE_T23
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(T)) +
                                                          (int64_t)c * 512 * KW * 3, 0, 512 * KW * 3, 0x00020000);
  const int o = (((j >> 2) * KW + kx) * 4 + (j & 3)) * 12;
  constexpr int bstep = 4 * KW * 4 * 12;
#pragma unroll
  for (int b = 0; b < 8; ++b) q[b] = __builtin_amdgcn_raw_buffer_load_b96(rsrc, o, b * bstep, DCTAE_T_LD_AUX);
#else
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T) + (int64_t)c * 512 * KW, 0, 512 * KW * 4,
                                                      0x00020000);
  const int o = t4_index(j, kx) * 16;   // band4 = 16 b + j
  constexpr int bstep = 16 * KW * 16;   // t4_index(16 b + j, kx) - t4_index(16 (b - 1) + j, kx), both layouts
#pragma unroll
  for (int b = 0; b < 8; ++b)
    q[b] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, b * bstep, DCTAE_T_LD_AUX));
#endif
}

__device__ __forceinline__ void cols512b_load(int c, int strip, const float* __restrict__ T, TPiece (&q)[8]) {
  const int tid = opaque_tid();
  const int G = tid >> 4, j = tid & 15;
  constexpr int KW = 448;
#if DCTAE_T23
  t_load_column(c, 14 * strip + min(G, 13), j, T, q);
#else
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T) + (int64_t)c * 512 * KW, 0, 512 * KW * 4,
                                                      0x00020000);
  const int kx = 14 * strip + min(G, 13);
  const int o = t4_index(j, kx) * 16;                                 // band4 = 16 b + j
  constexpr int bstep = 16 * KW * 16;   // t4_index(16 b + j, kx) - t4_index(16 (b - 1) + j, kx), both layouts
#if defined(DCTAE_PROFILING) && defined(DCTAE_C5B_ABL)
  if (DCTAE_C5B_ABL & 4) {   // profiling ablation: no T' loads (wrong outputs)
#pragma unroll
    for (int b = 0; b < 8; ++b) q[b] = make_float4(0.001f * (b + j), 0.002f * kx, 0.003f * c, 0.0004f * b);
    return;
  }
#endif
#pragma unroll
  for (int b = 0; b < 8; ++b)
    q[b] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, b * bstep, DCTAE_T_LD_AUX));
#endif
}

// PatchNorm-output epilogue of k_cols512b (the LFQ-projection encode's staged
// tokens, or returned normalised patches; qh = qw = 32): per tile row the
// PatchNorm (patchnorm.py:157-165, pn_forward's fp32 ops) on the (median, std)
// pairs this thread holds for the block's (channel, strip) -- loaded once per
// block, as the threshold path's tables, instead of 28 table loads per thread
// and image -- scores (FE:409-416), the optional sign codes (one codebook per
// tile row, MSB first), the values written back in place and stored as
// 16-byte pieces (cols_store_tokens)
__device__ __forceinline__ void cols512b_norm_epilogue(const ImgDesc& d, int c, int strip, float* Xf,
                                                       const float (&sb)[2], const float2 (&tn)[2][14],
                                                       const EncParams& ep, const TokenSinks& sk) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = tid & 15, jlc = min(jl, KS - 1);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int h = g16 + 16 * r;
    f2v* row = reinterpret_cast<f2v*>(Xf) + (KS * h + jlc) * (KS / 2);
    float y[KS];
    uint32_t am = 0, code = 0;
#pragma unroll
    for (int p = 0; p < KS / 2; ++p) {
      const f2v v2 = row[p];
      am = max(am, max(__float_as_uint(v2.x) & 0x7fffffffu, __float_as_uint(v2.y) & 0x7fffffffu));
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float x = e ? v2.y : v2.x;
        const float2 t = tn[r][2 * p + e];   // (median, std = b sqrt2 + eps)
        const float q = __fdiv_rn(__fsub_rn(x, t.x), t.y);
        const float v = (q != q) ? q : fminf(fmaxf(q, ep.min_val), ep.max_val);   // torch.clamp_ keeps NaN
        y[2 * p + e] = v;
        code = 2 * code + (v > 0.0f ? 1u : 0u);
      }
    }
    am = jl < KS ? am : 0u;
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x128, 0xf, 0xf, false));
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x124, 0xf, 0xf, false));
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x122, 0xf, 0xf, false));
    am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x121, 0xf, 0xf, false));
    const int64_t tok = cols_tok(d, c, strip, h, ep.C);
    if (jl == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(__uint_as_float(am), ep.mw), sb[r]);
    if (jl < KS) {
      if (sk.codes) sk.codes[tok * KS + jl] = (uint16_t)code;
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) row[p] = (f2v){y[2 * p], y[2 * p + 1]};
    }
  }
  __syncthreads();
  cols_store_tokens(d, c, strip, Xf, sk.norm, ep.C);
}

// (median, b sqrt2 + eps) of this thread's two tile rows h = g16 + 16 r, row jl
// (lanes 14 / 15: row 13) of the (channel, strip) item
__device__ __forceinline__ void cols_norm_tables(int c, int strip, const EncParams& ep, float2 (&tn)[2][14]) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jlc = min(tid & 15, KS - 1);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t tab = ((((int64_t)c * ep.maxph + g16 + 16 * r) * ep.maxpw) + strip) * (KS * KS) + (int64_t)jlc * KS;
    const float2* m2 = reinterpret_cast<const float2*>(ep.median + tab);
    const float2* b2 = reinterpret_cast<const float2*>(ep.b + tab);
#pragma unroll
    for (int p = 0; p < KS / 2; ++p) {
      const float2 mv = m2[p], bv = b2[p];
      tn[r][2 * p] = make_float2(mv.x, __fadd_rn(__fmul_rn(bv.x, 1.41421353816986083984375f), ep.eps));
      tn[r][2 * p + 1] = make_float2(mv.y, __fadd_rn(__fmul_rn(bv.y, 1.41421353816986083984375f), ep.eps));
    }
  }
}

template <bool THR, bool NORM = false>
__device__ __forceinline__ void cols512b_compute(const ImgDesc& d, int c, int strip, Cols512bLds& L,
                                                 const float4 (&q)[8], const float4 pcM, const float (&sb)[2],
                                                 const float2 (&thr_r)[2][7], const EncParams& ep,
                                                 const TokenSinks& sk, const float2 (*tn)[14] = nullptr) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14;
  const int tid = opaque_tid();
  const int G = tid >> 4, j = tid & 15;
  const int colc = min(G, KS - 1);
  const int s = sigma16(j);
  const bool self0 = (j == 0), self8 = (j == 15);
  cf v[16];
#pragma unroll
  for (int b = 0; b < 8; ++b) {   // q[b] = rows 64 b + 4 j + (0, 2, 3, 1)
    v[b] = (cf){q[b].x, q[b].y};
    v[15 - b] = (cf){mirror16(q[b].z), mirror16(q[b].w)};
  }
  fft256_group(v, L.u.xch[G], j, s, L.tw2);
  // X aliases the transpose regions: every group's pass-2 reads before any post write
  __syncthreads();
#if defined(DCTAE_PROFILING) && defined(DCTAE_C5B_ABL)
  if (DCTAE_C5B_ABL & 2) {   // profiling ablation: no Makhoul post, no epilogue (wrong outputs)
    cf acc = v[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) acc += v[i];
    L.u.X[tid] = acc.x + acc.y;
    __syncthreads();
    return;
  }
#endif
  float* xa = L.u.X + s * KS + colc;                 // X[s + 16 i] at + 224 i
  float* xb = L.u.X + (N - s) * KS + colc;           // X[N - s - 16 i] at - 224 i
  // steps in pairs, the next pair's coefficients read while this one computes
  float4 cn0 = L.pc[s], cn1 = L.pc[s + 16];
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const float4 c0 = cn0, c1 = cn1;
    if (i + 2 < 16) {
      cn0 = L.pc[s + 16 * (i + 2)];
      cn1 = L.pc[s + 16 * (i + 3)];
    }
    cf x0, x1;
    makhoul_step2(v, i, self0, self8, c0, c1, x0, x1);
    xa[224 * i] = x0.x;
    xa[224 * (i + 1)] = x1.x;
    // X[N - k] kept for k > 64; i = 4, s = 0 (k = 64) lands on the spare row 448
    if (i >= 4) xb[-224 * i] = x0.y;
    if (i + 1 >= 4) xb[-224 * (i + 1)] = x1.y;
  }
  if (self0) L.u.X[M * KS + colc] = (pcM.x + pcM.y) * v[0].x + (pcM.w - pcM.z) * v[0].y;
  __syncthreads();
#if defined(DCTAE_PROFILING) && defined(DCTAE_C5B_ABL)
  if (DCTAE_C5B_ABL & 1) return;   // profiling ablation: no token epilogue (wrong outputs)
#endif
  if (THR)
    cols512b_epilogue(d, c, strip, reinterpret_cast<const f2v*>(L.u.X), sb, thr_r, ep, sk);
  else if (NORM)
    cols512b_norm_epilogue(d, c, strip, L.u.X, sb, *reinterpret_cast<const float2(*)[2][14]>(tn), ep, sk);
  else
    cols_epilogue<false>(d, c, strip, reinterpret_cast<const f2v*>(L.u.X), sb, thr_r, ep, sk);
}

}  // namespace dctae
