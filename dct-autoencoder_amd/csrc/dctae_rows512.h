// Row pass of the 2-D DCT for images 512 pixels wide (the headline 512^2
// config): RGB -> IPT (util.py:70-82) -> orthonormal
// DCT-II of every row (torch_dct.dct over the last dim, util.py:333) -> the
// kept coefficients kx < Kw of T[c][y][kx] (row-major, read by the column
// pass).  One "item" = 16 rows of one image (256 threads); used by the
// two-kernel path (k_rows512, dctae_rows512.hip) and the persistent encode
// (k_enc512, dctae_enc512.hip).
//
// Makhoul: with v[n] = x[2n] (n < 256), v[511 - n] = x[2n + 1], the 512-point
// DCT-II is a 256-point complex FFT of z[m] = v[2m] + i v[2m + 1] followed by
// X[k] = Re W_k, X[N - k] = -Im W_k, W_k = alpha_k (Z[k] + conj Z[M - k]) +
// beta_k (Z[k] - conj Z[M - k]).  The FFT is two radix-16 Stockham passes.
//
// One 16-lane row group of a wave owns one image row (all 3 channels); lane j
// is pass-1 butterfly j.  Nothing goes through LDS before pass 1:
//  * lane j loads float4 x[64 b + 4 j .. + 3] of each 64-pixel block b (16-byte
//    coalesced loads, 256 B per row group) for R, G and B and converts them to
//    IPT in registers;
//  * its pass-1 inputs are z[j + 16 b] = (x[64 b + 4 j], x[64 b + 4 j + 2]) and
//    z[j + 16 (15 - b)] = (x[64 b + 63 - 4 j], x[64 b + 61 - 4 j]) — the .w / .y
//    of the mirror lane 15 - j: one DPP row_mirror per value;
//  * pass 1 (DFT16 in registers) -> ONE LDS transpose -> pass 2 (twiddles,
//    DFT16): lane l then holds Z[s + 16 i] for butterfly s = sigma(l);
//  * sigma pairs the Makhoul partners s, 16 - s on mirror lanes (l, 15 - l), so
//    conj Z[M - k] = the mirror lane's Z[(16 - s) + 16 (15 - i)] is again one
//    DPP row_mirror; s = 0 (lane 0) and s = 8 (lane 15) pair with themselves.
// LDS transpose slot of pass-1 output k1 of lane j: 16 k1 + (j ^ (k1 & 14)):
// the 16 ds_write_b64 of a row group cover one 128-byte row, and the 8
// ds_read_b128 of lane l (row s) hit 16 distinct 4-bank groups per lane group
// (s distinct, rows 32 banks apart by parity, j ^ (s & 14) spreads the rest).
#pragma once
#include "dctae_device.h"
#include "dctae_fft_common.h"

namespace dctae {

__device__ __forceinline__ float mirror16(float x) {   // lane l <- lane 15 - l of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xf, 0xf, false));
}
__device__ __forceinline__ float ror16(float x) {      // lane l <- lane l - 1 (mod 16)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x121, 0xf, 0xf, false));
}

__device__ __forceinline__ float ipt_pow(float x) {
  // sign(x) |x|^0.43 through v_log_f32 / v_exp_f32 (util.py:76-78)
  const float y = __builtin_amdgcn_exp2f(0.430000007152557373046875f * __builtin_amdgcn_logf(fabsf(x)));
  return __builtin_copysignf(y, x);
}

// transpose region of one row group: re plane at 0, im plane at + 256; 528
// floats apart (16 mod 32 banks), so the two row groups of a 32-lane
// ds_write_b32 land on opposite bank halves; the b128 reads stay conflict-free
// (a 16-bank shift keeps each lane group's 4-bank sets distinct)
constexpr int kXchStride = 528;

struct Rows512Xch {
  float xch[4][4][kXchStride];   // [wave][row group][re 256 | im 256 | pad]
};

// Row-pass tables (loaded once per block): W_256^{r s} and the Makhoul post
// coefficients (c1, c2, c3, c4) of rows512_item.
struct Rows512Tab {
  float2 tw2[16][16];
  float4 pc[257];
};

__device__ __forceinline__ void rows512_tables(Rows512Tab& L, const float2* __restrict__ tw,
                                               const float2* __restrict__ post) {
  const int tid = threadIdx.x;
  const int r = tid >> 4, s = tid & 15;
  L.tw2[r][s] = tw[r * s];
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int i = tid; i < 257; i += 256) {
    const float4 ab = p4[i];   // (al.x, al.y, be.x, be.y)
    L.pc[i] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
  }
}

// Makhoul post of k (A = Z[k], P = Z[M - k], alpha/beta as dctae_api.hip
// builds them): W = alpha (A + conj P) + beta (A - conj P), X[k] = Re W,
// X[N - k] = -Im W.  Expanded over (A.x, A.y, P.x, P.y):
//   X[k]     =  c1 A.x + c2 P.x - c3 A.y + c4 P.y
//   X[N - k] = -c1 A.y + c2 P.y - c3 A.x - c4 P.x
// with c1 = al.x + be.x, c2 = al.x - be.x, c3 = al.y + be.y, c4 = al.y - be.y
// (8 FMA-class operations per k instead of 2 complex adds + 2 complex products).
//
// Lane l of a row group is pass-2 butterfly l: it holds Z[l + 16 i].  The
// partner Z[M - k] = Z[(16 - l) + 16 (15 - i)] lives on lane 16 - l (l >= 1):
// D_i = rotate-right-by-one(mirror(reg[15 - i])).  Lane 0 (Z[16 i]) pairs
// with its own Z[16 ((16 - i) mod 16)] = reg[15 - (i - 1)]: the two DPP moves
// bring lane 0 its own register, so lane 0 uses D_{i-1} (D_15 at i = 0).
//
// rows512_item: rows y0 .. y0 + 15 of an image of H rows (rows past H compute
// a duplicate whose stores fall outside the buffer) -> T (channel planes of
// H x 448 floats, plane_bytes 0 drops every store).  The caller has loaded the
// tables and made them visible (a barrier) before the first item.  ABL bit 2
// (profiling builds only): no RGB loads.
template <int ABL = 0>
__device__ __forceinline__ void rows512_item(Rows512Xch& X, const Rows512Tab& L, const float* __restrict__ img, int H,
                                             int y0, float* T, uint32_t plane_bytes, const ColorMats& cm) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KW = 448;
  const int tid = threadIdx.x;
  const int wv = tid >> 6, g = (tid >> 4) & 3, j = tid & 15;
  const int y = y0 + 4 * wv + g;
  const int yl = min(y, H - 1);
  const int64_t hw = (int64_t)H * N;
  const float* src = img + (int64_t)yl * N + 4 * j;

  // ---- loads: R, G, B float4 of the 8 blocks
  float4 I[3][8];
  if (ABL & 2) {
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int c = 0; c < 3; ++c) I[c][b] = make_float4(0.001f * (j + b), 0.002f * c, 0.003f * yl, 0.0004f * b);
  } else {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      I[0][b] = *reinterpret_cast<const float4*>(src + 64 * b);
      I[1][b] = *reinterpret_cast<const float4*>(src + hw + 64 * b);
      I[2][b] = *reinterpret_cast<const float4*>(src + 2 * hw + 64 * b);
    }
  }
  // ---- IPT in place (util.py:70-82): LMS = Trgb2lms rgb, signed power, IPT = Mipt LMS'
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    float* r4 = reinterpret_cast<float*>(&I[0][b]);
    float* g4 = reinterpret_cast<float*>(&I[1][b]);
    float* b4 = reinterpret_cast<float*>(&I[2][b]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float l0 = ipt_pow(mat3_row(cm.rgb2lms, 0, r4[e], g4[e], b4[e]));
      const float l1 = ipt_pow(mat3_row(cm.rgb2lms, 1, r4[e], g4[e], b4[e]));
      const float l2 = ipt_pow(mat3_row(cm.rgb2lms, 2, r4[e], g4[e], b4[e]));
      r4[e] = mat3_row(cm.lms2ipt, 0, l0, l1, l2);
      g4[e] = mat3_row(cm.lms2ipt, 1, l0, l1, l2);
      b4[e] = mat3_row(cm.lms2ipt, 2, l0, l1, l2);
    }
  }

  float* xre = X.xch[wv][g];
  float* xim = X.xch[wv][g] + 256;
  const bool lane0 = (j == 0);
  // T stores: buffer stores on the channel plane (H x KW floats); rows y >= H
  // fall outside num_records and are dropped
  const int rowo = (y * KW + j) * 4;                     // X[j + 16 i] at + 64 i
  const int rown = (y * KW + (N - 15 * 16) - j) * 4;     // X[N - j - 16 i] at + 64 (15 - i)
  const int rown4 = j >= 1 ? rown : 0x7ffffff0;          // i = 4: k = 64 + j, X[N - k] kept iff j >= 1

#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // ---- pass 1 (Ns = 1): lane j's Makhoul pairs, DFT16 in registers
    float re[16], im[16];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float4 q = I[c][b];
      re[b] = q.x;
      im[b] = q.z;
      re[15 - b] = mirror16(q.w);
      im[15 - b] = mirror16(q.y);
    }
    dft16s(re, im);
    // ---- transpose through LDS: output k1 of lane j at slot 16 k1 + (j ^ (k1 & 12))
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      xre[16 * k1 + (j ^ (k1 & 12))] = re[k1];
      xim[16 * k1 + (j ^ (k1 & 12))] = im[k1];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- pass 2 (Ns = 16): butterfly j reads z1[j + 16 r] = lane r's output j
    {
      const float4* rr = reinterpret_cast<const float4*>(xre + 16 * j);
      const float4* ri = reinterpret_cast<const float4*>(xim + 16 * j);
      const int sw = (j >> 2) & 3;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 a = rr[q ^ sw], b = ri[q ^ sw];
        re[4 * q] = a.x, re[4 * q + 1] = a.y, re[4 * q + 2] = a.z, re[4 * q + 3] = a.w;
        im[4 * q] = b.x, im[4 * q + 1] = b.y, im[4 * q + 2] = b.z, im[4 * q + 3] = b.w;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();   // reads done before the next channel's writes
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      const float2 w = L.tw2[r][j];
      const float a = re[r], b = im[r];
      re[r] = a * w.x - b * w.y;
      im[r] = a * w.y + b * w.x;
    }
    dft16s(re, im);
    // ---- Makhoul post: k = j + 16 i
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(T + (int64_t)c * H * KW, 0, plane_bytes, 0x00020000);
    const float d15r = ror16(mirror16(re[0])), d15i = ror16(mirror16(im[0]));
    float pvr = d15r, pvi = d15i;   // D_{i-1}
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      // every lane runs both DPP moves (a DPP source lane must be active): D_i;
      // lane 0 takes D_{i-1} = its own Z[16 ((16 - i) mod 16)]
      const float dr = i == 15 ? d15r : ror16(mirror16(re[15 - i]));
      const float di = i == 15 ? d15i : ror16(mirror16(im[15 - i]));
      const float Pr = lane0 ? pvr : dr, Pi = lane0 ? pvi : di;
      pvr = dr;
      pvi = di;
      const float Ar = re[i], Ai = im[i];
      const float4 cc = L.pc[j + 16 * i];
      const float xk = cc.x * Ar + cc.y * Pr - cc.z * Ai + cc.w * Pi;
      const float xn = -cc.x * Ai + cc.y * Pi - cc.z * Ar - cc.w * Pr;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xk), rsrc, rowo, 64 * i, 0);
      if (i >= 5) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xn), rsrc, rown, 64 * (15 - i), 0);
      if (i == 4) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xn), rsrc, rown4, 64 * 11, 0);
    }
    // k = M (lane 0): A = P = Z[0]: X[M] = (c1 + c2) Z0.x + (c4 - c3) Z0.y
    {
      const float4 cc = L.pc[M];
      const float xm = (cc.x + cc.y) * re[0] + (cc.w - cc.z) * im[0];
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xm), rsrc, lane0 ? (y * KW + M) * 4 : 0x7ffffff0, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// Packed-f32 variant (rows_kernel 4).  The same transform as rows512_item with
// the VALU work issued as v_pk_{mul,fma,add}_f32 (two fp32 lanes per
// instruction, the 157 TF vector peak; the scalar item is ~2,850 VALU per wave
// and VALU-bound once T stays on chip):
//  * IPT: the channel mixes run on pixel pairs (0, 1) / (2, 3) of each float4
//    (adjacent registers) and write the pairs (0, 2) / (3, 1) -- exactly the
//    Makhoul (re, im) of z[j + 16 b] and the mirror lane's z[(15 - j) + 16 (15 - b)];
//    log / exp / copysign stay scalar (no packed form);
//  * pass 1 / pass 2: DFTV<16> on complex pairs, the transpose as ds_write_b64
//    (element (k1, lane r) at 16 k1 + (r ^ (k1 & 14))) / ds_read_b128 (lane of
//    row s reads chunk q at q ^ (s >> 1): 16 distinct 4-bank groups);
//  * pass 2 lane l runs butterfly s = sigma(l) (l < 8: l; 8 <= l < 15: l + 1;
//    15: 8) so the Makhoul partner 16 - s sits on the mirror lane 15 - l: one
//    DPP row_mirror per value (lanes 0 / 15, s = 0 / 8, pair with themselves);
//  * post: (X[k], X[N - k]) as one pair, four packed FMAs.
// Same rounding as rows512_item for the IPT (identical fma order per pixel);
// the FFT differs in operation order only (tolerance-tested).
// ---------------------------------------------------------------------------
#ifndef DCTAE_XCH_PK
#define DCTAE_XCH_PK 272
#endif
constexpr int kXchStridePk = DCTAE_XCH_PK;   // complex slots per row group: 2 KB + 128 B (row groups 0/1 on opposite bank halves)

struct Rows512XchPk {
  cf xch[4][4][kXchStridePk];
};

__device__ __forceinline__ cf splat_mix(const float* m, int i, cf a, cf b, cf c) {
  // packed mat3_row: fma(m2, c, fma(m1, b, m0 * a)) per half (same rounding)
  const cf m0 = (cf){m[3 * i], m[3 * i]}, m1 = (cf){m[3 * i + 1], m[3 * i + 1]}, m2 = (cf){m[3 * i + 2], m[3 * i + 2]};
  return __builtin_elementwise_fma(m2, c, __builtin_elementwise_fma(m1, b, m0 * a));
}

// (X[k], X[N - k]) = (c1 A.x + c2 P.x - c3 A.y + c4 P.y, -c1 A.y + c2 P.y - c3 A.x - c4 P.x)
// (the swaps / signs as VOP3P op_sel / neg modifiers; plain vector code
// materialises them with v_mov / v_xor)
__device__ __forceinline__ cf makhoul_pair(cf A, cf P, cf c12, cf c34) {
  cf t;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0] neg_hi:[1,0]" : "=v"(t) : "v"(A), "v"(c12));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(t) : "v"(P), "v"(c12), "v"(t));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
      : "=v"(t) : "v"(A), "v"(c34), "v"(t));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(t) : "v"(P), "v"(c34), "v"(t));
  return t;
}

__device__ __forceinline__ void rows512_item_pk(Rows512XchPk& X, const Rows512Tab& L, const float* __restrict__ img,
                                                int H, int y0, float* T, uint32_t plane_bytes, const ColorMats& cm) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KW = 448;
  const int tid = threadIdx.x;
  const int wv = tid >> 6, g = (tid >> 4) & 3, j = tid & 15;
  const int y = y0 + 4 * wv + g;
  const int yl = min(y, H - 1);
  const int64_t hw = (int64_t)H * N;
  const float* src = img + (int64_t)yl * N + 4 * j;

  float4 I[3][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    I[0][b] = *reinterpret_cast<const float4*>(src + 64 * b);
    I[1][b] = *reinterpret_cast<const float4*>(src + hw + 64 * b);
    I[2][b] = *reinterpret_cast<const float4*>(src + 2 * hw + 64 * b);
  }
  // ---- IPT (util.py:70-82): A[c][b] = (ipt_c(x0), ipt_c(x2)), B[c][b] = (ipt_c(x3), ipt_c(x1))
  cf A[3][8], B[3][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const cf r01 = (cf){I[0][b].x, I[0][b].y}, r23 = (cf){I[0][b].z, I[0][b].w};
    const cf g01 = (cf){I[1][b].x, I[1][b].y}, g23 = (cf){I[1][b].z, I[1][b].w};
    const cf b01 = (cf){I[2][b].x, I[2][b].y}, b23 = (cf){I[2][b].z, I[2][b].w};
    cf p02[3], p31[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const cf l01 = splat_mix(cm.rgb2lms, i, r01, g01, b01);
      const cf l23 = splat_mix(cm.rgb2lms, i, r23, g23, b23);
      // sign(x) |x|^0.43 (util.py:76-78): log scalar, the 0.43 scale packed, exp / copysign scalar
      const cf lg01 = (cf){__builtin_amdgcn_logf(fabsf(l01.x)), __builtin_amdgcn_logf(fabsf(l01.y))};
      const cf lg23 = (cf){__builtin_amdgcn_logf(fabsf(l23.x)), __builtin_amdgcn_logf(fabsf(l23.y))};
      const cf k = (cf){0.430000007152557373046875f, 0.430000007152557373046875f};
      const cf e01 = k * lg01, e23 = k * lg23;
      p02[i] = (cf){__builtin_copysignf(__builtin_amdgcn_exp2f(e01.x), l01.x),
                    __builtin_copysignf(__builtin_amdgcn_exp2f(e23.x), l23.x)};
      p31[i] = (cf){__builtin_copysignf(__builtin_amdgcn_exp2f(e23.y), l23.y),
                    __builtin_copysignf(__builtin_amdgcn_exp2f(e01.y), l01.y)};
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      A[c][b] = splat_mix(cm.lms2ipt, c, p02[0], p02[1], p02[2]);
      B[c][b] = splat_mix(cm.lms2ipt, c, p31[0], p31[1], p31[2]);
    }
  }

  cf* xr = X.xch[wv][g];
  const int s = j < 8 ? j : (j < 15 ? j + 1 : 8);   // sigma(j)
  const bool self0 = (j == 0), self8 = (j == 15);
  // T stores of butterfly s: X[s + 16 i] at + 64 i, X[N - s - 16 i] at + 64 (15 - i)
  const int rowo = (y * KW + s) * 4;
  const int rown = (y * KW + (N - 15 * 16) - s) * 4;
  const int rown4 = s >= 1 ? rown : 0x7ffffff0;   // i = 4: k = 64 + s, X[N - k] kept iff s >= 1

#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // ---- pass 1: lane j's z[j + 16 r]
    cf v[16];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      v[b] = A[c][b];
      v[15 - b] = (cf){mirror16(B[c][b].x), mirror16(B[c][b].y)};
    }
    DFTV<16>::run(v);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) xr[16 * k1 + (j ^ (k1 & 14))] = v[k1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- pass 2: butterfly s reads z1[s + 16 r] = lane r's output s
    {
      const float4* rr = reinterpret_cast<const float4*>(xr + 16 * s);
      const int sw = s >> 1;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 a = rr[q ^ sw];
        v[2 * q] = (cf){a.x, a.y};
        v[2 * q + 1] = (cf){a.z, a.w};
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();   // reads done before the next channel's writes
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      const float2 w = L.tw2[r][s];
      v[r] = cmul_pk(v[r], (cf){w.x, w.y});
    }
    DFTV<16>::run(v);
    // ---- Makhoul post: k = s + 16 i, A = Z[k] = v[i], P = Z[M - k]
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(T + (int64_t)c * H * KW, 0, plane_bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const cf m = (cf){mirror16(v[15 - i].x), mirror16(v[15 - i].y)};
      const cf own = self0 ? v[(16 - i) & 15] : v[15 - i];
      const cf P = (self0 || self8) ? own : m;
      const float4 cc = L.pc[s + 16 * i];
      const cf xx = makhoul_pair(v[i], P, (cf){cc.x, cc.y}, (cf){cc.z, cc.w});
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.x), rsrc, rowo, 64 * i, 0);
      if (i >= 5) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.y), rsrc, rown, 64 * (15 - i), 0);
      if (i == 4) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.y), rsrc, rown4, 64 * 11, 0);
    }
    // k = M (s = 0, lane 0): A = P = Z[0]: X[M] = (c1 + c2) Z0.x + (c4 - c3) Z0.y
    {
      const float4 cc = L.pc[M];
      const float xm = (cc.x + cc.y) * v[0].x + (cc.w - cc.z) * v[0].y;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xm), rsrc, self0 ? (y * KW + M) * 4 : 0x7ffffff0, 0, 0);
    }
  }
}

}  // namespace dctae

namespace dctae {

// ---------------------------------------------------------------------------
// Row pass + the column FFT's first pass (option rows_p1, k_rows512p1): one
// 512-thread block = the 32 rows of column butterfly j1 of one image,
//   q = 2 r + sub (r < 16, sub < 2), m = j1 + 16 r:
//   r < 8: row 4 m + 2 sub;  r >= 8: row 1023 - 4 m - 2 sub
// (exactly the rows the column kernel's pass-1 butterfly j1 reads: z[m] =
// (T[row(q = 2r)], T[row(q = 2r + 1)]) column by column).  Per channel: the
// row transform of rows512_item_pk, its 448 kept coefficients into the row
// group's own LDS region (aliasing its transpose buffer), a block barrier,
// then thread kx < 448 runs the column DFT16 over r and stores the 16
// outputs Y_j1[k1] as P1[c][j1][k1][kx] (float2; 448 contiguous per (c, j1,
// k1): coalesced).  P1 has T's size and takes T's workspace slot; the column
// kernel (k_fft_cols7p2) starts at pass 2.  Same arithmetic as
// k_rows512pk + k_fft_cols7, so the outputs are bit-identical.
// ---------------------------------------------------------------------------
struct Rows512P1Lds {
  cf xch[8][4][kXchStridePk];   // [wave][row group]: row transposes, then the row's 448 coefficients
  Rows512Tab t;
};

__device__ __forceinline__ void rows512_p1_tables(Rows512Tab& L, const float2* __restrict__ tw,
                                                  const float2* __restrict__ post) {
  const int tid = threadIdx.x;
  if (tid < 256) L.tw2[tid >> 4][tid & 15] = tw[(tid >> 4) * (tid & 15)];
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int i = tid; i < 257; i += 512) {
    const float4 ab = p4[i];
    L.pc[i] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
  }
}

__device__ __forceinline__ void rows512_p1_item(Rows512P1Lds& X, const float* __restrict__ img, int j1,
                                                float2* __restrict__ P1, const ColorMats& cm) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KW = 448;
  const int tid = threadIdx.x;
  const int wv = tid >> 6, g = (tid >> 4) & 3, j = tid & 15;
  const int q = 4 * wv + g, r = q >> 1, sub = q & 1;
  const int m = j1 + 16 * r;
  const int y = r < 8 ? 4 * m + 2 * sub : 1023 - 4 * m - 2 * sub;
  const int64_t hw = (int64_t)N * N;
  const float* src = img + (int64_t)y * N + 4 * j;

  float4 I[3][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    I[0][b] = *reinterpret_cast<const float4*>(src + 64 * b);
    I[1][b] = *reinterpret_cast<const float4*>(src + hw + 64 * b);
    I[2][b] = *reinterpret_cast<const float4*>(src + 2 * hw + 64 * b);
  }
  cf A[3][8], B[3][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const cf r01 = (cf){I[0][b].x, I[0][b].y}, r23 = (cf){I[0][b].z, I[0][b].w};
    const cf g01 = (cf){I[1][b].x, I[1][b].y}, g23 = (cf){I[1][b].z, I[1][b].w};
    const cf b01 = (cf){I[2][b].x, I[2][b].y}, b23 = (cf){I[2][b].z, I[2][b].w};
    cf p02[3], p31[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const cf l01 = splat_mix(cm.rgb2lms, i, r01, g01, b01);
      const cf l23 = splat_mix(cm.rgb2lms, i, r23, g23, b23);
      const cf lg01 = (cf){__builtin_amdgcn_logf(fabsf(l01.x)), __builtin_amdgcn_logf(fabsf(l01.y))};
      const cf lg23 = (cf){__builtin_amdgcn_logf(fabsf(l23.x)), __builtin_amdgcn_logf(fabsf(l23.y))};
      const cf k = (cf){0.430000007152557373046875f, 0.430000007152557373046875f};
      const cf e01 = k * lg01, e23 = k * lg23;
      p02[i] = (cf){__builtin_copysignf(__builtin_amdgcn_exp2f(e01.x), l01.x),
                    __builtin_copysignf(__builtin_amdgcn_exp2f(e23.x), l23.x)};
      p31[i] = (cf){__builtin_copysignf(__builtin_amdgcn_exp2f(e23.y), l23.y),
                    __builtin_copysignf(__builtin_amdgcn_exp2f(e01.y), l01.y)};
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      A[c][b] = splat_mix(cm.lms2ipt, c, p02[0], p02[1], p02[2]);
      B[c][b] = splat_mix(cm.lms2ipt, c, p31[0], p31[1], p31[2]);
    }
  }

  cf* xr = X.xch[wv][g];
  float* xl = reinterpret_cast<float*>(xr);   // the row's kept coefficients (after pass 2's reads)
  const int s = j < 8 ? j : (j < 15 ? j + 1 : 8);
  const bool self0 = (j == 0), self8 = (j == 15);
  // this thread's column in the column pass
  const int kx = tid;
  const bool colt = kx < KW;

#pragma unroll 1
  for (int c = 0; c < 3; ++c) {
    // channel c's IPT values are in A[0] / B[0] (rotated below: no dynamic
    // register indexing in the rolled channel loop, which would go to scratch)
    cf v[16];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      v[b] = A[0][b];
      v[15 - b] = (cf){mirror16(B[0][b].x), mirror16(B[0][b].y)};
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      A[0][b] = A[1][b];
      A[1][b] = A[2][b];
      B[0][b] = B[1][b];
      B[1][b] = B[2][b];
    }
    DFTV<16>::run(v);
    if (c > 0) __syncthreads();   // the previous channel's column-pass reads of every row region
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) xr[16 * k1 + (j ^ (k1 & 14))] = v[k1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
      const float4* rr = reinterpret_cast<const float4*>(xr + 16 * s);
      const int sw = s >> 1;
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) {
        const float4 a = rr[qq ^ sw];
        v[2 * qq] = (cf){a.x, a.y};
        v[2 * qq + 1] = (cf){a.z, a.w};
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();   // pass-2 reads done before the coefficients overwrite the region
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int rr2 = 1; rr2 < 16; ++rr2) {
      const float2 w = X.t.tw2[rr2][s];
      v[rr2] = cmul_pk(v[rr2], (cf){w.x, w.y});
    }
    DFTV<16>::run(v);
    // ---- Makhoul post -> the row's kept coefficients in LDS
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const cf mm = (cf){mirror16(v[15 - i].x), mirror16(v[15 - i].y)};
      const cf own = self0 ? v[(16 - i) & 15] : v[15 - i];
      const cf P = (self0 || self8) ? own : mm;
      const float4 cc = X.t.pc[s + 16 * i];
      const cf xx = makhoul_pair(v[i], P, (cf){cc.x, cc.y}, (cf){cc.z, cc.w});
      xl[s + 16 * i] = xx.x;
      // X[N - k] kept for k > 64; i = 4, s = 0 (k = 64) lands on slot 448, past the kept row
      if (i >= 4) xl[N - s - 16 * i] = xx.y;
    }
    if (self0) {
      const float4 cc = X.t.pc[M];
      xl[M] = (cc.x + cc.y) * v[0].x + (cc.w - cc.z) * v[0].y;
    }
    __syncthreads();   // every row's coefficients of channel c
    // ---- column pass 1: z[r'] = (row q = 2 r', row 2 r' + 1) of column kx, DFT16 over r'
    if (colt) {
      cf z[16];
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        const float* a = reinterpret_cast<const float*>(X.xch[r2 >> 1][(2 * r2) & 3]);
        const float* b2 = reinterpret_cast<const float*>(X.xch[r2 >> 1][(2 * r2 + 1) & 3]);
        z[r2] = (cf){a[kx], b2[kx]};
      }
      DFTV<16>::run(z);
      float2* dst = P1 + ((int64_t)(c * 16 + j1) * 16) * KW + kx;
#pragma unroll
      for (int k1 = 0; k1 < 16; ++k1) dst[k1 * KW] = make_float2(z[k1].x, z[k1].y);
    }
  }
}

}  // namespace dctae
