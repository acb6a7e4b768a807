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

}  // namespace dctae
