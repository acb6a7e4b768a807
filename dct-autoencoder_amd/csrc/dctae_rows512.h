// Row pass of the 2-D DCT for images 512 pixels wide (the headline 512^2
// config): RGB -> IPT (util.py:70-82) -> orthonormal
// DCT-II of every row (torch_dct.dct over the last dim, util.py:333) -> the
// kept coefficients kx < Kw of T[c][y][kx] (row-major, read by the column
// pass).  One "item" = 16 rows of one image (256 threads), run by k_rows512pk
// (dctae_rows512.hip).
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

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Layout of the band-layout T' (float4 = 4 rows of one column kx; band4 = y / 4):
//   2 (default): [band4 / 4][448 kx][16]  -- band16: a row block's channel is one
//       contiguous 28 KB piece (staged through LDS, 1 KB stores), a column
//       block's 14 columns are 896-byte runs;
//   0: [band4][448 kx][4]  -- direct 16-byte stores after a 4 x 4 cross-row
//       transpose; the column block reads 224-byte runs 7 KB apart.
// Measured (1024 x 512^2, same box): layout 0 rows 1.11 / cols 0.735 ms,
// layout 2 rows 1.08-1.09 / cols 0.607 ms.  Layout 2 at
// 207 VGPRs (2 waves / SIMD) still beats layout 0 at 156 (3 waves).
#ifndef DCTAE_TLAYOUT
#define DCTAE_TLAYOUT 2
#endif
// cache-policy bits of the band T' stores (k_rows512pk) and loads (k_cols512b /
// k_cols512w): 2 = nontemporal (default: T' is written once, read once; its
// 2.8 GB per 1024 images otherwise churn the L2 / MALL -- same-box A/B, rows
// 1.089-1.092 -> 1.053-1.054 ms with NT stores, the following sort / pack
// 0.128 -> 0.108 ms with NT loads), 0 = the default policy
#ifndef DCTAE_T_ST_AUX
#define DCTAE_T_ST_AUX 2
#endif
#ifndef DCTAE_T_LD_AUX
#define DCTAE_T_LD_AUX 2
#endif
// the decode's band U' (k_idct_cols512b stores, k_idct_rows512 loads): the
// stores nontemporal (default; same-box A/B r05: decode 2.07-2.12 -> 2.01-2.05
// ms, cols 0.88-0.90 -> 0.84-0.87, rows 1.10-1.12 -> 1.05-1.08), the loads at
// the default policy (nontemporal loads: rows 1.10 -> 1.29-1.33 ms)
#ifndef DCTAE_U_ST_AUX
#define DCTAE_U_ST_AUX 2
#endif
#ifndef DCTAE_U_LD_NT
#define DCTAE_U_LD_NT 0
#endif
static_assert(DCTAE_TLAYOUT == 0 || DCTAE_TLAYOUT == 2, "T' layouts: 0 or 2");

// T' as 12-byte records (DCTAE_T23, band16 layout only): the float4 of a
// band16 slot (4 rows of one column) is 4 x 23-bit signed mantissas and a
// nibble of the 8-bit exponent E shared by the record's 16 values (the 4
// slots of (band16, kx): the same column kx of 16 adjacent rows, so similar
// magnitudes); x = m 2^(E - 148), |m| < 2^22 against the record's |max| <
// 2^(E - 126): the largest value keeps 22-23 significant bits (fp32: 24), the
// others the same absolute step.  E = 255 marks a non-finite value in the
// record (decoded as NaN).  Slots 0 / 2 carry E's low nibble, 1 / 3 its high
// one.  T' is written once and read once: 2.06 instead of 2.75 MB per image.
// Off: measured slower (same box, 1024 x 512^2: rows 1.06 -> 1.10 ms, columns
// 0.60 -> 0.64 ms, encode 1.83 -> 1.91 ms; codes unchanged vs the oracle) --
// the pack / unpack VALU and the 12-byte accesses cost more than the 25 %
// fewer T' bytes save.
#ifndef DCTAE_T23
#define DCTAE_T23 0
#endif
static_assert(!DCTAE_T23 || DCTAE_TLAYOUT == 2, "12-byte T' records: band16 layout");
typedef unsigned v3u __attribute__((ext_vector_type(3)));

__device__ __forceinline__ uint32_t quad_max_u32(uint32_t x) {   // max over the 4 lanes of a DPP quad
  x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false));   // quad_perm [1, 0, 3, 2]
  x = max(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false));   // quad_perm [2, 3, 0, 1]
  return x;
}

// the record quarter of slot `slot` (the quad's lanes hold slots 0..3 of one record)
__device__ __forceinline__ v3u t23_pack(float4 f, int slot) {
  const uint32_t a = max(max(__float_as_uint(f.x) & 0x7fffffffu, __float_as_uint(f.y) & 0x7fffffffu),
                         max(__float_as_uint(f.z) & 0x7fffffffu, __float_as_uint(f.w) & 0x7fffffffu));
  const int e = (int)(quad_max_u32(a) >> 23);   // uint order: NaN > Inf > finite, so 255 = non-finite
  const int E = e < 22 ? 22 : e;
  const float qm = E == 255 ? 0.0f : __uint_as_float((uint32_t)(275 - E) << 23);   // 2^(148 - E), exact
  auto q = [&](float x) { return (uint32_t)min(max((int)__builtin_rintf(x * qm), -0x3fffff), 0x3fffff) & 0x7fffffu; };
  const uint32_t m0 = q(f.x), m1 = q(f.y), m2 = q(f.z), m3 = q(f.w);
  const uint32_t nib = (slot & 1) ? (uint32_t)E >> 4 : (uint32_t)E & 15u;
  return (v3u){m0 | (m1 << 23), (m1 >> 9) | (m2 << 14), (m2 >> 18) | (m3 << 5) | (nib << 28)};
}

// inverse of t23_pack; the 4 lanes of the quad hold the record's 4 slots
__device__ __forceinline__ float4 t23_unpack(v3u d, int slot) {
  const uint32_t own = d.z >> 28;
  const uint32_t oth = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0xB1, 0xf, 0xf, false);   // slot ^ 1's nibble
  const uint32_t E = (slot & 1) ? (oth | (own << 4)) : (own | (oth << 4));
  const float mul = E == 255u ? __int_as_float(0x7fc00000) : __uint_as_float((E - 21u) << 23);   // 2^(E - 148)
  const int m0 = (int)(d.x << 9) >> 9;
  const int m1 = (int)(__builtin_amdgcn_alignbit(d.y, d.x, 23) << 9) >> 9;
  const int m2 = (int)(__builtin_amdgcn_alignbit(d.z, d.y, 14) << 9) >> 9;
  const int m3 = (int)(d.z << 4) >> 9;
  return make_float4((float)m0 * mul, (float)m1 * mul, (float)m2 * mul, (float)m3 * mul);
}
__device__ __forceinline__ int t4_index(int band4, int kx) {
#if DCTAE_TLAYOUT == 0
  return band4 * 448 + kx;
#else
  return ((band4 >> 2) * 448 + kx) * 4 + (band4 & 3);
#endif
}

// The decode's band-layout U' (k_idct_cols512b -> k_idct_rows512<448, true>),
// natural row order in the float4: the same two layouts, chosen apart
// (DCTAE_ULAYOUT 2 = band16 [y / 16][kx][16], 0 = [y / 4][kx][4]).
#ifndef DCTAE_ULAYOUT
#define DCTAE_ULAYOUT 2
#endif
static_assert(DCTAE_ULAYOUT == 0 || DCTAE_ULAYOUT == 2, "U' layouts: 0 or 2");
__device__ __forceinline__ int u4_index(int band4, int kx) {
#if DCTAE_ULAYOUT == 0
  return band4 * 448 + kx;
#else
  return ((band4 >> 2) * 448 + kx) * 4 + (band4 & 3);
#endif
}

__device__ __forceinline__ float mirror16(float x) {   // lane l <- lane 15 - l of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xf, 0xf, false));
}

// Row-pass tables (loaded once per block): W_256^{r s} and the Makhoul post
// coefficients (c1, c2, c3, c4) of rows512_item_pk.
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

// ---------------------------------------------------------------------------
// The row item with the VALU work issued as v_pk_{mul,fma,add}_f32 (two fp32
// lanes per instruction, the 157 TF vector peak; a scalar restatement measured
// ~2,850 VALU per wave against 1,815):
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
// The IPT keeps the reference's per-pixel op order (util.py:70-82); the FFT
// is tolerance-tested against the oracle and the generic plan kernels.
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

// The 256-point complex FFT of one 16-lane row group: two radix-16 passes
// with ONE LDS transpose through the group's region xr.  In: v = z[j + 16 r]
// (lane j = pass-1 butterfly j); out: v = Z[s + 16 i], s = sigma(j).  Shared
// by the row kernel and the band-layout column kernel (k_cols512b).
__device__ __forceinline__ int sigma16(int j) { return j < 8 ? j : (j < 15 ? j + 1 : 8); }

__device__ __forceinline__ void fft256_group(cf (&v)[16], cf* xr, int j, int s, const float2 (&tw2)[16][16]) {
#pragma clang fp contract(fast)
  DFTV<16>::run(v);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) xr[16 * k1 + (j ^ (k1 & 14))] = v[k1];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // pass 2: butterfly s reads z1[s + 16 r] = lane r's output s
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
  __builtin_amdgcn_wave_barrier();   // reads done before the region is written again
#pragma unroll
  for (int r = 1; r < 16; ++r) {
    const float2 w = tw2[r][s];
    v[r] = cmul_pk(v[r], (cf){w.x, w.y});
  }
  DFTV<16>::run(v);
}

// Makhoul post of step i: (X[k], X[N - k]) for k = s + 16 i from Z[s + 16 i'] in v
__device__ __forceinline__ cf makhoul_step(const cf (&v)[16], int i, int s, bool self0, bool self8,
                                           const float4* pc) {
  const cf m = (cf){mirror16(v[15 - i].x), mirror16(v[15 - i].y)};
  const cf own = self0 ? v[(16 - i) & 15] : v[15 - i];
  const cf P = (self0 || self8) ? own : m;
  const float4 cc = pc[s + 16 * i];
  return makhoul_pair(v[i], P, (cf){cc.x, cc.y}, (cf){cc.z, cc.w});
}

// two independent Makhoul pairs with their VOP3P chains interleaved: every
// dependent op is one instruction behind its producer (the separate chains of
// makhoul_pair need an s_nop between their dependent ops)
__device__ __forceinline__ void makhoul_pair2(cf A0, cf P0, float4 c0, cf A1, cf P1, float4 c1, cf& t0, cf& t1) {
  const cf c12a = (cf){c0.x, c0.y}, c34a = (cf){c0.z, c0.w}, c12b = (cf){c1.x, c1.y}, c34b = (cf){c1.z, c1.w};
  asm("v_pk_mul_f32 %0, %2, %3 op_sel_hi:[1,0] neg_hi:[1,0]\n\t"
      "v_pk_mul_f32 %1, %6, %7 op_sel_hi:[1,0] neg_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %4, %3, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
      "v_pk_fma_f32 %1, %8, %7, %1 op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
      "v_pk_fma_f32 %0, %2, %5, %0 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
      "v_pk_fma_f32 %1, %6, %9, %1 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
      "v_pk_fma_f32 %0, %4, %5, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]\n\t"
      "v_pk_fma_f32 %1, %8, %9, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=&v"(t0), "=&v"(t1)
      : "v"(A0), "v"(c12a), "v"(P0), "v"(c34a), "v"(A1), "v"(c12b), "v"(P1), "v"(c34b));
}

// steps i and i + 1 of the Makhoul post with their coefficients c0 / c1
// already loaded (the caller keeps the next pair's LDS reads in flight)
__device__ __forceinline__ void makhoul_step2(const cf (&v)[16], int i, bool self0, bool self8, float4 c0, float4 c1,
                                              cf& x0, cf& x1) {
  // partner P = the mirror lane's v[15 - i] (lanes 1 .. 14) or the lane's own
  // value (lane 0: v[(16 - i) & 15], lane 15: v[15 - i]) -- self0 / self8 are
  // lanes 0 / 15 of every 16-lane row by construction, so both selects run on
  // constant lane masks in VCC: the own value by a v_cndmask_b32, then P by a
  // v_cndmask_b32 whose first source is read through the row_mirror DPP
  (void)self0;
  (void)self8;
  float p0x, p0y, p1x, p1y, q0x, q0y, q1x, q1y;
  asm("s_mov_b32 vcc_lo, 0x00010001\n\t"
      "s_mov_b32 vcc_hi, 0x00010001\n\t"
      "v_cndmask_b32 %4, %8, %12, vcc\n\t"
      "v_cndmask_b32 %5, %9, %13, vcc\n\t"
      "v_cndmask_b32 %6, %10, %8, vcc\n\t"
      "v_cndmask_b32 %7, %11, %9, vcc\n\t"
      "s_mov_b32 vcc_lo, 0x80018001\n\t"
      "s_mov_b32 vcc_hi, 0x80018001\n\t"
      "v_cndmask_b32_dpp %0, %8, %4, vcc row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %1, %9, %5, vcc row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %2, %10, %6, vcc row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %3, %11, %7, vcc row_mirror row_mask:0xf bank_mask:0xf"
      : "=&v"(p0x), "=&v"(p0y), "=&v"(p1x), "=&v"(p1y), "=&v"(q0x), "=&v"(q0y), "=&v"(q1x), "=&v"(q1y)
      : "v"(v[15 - i].x), "v"(v[15 - i].y), "v"(v[14 - i].x), "v"(v[14 - i].y), "v"(v[(16 - i) & 15].x),
        "v"(v[(16 - i) & 15].y)
      : "vcc");
  makhoul_pair2(v[i], (cf){p0x, p0y}, c0, v[i + 1], (cf){p1x, p1y}, c1, x0, x1);
}

// 4 x 4 transpose across the four 16-lane rows of a wave: on return r[k] at
// row g holds the input r[g] of row k.  v_permlane32_swap exchanges rows 2, 3
// of its first operand with rows 0, 1 of its second; v_permlane16_swap the odd
// rows of the first with the even rows of the second (VALU, no LDS).
__device__ __forceinline__ void xpose4_rows(float (&r)[4]) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(r[0]), __float_as_uint(r[2]), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(r[1]), __float_as_uint(r[3]), false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  r[0] = __uint_as_float(c[0]);
  r[1] = __uint_as_float(c[1]);
  r[2] = __uint_as_float(d[0]);
  r[3] = __uint_as_float(d[1]);
}

// Row pass output layouts (the channel plane is H x 448 floats either way):
//  * row-major T[c][y][kx] (band = false): read by the generic column kernels;
//  * band layout T'[c][y / 4][kx][slot] (band = true, H = 512 with the
//    columns on k_cols512b), rows 4 b + (0, 2, 3, 1) in slots 0..3 -- the
//    order of the Makhoul pairs (x0, x2) / (x3, x1) that the column kernel
//    needs in adjacent registers: the four rows of a wave are one band, so after a
//    4 x 4 cross-row transpose (xpose4_rows) every lane stores a float4
//    (rows 4b .. 4b + 3 of one column) and a wave's store covers 64 adjacent
//    columns = 1 KB contiguous (7 float4 stores + one 4-byte X[M] store per
//    lane and channel, against 29 scattered 4-byte stores); k_cols512b's
//    lane j of column kx then loads rows 64 b' + 4 j .. + 3 as one float4.
template <bool band>
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
  const int s = sigma16(j);
  const bool self0 = (j == 0), self8 = (j == 15);
  // row-major stores of butterfly s: X[s + 16 i] at + 64 i, X[N - s - 16 i] at + 64 (15 - i)
  const int rowo = (y * KW + s) * 4;
  const int rown = (y * KW + (N - 15 * 16) - s) * 4;
  const int rown4 = s >= 1 ? rown : 0x7ffffff0;   // i = 4: k = 64 + s, X[N - k] kept iff s >= 1
  // band stores (bytes): after xpose4_rows lane (g, s) of block q holds the
  // wave's four rows of column s + 16 (4 q + g) (X[k]) / N - s - 16 (4 q + g) (X[N - k])
  const int bnd = (y0 >> 2) + wv;
  int bkq[4], bnq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bkq[q] = t4_index(bnd, s + 16 * (4 * q + g)) * 16;
    bnq[q] = t4_index(bnd, N - s - 16 * (4 * q + g)) * 16;
  }
  bnq[1] = (g == 0 && s == 0) ? 0x7ffffff0 : bnq[1];   // column 448 (k = 64) is not kept
  const int bm = j == 0 ? t4_index(bnd, M) * 16 + 4 * ((0x2130 >> (4 * g)) & 3) : 0x7ffffff0;   // slot of row g: 0, 3, 1, 2

#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // ---- pass 1 inputs: lane j's z[j + 16 r]; FFT of the row group
    cf v[16];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      v[b] = A[c][b];
      v[15 - b] = (cf){mirror16(B[c][b].x), mirror16(B[c][b].y)};
    }
#if DCTAE_TLAYOUT == 2
    if (band && c > 0) __syncthreads();   // the previous channel's staged-output reads (aliased on xch)
    // lane indices made opaque per channel: the transpose addresses derived
    // from them are rebuilt in each channel instead of being held across all three
    int jo = j, so = s;
    if (band) asm volatile("" : "+v"(jo), "+v"(so));
    fft256_group(v, xr, jo, so, L.tw2);
#else
    fft256_group(v, xr, j, s, L.tw2);
#endif
    // ---- Makhoul post: k = s + 16 i, A = Z[k] = v[i], P = Z[M - k]
#if DCTAE_T23
    const auto rsrc = band ? __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(T) + (int64_t)c * H * KW * 3, 0,
                                                               plane_bytes / 4 * 3, 0x00020000)
                           : __builtin_amdgcn_make_buffer_rsrc(T + (int64_t)c * H * KW, 0, plane_bytes, 0x00020000);
#else
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(T + (int64_t)c * H * KW, 0, plane_bytes, 0x00020000);
#endif
#if DCTAE_TLAYOUT == 2
    if constexpr (band) {
      // band16 layout [y / 16][kx][16 rows]: the block's 16 rows of a channel are
      // one contiguous 28 KB piece; staged through LDS (aliasing the transpose
      // regions) so every wave stores whole 1 KB pieces.  Row r = 4 w + g of
      // column kx at kx 16 + 4 (w ^ ((kx >> 1) & 3)) + slot(g) (slots 0, 3, 1, 2:
      // the column kernel's Makhoul pairs (x0, x2) / (x3, x1) adjacent; the XOR
      // spreads a group's 16 lanes over 8 bank pairs)
      float* ob = reinterpret_cast<float*>(&X.xch[0][0][0]);
      const int sg = (0x2130 >> (4 * g)) & 3;
      // (kx >> 1) & 3 of kx = s + 16 i / N - s - 16 i does not depend on i
      float* oa = ob + s * 16 + 4 * (wv ^ ((s >> 1) & 3)) + sg;              // + 256 i
      float* on = ob + (N - s) * 16 + 4 * (wv ^ (((N - s) >> 1) & 3)) + sg;  // - 256 i
      __syncthreads();   // every group's pass-2 reads of xch
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
        oa[256 * i] = x0.x;
        oa[256 * (i + 1)] = x1.x;
        if (i >= 5 || (i == 4 && s >= 1)) on[-256 * i] = x0.y;
        if (i + 1 >= 5) on[-256 * (i + 1)] = x1.y;
        // without it the post-coefficient reads of later pairs are all hoisted up
        if ((i & 3) == 2) __builtin_amdgcn_sched_barrier(0);
      }
      if (self0) {
        const float4 cc = L.pc[M];
        ob[M * 16 + 4 * wv + sg] = (cc.x + cc.y) * v[0].x + (cc.w - cc.z) * v[0].y;   // (M >> 1) & 3 = 0
      }
      __syncthreads();
      // wave wv stores 16-column chunks wv * 7 .. wv * 7 + 6 (1 KB each)
      const int l = tid & 63;
      const int kx0 = 112 * wv + (l >> 2), qd = l & 3;   // + 16 it; (kx >> 1) & 3 = (l >> 3) & 3
      const float4* rd = reinterpret_cast<const float4*>(ob + kx0 * 16 + 4 * (qd ^ ((l >> 3) & 3)));
#if DCTAE_T23
      const int go = (((y0 >> 4) * KW + kx0) * 4 + qd) * 12;
#pragma unroll
      for (int it = 0; it < 7; ++it)
        __builtin_amdgcn_raw_buffer_store_b96(t23_pack(rd[64 * it], qd), rsrc, go, 768 * it, DCTAE_T_ST_AUX);
#else
      const int go = (((y0 >> 4) * KW + kx0) * 4 + qd) * 16;
#pragma unroll
      for (int it = 0; it < 7; ++it)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, rd[64 * it]), rsrc, go, 1024 * it, DCTAE_T_ST_AUX);
#endif
      __builtin_amdgcn_sched_barrier(0);   // keep the next channel's inputs from being built up here
    } else
#endif
    if constexpr (band) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float rk[4], rn[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const cf xx = makhoul_step(v, 4 * q + t, s, self0, self8, L.pc);
          rk[t] = xx.x;
          rn[t] = xx.y;
        }
        xpose4_rows(rk);
        __builtin_amdgcn_raw_buffer_store_b128(
            (v4u){__float_as_uint(rk[0]), __float_as_uint(rk[2]), __float_as_uint(rk[3]), __float_as_uint(rk[1])},
            rsrc, bkq[q], 0, 0);
        if (q >= 1) {   // X[N - k], k = s + 16 i, is kept for k > 64
          xpose4_rows(rn);
          __builtin_amdgcn_raw_buffer_store_b128(
              (v4u){__float_as_uint(rn[0]), __float_as_uint(rn[2]), __float_as_uint(rn[3]), __float_as_uint(rn[1])},
              rsrc, bnq[q], 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const cf xx = makhoul_step(v, i, s, self0, self8, L.pc);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.x), rsrc, rowo, 64 * i, 0);
        if (i >= 5) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.y), rsrc, rown, 64 * (15 - i), 0);
        if (i == 4) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xx.y), rsrc, rown4, 64 * 11, 0);
      }
    }
    // k = M (s = 0, lane 0): A = P = Z[0]: X[M] = (c1 + c2) Z0.x + (c4 - c3) Z0.y
    if (!(band && DCTAE_TLAYOUT == 2)) {   // band16: X[M] went through LDS
      const float4 cc = L.pc[M];
      const float xm = (cc.x + cc.y) * v[0].x + (cc.w - cc.z) * v[0].y;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xm), rsrc,
                                            band ? bm : (self0 ? (y * KW + M) * 4 : 0x7ffffff0), 0, 0);
    }
  }
}

}  // namespace dctae
