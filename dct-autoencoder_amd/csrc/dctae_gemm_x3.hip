// k_gemm_x3: the batched strided DCT GEMM of dctae_kernels.hip (k_gemm_f32,
//   O[c][m][n] = sum_k A[c][m][k] B[c][n][k])
// on the bf16 MFMA at fp32 accuracy.  Every operand element is split into
// three bf16 pieces a = a0 + a1 + a2 (a0 = bf16(a), a1 = bf16(a - a0),
// a2 = bf16(a - a0 - a1): 24 significant bits, as fp32) and the product keeps
// the six terms whose piece orders sum to <= 2,
//   a0 b0 + a0 b1 + a1 b0 + a1 b1 + a0 b2 + a2 b0,
// accumulated in fp32 by v_mfma_f32_32x32x16_bf16 (the dropped terms are
// ~2^-24 of |a b|).  Six bf16 MFMAs per 16-deep k step cost 6 x 32 cycles
// against 8 x 64 for the same step on v_mfma_f32_32x32x2_f32.  Measured
// against float64 on the orthonormal DCT: ~5e-8 of max |Y| (fp32 GEMM ~6e-7).
//
// Tiles as k_gemm_f32: 64 x 64 per workgroup, 4 waves of 32 x 32, K chunks of
// 32 (two k steps), the next chunk's global loads in flight during the MFMAs.
// Staging, per operand and channel:
//   * the shared DCT matrix comes pre-split (GemmProblem::Xs, three zero-padded
//     bf16 planes built once with the matrix): three 16-byte loads and LDS
//     writes per thread, no arithmetic;
//   * an fp32 operand whose k is contiguous: thread (row tid / 4, k 8 (tid % 4))
//     reads 8 floats as two 16-byte buffer loads;
//   * otherwise (row-contiguous, e.g. T of the column GEMM, stride +-Kw along
//     k): thread (row tid % 64, k 8 (tid / 64)), 8 four-byte loads that
//     coalesce across the wave's 64 rows;
//   then v_cvt_pk_bf16_f32 splits (the plain vector casts compile to it) and
//   three 16-byte LDS writes.  Buffer resources span exactly the operand's
//   element range, so rows past M / N and k past the range read 0; k past K
//   inside the range is zeroed in the last chunk only.
// LDS rows are 40 bf16 (80 bytes): the 32 lanes of a ds_read_b128 fragment
// group hit distinct banks, as do the 16-byte staging writes.
#include "dctae_launch.h"
#include "dctae_device.h"

#include <cmath>

namespace dctae {

namespace {

constexpr int XK = 32;        // k chunk
constexpr int kOob = 0x7ffffff0;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 hv8 __attribute__((ext_vector_type(8)));

// LDS image of one operand tile: three bf16 pieces of ROWS x 32 k, rows of
// 64 bytes, the 16-byte k group kq of row r at slot kq ^ swz(r).  With this
// swizzle the 16-lane groups of a ds_read_b128 fragment read, the 8-lane
// groups of the staging ds_write_b128 (two rows x four k groups, or eight rows
// x one k group) all hit distinct banks (exhaustive check over the lane
// groups of MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ int swz(int r) { return ((r >> 1) ^ (r >> 2)) & 3; }
__device__ __forceinline__ int lds_off(int r, int kq) { return r * XK + 8 * (kq ^ swz(r)); }

template <int ROWS, int NP = 3>
struct Pieces {
  uint16_t p[NP][ROWS * XK];
};

// one fp32 operand (64 rows x depth k) of one channel, as this thread stages it
struct Src {
  __amdgpu_buffer_rsrc_t rsrc;
  int voff;    // byte offset of this thread's (row, first k) from the range start; kOob for a row past the edge
  int kstep;   // bytes per k
  bool kc;     // k contiguous
  int kq;      // this thread's k group (8 kq)
  int row;     // this thread's row in the 64-row block
};

// rows [r0, r0 + 64) of X[r][k] = base[r * sr + k * sk], r < R, k < K
__device__ __forceinline__ Src make_src(const float* base, int64_t sr, int64_t sk, int r0, int R, int K) {
  Src s;
  s.kc = (sk == 1);
  const int tid = threadIdx.x;
  s.row = s.kc ? (tid >> 2) : (tid & 63);
  s.kq = s.kc ? (tid & 3) : (tid >> 6);
  // element range of the whole operand: [lo, hi]
  const int64_t lo = (sr < 0 ? (int64_t)(R - 1) * sr : 0) + (sk < 0 ? (int64_t)(K - 1) * sk : 0);
  const int64_t hi = (sr > 0 ? (int64_t)(R - 1) * sr : 0) + (sk > 0 ? (int64_t)(K - 1) * sk : 0);
  s.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + lo), 0, (int)((hi - lo + 1) * 4), 0x00020000);
  s.kstep = (int)(sk * 4);
  const int r = r0 + s.row;
  s.voff = r < R ? (int)(((int64_t)r * sr + (int64_t)(8 * s.kq) * sk - lo) * 4) : kOob;
  return s;
}

__device__ __forceinline__ f32x8 load_src(const Src& s, int k0, int K) {
  f32x8 v;
#if defined(DCTAE_PROFILING) && defined(DCTAE_GEMM_ABL) && (DCTAE_GEMM_ABL & 2)
  // profiling ablation: no fp32 operand loads (wrong output)
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.001f * (float)(s.row + e + k0);
  return v;
#endif
  if (s.kc) {
#if defined(DCTAE_PROFILING) && defined(DCTAE_GEMM_ABL) && (DCTAE_GEMM_ABL & 4)
    const int o = (s.voff + k0 * 4) & 0x3fff0;   // profiling ablation: every tile reads a 256 KB window (L2-resident)
#else
    const int o = s.voff + k0 * 4;
#endif
    const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(s.rsrc, o, 0, 0));
    const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(s.rsrc, o + 16, 0, 0));
    v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#if defined(DCTAE_PROFILING) && defined(DCTAE_GEMM_ABL) && (DCTAE_GEMM_ABL & 4)
      v[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(s.rsrc, (s.voff + (k0 + e) * s.kstep) & 0x3fffc, 0, 0));
#else
      v[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(s.rsrc, s.voff + (k0 + e) * s.kstep, 0, 0));
#endif
  }
  if (k0 + XK > K) {   // last chunk: k past K inside the range
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (k0 + 8 * s.kq + e >= K) v[e] = 0.0f;
  }
  return v;
}

template <int ROWS>
__device__ __forceinline__ void split_store(Pieces<ROWS, 3>& L, const Src& s, int rbase, f32x8 v, float) {
  const bfv8 h0 = __builtin_convertvector(v, bfv8);
  const f32x8 r1 = v - __builtin_convertvector(h0, f32x8);
  const bfv8 h1 = __builtin_convertvector(r1, bfv8);
  const f32x8 r2 = r1 - __builtin_convertvector(h1, f32x8);
  const bfv8 h2 = __builtin_convertvector(r2, bfv8);
  const int o = lds_off(rbase + s.row, s.kq);
  *reinterpret_cast<bfv8*>(&L.p[0][o]) = h0;
  *reinterpret_cast<bfv8*>(&L.p[1][o]) = h1;
  *reinterpret_cast<bfv8*>(&L.p[2][o]) = h2;
}

// k_gemm_h2: v scaled by the exact power of two `scale` (so its largest
// magnitude is below 2^14), then two fp16 pieces h0 = fp16(v), h1 = fp16(v - h0)
template <int ROWS>
__device__ __forceinline__ void split_store(Pieces<ROWS, 2>& L, const Src& s, int rbase, f32x8 v, float scale) {
  const f32x8 vs = v * scale;
  const hv8 h0 = __builtin_convertvector(vs, hv8);
#if defined(DCTAE_PROFILING) && defined(DCTAE_GEMM_ABL) && (DCTAE_GEMM_ABL & 1)
  const hv8 h1 = h0;   // profiling ablation: no residual piece (wrong output)
#else
  const f32x8 r1 = vs - __builtin_convertvector(h0, f32x8);
  const hv8 h1 = __builtin_convertvector(r1, hv8);
#endif
  const int o = lds_off(rbase + s.row, s.kq);
  *reinterpret_cast<hv8*>(&L.p[0][o]) = h0;
  *reinterpret_cast<hv8*>(&L.p[1][o]) = h1;
}

// pre-split planes, ROWS rows: thread slot i = tid + 256 j -> (row i / 4, k group i % 4)
template <int ROWS, int NP = 3>
struct PreSplit {
  u32x4 v[ROWS / 64][NP];
};

// buffer loads (a plain load through the pointer read from the problem struct
// compiles to flat_load, which also counts in lgkmcnt: the first LDS wait of
// the chunk's MFMAs then waited for these global loads too)
template <int ROWS, int NP>
__device__ __forceinline__ void load_pre(PreSplit<ROWS, NP>& q, const GemmProblem& p, int r0, int k0) {
  const int tid = threadIdx.x;
  const uint16_t* planes = NP == 3 ? p.Xs : p.Xh;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(planes), 0, (int)(NP * p.xs_plane * 2), 0x00020000);
#pragma unroll
  for (int j = 0; j < ROWS / 64; ++j) {
    const int o = ((r0 + 64 * j + (tid >> 2)) * p.xs_ld + k0 + 8 * (tid & 3)) * 2;
#pragma unroll
    for (int i = 0; i < NP; ++i)
      q.v[j][i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o + (int)(i * p.xs_plane * 2), 0, 0));
  }
}

template <int ROWS, int NP>
__device__ __forceinline__ void store_pre(Pieces<ROWS, NP>& L, const PreSplit<ROWS, NP>& q) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < ROWS / 64; ++j) {
    const int o = lds_off(64 * j + (tid >> 2), tid & 3);
#pragma unroll
    for (int i = 0; i < NP; ++i) *reinterpret_cast<u32x4*>(&L.p[i][o]) = q.v[j][i];
  }
}

template <int ROWS, int NP>
__device__ __forceinline__ void read_frag(bf16x8 (&f)[NP], const Pieces<ROWS, NP>& L, int r, int kq) {
  const int o = lds_off(r, kq);
#pragma unroll
  for (int q = 0; q < NP; ++q) f[q] = *reinterpret_cast<const bf16x8*>(&L.p[q][o]);
}

// k_gemm_h2: the three fp16 products of piece order <= 1, small terms first
__device__ __forceinline__ void mfma_pieces(floatx16& acc, const bf16x8 (&a)[2], const bf16x8 (&b)[2]) {
  const hv8 a0 = __builtin_bit_cast(hv8, a[0]), a1 = __builtin_bit_cast(hv8, a[1]);
  const hv8 b0 = __builtin_bit_cast(hv8, b[0]), b1 = __builtin_bit_cast(hv8, b[1]);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
}

// six split products, small terms first
__device__ __forceinline__ void mfma_pieces(floatx16& acc, const bf16x8 (&a)[3], const bf16x8 (&b)[3]) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

}  // namespace

// SH: 0 none shared (NC operands each, 64 x 64 tiles), 1 B shared (64 x 128
// tiles), 2 A shared (128 x 64 tiles): the tile is 128 wide along the shared
// operand, so the per-channel operand's split (the VALU part of the staging)
// serves twice the MFMAs.  PRE: the shared operand is read pre-split (p.Xs);
// the two forms are separate bodies so that only one form's staging registers
// are live.  4 waves in 2 x 2, each (TM / 2) x (TN / 2) of every channel.
template <int NC, int SH>
struct X3Shape {
  static constexpr int NA = SH == 2 ? 1 : NC, NB = SH == 1 ? 1 : NC;
  static constexpr int TM = SH == 2 ? 128 : 64, TN = SH == 1 ? 128 : 64;
};

template <int NC, int SH, bool PRE, int NP = 3>
__device__ __forceinline__ void gemm_x3_body(const GemmProblem& p, int tm, int tn,
                                             Pieces<X3Shape<NC, SH>::TM, NP> (&As)[X3Shape<NC, SH>::NA],
                                             Pieces<X3Shape<NC, SH>::TN, NP> (&Bs)[X3Shape<NC, SH>::NB]) {
  using S = X3Shape<NC, SH>;
  static_assert(NP == 3 || (PRE && SH != 0), "k_gemm_h2: the shared operand comes pre-split");
  // k_gemm_h2: the per-channel operand scaled by 2^ea so its |max| < 2^14 (fp16
  // range with headroom; |max| from p.amax, a non-finite or zero max leaves it
  // unscaled), the output unscaled by 2^-(ea + xh_exp): exact powers of two
  float scale = 1.0f, unscale = 1.0f;
  if constexpr (NP == 2) {
    const uint32_t mb = *p.amax;
    int ea = 0;
    if (mb != 0u && mb < 0x7f800000u) {
      int e;
      frexpf(__uint_as_float(mb), &e);   // max in [2^(e-1), 2^e)
      ea = min(max(14 - e, -100), 100);
    }
    scale = ldexpf(1.0f, ea);
    unscale = ldexpf(1.0f, -(ea + p.xh_exp));
  }
  constexpr int NA = S::NA, NB = S::NB, TM = S::TM, TN = S::TN;
  constexpr int BM = TM / 64, BN = TN / 64;   // 32 x 32 MFMA blocks per wave, per dimension
  constexpr bool preA = PRE && SH == 2, preB = PRE && SH == 1;
  constexpr int SAM = preA ? 0 : BM, SBN = preB ? 0 : BN;   // fp32 sources per channel
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int half = lane >> 5, l32 = lane & 31;

  Src sa[NA][SAM > 0 ? SAM : 1], sb[NB][SBN > 0 ? SBN : 1];
#pragma unroll
  for (int c = 0; c < NA; ++c)
#pragma unroll
    for (int j = 0; j < SAM; ++j) sa[c][j] = make_src(p.A + (int64_t)c * p.sAc, p.sAm, p.sAk, m0 + 64 * j, p.M, p.K);
#pragma unroll
  for (int c = 0; c < NB; ++c)
#pragma unroll
    for (int j = 0; j < SBN; ++j) sb[c][j] = make_src(p.B + (int64_t)c * p.sBc, p.sBn, p.sBk, n0 + 64 * j, p.N, p.K);

  floatx16 acc[NC][BM][BN];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < BM; ++i)
#pragma unroll
      for (int j = 0; j < BN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][i][j][r] = 0.0f;

  f32x8 va[NA][SAM > 0 ? SAM : 1], vb[NB][SBN > 0 ? SBN : 1];
  PreSplit<TM, NP> qa;
  PreSplit<TN, NP> qb;
  auto load = [&](int k0) {
    if constexpr (preA) load_pre(qa, p, m0, k0);
#pragma unroll
    for (int c = 0; c < NA; ++c)
#pragma unroll
      for (int j = 0; j < SAM; ++j) va[c][j] = load_src(sa[c][j], k0, p.K);
    if constexpr (preB) load_pre(qb, p, n0, k0);
#pragma unroll
    for (int c = 0; c < NB; ++c)
#pragma unroll
      for (int j = 0; j < SBN; ++j) vb[c][j] = load_src(sb[c][j], k0, p.K);
  };
  auto store = [&]() {
    if constexpr (preA) store_pre(As[0], qa);
#pragma unroll
    for (int c = 0; c < NA; ++c)
#pragma unroll
      for (int j = 0; j < SAM; ++j) split_store(As[c], sa[c][j], 64 * j, va[c][j], scale);
    if constexpr (preB) store_pre(Bs[0], qb);
#pragma unroll
    for (int c = 0; c < NB; ++c)
#pragma unroll
      for (int j = 0; j < SBN; ++j) split_store(Bs[c], sb[c][j], 64 * j, vb[c][j], scale);
  };
  load(0);
  store();
  __syncthreads();
  for (int k0 = 0; k0 < p.K; k0 += XK) {
    const bool more = k0 + XK < p.K;
    if (more) load(k0 + XK);
    if constexpr (SH != 0) {
      // Software-pipelined fragment reads: the chunk is 2 k steps x NC
      // channels = 2 NC units; a unit's MFMAs run while the next unit's
      // fragments are read (its "own" per-channel fragment, and at a step
      // boundary the next step's shared-matrix fragments), so a unit waits
      // only for LDS reads issued one unit earlier.  (Reads issued just
      // before the MFMAs that consume them capped the kernel at ~40 % of the
      // MFMA peak; with the reads removed it ran 1.54x faster.)
      constexpr int X = NB == 1 ? BN : BM;   // shared-side 32-blocks per wave
      auto rd_shared = [&](bf16x8 (&f)[X][NP], int st) {
        const int kq = 2 * st + half;
#pragma unroll
        for (int x = 0; x < X; ++x) {
          if constexpr (NB == 1) read_frag(f[x], Bs[0], wn * (TN / 2) + 32 * x + l32, kq);
          else read_frag(f[x], As[0], wm * (TM / 2) + 32 * x + l32, kq);
        }
      };
      auto rd_own = [&](bf16x8 (&f)[NP], int st, int c) {
        const int kq = 2 * st + half;
        if constexpr (NB == 1) read_frag(f, As[c], wm * (TM / 2) + l32, kq);
        else read_frag(f, Bs[c], wn * (TN / 2) + l32, kq);
      };
      auto mm = [&](const bf16x8 (&sh)[X][NP], const bf16x8 (&ow)[NP], int c) {
#pragma unroll
        for (int x = 0; x < X; ++x) {
          if constexpr (NB == 1) mfma_pieces(acc[c][0][x], ow, sh[x]);
          else mfma_pieces(acc[c][x][0], sh[x], ow);
        }
      };
      bf16x8 sh0[X][NP], sh1[X][NP], ow[2][NP];
      rd_shared(sh0, 0);
      rd_own(ow[0], 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < NC; ++c) {   // step 0: units 0 .. NC - 1
        if (c + 1 < NC) {
          rd_own(ow[(c + 1) & 1], 0, c + 1);
        } else {
          rd_shared(sh1, 1);
          rd_own(ow[(c + 1) & 1], 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the prefetch reads ahead of this unit's MFMAs
        mm(sh0, ow[c & 1], c);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {   // step 1: units NC .. 2 NC - 1
        if (c + 1 < NC) rd_own(ow[(NC + c + 1) & 1], 1, c + 1);
        __builtin_amdgcn_sched_barrier(0);
        mm(sh1, ow[(NC + c) & 1], c);
      }
    } else {
#pragma unroll
      for (int s = 0; s < XK / 16; ++s) {
        const int kq = 2 * s + half;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          bf16x8 a[NP], b[NP];
          read_frag(a, As[c], wm * 32 + l32, kq);
          read_frag(b, Bs[c], wn * 32 + l32, kq);
          mfma_pieces(acc[c][0][0], a, b);
        }
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  if constexpr (NP == 2) {
    uint32_t mx = 0;   // |max| of the outputs in uint order (NaN above Inf above finite)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < BM; ++i)
#pragma unroll
        for (int j = 0; j < BN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            acc[c][i][j][r] *= unscale;
            mx = max(mx, __float_as_uint(acc[c][i][j][r]) & 0x7fffffffu);
          }
    if (p.omax) {   // padded rows / columns accumulate zeros: no mask needed; one atomic per block
      __shared__ uint32_t part[4];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
      if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mx;
      __syncthreads();
      if (threadIdx.x == 0) atomicMax(p.omax, max(max(part[0], part[1]), max(part[2], part[3])));
    }
  }
  // C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  // Row-major outputs (a row's extent within the row stride): buffer stores
  // on the channel's output range, one 32-bit lane offset per (i, j) plus a
  // uniform row step; rows past M land past the range and columns past N get
  // an out-of-range offset, so no per-store predicate or 64-bit address math
  const int64_t ext = (int64_t)(p.M - 1) * p.sOm + (int64_t)(p.N - 1) * p.sOn + 1;
  if (p.sOm > 0 && p.sOn > 0 && p.sOm >= (int64_t)(p.N - 1) * p.sOn + 1 && (ext + 160 * p.sOm) * 4 < kOob) {
    const int sOm4 = (int)(p.sOm * 4);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.O + (int64_t)c * p.sOc, 0, (int)(ext * 4), 0x00020000);
#pragma unroll
      for (int i = 0; i < BM; ++i)
#pragma unroll
        for (int j = 0; j < BN; ++j) {
          const int gm = m0 + wm * (TM / 2) + 32 * i + 4 * half, gn = n0 + wn * (TN / 2) + 32 * j + l32;
          const int vo = gn < p.N ? gm * sOm4 + (int)(gn * p.sOn * 4) : kOob;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[c][i][j][r]), rsrc,
                                                  vo + ((r & 3) + 8 * (r >> 2)) * sOm4, 0, 0);
        }
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float* O = p.O + (int64_t)c * p.sOc;
#pragma unroll
    for (int i = 0; i < BM; ++i)
#pragma unroll
      for (int j = 0; j < BN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
          const int gm = m0 + wm * (TM / 2) + 32 * i + row, gn = n0 + wn * (TN / 2) + 32 * j + l32;
          if (gm < p.M && gn < p.N) O[(int64_t)gm * p.sOm + (int64_t)gn * p.sOn] = acc[c][i][j][r];
        }
  }
}

template <int NC, int SH>
__global__ __launch_bounds__(256, (SH == 0 && NC == 3) ? 1 : 2) void k_gemm_x3(const GemmProblem* __restrict__ probs,
                                                                             const TileRef* __restrict__ tiles) {
  using S = X3Shape<NC, SH>;
  __shared__ Pieces<S::TM> As[S::NA];
  __shared__ Pieces<S::TN> Bs[S::NB];
  const TileRef tr = tiles[blockIdx.x];
  if (tr.problem < 0) return;   // padding of an XCD-dealt list
  const GemmProblem p = probs[tr.problem];
  const int tm = tr.tile / p.tiles_n, tn = tr.tile % p.tiles_n;
  if (SH != 0 && p.Xs != nullptr)
    gemm_x3_body<NC, SH, true>(p, tm, tn, As, Bs);
  else
    gemm_x3_body<NC, SH, false>(p, tm, tn, As, Bs);
}

// k_gemm_h2: the encode's DCT GEMMs on fp16 MFMAs with two-piece operands and
// three products (a1 b0 + a0 b1 + a0 b0): each operand scaled by a power of
// two into the fp16 range, so a piece pair carries 22 significant bits and
// the dropped terms (a1 b1, the pieces' residuals) are <= 3 x 2^-22 |a b|
// (~0.1 of the fp32 rounding of k_gemm_f32's sums; half the MFMAs of k_gemm_x3)
#ifndef DCTAE_H2_WPE
#define DCTAE_H2_WPE 2
#endif
template <int NC, int SH>
__global__ __launch_bounds__(256, DCTAE_H2_WPE) void k_gemm_h2(const GemmProblem* __restrict__ probs,
                                                  const TileRef* __restrict__ tiles) {
  using S = X3Shape<NC, SH>;
  __shared__ Pieces<S::TM, 2> As[S::NA];
  __shared__ Pieces<S::TN, 2> Bs[S::NB];
  const TileRef tr = tiles[blockIdx.x];
  if (tr.problem < 0) return;   // padding of an XCD-dealt list
  const GemmProblem p = probs[tr.problem];
  const int tm = tr.tile / p.tiles_n, tn = tr.tile % p.tiles_n;
  gemm_x3_body<NC, SH, true, 2>(p, tm, tn, As, Bs);
}

// k_gemm_h2r: k_gemm_h2<3, 1> (the encode's row GEMM: A = the folded IPT of
// the three channels, k contiguous; B = the pre-split half DCT matrix) with
// both operands streamed global -> LDS by buffer_load ... lds: no staging
// registers and no store phase.  A two-stage LDS ring of [A fp32 3 x 64 x 32 |
// B fp16 2 planes x 128 x 32] (40 KB per stage: two blocks per CU), the next
// chunk in flight during the current one's MFMAs, one barrier per chunk; A's
// fp32 fragments are scaled and split into the two fp16 pieces in registers
// (k past K zeroed there).  The ablations of k_gemm_h2 put ~0.75
// ms of config 4's 2.3 ms row GEMM in its register-staged A loads.
// LDS slots: an A row is 8 slots of 4 floats, slot s of row r at s ^ ((r >> 1) & 7)
// (the 16 rows of a 16-lane ds_read_b128 group then cover the 16 slot
// positions of the 256-byte bank window: with s ^ (r & 7) rows r and r + 8
// collided, PMC 37 % of the kernel's LDS cycles in bank conflicts);
// a B row 4 slots of 8 halves at kq ^ swz(r), as Pieces.
#ifndef DCTAE_GEMM_DMA
#define DCTAE_GEMM_DMA 1
#endif
#ifndef DCTAE_GEMM_DMA_BR   // the matrix fragments in registers (needs NS >= 3)
#define DCTAE_GEMM_DMA_BR 0
#endif
#ifndef DCTAE_GEMM_DMA_NS   // ring stages
#define DCTAE_GEMM_DMA_NS 2
#endif
typedef __attribute__((address_space(3))) void lds_void_t;

// NS ring stages; BR: the pre-split matrix's fragments loaded straight into
// registers one chunk ahead (the ring then holds the image operand only)
template <int NS, bool BR>
struct H2rShape {
  static constexpr int NC = 3, TM = 64, TN = 128;
  static constexpr int A_CH = TM * XK * 4;                  // 8 KB per channel
  static constexpr int A_BYTES = NC * A_CH;                 // 24 KB
  static constexpr int B_PL = TN * XK * 2;                  // 8 KB per plane
  static constexpr int STAGE = A_BYTES + (BR ? 0 : 2 * B_PL);
  static constexpr int BPC = (160 * 1024) / (NS * STAGE) < 4 ? (160 * 1024) / (NS * STAGE) : 4;   // blocks per CU
  static constexpr int NDMA_A = 2 * NC;                     // buffer_load ... lds per wave per chunk: image
  static constexpr int NDMA = NDMA_A + (BR ? 0 : 4);        //   ... and matrix
};

// Workgroup barrier for LDS hand-offs only: this wave's LDS writes done, then
// s_barrier.  __syncthreads() is a release fence as well, which on gfx9
// (loads and stores share vmcnt) waits for EVERY outstanding vector memory
// operation -- the prefetched loads in flight included -- so with it no load
// or LDS-DMA chunk could stay in flight across a chunk's barriers.  Users wait
// for their own LDS-DMA chunks (wait_vm) before it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One 16-byte-per-lane buffer_load ... lds (lane i -> lds + 16 i), written
// out so the compiler does not see an LDS DMA in flight: it otherwise waits
// for every outstanding vector load (vmcnt(0)) before the next LDS read it
// cannot prove disjoint, prefetched register loads included.  The caller
// waits for the chunk (wait_vm) before its barrier.  rsrc: the raw buffer
// descriptor words (base, num_records, 0x00020000).
// The s_nop: nothing inside an asm string gets the wait states hipcc adds to
// its own instructions (cdna_hip_programming.md, "What hipcc does not do" 2):
// an LDS DMA needs one after the s_mov to M0, and a descriptor or soffset SGPR
// written by VALU (readfirstlane) needs five before a buffer instruction reads
// it.  Without them a piece could land at the previous M0 -- seen as rare
// run-to-run differences of a few tokens on the config-4 batch.
__device__ __forceinline__ void dma_lds16(u32x4 rsrc, const void* lds, int voff) {
  const uint32_t m0 = (uint32_t)(uintptr_t)lds;
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc), "{m0}"(m0) : "memory");
}
__device__ __forceinline__ u32x4 rsrc_words(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  u32x4 r;
  r[0] = (uint32_t)a;
  r[1] = (uint32_t)(a >> 32) & 0xffffu;   // stride 0
  r[2] = bytes;
  r[3] = 0x00020000u;
  return r;
}

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt in bits 3:0 and 15:14, expcnt and lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int NS, bool BR>
__global__ __launch_bounds__(256, (H2rShape<NS, BR>::BPC)) void k_gemm_h2r(const GemmProblem* __restrict__ probs,
                                                                        const TileRef* __restrict__ tiles) {
  using S = H2rShape<NS, BR>;
  constexpr int NC = S::NC, TM = S::TM, TN = S::TN, A_CH = S::A_CH, A_BYTES = S::A_BYTES, B_PL = S::B_PL;
  constexpr int STAGE = S::STAGE;
  static_assert(S::BPC >= 1 && NS >= 2, "k_gemm_h2r: ring");
  static_assert(!BR || NS >= 3, "k_gemm_h2r: BR waits assume a chunk in flight behind the matrix loads");
  __shared__ __attribute__((aligned(16))) uint8_t ring[NS * STAGE];
  const TileRef tr = tiles[blockIdx.x];
  if (tr.problem < 0) return;   // padding of an XCD-dealt list
  const GemmProblem p = probs[tr.problem];
  const int tm = tr.tile / p.tiles_n, tn = tr.tile % p.tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1, half = lane >> 5, l32 = lane & 31;
  // the per-channel operand scaled by 2^ea (|max| < 2^14), the output unscaled (gemm_x3_body)
  // (v_ldexp_f32 on the fragments: exact as the multiply, and beside MFMAs a
  // packed f32 multiply costs ~5x its issue slot, MI355X_MICROARCH.md)
  int ea = 0;
  {
    const uint32_t mb = *p.amax;
    if (mb != 0u && mb < 0x7f800000u) {
      int e;
      frexpf(__uint_as_float(mb), &e);
      ea = min(max(14 - e, -100), 100);
    }
  }
  const float unscale = ldexpf(1.0f, -(ea + p.xh_exp));
  // A: channel c's element range [0, (M - 1) sAm + K - 1] (sAk = 1, sAm > 0);
  // wave-instruction j of this wave: channel j / 2, rows 8 rg + lane / 8 with
  // rg = 4 (j & 1) + wave, LDS slot lane % 8 = k slot (lane % 8) ^ ((row >> 1) & 7);
  // rows past M: an offset past the range (the load returns 0, no access)
  const int64_t a_ext = (int64_t)(p.M - 1) * p.sAm + p.K;
  // (with a template-dependent size this array made the host pass drop the
  // kernel's launch stub without a diagnostic: undefined symbol at load time)
  __amdgpu_buffer_rsrc_t arsrc[3];
#pragma unroll
  for (int c = 0; c < NC; ++c)
    arsrc[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.A + (int64_t)c * p.sAc), 0, (int)(a_ext * 4),
                                                 0x00020000);
  int aoff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * (4 * h + wave) + (lane >> 3), s8 = (lane & 7) ^ ((row >> 1) & 7);
    aoff[h] = m0 + row < p.M ? (int)(((int64_t)(m0 + row) * p.sAm + 4 * s8) * 4) : kOob;
  }
  // B: the planes are padded (Rp rows, xs_ld k), so every matrix load of a tile is in range
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.Xh), 0, (int)(2 * p.xs_plane * 2),
                                                      0x00020000);
  const int xsp2 = (int)(p.xs_plane * 2);
  // in the ring: plane j / 2, rows 16 rg + lane / 4 (rg = 4 (j & 1) + wave), LDS
  // slot lane % 4 = k quad (lane % 4) ^ swz(row)
  int boff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 16 * (4 * h + wave) + (lane >> 2), kq = (lane & 3) ^ swz(row);
    boff[h] = ((n0 + row) * p.xs_ld + 8 * kq) * 2;
  }
  // in registers (BR): this lane's fragments, rows wn 64 + 32 x + l32, k quad 2 ks + half
  const int bro = ((n0 + wn * 64 + l32) * p.xs_ld + 8 * half) * 2;
  auto dma = [&](int st, int k0) {
    uint8_t* base = ring + st * STAGE;
#pragma unroll
    for (int j = 0; j < 2 * NC; ++j) {
      const int c = j >> 1, h = j & 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc[c], (lds_void_t*)(base + c * A_CH + (4 * h + wave) * 1024), 16,
                                               (int)((uint32_t)aoff[h] + (uint32_t)k0 * 4u), 0, 0, 0);
    }
    if constexpr (!BR) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pl = j >> 1, h = j & 1;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void_t*)(base + A_BYTES + pl * B_PL + (4 * h + wave) * 1024),
                                                 16, boff[h] + k0 * 2 + pl * xsp2, 0, 0, 0);
      }
    }
  };
  typedef bf16x8 BFrag[XK / 16][2][2];   // [ks][x][plane]
  auto load_b = [&](BFrag& f, int k0) {
#pragma unroll
    for (int ks = 0; ks < XK / 16; ++ks)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          f[ks][x][pl] = __builtin_bit_cast(
              bf16x8, __builtin_amdgcn_raw_buffer_load_b128(brsrc, bro + (32 * x * p.xs_ld + k0 + 16 * ks) * 2 + pl * xsp2,
                                                            0, 0));
  };
  floatx16 acc[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][x][r] = 0.0f;
  const int ra = wm * 32 + l32;   // this lane's A row in the tile
  auto compute = [&](int st, int k0, const BFrag& bf) {
    const uint8_t* base = ring + st * STAGE;
    const float* Af = reinterpret_cast<const float*>(base);
    const uint16_t* Bp = reinterpret_cast<const uint16_t*>(base + A_BYTES);
#pragma unroll
    for (int ks = 0; ks < XK / 16; ++ks) {
      const int kq = 2 * ks + half;
      bf16x8 b[2][2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int rb = wn * 64 + 32 * x + l32;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          b[x][pl] = BR ? bf[ks][x][pl] : *reinterpret_cast<const bf16x8*>(Bp + pl * (B_PL / 2) + rb * XK + 8 * (kq ^ swz(rb)));
      }
      const int kb = k0 + 8 * kq;   // this lane's first k
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float* ar = Af + c * (A_CH / 4) + ra * XK;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(ar + 4 * ((2 * kq) ^ ((ra >> 1) & 7)));
        const f32x4 hi = *reinterpret_cast<const f32x4*>(ar + 4 * ((2 * kq + 1) ^ ((ra >> 1) & 7)));
        f32x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        if (k0 + XK > p.K) {   // the last chunk (uniform): k past K (the bytes after the row's range) -> 0
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = kb + e < p.K ? v[e] : 0.0f;
        }
        f32x8 vs;
#pragma unroll
        for (int e = 0; e < 8; ++e) vs[e] = ldexpf(v[e], ea);
        const hv8 h0 = __builtin_convertvector(vs, hv8);
        // the residual vs - h0 (exact) as one mixed-precision FMA per value
        // (written out: the compiler forms cvt + sub, then packs the subs)
        const u32x4 hw = __builtin_bit_cast(u32x4, h0);
        f32x8 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r[2 * e]) : "v"(hw[e]), "v"(vs[2 * e]));
          asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r[2 * e + 1]) : "v"(hw[e]), "v"(vs[2 * e + 1]));
        }
        const hv8 h1 = __builtin_convertvector(r, hv8);
        const bf16x8 a[2] = {__builtin_bit_cast(bf16x8, h0), __builtin_bit_cast(bf16x8, h1)};
#pragma unroll
        for (int x = 0; x < 2; ++x) mfma_pieces(acc[c][x], a, b[x]);
      }
    }
  };
  // NS - 1 image chunks in flight: chunk i lands in stage i % NS.  Issue
  // order per iteration i: [matrix chunk i + 1 (BR)] [image chunk i + NS - 1];
  // at the top of iteration i this wave's chunk-i loads (and the matrix's) are
  // done once at most the younger image chunks' loads are outstanding (all,
  // near the end); the barrier makes that every wave's and frees stage
  // (i - 1) % NS for chunk i + NS - 1
  const int nk = (p.K + XK - 1) / XK;
  BFrag bf0, bf1;
  if constexpr (BR) load_b(bf0, 0);
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nk) dma(i, i * XK);
  auto step = [&](int i, const BFrag& cur, BFrag& nxt) {
    if (NS == 2 || i + NS - 2 >= nk)
      wait_vm<0>();
    else if (BR)
      wait_vm<S::NDMA_A>();   // image chunk i + 1 (NS = 3) may be outstanding
    else
      wait_vm<S::NDMA * (NS - 2)>();
    __syncthreads();
    if constexpr (BR)
      if (i + 1 < nk) load_b(nxt, (i + 1) * XK);
    if (i + NS - 1 < nk) dma((i + NS - 1) % NS, (i + NS - 1) * XK);
    compute(i % NS, i * XK, cur);
  };
  for (int i = 0; i < nk; i += 2) {
    step(i, bf0, bf1);
    if (i + 1 < nk) step(i + 1, bf1, bf0);
  }
  __syncthreads();   // the ring is reused below
  uint32_t mx = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[c][x][r] *= unscale;
        mx = max(mx, __float_as_uint(acc[c][x][r]) & 0x7fffffffu);
      }
  if (p.omax) {   // T's |max| for the column GEMM; one atomic per block (partials in the freed ring)
    uint32_t* part = reinterpret_cast<uint32_t*>(ring);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane == 0) part[wave] = mx;
    __syncthreads();
    if (tid == 0) atomicMax(p.omax, max(max(part[0], part[1]), max(part[2], part[3])));
  }
  // C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5); row-major
  // outputs through buffer stores on the channel's range (gemm_x3_body)
  const int64_t ext = (int64_t)(p.M - 1) * p.sOm + (int64_t)(p.N - 1) * p.sOn + 1;
  if (p.sOm > 0 && p.sOn > 0 && p.sOm >= (int64_t)(p.N - 1) * p.sOn + 1 && (ext + 160 * p.sOm) * 4 < kOob) {
    const int sOm4 = (int)(p.sOm * 4);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.O + (int64_t)c * p.sOc, 0, (int)(ext * 4), 0x00020000);
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int gm = m0 + wm * 32 + 4 * half, gn = n0 + wn * 64 + 32 * x + l32;
        const int vo = gn < p.N ? gm * sOm4 + (int)(gn * p.sOn * 4) : kOob;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[c][x][r]), rsrc, vo + ((r & 3) + 8 * (r >> 2)) * sOm4,
                                                0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float* O = p.O + (int64_t)c * p.sOc;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half, gn = n0 + wn * 64 + 32 * x + l32;
        if (gm < p.M && gn < p.N) O[(int64_t)gm * p.sOm + (int64_t)gn * p.sOn] = acc[c][x][r];
      }
  }
}

// k_gemm_h2c: k_gemm_h2<3, 2> (the encode's column GEMM: A = the pre-split
// half DCT matrix of H, shared; B = T per channel, n = kx contiguous, k = y
// strided by +-Kw) with both operands streamed by LDS DMA into a two-stage
// ring: the matrix as k_gemm_h2r's (128 rows x 32 k x 2 planes), T as 32
// k-rows x 64 columns of fp32 per channel, four rows per 1 KB wave-instruction
// (24 KB a stage, 40 KB with the matrix: two blocks per CU).  The MFMA
// fragment of T (8 consecutive k of one column) is 8 ds_read_b32 down a
// column; the 16-byte column groups of rows with (k >> 3) odd are swapped by
// 8 slots, so the two half-waves (k groups 8 apart) read disjoint banks.  The
// fragment is split in registers as k_gemm_h2r's; products and their order
// are k_gemm_h2's (bit-identical, option cols_dma).
__global__ __launch_bounds__(256, 2) void k_gemm_h2c(const GemmProblem* __restrict__ probs,
                                                    const TileRef* __restrict__ tiles) {
  constexpr int NC = 3, TM = 128, TN = 64;
  constexpr int A_PL = TM * XK * 2;          // 8 KB per matrix plane
  constexpr int A_BYTES = 2 * A_PL;          // 16 KB
  constexpr int B_CH = XK * TN * 4;          // 8 KB per channel: 32 rows of 256 bytes
  constexpr int STAGE = A_BYTES + NC * B_CH;   // 40 KB
  __shared__ __attribute__((aligned(16))) uint8_t ring[2 * STAGE];
  const TileRef tr = tiles[blockIdx.x];
  if (tr.problem < 0) return;   // padding of an XCD-dealt list
  const GemmProblem p = probs[tr.problem];
  const int tm = tr.tile / p.tiles_n, tn = tr.tile % p.tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int ea = 0;   // T scaled by 2^ea (|max| < 2^14), the output unscaled (gemm_x3_body)
  {
    const uint32_t mb = *p.amax;
    if (mb != 0u && mb < 0x7f800000u) {
      int e;
      frexpf(__uint_as_float(mb), &e);
      ea = min(max(14 - e, -100), 100);
    }
  }
  const float unscale = ldexpf(1.0f, -(ea + p.xh_exp));
  // the matrix: plane j / 2, rows 16 rg + lane / 4 with rg = wave + 4 (j & 1), slot lane % 4 = k quad ^ swz(row)
  const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.Xh), 0, (int)(2 * p.xs_plane * 2),
                                                      0x00020000);
  int aoff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 16 * (wave + 4 * h) + (lane >> 2), kq = (lane & 3) ^ swz(row);
    aoff[h] = ((m0 + row) * p.xs_ld + 8 * kq) * 2;
  }
  const int xsp2 = (int)(p.xs_plane * 2);
  // T: channel c's element range [lo, hi] (sBn = 1, sBk = +-Kw) plus 64 floats,
  // so a 16-byte piece straddling its end is read whole (it stays inside the
  // workspace's padded regions); wave-instruction j: channel j / 2, rows
  // 4 g + lane / 16 with g = wave + 4 (j & 1), LDS slot lane % 16 = column
  // group (lane % 16) ^ (8 ((row >> 3) & 1)); k past K is zeroed at the split
  const int64_t lo = p.sBk < 0 ? (int64_t)(p.K - 1) * p.sBk : 0;
  const int64_t hi = (int64_t)(p.N - 1) + (p.sBk > 0 ? (int64_t)(p.K - 1) * p.sBk : 0);
  __amdgpu_buffer_rsrc_t brsrc[3];
#pragma unroll
  for (int c = 0; c < NC; ++c)
    brsrc[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B + (int64_t)c * p.sBc + lo), 0,
                                                 (int)((hi - lo + 1 + 64) * 4), 0x00020000);
  int boff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 4 * (wave + 4 * h) + (lane >> 4), q = (lane & 15) ^ (8 * ((row >> 3) & 1));
    boff[h] = (int)(((int64_t)row * p.sBk + n0 + 4 * q - lo) * 4);
  }
  const int bstep = (int)(p.sBk * 4);   // bytes per k row (negative for the odd parity's descending rows)
  auto dma = [&](int st, int k0) {
    uint8_t* base = ring + st * STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pl = j >> 1, h = j & 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void_t*)(base + pl * A_PL + (wave + 4 * h) * 1024), 16,
                                               aoff[h] + k0 * 2 + pl * xsp2, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2 * NC; ++j) {
      const int c = j >> 1, h = j & 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc[c], (lds_void_t*)(base + A_BYTES + c * B_CH + (wave + 4 * h) * 1024),
                                               16, boff[h] + k0 * bstep, 0, 0, 0);
    }
  };
  floatx16 acc[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][x][r] = 0.0f;
  const int nb = wn * 32 + l32;   // this lane's T column in the tile
  const int bcol = 4 * ((nb >> 2) ^ (8 * half)) + (nb & 3);   // its float within a 64-float row (rows 8 half + e)
  auto compute = [&](int st, int k0) {
    const uint8_t* base = ring + st * STAGE;
    const uint16_t* Ap = reinterpret_cast<const uint16_t*>(base);
    const float* Bf = reinterpret_cast<const float*>(base + A_BYTES);
#pragma unroll
    for (int ks = 0; ks < XK / 16; ++ks) {
      const int kq = 2 * ks + half;
      bf16x8 a[2][2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int ra = wm * 64 + 32 * x + l32;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) a[x][pl] = *reinterpret_cast<const bf16x8*>(Ap + pl * (A_PL / 2) + lds_off(ra, kq));
      }
      const int kb = k0 + 8 * kq;   // this lane's first k
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float* bc = Bf + c * (B_CH / 4) + (8 * kq) * TN + bcol;
        f32x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = bc[e * TN];
        if (k0 + XK > p.K) {   // the last chunk (uniform): k past K -> 0
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = kb + e < p.K ? v[e] : 0.0f;
        }
        f32x8 vs;
#pragma unroll
        for (int e = 0; e < 8; ++e) vs[e] = ldexpf(v[e], ea);
        const hv8 h0 = __builtin_convertvector(vs, hv8);
        const u32x4 hw = __builtin_bit_cast(u32x4, h0);
        f32x8 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r[2 * e]) : "v"(hw[e]), "v"(vs[2 * e]));
          asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r[2 * e + 1]) : "v"(hw[e]), "v"(vs[2 * e + 1]));
        }
        const hv8 h1 = __builtin_convertvector(r, hv8);
        const bf16x8 b[2] = {__builtin_bit_cast(bf16x8, h0), __builtin_bit_cast(bf16x8, h1)};
#pragma unroll
        for (int x = 0; x < 2; ++x) mfma_pieces(acc[c][x], a[x], b);
      }
    }
  };
  const int nk = (p.K + XK - 1) / XK;
  dma(0, 0);
  for (int i = 0; i < nk; ++i) {
    wait_vm<0>();
    __syncthreads();
    if (i + 1 < nk) dma((i + 1) & 1, (i + 1) * XK);
    compute(i & 1, i * XK);
  }
  // C/D map: column = lane & 31 (n), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (m);
  // row-major outputs through buffer stores on the channel's range (gemm_x3_body)
  const int64_t ext = (int64_t)(p.M - 1) * p.sOm + (int64_t)(p.N - 1) * p.sOn + 1;
  if (p.sOm > 0 && p.sOn > 0 && p.sOm >= (int64_t)(p.N - 1) * p.sOn + 1 && (ext + 160 * p.sOm) * 4 < kOob) {
    const int sOm4 = (int)(p.sOm * 4);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.O + (int64_t)c * p.sOc, 0, (int)(ext * 4), 0x00020000);
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int gm = m0 + wm * 64 + 32 * x + 4 * half, gn = n0 + nb;
        const int vo = gn < p.N ? gm * sOm4 + (int)(gn * p.sOn * 4) : kOob;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[c][x][r] * unscale), rsrc,
                                                vo + ((r & 3) + 8 * (r >> 2)) * sOm4, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float* O = p.O + (int64_t)c * p.sOc;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 64 + 32 * x + (r & 3) + 8 * (r >> 2) + 4 * half, gn = n0 + nb;
        if (gm < p.M && gn < p.N) O[(int64_t)gm * p.sOm + (int64_t)gn * p.sOn] = acc[c][x][r] * unscale;
      }
  }
}

void launch_gemm_h2(const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share, bool dma,
                    bool dma_cols) {
  if (n_tiles <= 0) return;
  if (share == 1 && dma && DCTAE_GEMM_DMA)
    hipLaunchKernelGGL((k_gemm_h2r<DCTAE_GEMM_DMA_NS, DCTAE_GEMM_DMA_BR != 0>), dim3(n_tiles), dim3(256), 0, s, probs,
                       tiles);
  else if (share == 1)
    hipLaunchKernelGGL((k_gemm_h2<3, 1>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else if (dma_cols)
    hipLaunchKernelGGL(k_gemm_h2c, dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else
    hipLaunchKernelGGL((k_gemm_h2<3, 2>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
}

// ---------------------------------------------------------------------------
// k_rows_fused: colour transform, (x, y) folds and row GEMM of both parities
// in one pass, for the images whose rows and columns both run on the GEMM DCT
// (ImgDesc::tperm; reference util.py:70-82 then util.py:333).  The separate
// path writes the folded IPT (k_rgb_to_ipt, 3.4 GB on config 4) and reads it
// back in the row GEMM.  Here a block owns 16 row pairs (y, H-1-y) -- 32
// folded rows: 16 sums, 16 differences -- and every output column of both
// parities (N <= 256 each: Kw <= 512).  Per 32-deep k chunk each of its 512
// threads loads the 4 pixels (y, k), (y, W-1-k), (H-1-y, k), (H-1-y, W-1-k),
// computes their IPT and the folds of both parities in registers
// (k_rgb_to_ipt's arithmetic, value for value: every pixel is transformed
// once), and writes the fp16 pieces to LDS; waves 0-3 run the even-kx
// columns against the even half DCT matrix, waves 4-7 the odd ones (64
// columns of 32 rows and 3 channels each, 96 accumulator VGPRs).  The
// matrices stream through a two-stage LDS ring (LDS DMA), the pixels two
// chunks ahead in registers.
// Scale: the image's |max| (k_gemm_h2's operand scale) is unknown before the
// transform, so the first pass splits at a fixed 2^DCTAE_FUSED_SE and records
// the |max| of the folded values; an image with a value outside the safe fp16
// range (|v| 2^SE >= 2^15, or not finite) is flagged, and the fix-up launch
// (fix = 1, flagged images only, grid-stride) redoes it at the scale k_gemm_h2
// derives from that |max| -- the old path's arithmetic for those images.
// ---------------------------------------------------------------------------
#ifndef DCTAE_FUSED_SE
#define DCTAE_FUSED_SE 11
#endif
// 1: the colour transform of chunk i + 1 interleaved with chunk i's MFMAs
// (double-buffered pieces; TN = 224 so that the ring and both piece buffers
// fit 160 KB of LDS), 0: transform and MFMA phases between two barriers.
// Off: on the config-4 batch the interleaved form encoded 3-6 % of calls
// differently from the first call (whole coefficient columns of the first
// images' low kx -- stale or unwritten matrix rows read by the MFMAs; NaN on
// a fresh GPU without the persistent loop), the two-barrier form 0 of 690
// (tools/c4_stress.py); with vmcnt(0) at each step top 0 of 100, but slower
#ifndef DCTAE_FUSED_PIPE
#define DCTAE_FUSED_PIPE 0
#endif
#ifndef DCTAE_FUSED_DYN
#define DCTAE_FUSED_DYN 1   // persistent first pass with per-XCD tile counters (below)
#endif
constexpr int kFusedPairs = 16;    // row pairs per block
constexpr int kFusedTN = 256;      // output columns per parity

__global__ __launch_bounds__(512, 1) void k_rows_fused(const GemmProblem* __restrict__ probs,
                                                      const TileRef* __restrict__ tiles, int n_tiles,
                                                      const ImgDesc* __restrict__ imgs, const float* __restrict__ rgb,
                                                      ColorMats cm, uint32_t* __restrict__ amax, int* __restrict__ flags,
                                                      int n_img, int fix) {
  constexpr bool PIPE = DCTAE_FUSED_PIPE != 0;
  constexpr int TN = PIPE ? 224 : kFusedTN, NPR = kFusedPairs;
  constexpr int B_PL = TN * XK * 2;          // 16 KB: one plane of one parity's matrix chunk
  constexpr int B_ST = 4 * B_PL;             // 64 KB (56 KB, PIPE): 2 parities x 2 planes
  constexpr int A_CQ = 2 * NPR * XK;         // halves per (parity, channel, piece): 32 rows x 32 k
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * B_ST + (PIPE ? 2 : 1) * 12 * A_CQ * 2];   // 152 / 160 KB
  uint16_t* As = reinterpret_cast<uint16_t*>(lds + 2 * B_ST);
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, l32 = lane & 31;
  // the wave index as a uniform value: the parity's matrix descriptor and the
  // column-range tests stay scalar (from tid they were per-lane: a waterfall
  // loop around every matrix load and a divergent branch around every MFMA)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pw = wave >> 2, wc = wave & 3;   // this wave's parity and 64-column slice
  const float gam = 0.430000007152557373046875f;
  if (fix && flags[n_img] == 0) return;      // fix-up: no image of the job flagged
  // DCTAE_FUSED_DYN (first pass): a persistent grid taking tiles from
  // per-XCD counters (flags[n_img + 1 + x]): block b runs on XCD b % 8 and
  // takes the dealt list's positions x + 8 k of its XCD lane in counter order,
  // so the image-per-XCD dealing holds without a static split's imbalance, and
  // the next tile's counter value is fetched while this tile runs
  const bool dyn = DCTAE_FUSED_DYN && !fix;
  const int xl = (int)(blockIdx.x & 7);
  int* ctr = flags + n_img + 1 + xl;
  for (int t = blockIdx.x; t < n_tiles;) {
    int t_next = 0;   // (dyn, thread 0) the next position of this XCD lane
    if (dyn && tid == 0) t_next = xl + 8 * ((int)(gridDim.x >> 3) + atomicAdd(ctr, 1));
    const TileRef tr = tiles[t];
    const GemmProblem pu = probs[max(tr.problem, 0)], pv = probs[max(tr.problem, 0) + 1];   // even and odd parity
    const int li = pu.pad2;
    // padding of an XCD-dealt list, or (fix-up) an image not flagged: the next tile
    if (tr.problem < 0 || (fix && flags[li] == 0)) {
      if (dyn) {
        uint32_t* part = reinterpret_cast<uint32_t*>(lds);
        __syncthreads();
        if (tid == 0) part[24] = (uint32_t)t_next;
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane((int)part[24]);   // uniform: the descriptors stay scalar
        __syncthreads();
      } else {
        t += (int)gridDim.x;
      }
      continue;
    }
    const ImgDesc d = imgs[li];
    const int H = d.H, W = d.W, Hh = (H + 1) >> 1, Ku = pu.K, Kv = pv.K;
    const int j0 = tr.tile * NPR;
    // operand scale 2^se: fixed in the first pass, k_gemm_h2's rule on the recorded |max| in the fix-up
    int se = DCTAE_FUSED_SE;
    if (fix) {
      const uint32_t mb = amax[2 * li];
      se = 0;
      if (mb != 0u && mb < 0x7f800000u) {
        int e;
        frexpf(__uint_as_float(mb), &e);
        se = min(max(14 - e, -100), 100);
      }
    }
    // the matrices: wave-instruction j: parity j / 4, plane (j / 2) % 2, rows
    // 16 rg + lane / 4 with rg = wave + 8 (j % 2) (16 rows of 64 bytes per 1 KB),
    // LDS slot lane % 4 = k quad (lane % 4) ^ swz(row), as k_gemm_h2r
    const u32x4 brs[2] = {rsrc_words(pu.Xh, (uint32_t)(2 * pu.xs_plane * 2)),
                          rsrc_words(pv.Xh, (uint32_t)(2 * pv.xs_plane * 2))};
    int boff[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * (wave + 8 * h) + (lane >> 2), kq = (lane & 3) ^ swz(row);
      boff[0][h] = (row * pu.xs_ld + 8 * kq) * 2;
      boff[1][h] = (row * pv.xs_ld + 8 * kq) * 2;
    }
    const int xsp2[2] = {(int)(pu.xs_plane * 2), (int)(pv.xs_plane * 2)};
    const int nrow[2] = {(pu.N + 31) & ~31, (pv.N + 31) & ~31};   // matrix rows the MFMAs read
    auto dma_b = [&](int st, int k0) {
#if defined(DCTAE_PROFILING) && defined(DCTAE_FUSED_ABL) && (DCTAE_FUSED_ABL & 8)
      return;   // profiling ablation: no matrix loads (wrong output)
#endif
      uint8_t* base = lds + st * B_ST;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int par = j >> 2, pl = (j >> 1) & 1, h = j & 1;
        if (16 * (wave + 8 * h) < nrow[par])   // rows past the parity's N (rounded to the MFMA blocks) are never read
          dma_lds16(brs[par], base + (2 * par + pl) * B_PL + (wave + 8 * h) * 1024,
                    boff[par][h] + k0 * 2 + pl * xsp2[par]);
      }
    };
    // the pixels: row pair pr = tid / 32 (y = j0 + pr, y2 = H-1-y), column k = k0 + tid % 32 and W-1-k
    const int pr = tid >> 5, kk0 = tid & 31;
    const int y = j0 + pr;
    const bool vy = y < Hh;
    const int yy = vy ? y : 0, y2 = H - 1 - yy;
    const bool yp = y2 != yy;
    const int hw = H * W;
    const auto rrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rgb + d.rgb_off), 0, 3 * hw * 4, 0x00020000);
    typedef float Px[4][3];
    Px pxa, pxb;
    auto load_rgb = [&](Px& px, int k0) {
#if defined(DCTAE_PROFILING) && defined(DCTAE_FUSED_ABL) && (DCTAE_FUSED_ABL & 4)
#pragma unroll
      for (int q = 0; q < 4; ++q)   // profiling ablation: no pixel loads (wrong output)
#pragma unroll
        for (int c = 0; c < 3; ++c) px[q][c] = 0.001f * (float)(k0 + q + c + kk0);
      return;
#endif
      const int k = k0 + kk0, kk = k < Ku ? k : 0, x2 = W - 1 - kk;
      const int o[4] = {yy * W + kk, yy * W + x2, y2 * W + kk, y2 * W + x2};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          px[q][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrsrc, (c * hw + o[q]) * 4, 0, 0));
    };
    bool bad = false;
    uint32_t fmx = 0;   // |max| of the folded values (the fix-up's scale)
    float pi[4][3];     // the IPT of the chunk position's 4 pixels
    // the colour transform of pixel q (util.py:70-82, k_rgb_to_ipt's arithmetic)
    auto pix = [&](const Px& px, int q) {
      const float r = px[q][0], g = px[q][1], b = px[q][2];
      const float l0 = signed_pow_fast(mat3_row(cm.rgb2lms, 0, r, g, b), gam);
      const float l1 = signed_pow_fast(mat3_row(cm.rgb2lms, 1, r, g, b), gam);
      const float l2 = signed_pow_fast(mat3_row(cm.rgb2lms, 2, r, g, b), gam);
#pragma unroll
      for (int c = 0; c < 3; ++c) pi[q][c] = mat3_row(cm.lms2ipt, c, l0, l1, l2);
    };
    // k_rgb_to_ipt's folds of channel c: row y (sum) and row H-1-y (difference)
    // of both parities, split into fp16 pieces into Ab
    auto fold = [&](int k0, int c, uint16_t* Ab) {
      const int k = k0 + kk0;
      const int kk = k < Ku ? k : 0;
      const bool xp = W - 1 - kk != kk;
      const bool oku = vy && k < Ku, okv = vy && k < Kv;
      const int kq = (k & 31) >> 3, kw = k & 7;
      const float pb = xp ? pi[1][c] : 0.0f, pd = xp ? pi[3][c] : 0.0f;
      const float a = yp ? pi[0][c] + pi[2][c] : pi[0][c];
      const float bb = yp ? pb + pd : pb;
      const float c2 = pi[0][c] - pi[2][c], d2 = pb - pd;
      const float v[2][2] = {{oku ? (xp ? a + bb : a) : 0.0f, oku && yp ? (xp ? c2 + d2 : c2) : 0.0f},
                             {okv ? a - bb : 0.0f, okv && yp ? c2 - d2 : 0.0f}};
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const float vv = v[par][rr];
          fmx = max(fmx, __float_as_uint(vv) & 0x7fffffffu);
          const float vsc = ldexpf(vv, se);
          bad |= !(fabsf(vsc) < 32768.0f);
          const _Float16 h0 = (_Float16)vsc;
          const _Float16 h1 = (_Float16)(vsc - (float)h0);
          const int row = pr + NPR * rr;
          const int o = row * XK + 8 * (kq ^ swz(row)) + kw;
          Ab[((par * 3 + c) * 2 + 0) * A_CQ + o] = __builtin_bit_cast(uint16_t, h0);
          Ab[((par * 3 + c) * 2 + 1) * A_CQ + o] = __builtin_bit_cast(uint16_t, h1);
        }
    };
    auto transform = [&](const Px& px, int k0, uint16_t* Ab) {
#if defined(DCTAE_PROFILING) && defined(DCTAE_FUSED_ABL) && (DCTAE_FUSED_ABL & 1)
      // profiling ablation: no colour transform / folds / split (wrong output)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int pq = 0; pq < 8; ++pq) {
          const int row = pr + NPR * (pq & 1);
          const int o = row * XK + 8 * (((kk0 >> 3)) ^ swz(row)) + (kk0 & 7);
          Ab[((pq >> 2) * 3 + c) * 2 * A_CQ + ((pq >> 1) & 1) * A_CQ + o] =
              (uint16_t)(__float_as_uint(px[pq & 3][c]) & 0x3bffu);
        }
      return;
#endif
#pragma unroll
      for (int q = 0; q < 4; ++q) pix(px, q);
#pragma unroll
      for (int c = 0; c < 3; ++c) fold(k0, c, Ab);
    };
    floatx16 acc[3][2];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][x][r] = 0.0f;
    const int nw = pw ? pv.N : pu.N;   // this wave's parity's output columns
    // the MFMAs of k step ks and channel c of one chunk (stage st, pieces Ab)
    auto mfma_unit = [&](int st, const uint16_t* Ab, int ks, int c) {
#if defined(DCTAE_PROFILING) && defined(DCTAE_FUSED_ABL) && (DCTAE_FUSED_ABL & 2)
      return;   // profiling ablation: no MFMAs (wrong output)
#endif
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(lds + st * B_ST + 2 * pw * B_PL);
      const int kq = 2 * ks + half;
      bf16x8 a[2];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        a[q] = *reinterpret_cast<const bf16x8*>(Ab + ((pw * 3 + c) * 2 + q) * A_CQ + lds_off(l32, kq));
#pragma unroll
      for (int x = 0; x < 2; ++x)
        if (wc * 64 + 32 * x < nw) {   // (wave-uniform) columns past N: none
          const int rb = wc * 64 + 32 * x + l32;
          bf16x8 b[2];
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            b[pl] = *reinterpret_cast<const bf16x8*>(Bp + pl * (B_PL / 2) + lds_off(rb, kq));
          mfma_pieces(acc[c][x], a, b);
        }
    };
    const int nk = (Ku + XK - 1) / XK;
    if constexpr (!PIPE) {
      // Pixels two chunks ahead (pxa: even chunks, pxb: odd), the matrices one;
      // issue order per step i: [matrices i + 1] [pixels i + 2], so at its top at
      // most pixels i + 1's 12 loads may be outstanding.  Every step issues the
      // same loads (past the last chunk: clamped pixels, matrix offsets reading
      // zeros), and the loop body is unconditional, so the compiler's own waits
      // on the pixel registers count exactly.
      auto step = [&](int i, Px& cur) {
        wait_vm<12>();      // this wave's pixels and matrix chunk i
        lds_barrier();      // every wave's; chunk i - 1's MFMAs done (the pieces and stage (i + 1) % 2 free)
        dma_b((i + 1) & 1, (i + 1) * XK);
        transform(cur, i * XK, As);
        load_rgb(cur, (i + 2) * XK);
        lds_barrier();      // the pieces of chunk i
#pragma unroll
        for (int ks = 0; ks < XK / 16; ++ks)
#pragma unroll
          for (int c = 0; c < 3; ++c) mfma_unit(i & 1, As, ks, c);
      };
      load_rgb(pxa, 0);
      dma_b(0, 0);
      load_rgb(pxb, XK);
      int i = 0;
      for (; i + 1 < nk; i += 2) {
        step(i, pxa);
        step(i + 1, pxb);
      }
      if (i < nk) step(i, pxa);
    } else {
      // DCTAE_FUSED_PIPE: the transform of chunk i + 1 interleaved with chunk i's
      // MFMAs (double-buffered pieces As / As + 12 A_CQ), one barrier per chunk.
      // Issue order per step i: [matrices i + 1] [pixels i + 3]; at its top the
      // wave needs matrices i and pixels i + 1, pixels i + 2 may be in flight.
      uint16_t* A0 = As;
      uint16_t* A1 = As + 12 * A_CQ;
      auto step = [&](int i, Px& cur, const uint16_t* Ac, uint16_t* An) {
#ifdef DCTAE_FUSED_SB   // pin the issue order the counted wait assumes (no load moved across it)
        __builtin_amdgcn_sched_barrier(0);
#endif
#if defined(DCTAE_FUSED_WAIT0)
        wait_vm<0>();
#elif !defined(DCTAE_FUSED_EARLYWAIT)
        wait_vm<12>();
#endif
        lds_barrier();      // pieces of chunk i from every wave; chunk i - 1's MFMAs done (An, stage (i + 1) % 2 free)
        dma_b((i + 1) & 1, (i + 1) * XK);
        const int kn = (i + 1) * XK;
        mfma_unit(i & 1, Ac, 0, 0);
        pix(cur, 0);
        mfma_unit(i & 1, Ac, 0, 1);
        pix(cur, 1);
        mfma_unit(i & 1, Ac, 0, 2);
        pix(cur, 2);
        mfma_unit(i & 1, Ac, 1, 0);
        pix(cur, 3);
#ifdef DCTAE_FUSED_EARLYWAIT
        // (experiment) the pixels of chunk i + 3 issued as soon as cur is
        // consumed, and the wait for matrices i + 1 two MFMA units before the
        // next barrier instead of right before it
        load_rgb(cur, (i + 3) * XK);
        mfma_unit(i & 1, Ac, 1, 1);
        fold(kn, 0, An);
        fold(kn, 1, An);
#ifdef DCTAE_FUSED_SB
        __builtin_amdgcn_sched_barrier(0);
#endif
        wait_vm<12>();
        mfma_unit(i & 1, Ac, 1, 2);
        fold(kn, 2, An);
#else
        mfma_unit(i & 1, Ac, 1, 1);
        fold(kn, 0, An);
        fold(kn, 1, An);
        mfma_unit(i & 1, Ac, 1, 2);
        fold(kn, 2, An);
        load_rgb(cur, (i + 3) * XK);
#endif
      };
      load_rgb(pxa, 0);
      load_rgb(pxb, XK);
      dma_b(0, 0);
      transform(pxa, 0, A0);
      load_rgb(pxa, 2 * XK);
#ifdef DCTAE_FUSED_EARLYWAIT
      wait_vm<12>();   // matrices 0
#endif
      int i = 0;
      for (; i + 1 < nk; i += 2) {
        step(i, pxb, A0, A1);
        step(i + 1, pxa, A1, A0);
      }
      if (i < nk) step(i, pxb, A0, A1);
    }
    wait_vm<0>();   // no LDS DMA may outlive the loop (the LDS is reused, and released at exit)
    const GemmProblem& p = pw ? pv : pu;
    const int N = p.N;
    const float unscale = ldexpf(1.0f, -(se + p.xh_exp));
    // C/D map: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5):
    // rows < 16 are the sums (T row j0 + row), the rest the differences (T row
    // H - 1 - (j0 + row - 16)); the middle row of an odd H has no difference
    uint32_t mx = 0;
    int trow[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * half;
      const int j = j0 + (rr & (NPR - 1));
      const int ty = rr < NPR ? j : H - 1 - j;
      trow[r] = (j < Hh && (rr < NPR || ty != j)) ? ty : -1;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const bool vn = wc * 64 + 32 * x + l32 < N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          acc[c][x][r] *= unscale;
          if (vn && trow[r] >= 0) mx = max(mx, __float_as_uint(acc[c][x][r]) & 0x7fffffffu);
        }
      }
    // block reductions: flag, |max| of the folded values, |max| of T
    uint32_t* part = reinterpret_cast<uint32_t*>(lds);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
      fmx = max(fmx, (uint32_t)__shfl_xor((int)fmx, o));
    }
    const bool wbad = __ballot(bad) != 0;   // (__syncthreads_or brings 256 bytes of LDS of its own)
    __syncthreads();   // every wave past its last LDS read: the partials alias the ring
    if (lane == 0) {
      part[wave] = mx;
      part[8 + wave] = fmx;
      part[16 + wave] = wbad ? 1u : 0u;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t m = 0, f = 0, any_bad = 0;
      for (int w = 0; w < 8; ++w) {
        m = max(m, part[w]);
        f = max(f, part[8 + w]);
        any_bad |= part[16 + w];
      }
      if (!fix) {
        if (f) atomicMax(amax + 2 * li, f);
        if (any_bad) {
          flags[li] = 1;
          flags[n_img] = 1;   // the job's "any" word, read first by the fix-up
        }
      }
      // T's |max| for the column GEMM; a flagged block leaves it to the fix-up
      if (pu.omax && (fix || !any_bad)) atomicMax(pu.omax, m);
    }
    const int64_t ext = (int64_t)(p.M - 1) * p.sOm + (int64_t)(N - 1) * p.sOn + 1;
    const int sOm4 = (int)(p.sOm * 4);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(p.O + (int64_t)c * p.sOc, 0, (int)(ext * 4), 0x00020000);
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int n = wc * 64 + 32 * x + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int vo = (n < N && trow[r] >= 0) ? trow[r] * sOm4 + n * 4 : kOob;
#if defined(DCTAE_PROFILING) && defined(DCTAE_FUSED_ABL) && (DCTAE_FUSED_ABL & 16)
          if (acc[c][x][r] == 1.2345f)   // profiling ablation: (almost) no T stores (wrong output)
#endif
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[c][x][r]), rsrc, vo, 0, 0);
        }
      }
    }
    if (dyn) {
      uint32_t* part = reinterpret_cast<uint32_t*>(lds);
      if (tid == 0) part[24] = (uint32_t)t_next;
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane((int)part[24]);   // uniform: the descriptors stay scalar
    } else {
      t += (int)gridDim.x;
    }
    __syncthreads();   // the partials / LDS reused by the next tile
  }
}

int fused_pairs_per_block() { return kFusedPairs; }
int fused_max_n() { return DCTAE_FUSED_PIPE ? 224 : kFusedTN; }

void launch_rows_fused(const GemmProblem* probs, const TileRef* tiles, int n_tiles, const ImgDesc* imgs,
                       const float* rgb, const ColorMats& cm, uint32_t* amax, int* flags, int n_img, hipStream_t s,
                       bool fixup) {
  if (n_tiles <= 0) return;
  // the fix-up: a short grid-stride launch (every block exits at once when no image is flagged)
  const int g = fixup || DCTAE_FUSED_DYN ? std::min((n_tiles + 7) & ~7, 256) : n_tiles;
  hipLaunchKernelGGL(k_rows_fused, dim3(g), dim3(512), 0, s, probs, tiles, n_tiles, imgs, rgb, cm, amax, flags, n_img,
                     fixup ? 1 : 0);
}

void launch_gemm_x3(int nc, const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share) {
  if (n_tiles <= 0) return;
  if (nc == 3 && share == 1)
    hipLaunchKernelGGL((k_gemm_x3<3, 1>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else if (nc == 3 && share == 2)
    hipLaunchKernelGGL((k_gemm_x3<3, 2>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else if (nc == 3)
    hipLaunchKernelGGL((k_gemm_x3<3, 0>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else
    hipLaunchKernelGGL((k_gemm_x3<1, 0>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
}

// host: three bf16 planes [3][Rp][Kp] of a row-major fp32 matrix (R x K),
// zero padded to Rp = ceil128(R), Kp = ceil32(K); the same round-to-nearest-
// even split the kernel applies to fp32 operands
static uint16_t host_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float host_f32(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

void split_matrix_x3(const float* m, int R, int K, std::vector<uint16_t>& out, int* Rp, int* Kp) {
  *Rp = (R + 127) / 128 * 128;
  *Kp = (K + XK - 1) / XK * XK;
  const size_t plane = (size_t)*Rp * *Kp;
  out.assign(3 * plane, 0);
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < K; ++k) {
      const float v = m[(size_t)r * K + k];
      const uint16_t h0 = host_bf16(v);
      const float r1 = v - host_f32(h0);
      const uint16_t h1 = host_bf16(r1);
      const float r2 = r1 - host_f32(h1);
      const size_t o = (size_t)r * *Kp + k;
      out[o] = h0;
      out[plane + o] = h1;
      out[2 * plane + o] = host_bf16(r2);
    }
}

// host: two fp16 planes [2][Rp][Kp] of the matrix scaled by 2^e, e chosen so
// the largest |value| * 2^e lies in [2^13, 2^14) (k_gemm_h2's operand range)
void split_matrix_h2(const float* m, int R, int K, std::vector<uint16_t>& out, int* Rp, int* Kp, int* e_out) {
  *Rp = (R + 127) / 128 * 128;
  *Kp = (K + XK - 1) / XK * XK;
  const size_t plane = (size_t)*Rp * *Kp;
  out.assign(2 * plane, 0);
  float mx = 0.0f;
  for (size_t i = 0; i < (size_t)R * K; ++i) mx = std::max(mx, std::fabs(m[i]));
  int e = 0;
  if (mx > 0.0f && std::isfinite(mx)) {
    int ex;
    std::frexp(mx, &ex);
    e = 14 - ex;
  }
  *e_out = e;
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < K; ++k) {
      const float v = std::ldexp(m[(size_t)r * K + k], e);
      const _Float16 h0 = (_Float16)v;
      const _Float16 h1 = (_Float16)(v - (float)h0);
      const size_t o = (size_t)r * *Kp + k;
      out[o] = __builtin_bit_cast(uint16_t, h0);
      out[plane + o] = __builtin_bit_cast(uint16_t, h1);
    }
}

}  // namespace dctae
