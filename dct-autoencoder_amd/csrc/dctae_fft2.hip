// Compile-time specialised two-pass FFT-DCT kernels (M = N/2 = R1 * R2,
// at most 64/3 butterflies per job and pass) for the headline image sizes:
//   N = 512: M = 256 = 16 x 16        N = 224: M = 112 = 16 x 7
// Same maths as dctae_fft.hip (Makhoul + Stockham), but every index is a
// compile-time expression, passes are done in place (register staged), and
// the row kernel gives each image row to one wave (no block barriers).
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_launch.h"
#include "dctae_spec512.h"

// config 2's T with the nontemporal hint: on for k_rows224p's stores (rows
// 0.060 -> 0.057 ms), off for k_cols224's loads (their strided 8-byte reads
// share lines through L2: cols 0.052 -> 0.069 ms with it), same-box A/B r05.
#ifndef DCTAE_T224_ST_NT
#define DCTAE_T224_ST_NT 1
#endif
#ifndef DCTAE_T224_LD_NT
#define DCTAE_T224_LD_NT 0
#endif


namespace dctae {

// padded complex slot of element m: one spare slot every 16 keeps the
// stride-16 Stockham accesses on distinct LDS banks
__device__ __forceinline__ constexpr int pad16(int m) { return m + (m >> 4); }

// ---------------------------------------------------------------------------
// rows: one wave = one image row, its 3 IPT channels are 3 jobs.  A row item
// is 16 rows (4 waves x RPW rows); T points at channel 0, row 0 of the
// image's row-pass output (row-major [c][y][kx]).
// ---------------------------------------------------------------------------
template <int N>
struct RowsLds {
  static constexpr int M = N / 2;
  static constexpr int MP = pad16(M - 1) + 2;
  float2 z[4][3][MP];
};

template <int N, int R1, int R2>
__device__ __forceinline__ void rows2_item(const ImgDesc& d, int y_first, const float* __restrict__ rgb,
                                           float* __restrict__ T, RowsLds<N>& L, const float2* post_s,
                                           const float2* tw_s, const ColorMats& cm) {
  constexpr int M = N / 2;
  constexpr int MP = RowsLds<N>::MP;
  constexpr int B1 = M / R1, B2 = M / R2;
  constexpr int PX = (N + 63) / 64;        // pixels per lane and row
  constexpr int KI = (M + 63) / 64;        // k = lane + 64 i, i < KI, covers k < M (k = M by lane 0)
#ifndef DCTAE_RPW224
#define DCTAE_RPW224 1   // 224-wide rows: one row per wave (0.074 vs 0.081 ms at 4 rows per wave, config 2)
#endif
  constexpr int RPW = N == 224 ? DCTAE_RPW224 : 4;   // rows per wave (block = 4 RPW rows)
  static_assert(R1 * R2 == M, "two-pass plan");
  static_assert(3 * B1 <= 64 && 3 * B2 <= 64, "one butterfly per lane per pass");
  static_assert(R1 == 16, "first radix 16 (Ns of pass 2 = 16)");
  const int tid = opaque_tid();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  float2(*z)[MP] = L.z[wave];
  float* zf0 = reinterpret_cast<float*>(z[0]);
  float* zf1 = reinterpret_cast<float*>(z[1]);
  float* zf2 = reinterpret_cast<float*>(z[2]);
  const int H = d.H, Kw = d.Kw;
  const int64_t hw = (int64_t)H * N;
  const float* src = rgb + d.rgb_off;
  const float gam = 0.430000007152557373046875f;
  // ---- lane-invariant index maps (the same for every row)
  int zo[PX];                               // Makhoul slot of pixel lane + 64 i
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int px = lane + 64 * i;
    const int v = (px & 1) ? (N - 1 - (px >> 1)) : (px >> 1);
    zo[i] = 2 * pad16(v >> 1) + (v & 1);
  }
  // T offset of coefficient kx within (channel, row); -1 = not kept
  int oa[KI], ob[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    const int kx2 = N - k;
    oa[i] = (k < Kw) ? k : -1;
    ob[i] = (k >= 1 && kx2 < Kw) ? kx2 : -1;
  }
  const int oM = (M < Kw) ? M : -1;
  const int ystride = Kw;                   // T offset step per row
  const int64_t cstride = (int64_t)H * Kw;  // per channel
  float pr[PX], pg[PX], pb[PX];
  auto fetch = [&](int y) {
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int px = lane + 64 * i;
      if (px < N && y < H) {
        const int64_t o = (int64_t)y * N + px;
        pr[i] = src[o];
        pg[i] = src[hw + o];
        pb[i] = src[2 * hw + o];
      }
    }
  };
  int y = y_first + wave;
#pragma unroll 1
  for (int rr = 0; rr < RPW; ++rr, y += 4) {
    if (y >= H) break;
    fetch(y);
    // ---- IPT (util.py:70-82) + Makhoul reorder into LDS
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      if (lane + 64 * i < N) {
        const float l0 = signed_pow_fast(mat3_row(cm.rgb2lms, 0, pr[i], pg[i], pb[i]), gam);
        const float l1 = signed_pow_fast(mat3_row(cm.rgb2lms, 1, pr[i], pg[i], pb[i]), gam);
        const float l2 = signed_pow_fast(mat3_row(cm.rgb2lms, 2, pr[i], pg[i], pb[i]), gam);
        zf0[zo[i]] = mat3_row(cm.lms2ipt, 0, l0, l1, l2);
        zf1[zo[i]] = mat3_row(cm.lms2ipt, 1, l0, l1, l2);
        zf2[zo[i]] = mat3_row(cm.lms2ipt, 2, l0, l1, l2);
      }
    }
    // ---- pass 1: radix R1, Ns = 1 (no twiddles); in place, one butterfly per lane
    if (lane < 3 * B1) {
      const int c = lane / B1, j = lane - c * B1;
      float2 v[R1];
#pragma unroll
      for (int r = 0; r < R1; ++r) v[r] = z[c][pad16(j + r * B1)];
      DFT<R1>::run(v);
#pragma unroll
      for (int r = 0; r < R1; ++r) z[c][pad16(j * R1 + r)] = v[r];
    }
    // ---- pass 2: radix R2, Ns = R1; twiddle W_M^{r*j}
    if (lane < 3 * B2) {
      const int c = lane / B2, j = lane - c * B2;
      float2 v[R2];
#pragma unroll
      for (int r = 0; r < R2; ++r) v[r] = z[c][pad16(j + r * B2)];
#pragma unroll
      for (int r = 1; r < R2; ++r) v[r] = cmul(v[r], tw_s[r * j]);
      DFT<R2>::run(v);
#pragma unroll
      for (int r = 0; r < R2; ++r) z[c][pad16(j + r * R1)] = v[r];
    }
    // ---- Makhoul post-processing -> T (k = lane + 64 i; X[k] = Re W_k, X[N-k] = -Im W_k)
#pragma unroll 1
    for (int c = 0; c < 3; ++c) {
      float* tb = T + c * cstride + (int64_t)y * ystride;
#pragma unroll
      for (int i = 0; i < KI; ++i) {
        const int k = lane + 64 * i;
        if (k < M) {
          const float2 A = z[c][pad16(k)];
          float2 B = z[c][pad16(k == 0 ? 0 : M - k)];
          B.y = -B.y;
          const float2 al = post_s[2 * k], be = post_s[2 * k + 1];
          const float2 W = cadd(cmul(al, cadd(A, B)), cmul(be, csub(A, B)));
          if (oa[i] >= 0) tb[oa[i]] = W.x;
          if (ob[i] >= 0) tb[ob[i]] = -W.y;
        }
        __builtin_amdgcn_sched_barrier(0);  // bound register pressure: one k-slice in flight
      }
      if (lane == 0 && oM >= 0) {  // k = M: A = B = conj-paired Z[0]
        const float2 A = z[c][0];
        const float2 B = make_float2(A.x, -A.y);
        const float2 W = cadd(cmul(post_s[2 * M], cadd(A, B)), cmul(post_s[2 * M + 1], csub(A, B)));
        tb[oM] = W.x;
      }
    }
  }
}

template <int N, int R1, int R2>
__global__ __launch_bounds__(256) void k_fft_rows2(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                   const float* __restrict__ rgb, float* __restrict__ ws,
                                                   const float2* __restrict__ tw, const float2* __restrict__ post,
                                                   ColorMats cm) {
  constexpr int M = N / 2;
  __shared__ RowsLds<N> L;
  __shared__ float2 post_s[2 * (M + 1)];
  __shared__ float2 tw_s[M];
  for (int i = threadIdx.x; i < 2 * (M + 1); i += 256) post_s[i] = post[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  __syncthreads();
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  rows2_item<N, R1, R2>(d, jb.y, rgb, ws + d.ws_t, L, post_s, tw_s, cm);
}

// ---------------------------------------------------------------------------
// k_rows224p<RW>: the row pass of 224-wide images (config 2) with RW = 2 or 3
// rows per wave (3 RW channel-rows) instead of rows2_item's one: pass 1 (radix
// 16, 7 butterflies per channel-row) fills 42 / 63 of 64 lanes instead of 21,
// a wave's RW contiguous rows are 7 / 10.5 pixels per lane instead of 3.5 of 4,
// the colour mix runs on pixel pairs (v_pk_fma_f32, splat_mix) and the Makhoul
// post is makhoul_pair on the (c1, c2, c3, c4) coefficients (4 VALU per
// coefficient pair).  A block is 4 RW rows; no block barrier after the tables.
// ---------------------------------------------------------------------------
template <int RW>
struct Rows224pLds {
  static constexpr int MP = RowsLds<224>::MP;
  float2 z[4][3 * RW][MP];
};

template <int RW>
__global__ __launch_bounds__(256) void k_rows224p(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                  const float* __restrict__ rgb, float* __restrict__ ws,
                                                  const float2* __restrict__ tw, const float2* __restrict__ post,
                                                  ColorMats cm) {
  constexpr int N = 224, M = 112, R1 = 16, R2 = 7, B1 = 7, B2 = 16;
  static_assert(RW == 2 || RW == 3, "rows per wave");
  constexpr int CR = 3 * RW;                 // channel-rows per wave
  constexpr int MP = Rows224pLds<RW>::MP;
  constexpr int PX = (RW * N + 63) / 64;   // pixels per lane: 7 (RW = 2) or 11 (the last half-populated)
  constexpr int KI = (M + 63) / 64;
  __shared__ Rows224pLds<RW> L;
  __shared__ float4 pc[M + 1];
  __shared__ float2 tw_s[M];
  // the wave's pixel loads are issued first: the table loads, their LDS
  // stores and the block barrier overlap them instead of preceding them
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const int tid = opaque_tid();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int H = d.H, Kw = d.Kw;
  const int y0 = jb.y + RW * wave;
  const bool live = y0 < H;   // wave-uniform; dead waves still reach the barrier
  float2(*z)[MP] = L.z[wave];
  float* zf = reinterpret_cast<float*>(&z[0][0]);
  const int64_t hw = (int64_t)H * N;
  const float* src = rgb + d.rgb_off + (int64_t)(live ? y0 : 0) * N;   // the wave's rows are contiguous
  const int nq = live ? min(RW, H - y0) * N : 0;
  float pr[PX + 1], pg[PX + 1], pb[PX + 1];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    // unconditional loads (pixels past the image's last row re-read pixel
    // lane; their results are never stored): no per-element control flow
    const int q = lane + 64 * i, qq = q < nq ? q : lane;
    pr[i] = src[qq];
    pg[i] = src[hw + qq];
    pb[i] = src[2 * hw + qq];
  }
  {
    const float4* p4 = reinterpret_cast<const float4*>(post);
    for (int i = threadIdx.x; i < M + 1; i += 256) {
      const float4 ab = p4[i];   // (al.x, al.y, be.x, be.y)
      pc[i] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
    }
    for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  }
  __syncthreads();
  if (!live) return;   // no block barrier follows
  pr[PX] = pg[PX] = pb[PX] = 0.0f;
  // ---- IPT (util.py:70-82) on pixel pairs + Makhoul reorder into LDS.  The
  //      LDS slot of pixel q = lane + 64 i repeats with period 7 in i (448 =
  //      7 x 64 pixels = two rows): slot(i + 7) = slot(i) + two rows' channels
  const float gam = 0.430000007152557373046875f;
  int slot7[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int q = lane + 64 * i;
    const int r = (q >= N ? 1 : 0) + (q >= 2 * N ? 1 : 0);
    const int px = q - N * r;
    const int v = (px & 1) ? (N - 1 - (px >> 1)) : (px >> 1);
    slot7[i] = (3 * r) * 2 * MP + 2 * pad16(v >> 1) + (v & 1);
  }
#pragma unroll
  for (int i = 0; i < PX; i += 2) {
    const cf r2 = (cf){pr[i], pr[i + 1]}, g2 = (cf){pg[i], pg[i + 1]}, b2 = (cf){pb[i], pb[i + 1]};
    const cf l0 = splat_mix(cm.rgb2lms, 0, r2, g2, b2), l1 = splat_mix(cm.rgb2lms, 1, r2, g2, b2),
             l2 = splat_mix(cm.rgb2lms, 2, r2, g2, b2);
    const cf q0 = (cf){signed_pow_fast(l0.x, gam), signed_pow_fast(l0.y, gam)};
    const cf q1 = (cf){signed_pow_fast(l1.x, gam), signed_pow_fast(l1.y, gam)};
    const cf q2 = (cf){signed_pow_fast(l2.x, gam), signed_pow_fast(l2.y, gam)};
    const cf o0 = splat_mix(cm.lms2ipt, 0, q0, q1, q2), o1 = splat_mix(cm.lms2ipt, 1, q0, q1, q2),
             o2 = splat_mix(cm.lms2ipt, 2, q0, q1, q2);
#pragma unroll
    for (int h = 0; h < 2 && i + h < PX; ++h) {
      const int q = lane + 64 * (i + h);
      if (q < RW * N) {
        float* zr = zf + (i + h < 7 ? slot7[i + h] : slot7[i + h - 7] + 6 * 2 * MP);
        zr[0] = h ? o0.y : o0.x;
        zr[2 * MP] = h ? o1.y : o1.x;
        zr[4 * MP] = h ? o2.y : o2.x;
      }
    }
  }
  wave_lds_sync();   // the reorder stores of other lanes
  // ---- pass 1: radix 16, Ns = 1; in place, one butterfly per lane (63 of 64)
  if (lane < CR * B1) {
    const int c = lane / B1, j = lane - c * B1;
    cf v[R1];
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const float2 x = z[c][pad16(j + r * B1)];
      v[r] = (cf){x.x, x.y};
    }
    DFTV<R1>::run(v);
#pragma unroll
    for (int r = 0; r < R1; ++r) z[c][pad16(j * R1 + r)] = make_float2(v[r].x, v[r].y);
  }
  wave_lds_sync();
  // ---- pass 2: radix 7, Ns = 16; twiddle W_M^{r j}; 144 butterflies in 3 rounds
#pragma unroll
  for (int t = 0; t < (CR * B2 + 63) / 64; ++t) {
    const int b = lane + 64 * t;
    if (b < CR * B2) {
      const int c = b >> 4, j = b & 15;
      cf v[R2];
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        const float2 x = z[c][pad16(j + r * B2)];
        v[r] = (cf){x.x, x.y};
      }
#pragma unroll
      for (int r = 1; r < R2; ++r) {
        const float2 w = tw_s[r * j];
        v[r] = cmul_pk(v[r], (cf){w.x, w.y});
      }
      DFTV<R2>::run(v);
#pragma unroll
      for (int r = 0; r < R2; ++r) z[c][pad16(j + r * R1)] = make_float2(v[r].x, v[r].y);
    }
  }
  wave_lds_sync();
  // ---- Makhoul post -> T: (X[k], X[N - k]) = makhoul_pair(Z[k], Z[M - k]), k = lane + 64 i
  int oa[KI], ob[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    oa[i] = (k < M && k < Kw) ? k : -1;
    ob[i] = (k < M && k >= 1 && N - k < Kw) ? N - k : -1;
  }
  const int64_t cstride = (int64_t)H * Kw;
  float* T = ws + d.ws_t;
#pragma unroll 1
  for (int cr = 0; cr < CR; ++cr) {
    const int rr = cr / 3, c = cr - 3 * rr;
    const int y = y0 + rr;
    if (y >= H) break;
    float* tb = T + c * cstride + (int64_t)y * Kw;
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = lane + 64 * i;
      if (k < M) {
        const float4 cc = pc[k];
        const float2 A = z[cr][pad16(k)], P = z[cr][pad16(k == 0 ? 0 : M - k)];
        const cf t = makhoul_pair((cf){A.x, A.y}, (cf){P.x, P.y}, (cf){cc.x, cc.y}, (cf){cc.z, cc.w});
#if DCTAE_T224_ST_NT
        if (oa[i] >= 0) __builtin_nontemporal_store(t.x, tb + oa[i]);
        if (ob[i] >= 0) __builtin_nontemporal_store(t.y, tb + ob[i]);
#else
        if (oa[i] >= 0) tb[oa[i]] = t.x;
        if (ob[i] >= 0) tb[ob[i]] = t.y;
#endif
      }
    }
    if (lane == 0 && M < Kw) {   // k = M: Z[0] with itself
      const float2 A = z[cr][0];
      const float4 cc = pc[M];
      tb[M] = makhoul_pair((cf){A.x, A.y}, (cf){A.x, A.y}, (cf){cc.x, cc.y}, (cf){cc.z, cc.w}).x;
    }
  }
}

// ---------------------------------------------------------------------------
// cols, linear-address form: every LDS address is (lane base) + (compile-time
// constant), so address arithmetic folds into the ds_read / ds_write offset
// fields instead of costing VALU (the column kernel is VALU-issue bound).
//  * the T slice is copied to LDS in natural row order (row y at y*KSP);
//  * Makhoul's reorder v[n] = x[2n] / x[2N-1-2n] is applied by pass 1's read
//    addresses: z[m] = (v[2m], v[2m+1]) with m = jj + B1 r is rows
//    4jj + 4B1 r (+2) for r < 8 and 2N-1-4jj-4B1 r (-2) for r >= 8;
//  * passes and post-processing use the padded complex layout pad16(m),
//    which is linear in the unrolled index for every access made here.
// Row-major T only (t_layout 0); P = 14 tile columns per block.
// ---------------------------------------------------------------------------
template <int N>
struct ColsLds {
  static constexpr int M = N / 2;
  static constexpr int KSP = 15;
  static constexpr int ZROWS = 2 * (pad16(M - 1) + 1);
  float z[ZROWS * KSP];
};

typedef float c4f2 __attribute__((ext_vector_type(2)));

// the T slice of column item (d, c, strip): thread (y0 = t / 7, p = t % 7)
// holds float2 p of rows y0 + 32 k (threads t < 32 * KS / 2)
template <int N, int KS>
__device__ __forceinline__ void cols4_fetch(const ImgDesc& d, int c, int strip, const float* __restrict__ T,
                                            c4f2 (&tv)[N / 32]) {
  const int tid = opaque_tid();
  if (tid < 32 * (KS / 2)) {
    const int y0 = tid / (KS / 2), p = tid - y0 * (KS / 2);
    const c4f2* src = reinterpret_cast<const c4f2*>(T + ((int64_t)c * d.H + y0) * d.Kw + strip * KS) + p;
    const int64_t rstep = (int64_t)16 * d.Kw;   // 32 rows, in float2
#pragma unroll
    for (int k = 0; k < N / 32; ++k) tv[k] = src[k * rstep];
  }
}

// one column item: (image d, channel c, tile column strip); T = the image's
// row-pass output (channel 0, row 0).  Caller: post_s / tw_s loaded, a block
// barrier since the previous use of zs and sbias.
template <int N, int R2, int KS, bool THR>
__device__ __forceinline__ void cols4_item(const ImgDesc& d, int c, int strip, const float* __restrict__ T, float* zs,
                                           const float2* post_s, const float2* tw_s, float* sbias,
                                           const EncParams& ep, const TokenSinks& sk) {
#pragma clang fp contract(fast)
  constexpr int R1 = 16;
  constexpr int M = N / 2;
  constexpr int B1 = M / R1, B2 = M / R2;
  constexpr int KSP = KS | 1;
  constexpr int ZROWS = 2 * (pad16(M - 1) + 1);
  constexpr int M16 = M / 16;
  static_assert(M % 16 == 0 && B2 == 16 && B1 <= 16 && KS == 14, "plan shape");
  static_assert(N * KSP <= ZROWS * KSP, "natural rows fit the complex layout");
  static_assert(KSP == ColsLds<N>::KSP, "LDS image");
  const int tid = opaque_tid();
  // LFQ-bit thresholds of this thread's epilogue rows (latency hidden behind the transform)
  constexpr int EPR = 2;
  const int g16 = tid >> 4, jl = tid & 15;
  float2 thr_r[EPR][KS / 2];
  auto load_thr = [&]() {
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int h = g16 + 16 * r;
      if (h < d.qh && jl < KS) {
        const float2* t2 = reinterpret_cast<const float2*>(
            ep.thr + ((((int64_t)c * ep.maxph + h) * ep.maxpw) + strip) * (KS * KS) + (int64_t)jl * KS);
#pragma unroll
        for (int p = 0; p < KS / 2; ++p) thr_r[r][p] = t2[p];
      }
    }
  };
  if (THR) load_thr();
  if (THR && tid < 32) sbias[tid] = __fdiv_rn(-(float)(tid + strip), ep.ci[c]);
  // ---- T slice -> LDS, natural row order
  c4f2 tv[N / 32];
  cols4_fetch<N, KS>(d, c, strip, T, tv);
  if (tid < 32 * (KS / 2)) {
    // row-major: thread (y0 = t / 7, p = t % 7) copies float2 p of rows y0 + 32k
    const int y0 = tid / (KS / 2), p = tid - y0 * (KS / 2);
    float* dst = zs + y0 * KSP + 2 * p;
#pragma unroll
    for (int k = 0; k < N / 32; ++k) {
      dst[32 * KSP * k] = tv[k].x;
      dst[32 * KSP * k + 1] = tv[k].y;
    }
  }
  __syncthreads();
  const int jj = tid & 15, col = tid >> 4;
  const bool on_col = col < KS;
  // ---- pass 1 (Ns = 1), Makhoul reorder folded into the read addresses
  {
    cf v[R1];
    const bool on = on_col && jj < B1;
    if (on) {
      // rows 4jj + 4B1 r (+2) for r < 8; rows 2N-1-4jj-4B1 r (-2) for r >= 8, addressed
      // upwards from the lowest one (LDS offsets are unsigned immediates)
      const float* lo = zs + 4 * jj * KSP + col;
      const float* hi = zs + (2 * N - 3 - 4 * jj - 4 * B1 * (R1 - 1)) * KSP + col;
#pragma unroll
      for (int r = 0; r < R1 / 2; ++r) v[r] = (cf){lo[4 * B1 * r * KSP], lo[(4 * B1 * r + 2) * KSP]};
#pragma unroll
      for (int r = R1 / 2; r < R1; ++r)
        v[r] = (cf){hi[(4 * B1 * (R1 - 1 - r) + 2) * KSP], hi[4 * B1 * (R1 - 1 - r) * KSP]};
      DFTV<R1>::run(v);
    }
    __syncthreads();
    if (on) {
      float* o = zs + 2 * 17 * jj * KSP + col;                     // z[16 jj + r]: pad16 = 17 jj + r
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        o[2 * r * KSP] = v[r].x;
        o[(2 * r + 1) * KSP] = v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- pass 2 (Ns = 16): z[jj + 16 r], pad16 = jj + 17 r
  {
    cf v[R2];
    const bool on = on_col;
    float* z = zs + 2 * jj * KSP + col;
    if (on) {
#pragma unroll
      for (int r = 0; r < R2; ++r) v[r] = (cf){z[2 * 17 * r * KSP], z[(2 * 17 * r + 1) * KSP]};
#pragma unroll
      for (int r = 1; r < R2; ++r) {
        const float2 w = tw_s[r * jj];
        v[r] = cmulv(v[r], (cf){w.x, w.y});
      }
      DFTV<R2>::run(v);
    }
    __syncthreads();
    if (on) {
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        z[2 * 17 * r * KSP] = v[r].x;
        z[(2 * 17 * r + 1) * KSP] = v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- Makhoul post-processing: k = jj + 16 i, A = Z[k] (pad16 = jj + 17 i),
  //      B = conj Z[M - k] (pad16 = bb - 17 i); k = 0 and k = M use Z[0]
  constexpr int KPL = M16 + 1;
  cf wv[KPL];
  if (on_col) {
    const float* za = zs + 2 * jj * KSP + col;
    const int bb = M + M16 - 1 - jj + (jj == 0 ? 1 : 0);
    const float* zb = zs + 2 * (bb - 17 * (M16 - 1)) * KSP + col;   // Z[M - k] for i = M16 - 1; others above it
    const cf* ps = reinterpret_cast<const cf*>(post_s) + 2 * jj;
#pragma unroll
    for (int i = 0; i < M16; ++i) {
      const cf A = (cf){za[2 * 17 * i * KSP], za[(2 * 17 * i + 1) * KSP]};
      cf B;
      if (i == 0) {
        const float* zb0 = jj == 0 ? zs + col : zb + 2 * 17 * (M16 - 1) * KSP;
        B = (cf){zb0[0], -zb0[KSP]};
      } else {
        B = (cf){zb[2 * 17 * (M16 - 1 - i) * KSP], -zb[(2 * 17 * (M16 - 1 - i) + 1) * KSP]};
      }
      // W = al (A + B) + be (A - B), as (re, im) pairs: one pk_mul + pk_fma per product
      const cf s1 = A + B, d1 = A - B, al = ps[32 * i], be = ps[32 * i + 1];
      wv[i] = s1.xx * al + s1.yy * (cf){-al.y, al.x} + d1.xx * be + d1.yy * (cf){-be.y, be.x};
    }
    if (jj == 0) {  // k = M
      const cf A = (cf){zs[col], zs[KSP + col]};
      const cf B = (cf){A.x, -A.y};
      const cf* pm = reinterpret_cast<const cf*>(post_s) + 2 * M;
      wv[M16] = cmulv(A + B, pm[0]) + cmulv(A - B, pm[1]);
    }
  }
  __syncthreads();
  const int Kh = d.Kh;
  if (on_col) {
    float* xo = zs + jj * KSP + col;                 // X[k] at row k (natural layout)
    float* xn = zs + (N - jj - 16 * (M16 - 1)) * KSP + col;   // X[N - k], addressed from the lowest row
#pragma unroll
    for (int i = 0; i < M16; ++i) {
      const int k = jj + 16 * i;
      if (k < Kh) xo[16 * i * KSP] = wv[i].x;
      if (k >= 1 && N - k < Kh) xn[16 * (M16 - 1 - i) * KSP] = -wv[i].y;
    }
    if (jj == 0 && M < Kh) zs[M * KSP + col] = wv[M16].x;
  }
  __syncthreads();
  // ---- token epilogue: tile (h, strip) of channel c, one 16-lane group per tile
  if (THR) {
    // codes from the exact LFQ thresholds; amax as an integer max of |x| bit
    // patterns (NaN patterns order above inf: NaN-propagating like torch.amax)
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int h = g16 + 16 * r;
      if (h < d.qh) {
        const float* row = zs + (KS * h + jl) * KSP;   // lanes jl >= KS read in-bounds junk, masked below
        uint32_t am = 0, code = 0;
#pragma unroll
        for (int p = 0; p < KS / 2; ++p) {
          const float v0 = row[2 * p], v1 = row[2 * p + 1];
          am = max(am, max(__float_as_uint(v0) & 0x7fffffffu, __float_as_uint(v1) & 0x7fffffffu));
          code = 2 * code + (v0 >= thr_r[r][p].x ? 1u : 0u);   // MSB-first (lfq.py:187)
          code = 2 * code + (v1 >= thr_r[r][p].y ? 1u : 0u);
        }
        am = jl < KS ? am : 0u;
        // 16-lane row max by DPP row rotations (as cols_epilogue, dctae_spec512.h)
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x128, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x124, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x122, 0xf, 0xf, false));
        am = max(am, (uint32_t)__builtin_amdgcn_mov_dpp((int)am, 0x121, 0xf, 0xf, false));
        const int64_t tok = d.tok_off + (h * d.qw + strip) * ep.C + c;
        if (jl == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(__uint_as_float(am), ep.mw), sbias[h]);
        if (jl < KS && sk.codes) sk.codes[tok * KS + jl] = (uint16_t)code;
        if (sk.raw && jl < KS) {
#pragma unroll
          for (int p2 = 0; p2 < KS; ++p2) sk.raw[tok * KS * KS + jl * KS + p2] = row[p2];
        }
      }
    }
  } else {
    for (int h = g16; h < d.qh; h += 16) {
      float vals[KS];
      const float* row = zs + (KS * h + jl) * KSP;
#pragma unroll
      for (int p2 = 0; p2 < KS; ++p2) vals[p2] = row[p2];
      const int f = (h * d.qw + strip) * ep.C + c;
      token_epilogue_p<KS>(ep, c, h, strip, jl, vals, d.tok_off + f, sk);
    }
  }
}

// one cols7 workgroup (block index b of the column grid): (channel, tile
// column) item t and IPB consecutive images of the list
template <bool THR, int IPB, bool PF>
__device__ __forceinline__ void cols7_block(int b, const ImgDesc* __restrict__ imgs, const int* __restrict__ list,
                                            int n_list, int n_items, int qw, const float* __restrict__ ws,
                                            const float2* __restrict__ tw, const float2* __restrict__ post,
                                            const EncParams& ep, const TokenSinks& sk, Cols7Lds& L, float4* post4,
                                            float2* tw_s, float* sbias) {
  constexpr int M = 256;
  const int per_x = (n_items + 7) / 8;
  const int slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, g = slot / per_x;
  const int k0 = g * IPB;
  if (t >= n_items || k0 >= n_list) return;
  const int c = t / qw, strip = t - c * qw;
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int i = threadIdx.x; i < M + 1; i += 256) post4[i] = p4[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  float2 thr_r[2][7];
  cols_thresholds<THR>(imgs[list[k0]], c, strip, ep, thr_r, sbias);
  float va[16], vb[16];
  {
    const ImgDesc d0 = imgs[list[k0]];
    cols7_load(d0, c, strip, ws + d0.ws_t, va, vb);
  }
  __syncthreads();   // tables
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int k = k0 + u;
    if (k < n_list) {
      const ImgDesc dk = imgs[list[k]];
      if (u > 0 && !PF) cols7_load(dk, c, strip, ws + dk.ws_t, va, vb);
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(va[r]), "+v"(vb[r]));   // see k_cols512b
      float na[16], nb[16];
      if (PF && u + 1 < IPB) {   // unconditional (the last image reloads itself), see k_cols512b
        const ImgDesc dn = imgs[list[min(k + 1, n_list - 1)]];
        cols7_load(dn, c, strip, ws + dn.ws_t, na, nb);   // in flight during the transform
      }
      cols7_compute<THR>(dk, c, strip, L, va, vb, post4, tw_s, sbias, thr_r, ep, sk);
      __syncthreads();
      if (PF && u + 1 < IPB) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          va[r] = na[r];
          vb[r] = nb[r];
        }
      }
    }
  }
}

template <bool THR, int IPB, bool PF>
__global__ __launch_bounds__(256) void k_fft_cols7(const ImgDesc* __restrict__ imgs, const int* __restrict__ list,
                                                   int n_list, int n_items, int qw,
                                                   const float* __restrict__ ws, const float2* __restrict__ tw,
                                                   const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  __shared__ Cols7Lds L;
  __shared__ float4 post4[257];
  __shared__ float2 tw_s[256];
  __shared__ float sbias[32];
  cols7_block<THR, IPB, PF>(blockIdx.x, imgs, list, n_list, n_items, qw, ws, tw, post, ep, sk, L, post4, tw_s, sbias);
}

// k_cols512b: the band-layout column pass (dctae_spec512.h).  Block b of the
// grid: (channel, tile strip) item t and IPB consecutive images of `list`;
// XCD-aware: blocks b and b + 8 share an XCD, each XCD lane owns 12 adjacent
// items (neighbouring strips share L2 lines; their threshold tables stay in
// that XCD's L2), the next image's T' loads in flight during the transform.
// Images per block, same-box A/B (1024 x 512^2, NT T', round 5): 2 -> 0.588-
// 0.590 ms, 3 -> 0.570-0.571 (default: a block's first image, whose loads
// nothing hides, is a third of its work instead of half), 4 -> 0.581, 6 ->
// 0.575-0.577, 8 -> 0.579-0.580.
#ifndef DCTAE_C5B_IPB
#define DCTAE_C5B_IPB 3
#endif
// PatchNorm-output columns (cols512b_norm_epilogue): 1 = on, 0 = the generic
// token epilogue; images per block
#ifndef DCTAE_C5B_NORM
#define DCTAE_C5B_NORM 1
#endif
#ifndef DCTAE_C5B_NORM_IPB
#define DCTAE_C5B_NORM_IPB 3
#endif
template <bool THR, int IPB, bool NORM = false>
__global__ __launch_bounds__(256) void k_cols512b(const ImgDesc* __restrict__ imgs, const int* __restrict__ list,
                                                  int n_list, const float* __restrict__ ws,
                                                  const float2* __restrict__ tw, const float2* __restrict__ post,
                                                  EncParams ep, TokenSinks sk) {
  constexpr int M = 256, per_x = 12;   // 96 items = 3 channels x 32 strips, 12 per XCD lane
  __shared__ Cols512bLds L;
  const int b = blockIdx.x;
  const int slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, k0 = (slot / per_x) * IPB;
  if (k0 >= n_list) return;
  const int c = t >> 5, strip = t & 31;
  const int tid = threadIdx.x;
  L.tw2[tid >> 4][tid & 15] = tw[(tid >> 4) * (tid & 15)];
  const float4* p4 = reinterpret_cast<const float4*>(post);
  {
    const float4 ab = p4[tid];   // (al.x, al.y, be.x, be.y) -> c1..c4
    L.pc[tid] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
  }
  const float4 abM = p4[M];
  const float4 pcM = make_float4(abM.x + abM.z, abM.x - abM.z, abM.y + abM.w, abM.y - abM.w);
  float2 thr_r[2][7];
  cols_thresholds<THR>(imgs[list[k0]], c, strip, ep, thr_r, nullptr);
  float sb[2] = {0.0f, 0.0f};
  if (THR || NORM) {
    const int g16 = tid >> 4;
    sb[0] = __fdiv_rn(-(float)(g16 + strip), ep.ci[c]);
    sb[1] = __fdiv_rn(-(float)(g16 + 16 + strip), ep.ci[c]);
  }
  float2 tn[NORM ? 2 : 1][14];
  if constexpr (NORM) cols_norm_tables(c, strip, ep, tn);
  TPiece qa[8];
  cols512b_load(c, strip, ws + imgs[list[k0]].ws_t, qa);
  __syncthreads();   // tables
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int k = k0 + u;
    if (k < n_list) {
      const ImgDesc dk = imgs[list[k]];
      // the loads of this image (prefetched during the previous one) become
      // opaque values here: without it the compiler moves their register
      // shuffles up to the loads and waits for the NEXT image's prefetch
      // before computing this one (no overlap at all)
      t_opaque(qa);
      // the next image's loads in flight during this one; unconditional (the
      // last image of the list reloads itself): a conditional load makes the
      // compiler merge qn / qa with register copies right behind the loads
      TPiece qn[8];
      if (u + 1 < IPB) cols512b_load(c, strip, ws + imgs[list[min(k + 1, n_list - 1)]].ws_t, qn);
      float4 qf[8];
      t_decode(qa, qf);
      cols512b_compute<THR, NORM>(dk, c, strip, L, qf, pcM, sb, thr_r, ep, sk, tn);
      __syncthreads();   // epilogue reads of X before the next image's transposes
      if (u + 1 < IPB) {
#pragma unroll
        for (int r = 0; r < 8; ++r) qa[r] = qn[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_cols512w: k_cols512b's codes-only (THR) path with no idle lanes.  A block
// of 7 waves = 28 16-lane groups covers TWO tile strips (28 columns) of one
// channel, so every group transforms a distinct column (k_cols512b's 16
// groups over one 14-column strip repeat column 13 twice: 1/8 of its FFT and
// epilogue work).  The epilogue maps thread t to tile row (h, jl) = (t / 14,
// t % 14) of both strips (448 = 32 x 14 threads, two rows each, no repeated
// lanes); the row maxima go through LDS (rmax) and the 64 tile scores are
// finished by wave 0 after the block barrier that ends the image.
// ---------------------------------------------------------------------------
struct Cols512wLds {
  union {
    cf xch[28][kXchStridePk];   // per group transpose region (60,928 B)
    float X[2][449 * 14];       // the two strips' 448 x 14 coefficients (+ the spare row of the k = 64 store)
  } u;
  uint32_t rmax[2][32][14];     // row |max| bits (uint order: +NaN above Inf above finite)
  float2 tw2[16][16];
  float4 pc[256];
};                              // 70,656 B: 2 blocks per CU

__device__ __forceinline__ void cols512w_load(int c, int kx, const float* __restrict__ T, TPiece (&q)[8]) {
  t_load_column(c, kx, opaque_tid() & 15, T, q);
}

// the transform of group G = column col of strip 2 sp + sg, image k: band T'
// in qa -> X[sg] (lane indices from a fresh opaque_tid: the compiler rebuilds
// the addresses per phase instead of holding them across the image loop)
__device__ __forceinline__ void cols512w_transform(Cols512wLds& L, const float4 (&qa)[8], float4 pcM) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14;
  const int tid = opaque_tid();
  const int G = tid >> 4, j = tid & 15;
  const int sg = G >= KS ? 1 : 0, col = G - KS * sg;
  const int s = sigma16(j);
  const bool self0 = (j == 0), self8 = (j == 15);
  cf v[16];
#pragma unroll
  for (int bb = 0; bb < 8; ++bb) {   // qa[bb] = rows 64 bb + 4 j + (0, 2, 3, 1)
    v[bb] = (cf){qa[bb].x, qa[bb].y};
    v[15 - bb] = (cf){mirror16(qa[bb].z), mirror16(qa[bb].w)};
  }
  fft256_group(v, L.u.xch[G], j, s, L.tw2);
  __syncthreads();   // X aliases the transpose regions
  float* xs = L.u.X[sg];
  float* xa = xs + s * KS + col;         // X[s + 16 i] at + 224 i
  float* xb = xs + (N - s) * KS + col;   // X[N - s - 16 i] at - 224 i
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
    if (i >= 4) xb[-224 * i] = x0.y;
    if (i + 1 >= 4) xb[-224 * (i + 1)] = x1.y;
  }
  if (self0) xs[M * KS + col] = (pcM.x + pcM.y) * v[0].x + (pcM.w - pcM.z) * v[0].y;
}

// codes of tile row (h, jl) = (t / 14, t % 14) in both strips, the rows' |max| into rmax
__device__ __forceinline__ void cols512w_epilogue(Cols512wLds& L, const ImgDesc& dk, int c, int sp,
                                                  const float2 (&thr_r)[2][7], const EncParams& ep,
                                                  const TokenSinks& sk) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
  const int eh = tid / KS, ejl = tid - KS * eh;
  const f2v* row0 = reinterpret_cast<const f2v*>(L.u.X[0]) + (KS * eh + ejl) * (KS / 2);
  const f2v* row1 = reinterpret_cast<const f2v*>(L.u.X[1]) + (KS * eh + ejl) * (KS / 2);
  uint32_t code0 = 0, code1 = 0;
  float am0 = 0.0f, am1 = 0.0f;
#pragma unroll
  for (int p = 0; p < KS / 2; ++p) code_bits4(code0, code1, am0, am1, row0[p], row1[p], thr_r[0][p], thr_r[1][p]);
  L.rmax[0][eh][ejl] = __float_as_uint(am0);
  L.rmax[1][eh][ejl] = __float_as_uint(am1);
  if (sk.codes) {
    sk.codes[cols_tok(dk, c, 2 * sp, eh, ep.C) * KS + ejl] = (uint16_t)code0;
    sk.codes[cols_tok(dk, c, 2 * sp + 1, eh, ep.C) * KS + ejl] = (uint16_t)code1;
  }
  if (sk.raw) {   // both strips' tokens as 16-byte pieces (cols_store_tokens over 448 threads)
    for (int e = tid; e < 2 * 32 * 49; e += 448) {
      const int r = e / (32 * 49), e2 = e - r * 32 * 49, h = e2 / 49, q = e2 - h * 49;
      reinterpret_cast<float4*>(sk.raw + cols_tok(dk, c, 2 * sp + r, h, ep.C) * (KS * KS))[q] =
          reinterpret_cast<const float4*>(L.u.X[r] + KS * KS * h)[q];
    }
  }
}

// wave 0: the 64 tile scores of image dk from rmax (FE:409-416)
__device__ __forceinline__ void cols512w_scores(const Cols512wLds& L, const ImgDesc& dk, int c, int sp,
                                                const EncParams& ep, const TokenSinks& sk) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
  if (tid < 64) {
    const int r = tid >> 5, h = tid & 31;
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < KS; ++q) m = max(m, L.rmax[r][h][q]);
    const float sb = __fdiv_rn(-(float)(h + 2 * sp + r), ep.ci[c]);
    sk.scores[cols_tok(dk, c, 2 * sp + r, h, ep.C)] = __fadd_rn(__fmul_rn(__uint_as_float(m), ep.mw), sb);
  }
}

template <int IPB>
__global__ __launch_bounds__(448) __attribute__((amdgpu_waves_per_eu(4))) void k_cols512w(
    const ImgDesc* __restrict__ imgs, const int* __restrict__ list, int n_list, const float* __restrict__ ws,
    const float2* __restrict__ tw, const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  constexpr int M = 256, KS = 14, per_x = 6;   // 48 items = 3 channels x 16 strip pairs, 6 per XCD lane
  __shared__ Cols512wLds L;
  const int b = blockIdx.x;
  const int slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, k0 = (slot / per_x) * IPB;
  if (k0 >= n_list) return;
  const int c = t >> 4, sp = t & 15;
  {
    const int tid = threadIdx.x;
    if (tid < 256) {
      L.tw2[tid >> 4][tid & 15] = tw[(tid >> 4) * (tid & 15)];
      const float4 ab = reinterpret_cast<const float4*>(post)[tid];   // (al.x, al.y, be.x, be.y) -> c1..c4
      L.pc[tid] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
    }
  }
  const float4 abM = reinterpret_cast<const float4*>(post)[M];
  const float4 pcM = make_float4(abM.x + abM.z, abM.x - abM.z, abM.y + abM.w, abM.y - abM.w);
  float2 thr_r[2][7];   // the thread's epilogue rows' thresholds (image-independent; band images: qh = qw = 32)
  {
    const int tid = opaque_tid();
    const int eh = tid / KS, ejl = tid - KS * eh;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float2* t2 = reinterpret_cast<const float2*>(
          ep.thr + ((((int64_t)c * ep.maxph + eh) * ep.maxpw) + 2 * sp + r) * (KS * KS) + (int64_t)ejl * KS);
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) thr_r[r][p] = t2[p];
    }
  }
  const int kx = [&] {
    const int G = opaque_tid() >> 4, sg = G >= KS ? 1 : 0;
    return KS * (2 * sp + sg) + G - KS * sg;
  }();
  TPiece qa[8];
  cols512w_load(c, kx, ws + imgs[list[k0]].ws_t, qa);
  __syncthreads();   // tables
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int k = k0 + u;
    if (k >= n_list) break;   // block-uniform
    t_opaque(qa);
    TPiece qn[8];
    if (u + 1 < IPB) cols512w_load(c, kx, ws + imgs[list[min(k + 1, n_list - 1)]].ws_t, qn);
    // the previous image's scores (its rmax was written before the barrier that ended it)
    if (u > 0) cols512w_scores(L, imgs[list[k - 1]], c, sp, ep, sk);
    float4 qf[8];
    t_decode(qa, qf);
    cols512w_transform(L, qf, pcM);
    __syncthreads();
    cols512w_epilogue(L, imgs[list[k]], c, sp, thr_r, ep, sk);
    __syncthreads();   // X / rmax reads before the next image's transposes and the score reads
    if (u + 1 < IPB) {
#pragma unroll
      for (int r = 0; r < 8; ++r) qa[r] = qn[r];
    }
  }
  cols512w_scores(L, imgs[list[min(k0 + IPB, n_list) - 1]], c, sp, ep, sk);
}

void launch_cols512b(const ImgDesc* imgs, const int* list, int n_list, const float* ws, const float2* tw,
                     const float2* post, const EncParams& ep, const TokenSinks& sk, hipStream_t s, bool wide) {
  if (n_list <= 0) return;
  const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
  // PatchNorm output (LFQ projections' staging, returned patches) with the
  // tables held per block: no raw copy, codes (if any) one codebook per tile row
  const bool norm = DCTAE_C5B_NORM && !thr && sk.norm && ep.median && !sk.raw && ep.maxph == 32 && ep.maxpw == 32 &&
                    (!sk.codes || (ep.cb_dim == 14 && ep.ncb == 14));
  const int ipb = thr ? DCTAE_C5B_IPB : norm ? DCTAE_C5B_NORM_IPB : 2;
  const int grid = 96 * ((n_list + ipb - 1) / ipb);
  if (thr && wide) {   // two strips per 7-wave block: 48 items
    hipLaunchKernelGGL((k_cols512w<DCTAE_C5B_IPB>), dim3(48 * ((n_list + DCTAE_C5B_IPB - 1) / DCTAE_C5B_IPB)), dim3(448),
                       0, s, imgs, list, n_list, ws, tw, post, ep, sk);
    return;
  }
  if (thr)
    hipLaunchKernelGGL((k_cols512b<true, DCTAE_C5B_IPB>), dim3(grid), dim3(256), 0, s, imgs, list, n_list, ws, tw,
                       post, ep, sk);
  else if (norm)
    hipLaunchKernelGGL((k_cols512b<false, DCTAE_C5B_NORM_IPB, true>), dim3(grid), dim3(256), 0, s, imgs, list, n_list,
                       ws, tw, post, ep, sk);
  else
    hipLaunchKernelGGL((k_cols512b<false, 2>), dim3(grid), dim3(256), 0, s, imgs, list, n_list, ws, tw, post, ep, sk);
}

int cols7_grid(int n_list, int qw, int ipb) {
  const int n_items = 3 * qw, per_x = (n_items + 7) / 8;
  return 8 * per_x * ((n_list + ipb - 1) / ipb);
}

template <int N, int R2, int KS, bool THR>
__global__ __launch_bounds__(256) void k_fft_cols4(const ImgDesc* __restrict__ imgs, const int4* __restrict__ blocks,
                                                   const float* __restrict__ ws, const float2* __restrict__ tw,
                                                   const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  constexpr int M = N / 2;
  __shared__ ColsLds<N> L;
  __shared__ float2 post_s[2 * (M + 1)];
  __shared__ float2 tw_s[M];
  __shared__ float sbias[32];   // -(h + strip) / ci[c] per tile row h (fp32 division, FE:411-416)
  for (int i = threadIdx.x; i < 2 * (M + 1); i += 256) post_s[i] = post[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  const int4 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  cols4_item<N, R2, KS, THR>(d, jb.y, jb.z, ws + d.ws_t, L.z, post_s, tw_s, sbias, ep, sk);
}

// ---------------------------------------------------------------------------
// k_cols224: the column pass of 224-high images (config 2), two column items
// (image, channel, tile-column strip) per block and 8 lanes per column instead
// of k_fft_cols4's 16.  k_fft_cols4<224> is VALU-issue bound (666 VALU per
// wave for 3.5 columns, 1 block per item); here, per wave of 7 columns:
//  * pass 1 (radix 16, 7 butterflies per column) runs on 7 / 8 of the lanes
//    instead of 7 / 16; pass 2 (radix 7, 16 butterflies) is two per lane;
//  * the Makhoul post is makhoul_pair2 on the (c1, c2, c3, c4) coefficients
//    (VOP3P modifiers for the conjugates and swaps: 4 VALU per coefficient
//    pair, as the 512 kernels);
//  * the THR epilogue is cols512b_epilogue's (v_cmp + v_addc code bits, one
//    v_maximum3_f32 per two |x|, buffer stores), one tile row of each item per
//    thread; with an odd item count the second item repeats the first (the
//    same values to the same addresses, no branches).
// ---------------------------------------------------------------------------
template <bool THR>
__global__ __launch_bounds__(256) void k_cols224(const ImgDesc* __restrict__ imgs, const int4* __restrict__ blocks,
                                                 int n_items, const float* __restrict__ ws,
                                                 const float2* __restrict__ tw, const float2* __restrict__ post,
                                                 EncParams ep, TokenSinks sk) {
#pragma clang fp contract(fast)
  constexpr int N = 224, M = 112, R1 = 16, R2 = 7, B1 = 7, KS = 14;
#ifndef DCTAE_C224_KSP
#define DCTAE_C224_KSP 30
#endif
  // LDS row stride (28 columns + pad): ds_read/write_b32 bank = dword mod 32 per
  // 32-lane half (4 columns x 8 lanes jj): pass 2 and the post step jj by 2 KSP
  // and pass 1's stores by 34 KSP, conflict-free when those are 4 x odd mod 32,
  // i.e. KSP = 2 mod 4 (30); 29 made them 2-way (PMC: 0.36 conflict share)
  constexpr int KSP = DCTAE_C224_KSP;
  static_assert(KSP >= 2 * KS, "28 columns");
  constexpr int ZROWS = 2 * (pad16(M - 1) + 1);   // padded complex layout, in floats per column
  static_assert(N <= ZROWS, "natural rows fit the complex layout");
  __shared__ float zs[ZROWS * KSP];
  __shared__ float4 pc[M + 1];     // (c1, c2, c3, c4) of makhoul_pair (rows512_tables)
  __shared__ float2 tw_s[M];
  __shared__ float sbias[2][16];   // -(h + strip) / ci[c] per item and tile row h (fp32 division, FE:411-416)
  {
    const float4* p4 = reinterpret_cast<const float4*>(post);
    for (int i = threadIdx.x; i < M + 1; i += 256) {
      const float4 ab = p4[i];   // (al.x, al.y, be.x, be.y)
      pc[i] = make_float4(ab.x + ab.z, ab.x - ab.z, ab.y + ab.w, ab.y - ab.w);
    }
    for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  }
  // XCD-dealt pairs: XCD x (blocks b = x + 8 s) runs pairs [x per_x, (x + 1)
  // per_x) in order, so the neighbouring strips of one (image, channel), which
  // share T's 128-byte lines, are read through the same L2 at about the same time
  const int n_pairs = (n_items + 1) / 2, per_x = (n_pairs + 7) / 8;
  const int pidx = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (pidx >= n_pairs) return;   // block-uniform, before any barrier
  const int tid = opaque_tid();
  const int i0 = 2 * pidx;
  const int4 ja = blocks[i0], jb = blocks[i0 + 1 < n_items ? i0 + 1 : i0];
  const ImgDesc da = imgs[ja.x], db = imgs[jb.x];
  const int g16 = tid >> 4, jl = tid & 15, jlc = min(jl, KS - 1);
  if (THR) {
    if (tid < 32) {
      const int u = tid >> 4, h = tid & 15;
      const int c = u ? jb.y : ja.y, strip = u ? jb.z : ja.z;
      sbias[u][h] = __fdiv_rn(-(float)(h + strip), ep.ci[c]);
    }
  }
  // ---- T slices -> LDS, natural row order: thread t < 224 of item u = t / 112
  //      holds float2 p = t % 7 of rows y0 + 16 k, y0 = (t % 112) / 7
  if (tid < 224) {
    const int u = tid >= 112 ? 1 : 0, t = tid - 112 * u;
    const int y0 = t / (KS / 2), p = t - y0 * (KS / 2);
    const int c = u ? jb.y : ja.y, strip = u ? jb.z : ja.z;
    const int64_t tbase = u ? db.ws_t : da.ws_t;
    const int H = u ? db.H : da.H, Kw = u ? db.Kw : da.Kw;
    const c4f2* src = reinterpret_cast<const c4f2*>(ws + tbase + ((int64_t)c * H + y0) * Kw + strip * KS) + p;
    const int64_t rstep = (int64_t)8 * Kw;   // 16 rows, in float2
    c4f2 tv[N / 16];
#pragma unroll
    for (int k = 0; k < N / 16; ++k) {
#if DCTAE_T224_LD_NT
      tv[k] = __builtin_nontemporal_load(src + k * rstep);
#else
      tv[k] = src[k * rstep];
#endif
    }
    float* dst = zs + y0 * KSP + KS * u + 2 * p;
#pragma unroll
    for (int k = 0; k < N / 16; ++k) {
      dst[16 * KSP * k] = tv[k].x;
      dst[16 * KSP * k + 1] = tv[k].y;
    }
  }
  __syncthreads();
  const int jj = tid & 7, col = tid >> 3;   // column col of the 28 (item col / 14)
  const bool on_col = col < 2 * KS;
  // ---- pass 1 (radix 16, Ns = 1), Makhoul reorder folded into the read addresses (as cols4_item)
  {
    cf v[R1];
    const bool on = on_col && jj < B1;
    if (on) {
      const float* lo = zs + 4 * jj * KSP + col;
      const float* hi = zs + (2 * N - 3 - 4 * jj - 4 * B1 * (R1 - 1)) * KSP + col;
#pragma unroll
      for (int r = 0; r < R1 / 2; ++r) v[r] = (cf){lo[4 * B1 * r * KSP], lo[(4 * B1 * r + 2) * KSP]};
#pragma unroll
      for (int r = R1 / 2; r < R1; ++r)
        v[r] = (cf){hi[(4 * B1 * (R1 - 1 - r) + 2) * KSP], hi[4 * B1 * (R1 - 1 - r) * KSP]};
      DFTV<R1>::run(v);
    }
    __syncthreads();
    if (on) {
      float* o = zs + 2 * 17 * jj * KSP + col;   // z[16 jj + r]: pad16 = 17 jj + r
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        o[2 * r * KSP] = v[r].x;
        o[(2 * r + 1) * KSP] = v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- pass 2 (radix 7, Ns = 16): butterflies j = jj and jj + 8, z[j + 16 r] at pad16 = j + 17 r
  {
    cf v[2][R2];
    if (on_col) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = jj + 8 * h;
        const float* z = zs + 2 * jj * KSP + 16 * h * KSP + col;
#pragma unroll
        for (int r = 0; r < R2; ++r) v[h][r] = (cf){z[2 * 17 * r * KSP], z[(2 * 17 * r + 1) * KSP]};
#pragma unroll
        for (int r = 1; r < R2; ++r) {
          const float2 w = tw_s[r * j];
          v[h][r] = cmul_pk(v[h][r], (cf){w.x, w.y});
        }
        DFTV<R2>::run(v[h]);
      }
    }
    __syncthreads();
    if (on_col) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float* z = zs + 2 * jj * KSP + 16 * h * KSP + col;
#pragma unroll
        for (int r = 0; r < R2; ++r) {
          z[2 * 17 * r * KSP] = v[h][r].x;
          z[(2 * 17 * r + 1) * KSP] = v[h][r].y;
        }
      }
    }
    __syncthreads();
  }
  // ---- LFQ-bit thresholds of this thread's epilogue row in each item (lanes
  //      14 / 15 repeat row 13, as cols_thresholds): loaded here, in flight
  //      during the post-processing (at the top of the kernel they held 28
  //      VGPRs through both passes: 138 VGPRs, 3 waves / SIMD)
  float2 thr_r[2][KS / 2];
  if (THR) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const ImgDesc& d = u ? db : da;
      const int c = u ? jb.y : ja.y, strip = u ? jb.z : ja.z;
      if (g16 < d.qh) {
        const float2* t2 = reinterpret_cast<const float2*>(
            ep.thr + ((((int64_t)c * ep.maxph + g16) * ep.maxpw) + strip) * (KS * KS) + (int64_t)jlc * KS);
#pragma unroll
        for (int p = 0; p < KS / 2; ++p) thr_r[u][p] = t2[p];
      }
    }
  }
  // ---- Makhoul post-processing: (X[k], X[N - k]) = makhoul_pair(Z[k], Z[M - k])
  //      for k = jj + 8 i (i < 14): Z[k] at pad16 = jj + 8 i + i / 2; Z[M - k]
  //      at pad16 = 8 (14 - i) - jj + (13 - i) / 2 for jj >= 1, one more for
  //      jj = 0 and even i; k = 0 and k = M pair Z[0] with itself
  constexpr int M8 = M / 8;
  cf wv[M8 + 1];
  if (on_col) {
    const float* za = zs + 2 * jj * KSP + col;
    const int e = jj == 0 ? 1 : 0;
    const float* zbo = zs + 2 * (8 - jj) * KSP + col;       // odd i: + 8 (13 - i) + (13 - i) / 2
    const float* zbe = zs + 2 * (8 - jj + e) * KSP + col;   // even i >= 2
    const float* zb0 = jj == 0 ? zs + col : zs + 2 * (118 - jj) * KSP + col;   // i = 0: Z[112 - jj] or Z[0]
    const float4* pcl = pc + jj;
#pragma unroll
    for (int i = 0; i < M8; i += 2) {
      cf A[2], P[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ii = i + h;
        const int pa = 8 * ii + (ii >> 1);
        A[h] = (cf){za[2 * pa * KSP], za[(2 * pa + 1) * KSP]};
        const int pb = 8 * (13 - ii) + ((13 - ii) >> 1);
        const float* zb = ii == 0 ? zb0 : ((ii & 1) ? zbo + 2 * pb * KSP : zbe + 2 * pb * KSP);
        P[h] = (cf){zb[0], zb[KSP]};
      }
      makhoul_pair2(A[0], P[0], pcl[8 * i], A[1], P[1], pcl[8 * i + 8], wv[i], wv[i + 1]);
      if ((i & 3) == 2) __builtin_amdgcn_sched_barrier(0);   // bound the LDS reads in flight (registers)
    }
    if (jj == 0) {   // k = M: Z[0] with itself
      const cf Z0 = (cf){zs[col], zs[KSP + col]};
      const float4 cm = pc[M];
      wv[M8] = makhoul_pair(Z0, Z0, (cf){cm.x, cm.y}, (cf){cm.z, cm.w});
    }
  }
  __syncthreads();
  if (on_col) {
    float* xo = zs + jj * KSP + col;                          // X[k] at row k
    float* xn = zs + (N - jj - 8 * (M8 - 1)) * KSP + col;     // X[N - k], from the lowest row
    if (da.Kh >= N && db.Kh >= N) {   // every row kept (wave-uniform): no per-row compares
#pragma unroll
      for (int i = 0; i < M8; ++i) {
        xo[8 * i * KSP] = wv[i].x;
        if (i > 0 || jj > 0) xn[8 * (M8 - 1 - i) * KSP] = wv[i].y;
      }
      if (jj == 0) zs[M * KSP + col] = wv[M8].x;
    } else {
      const int Kh = col >= KS ? db.Kh : da.Kh;
#pragma unroll
      for (int i = 0; i < M8; ++i) {
        const int k = jj + 8 * i;
        if (k < Kh) xo[8 * i * KSP] = wv[i].x;
        if (k >= 1 && N - k < Kh) xn[8 * (M8 - 1 - i) * KSP] = wv[i].y;
      }
      if (jj == 0 && M < Kh) zs[M * KSP + col] = wv[M8].x;
    }
  }
  __syncthreads();
  // ---- token epilogue: tile (h = g16, strip) of each item
  if (THR) {
    const float* row0 = zs + (KS * g16 + jlc) * KSP;   // item 0: columns 0 .. 13; item 1: 14 .. 27
    uint32_t code0 = 0, code1 = 0;
    float am0 = 0.0f, am1 = 0.0f;
#pragma unroll
    for (int p = 0; p < KS / 2; ++p)
      code_bits4(code0, code1, am0, am1, (f2v){row0[2 * p], row0[2 * p + 1]},
                 (f2v){row0[KS + 2 * p], row0[KS + 2 * p + 1]}, thr_r[0][p], thr_r[1][p]);
    uint32_t u0 = __float_as_uint(am0), u1 = __float_as_uint(am1);
#define DCTAE_ROR_MAX(ctl)                                                        \
  u0 = max(u0, (uint32_t)__builtin_amdgcn_mov_dpp((int)u0, ctl, 0xf, 0xf, false)); \
  u1 = max(u1, (uint32_t)__builtin_amdgcn_mov_dpp((int)u1, ctl, 0xf, 0xf, false));
    DCTAE_ROR_MAX(0x128) DCTAE_ROR_MAX(0x124) DCTAE_ROR_MAX(0x122) DCTAE_ROR_MAX(0x121)
#undef DCTAE_ROR_MAX
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const ImgDesc& d = u ? db : da;
      const int c = u ? jb.y : ja.y, strip = u ? jb.z : ja.z;
      if (g16 < d.qh) {
        const int64_t tok = cols_tok(d, c, strip, g16, ep.C);
        sk.scores[tok] = __fadd_rn(__fmul_rn(__uint_as_float(u ? u1 : u0), ep.mw), sbias[u][g16]);
        if (sk.codes) sk.codes[tok * KS + jlc] = (uint16_t)(u ? code1 : code0);
        if (sk.raw) {
          const float* row = row0 + KS * u;
#pragma unroll
          for (int p2 = 0; p2 < KS; ++p2) sk.raw[tok * KS * KS + jlc * KS + p2] = row[p2];
        }
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const ImgDesc& d = u ? db : da;
      const int c = u ? jb.y : ja.y, strip = u ? jb.z : ja.z;
      for (int h = g16; h < d.qh; h += 16) {
        float vals[KS];
        const float* row = zs + (KS * h + jl) * KSP + KS * u;
#pragma unroll
        for (int p2 = 0; p2 < KS; ++p2) vals[p2] = row[p2];
        token_epilogue_p<KS>(ep, c, h, strip, jl, vals, cols_tok(d, c, strip, h, ep.C), sk);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------

int fft_spec_id(int N, const int* radix, int npass, int P) {
  if (P != 14 || npass != 2) return 0;
  if (N == 512 && radix[0] == 16 && radix[1] == 16) return 1;
  if (N == 224 && radix[0] == 16 && radix[1] == 7) return 2;
  return 0;
}

#ifndef DCTAE_ROWS224P
#define DCTAE_ROWS224P 2   // rows per wave of k_rows224p (2 or 3; 0: k_fft_rows2<224>)
#endif
int fft_spec_rows_per_block(int spec) {
  return spec == 2 ? (DCTAE_ROWS224P ? 4 * DCTAE_ROWS224P : 4 * DCTAE_RPW224) : (spec ? 16 : 0);
}

void launch_fft_rows_spec(int spec, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                          const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s) {
  if (n_blocks <= 0) return;
  if (spec == 1)
    hipLaunchKernelGGL((k_fft_rows2<512, 16, 16>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
  else if (spec == 2 && DCTAE_ROWS224P)
    hipLaunchKernelGGL((k_rows224p<DCTAE_ROWS224P == 3 ? 3 : 2>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb,
                       ws, tw, post, cm);
  else if (spec == 2)
    hipLaunchKernelGGL((k_fft_rows2<224, 16, 7>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
}

// spec 1 (N = 512): k_fft_cols7 over `list` (the job's 512-high images, one
// tile-column count qw) when given, else one k_fft_cols4 block per item;
// spec 2 (N = 224): k_fft_cols4.  thr: codes-only encode on the exact LFQ
// thresholds (14 x 14 codes), else the generic token epilogue.
void launch_fft_cols_spec(int spec, const ImgDesc* imgs, const int4* blocks, int n_blocks, const float* ws,
                          const float2* tw, const float2* post, const EncParams& ep, const TokenSinks& sk,
                          hipStream_t s, const int* list, int n_list, int qw) {
  if (n_blocks <= 0) return;
  const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
  if (spec == 1 && list && n_list > 0) {
    const int n_items = 3 * qw;
#ifndef DCTAE_C7_IPB
#define DCTAE_C7_IPB 2
#endif
    const int grid = cols7_grid(n_list, qw, thr ? DCTAE_C7_IPB : 2);
    if (thr)
      hipLaunchKernelGGL((k_fft_cols7<true, DCTAE_C7_IPB, true>), dim3(grid), dim3(256), 0, s, imgs, list, n_list,
                         n_items, qw, ws, tw, post, ep, sk);
    else
      hipLaunchKernelGGL((k_fft_cols7<false, 2, true>), dim3(grid), dim3(256), 0, s, imgs, list, n_list, n_items, qw,
                         ws, tw, post, ep, sk);
    return;
  }
#define DCTAE_COLS4(NN, RR, T)                                                                                  \
  hipLaunchKernelGGL((k_fft_cols4<NN, RR, 14, T>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk)
  if (spec == 1 && thr) DCTAE_COLS4(512, 16, true);
  else if (spec == 1) DCTAE_COLS4(512, 16, false);
#ifndef DCTAE_COLS224
#define DCTAE_COLS224 1
#endif
  else if (spec == 2 && DCTAE_COLS224 && thr)
    hipLaunchKernelGGL((k_cols224<true>), dim3(8 * (((n_blocks + 1) / 2 + 7) / 8)), dim3(256), 0, s, imgs, blocks,
                       n_blocks, ws, tw, post, ep, sk);
  else if (spec == 2 && DCTAE_COLS224)
    hipLaunchKernelGGL((k_cols224<false>), dim3(8 * (((n_blocks + 1) / 2 + 7) / 8)), dim3(256), 0, s, imgs, blocks,
                       n_blocks, ws, tw, post, ep, sk);
  else if (spec == 2 && thr) DCTAE_COLS4(224, 7, true);
  else if (spec == 2) DCTAE_COLS4(224, 7, false);
#undef DCTAE_COLS4
}

}  // namespace dctae
