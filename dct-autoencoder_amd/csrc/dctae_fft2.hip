// Compile-time specialised two-pass FFT-DCT kernels (M = N/2 = R1 * R2,
// at most 64/3 butterflies per job and pass) for the headline image sizes:
//   N = 512: M = 256 = 16 x 16        N = 224: M = 112 = 16 x 7
// Same maths as dctae_fft.hip (Makhoul + Stockham), but every index is a
// compile-time expression, passes are done in place (register staged), and
// the row kernel gives each image row to one wave (no block barriers).
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_launch.h"

// profiling builds only (tools/gpu_ablate.sh): skip parts of the column kernel
#ifndef DCTAE_THR_AT
#define DCTAE_THR_AT 2
#endif
#ifndef DCTAE_ABLATE
#define DCTAE_ABLATE 0
#endif

namespace dctae {

// padded complex slot of element m: one spare slot every 16 keeps the
// stride-16 Stockham accesses on distinct LDS banks
__device__ __forceinline__ constexpr int pad16(int m) { return m + (m >> 4); }

// ---------------------------------------------------------------------------
// rows: one wave = one image row, its 3 IPT channels are 3 jobs.  A row item
// is 16 rows (4 waves x RPW rows); T points at channel 0, row 0 of the
// image's row-pass output.  NT: RGB read with non-temporal loads (streamed
// once; keeps the XCD's L2 for T in the fused kernel).
// ---------------------------------------------------------------------------
template <int N>
struct RowsLds {
  static constexpr int M = N / 2;
  static constexpr int MP = pad16(M - 1) + 2;
  float2 z[4][3][MP];
};

// threadIdx.x through a volatile asm: not loop-invariant to the compiler, so
// the lane-derived LDS addresses of an item body are rebuilt per item instead
// of being hoisted out of the fused kernel's item loop (and kept live in VGPRs)
__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

template <int N, int R1, int R2, bool PF, bool NT>
__device__ __forceinline__ void rows2_item(const ImgDesc& d, int y_first, const float* __restrict__ rgb,
                                           float* __restrict__ T, RowsLds<N>& L, const float2* post_s,
                                           const float2* tw_s, const ColorMats& cm) {
  constexpr int M = N / 2;
  constexpr int MP = RowsLds<N>::MP;
  constexpr int B1 = M / R1, B2 = M / R2;
  constexpr int PX = (N + 63) / 64;        // pixels per lane and row
  constexpr int KI = (M + 63) / 64;        // k = lane + 64 i, i < KI, covers k < M (k = M by lane 0)
  constexpr int RPW = 4;                   // rows per wave (block = 16 rows)
  static_assert(R1 * R2 == M, "two-pass plan");
  static_assert(3 * B1 <= 64 && 3 * B2 <= 64, "one butterfly per lane per pass");
  static_assert(R1 == 16, "first radix 16 (Ns of pass 2 = 16)");
  const int tid = opaque_tid();
  const int wave = tid >> 6, lane = tid & 63;
  float2(*z)[MP] = L.z[wave];
  float* zf0 = reinterpret_cast<float*>(z[0]);
  float* zf1 = reinterpret_cast<float*>(z[1]);
  float* zf2 = reinterpret_cast<float*>(z[2]);
  const int H = d.H, Kw = d.Kw;
  const int64_t hw = (int64_t)H * N;
  const float* src = rgb + d.rgb_off;
  const float gam = 0.430000007152557373046875f;
  const int lay = d.t_strips;               // 0 row-major, 1 strips of 14, 2 strips padded to 16, 3 padded row-major
  const int SW = (lay >= 2) ? 16 : 14;       // strip row width (floats)
  // ---- lane-invariant index maps (the same for every row)
  int zo[PX];                               // Makhoul slot of pixel lane + 64 i
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int px = lane + 64 * i;
    const int v = (px & 1) ? (N - 1 - (px >> 1)) : (px >> 1);
    zo[i] = 2 * pad16(v >> 1) + (v & 1);
  }
  // T offset of coefficient kx within (channel, row): strips: (kx/14)*H*14 + kx%14, else kx; -1 = not kept
  int oa[KI], ob[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = lane + 64 * i;
    const int kx2 = N - k;
    oa[i] = (k < Kw) ? (lay == 3 ? (k / 14) * 16 + k % 14 : lay ? (k / 14) * H * SW + k % 14 : k) : -1;
    ob[i] = (k >= 1 && kx2 < Kw) ? (lay == 3 ? (kx2 / 14) * 16 + kx2 % 14 : lay ? (kx2 / 14) * H * SW + kx2 % 14 : kx2)
                                 : -1;
  }
  const int oM = (M < Kw) ? (lay == 3 ? (M / 14) * 16 + M % 14 : lay ? (M / 14) * H * SW + M % 14 : M) : -1;
  const int ystride = lay == 3 ? (Kw / 14) * 16 : lay ? SW : Kw;   // T offset step per row
  const int64_t cstride = lay >= 2 ? (int64_t)H * (Kw / 14) * 16 : (int64_t)H * Kw;  // per channel
  float pr[PX], pg[PX], pb[PX];
  auto fetch = [&](int y) {
    if (DCTAE_ABLATE & 64) {
#pragma unroll
      for (int i = 0; i < PX; ++i) pr[i] = pg[i] = pb[i] = 0.001f * (lane + 64 * i + y);
      return;
    }
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int px = lane + 64 * i;
      if (px < N && y < H) {
        const int64_t o = (int64_t)y * N + px;
        if (NT) {
          pr[i] = ld_nt(src + o);
          pg[i] = ld_nt(src + hw + o);
          pb[i] = ld_nt(src + 2 * hw + o);
        } else {
          pr[i] = src[o];
          pg[i] = src[hw + o];
          pb[i] = src[2 * hw + o];
        }
      }
    }
  };
  int y = y_first + wave;
  if (PF) fetch(y);
#pragma unroll 1
  for (int rr = 0; rr < RPW; ++rr, y += 4) {
    if (y >= H) break;
    if (!PF) fetch(y);
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
    if (PF) {
      __builtin_amdgcn_sched_barrier(0);
      fetch(y + 4);  // next row of this wave: in flight while this one is transformed
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
          if (!(DCTAE_ABLATE & 32)) {
            if (oa[i] >= 0) tb[oa[i]] = W.x;
            if (ob[i] >= 0) tb[ob[i]] = -W.y;
          } else if (W.x == 12345.0f) {
            tb[0] = W.y;   // keep the work alive
          }
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

template <int N, int R1, int R2, bool PF>
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
  rows2_item<N, R1, R2, PF, false>(d, jb.y, rgb, ws + d.ws_t, L, post_s, tw_s, cm);
}

// ---------------------------------------------------------------------------
// cols: one block = (image, channel, tile column); KS = P columns of T.
// LDS column layout: complex m of column col at re [2*pad16(m)*KSP + col],
// im [+KSP], KSP odd: with 16 butterflies of one column on consecutive lanes
// every Stockham read and write of a half-wave hits 32 distinct banks.
// ---------------------------------------------------------------------------
template <int N, int R1, int R2, int KS>
__global__ __launch_bounds__(256) void k_fft_cols2(const ImgDesc* __restrict__ imgs, const int4* __restrict__ blocks,
                                                   const float* __restrict__ ws, const float2* __restrict__ tw,
                                                   const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  constexpr int M = N / 2;
  constexpr int B1 = M / R1, B2 = M / R2;
  constexpr int KSP = KS | 1;              // odd row stride
  constexpr int ZROWS = 2 * (pad16(M - 1) + 1);
  static_assert(KS * 16 <= 256, "16 butterfly lanes per column");
  static_assert(B1 <= 16 && B2 <= 16 && R1 == 16, "plan shape");
  __shared__ float zs[ZROWS * KSP];
  __shared__ float2 post_s[2 * (M + 1)];
  __shared__ float2 tw_s[M];
  const int tid = threadIdx.x;
  const int4 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const int c = jb.y, strip = jb.z;
  const int Kw = d.Kw;
  // LFQ-bit thresholds of this thread's epilogue rows, fetched now so their
  // latency hides behind the transform (tiles h = g16 + 16 r, row jl)
  constexpr int EPR = 2;                    // epilogue rounds (qh <= 32 tiles, 16 groups)
  const int g16 = tid >> 4, jl = tid & 15;
  const bool use_thr = ep.median && ep.thr && !sk.norm && (KS % 2 == 0);
  float2 thr_r[EPR][KS / 2];
  if (use_thr) {
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
  }
  for (int i = tid; i < 2 * (M + 1); i += 256) post_s[i] = post[i];
  for (int i = tid; i < M; i += 256) tw_s[i] = tw[i];
  auto zre = [&](int m, int col) -> float& { return zs[2 * pad16(m) * KSP + col]; };
  auto zim = [&](int m, int col) -> float& { return zs[(2 * pad16(m) + 1) * KSP + col]; };
  auto put = [&](int y, int j, float v) {
    const int vv = (y & 1) ? (N - 1 - (y >> 1)) : (y >> 1);
    zs[(2 * pad16(vv >> 1) + (vv & 1)) * KSP + j] = v;
  };
  if (d.t_strips == 2) {
    // padded strips: row y of strip (c, w) = 16 floats at 64-byte alignment, 14 used
    const float4* T4 = reinterpret_cast<const float4*>(ws + d.ws_t + (int64_t)c * d.H * (Kw / KS) * 16 +
                                                       (int64_t)strip * N * 16);
#pragma unroll
    for (int q = tid; q < N * 4; q += 256) {
      const float4 t4 = T4[q];
      const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
      const int y = q >> 2, j0 = (q & 3) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j0 + u < KS) put(y, j0 + u, tv[u]);
    }
  } else if (d.t_strips) {
    const float4* T4 = reinterpret_cast<const float4*>(ws + d.ws_t + (int64_t)c * d.H * Kw + (int64_t)strip * N * KS);
    static_assert((N * KS) % 4 == 0, "strip of whole float4s");
#pragma unroll
    for (int q = tid; q < N * KS / 4; q += 256) {
      const float4 t4 = T4[q];
      const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = 4 * q + u;
        const int y = e / KS, j = e - y * KS;
        put(y, j, tv[u]);
      }
    }
  } else if ((KS & 1) == 0 && (Kw & 1) == 0) {
    // row-major T: KS/2 float2 per row (8-byte aligned: KS and Kw even)
    const float2* T2 = reinterpret_cast<const float2*>(ws + d.ws_t + (int64_t)c * d.H * Kw + strip * KS);
    const int rs = Kw / 2;
#pragma unroll 2
    for (int q = tid; q < N * (KS / 2); q += 256) {
      const int y = q / (KS / 2), p = q - y * (KS / 2);
      const float2 t2 = T2[(int64_t)y * rs + p];
      put(y, 2 * p, t2.x);
      put(y, 2 * p + 1, t2.y);
    }
  } else {
    const float* T = ws + d.ws_t + (int64_t)c * d.H * Kw + strip * KS;
#pragma unroll 4
    for (int e = tid; e < N * KS; e += 256) {
      const int y = e / KS, j = e - y * KS;
      put(y, j, T[(int64_t)y * Kw + j]);
    }
  }
  __syncthreads();
  const int jj = tid & 15, col = tid >> 4;   // butterfly on the lane, column across 16-lane groups
  const bool on_col = col < KS;
  // ---- pass 1 (Ns = 1)
  {
    float2 v[R1];
    const bool on = on_col && jj < B1;
    if (on) {
#pragma unroll
      for (int r = 0; r < R1; ++r) v[r] = make_float2(zre(jj + r * B1, col), zim(jj + r * B1, col));
      DFT<R1>::run(v);
    }
    __syncthreads();
    if (on) {
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        zre(jj * R1 + r, col) = v[r].x;
        zim(jj * R1 + r, col) = v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- pass 2 (Ns = R1)
  {
    float2 v[R2];
    const bool on = on_col && jj < B2;
    if (on) {
#pragma unroll
      for (int r = 0; r < R2; ++r) v[r] = make_float2(zre(jj + r * B2, col), zim(jj + r * B2, col));
#pragma unroll
      for (int r = 1; r < R2; ++r) v[r] = cmul(v[r], tw_s[r * jj]);
      DFT<R2>::run(v);
    }
    __syncthreads();
    if (on) {
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        zre(jj + r * R1, col) = v[r].x;
        zim(jj + r * R1, col) = v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- Makhoul post-processing into registers, then X[ky][col] (row stride KSP) in place
  constexpr int KPL = (M + 1 + 15) / 16;   // k values per lane
  float2 wv[KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = jj + 16 * i;
    if (on_col && k <= M) {
      const int ka = (k == M) ? 0 : k, kb = (k == 0) ? 0 : M - k;
      const float2 A = make_float2(zre(ka, col), zim(ka, col));
      const float2 B = make_float2(zre(kb, col), -zim(kb, col));
      const float2 al = post_s[2 * k], be = post_s[2 * k + 1];
      wv[i] = cadd(cmul(al, cadd(A, B)), cmul(be, csub(A, B)));
    }
  }
  __syncthreads();
  const int Kh = d.Kh;
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = jj + 16 * i;
    if (on_col && k <= M) {
      if (k < Kh) zs[k * KSP + col] = wv[i].x;
      if (k >= 1 && k < M && N - k < Kh) zs[(N - k) * KSP + col] = -wv[i].y;
    }
  }
  __syncthreads();
  // ---- token epilogue: tile (h, strip) of channel c, one 16-lane group per tile
  if (use_thr && d.qh <= 16 * EPR) {
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int h = g16 + 16 * r;
      if (h < d.qh) {
        float vals[KS];
#pragma unroll
        for (int p2 = 0; p2 < KS; ++p2) vals[p2] = (jl < KS) ? zs[(KS * h + jl) * KSP + p2] : 0.0f;
        const int f = (h * d.qw + strip) * ep.C + c;
        token_epilogue_thr<KS>(ep, c, h, strip, jl, vals, thr_r[r], d.tok_off + f, sk);
      }
    }
  } else {
    for (int h = g16; h < d.qh; h += 16) {
      float vals[KS];
#pragma unroll
      for (int p2 = 0; p2 < KS; ++p2) vals[p2] = (jl < KS) ? zs[(KS * h + jl) * KSP + p2] : 0.0f;
      const int f = (h * d.qw + strip) * ep.C + c;
      token_epilogue_p<KS>(ep, c, h, strip, jl, vals, d.tok_off + f, sk);
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

// one column item: (image d, channel c, tile column strip); T = the image's
// row-pass output (channel 0, row 0).  NTL: T read with non-temporal loads,
// which bypass the CU's L1 (the fused kernel reads T that other CUs of the
// XCD have just written).  Caller: post_s / tw_s loaded, a block barrier
// since the previous use of zs.
template <int N, int R2, int KS, bool THR, bool NTL, int THR_AT = 0>
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
  if (THR && THR_AT == 0) load_thr();
  if (THR && tid < 32) sbias[tid] = __fdiv_rn(-(float)(tid + strip), ep.ci[c]);
  // ---- T slice -> LDS, natural row order
  if (d.t_strips == 3) {
    // padded row-major: the slice row is one aligned 64-B segment (14 of 16 floats used);
    // thread (y0 = t / 4, q = t % 4) copies float4 q of rows y0 + 64 k
    const int q = tid & 3, y0 = tid >> 2;
    const int64_t rs = (int64_t)(d.Kw / KS) * 16;
    const float4* src = reinterpret_cast<const float4*>(T + ((int64_t)c * d.H + y0) * rs + strip * 16) + q;
    constexpr int NK4 = (N + 63) / 64;
    float4 tv[NK4];
#pragma unroll
    for (int k = 0; k < NK4; ++k)
      if (N % 64 == 0 || y0 + 64 * k < N) tv[k] = src[k * 16 * rs];
    float* dst = zs + y0 * KSP + 4 * q;
#pragma unroll
    for (int k = 0; k < NK4; ++k) {
      if (N % 64 != 0 && y0 + 64 * k >= N) continue;
      dst[64 * KSP * k] = tv[k].x;
      dst[64 * KSP * k + 1] = tv[k].y;
      if (q < 3) {
        dst[64 * KSP * k + 2] = tv[k].z;
        dst[64 * KSP * k + 3] = tv[k].w;
      }
    }
  } else if (!(DCTAE_ABLATE & 1) && tid < 32 * (KS / 2)) {
    // row-major: thread (y0 = t / 7, p = t % 7) copies float2 p of rows y0 + 32k
    const int y0 = tid / (KS / 2), p = tid - y0 * (KS / 2);
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v* src = reinterpret_cast<const f2v*>(T + ((int64_t)c * d.H + y0) * d.Kw + strip * KS) + p;
    const int64_t rstep = (int64_t)16 * d.Kw;   // 32 rows, in float2
    float* dst = zs + y0 * KSP + 2 * p;
    f2v tv[N / 32];
#pragma unroll
    for (int k = 0; k < N / 32; ++k) tv[k] = NTL ? ld_nt(src + k * rstep) : src[k * rstep];
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
    const bool on = on_col && jj < B1 && !(DCTAE_ABLATE & 2);
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
    const bool on = on_col && !(DCTAE_ABLATE & 4);
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
  if (THR && THR_AT == 1) load_thr();
  // ---- Makhoul post-processing: k = jj + 16 i, A = Z[k] (pad16 = jj + 17 i),
  //      B = conj Z[M - k] (pad16 = bb - 17 i); k = 0 and k = M use Z[0]
  constexpr int KPL = M16 + 1;
  cf wv[KPL];
  if (on_col && !(DCTAE_ABLATE & 8)) {
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
  if (on_col && !(DCTAE_ABLATE & 8)) {
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
  if (THR && THR_AT == 2) load_thr();
  // ---- token epilogue: tile (h, strip) of channel c, one 16-lane group per tile
  if (DCTAE_ABLATE & 16) return;
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
          code |= (v0 >= thr_r[r][p].x ? 1u : 0u) << (KS - 1 - 2 * p);   // MSB-first (lfq.py:187)
          code |= (v1 >= thr_r[r][p].y ? 1u : 0u) << (KS - 2 - 2 * p);
        }
        am = jl < KS ? am : 0u;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o, 64));
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

// ---------------------------------------------------------------------------
// cols, complex-pair LDS form (N = 512, P = 14): every complex value is one
// 8-byte LDS word, so each butterfly operand is one ds_read_b64 / ds_write_b64
// (half the LDS instructions of the split re/im rows of cols4).
//   z[m][col] at float2 index pad16(m) * 14 + col: the stride-16 Stockham
//   accesses of a half-wave (16 butterflies x 2 columns) hit 32 distinct
//   8-byte bank pairs (14 jj mod 32 distinct and even, col parity odd/even);
//   the Makhoul reorder is applied while copying T in: z[m] = (x[4m], x[4m+2])
//   for m < M/2, (x[2N-1-4m], x[2N-3-4m]) above;
//   X[k][col] (real, after the post-processing) at float index k * 14 + col,
//   in place; the epilogue reads a tile row as 7 ds_read_b64.
// ---------------------------------------------------------------------------
// float2 slot of complex element m of column 0 (column col at + col):
//   zaddr(m) = 15 (m % 16) + 257 (m / 16)
// * stride-16 reads z[jj + 16 r] (16 butterflies x 2 columns per half-wave):
//   15 jj + col distinct mod 32 but for one pair -> ds_read_b64 ~conflict-free;
// * pass-1 writes z[16 jj + r] (257 jj = jj mod 16) and pass-2 writes
//   z[jj + 16 r] (15 jj) hit 16 distinct 8-byte slots per 16-lane store group;
// * the m + 16 step (257 x 8 bytes) is beyond ds_read2_b64's 8-bit offset, so
//   butterfly operands are not paired into ds_read2_b64 (8 LDS cycles for the
//   pair against 2 + 2 for two ds_read_b64).
__device__ __forceinline__ constexpr int zaddr(int m) { return 15 * (m & 15) + 257 * (m >> 4); }

struct Cols5Lds {
  static constexpr int KS = 14;
  float2 z[zaddr(255) + KS];
};

typedef float f2v __attribute__((ext_vector_type(2)));

// cols5 pieces.  Thresholds of this thread's epilogue rows: tiles h = g16 + 16 r, row jl.
template <bool THR>
__device__ __forceinline__ void cols5_thresholds(const ImgDesc& d, int c, int strip, const EncParams& ep,
                                                 float2 (&thr_r)[2][7], float* sbias) {
  constexpr int KS = 14, EPR = 2;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = tid & 15;
  if (THR) {
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
  }
  if (THR && tid < 32) sbias[tid] = __fdiv_rn(-(float)(tid + strip), ep.ci[c]);
}

// the T slice (512 rows x 14 columns) of (c, strip) into registers: item i = (m, p)
template <bool NTL>
__device__ __forceinline__ void cols5_load(const ImgDesc& d, int c, int strip, const float* __restrict__ T,
                                           f2v (&va)[7], f2v (&vb)[7]) {
  constexpr int N = 512, M = 256, KS = 14;
  const int tid = opaque_tid();
  const f2v* base = reinterpret_cast<const f2v*>(T + (int64_t)c * d.H * d.Kw + strip * KS);
  const int rs = d.Kw >> 1;
#pragma unroll
  for (int u = 0; u < 7; ++u) {
    if (DCTAE_ABLATE & 1) { va[u] = vb[u] = (f2v){1.0f, 2.0f}; continue; }
    const int i = tid + 256 * u;
    const int m = i / 7, p = i - m * 7;
    const int ya = m < M / 2 ? 4 * m : 2 * N - 1 - 4 * m;
    const f2v* pa = base + ya * rs + p;
    const f2v* pb = base + (m < M / 2 ? ya + 2 : ya - 2) * rs + p;
    va[u] = NTL ? ld_nt(pa) : *pa;
    vb[u] = NTL ? ld_nt(pb) : *pb;
  }
}

// registers -> z, Makhoul reorder: z[m] = (x[4m], x[4m+2]) / (x[2N-1-4m], x[2N-3-4m])
__device__ __forceinline__ void cols5_stage(float2* zc, const f2v (&va)[7], const f2v (&vb)[7]) {
  constexpr int KS = 14;
  const int tid = opaque_tid();
#pragma unroll
  for (int u = 0; u < 7; ++u) {
    const int i = tid + 256 * u;
    const int m = i / 7, p = i - m * 7;
    f2v* z = reinterpret_cast<f2v*>(zc + zaddr(m) + 2 * p);
    z[0] = (f2v){va[u].x, vb[u].x};
    z[1] = (f2v){va[u].y, vb[u].y};
  }
}

// token epilogue of one (channel, tile column) item: X2 = the 448 x 14 kept
// coefficients (float index k * 14 + col) in LDS; tile (h, strip) per 16-lane
// group g16 (+16 r), tile row jl; codes from the thresholds held in registers
template <bool THR>
__device__ __forceinline__ void cols5_epilogue(const ImgDesc& d, int c, int strip, const f2v* X2, const float* sbias,
                                               const float2 (&thr_r)[2][7], const EncParams& ep,
                                               const TokenSinks& sk) {
  constexpr int KS = 14, EPR = 2;
  const int tid = opaque_tid();
  const int g16 = tid >> 4, jl = tid & 15;
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
          code |= (v2.x >= thr_r[r][p].x ? 1u : 0u) << (KS - 1 - 2 * p);   // MSB-first (lfq.py:187)
          code |= (v2.y >= thr_r[r][p].y ? 1u : 0u) << (KS - 2 - 2 * p);
        }
        am = jl < KS ? am : 0u;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o, 64));
        const int64_t tok = d.tok_off + (h * d.qw + strip) * ep.C + c;
        if (jl == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(__uint_as_float(am), ep.mw), sbias[h]);
        if (jl < KS && sk.codes) sk.codes[tok * KS + jl] = (uint16_t)code;
        if (sk.raw && jl < KS) {
#pragma unroll
          for (int p = 0; p < KS / 2; ++p) {
            const f2v v2 = row[p];
            sk.raw[tok * KS * KS + jl * KS + 2 * p] = v2.x;
            sk.raw[tok * KS * KS + jl * KS + 2 * p + 1] = v2.y;
          }
        }
      }
    }
  } else {
    for (int h = g16; h < d.qh; h += 16) {
      float vals[KS];
      const f2v* row = X2 + (KS * h + (jl < KS ? jl : 0)) * (KS / 2);
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) {
        const f2v v2 = row[p];
        vals[2 * p] = v2.x;
        vals[2 * p + 1] = v2.y;
      }
      const int f = (h * d.qw + strip) * ep.C + c;
      token_epilogue_p<KS>(ep, c, h, strip, jl, vals, d.tok_off + f, sk);
    }
  }
}

// z staged (and a barrier since): column FFT-DCT, post-processing, token epilogue
template <bool THR>
__device__ __forceinline__ void cols5_compute(const ImgDesc& d, int c, int strip, float2* zc, const float4* post4,
                                              const float2* tw_s, const float* sbias, const float2 (&thr_r)[2][7],
                                              const EncParams& ep, const TokenSinks& sk) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14, M16 = 16, EPR = 2;
  const int tid = opaque_tid();
  const int jj = tid & 15, col = tid >> 4;
  const bool on_col = col < KS;
  const int g16 = tid >> 4, jl = tid & 15;
  constexpr int S16 = 257;   // float2 step of m + 16 (zaddr)
  const cf* zr = reinterpret_cast<const cf*>(zc) + 15 * jj + col;   // z[jj + 16 r] = 15 jj + 257 r
  // ---- pass 1 (Ns = 1): z[jj + 16 r] -> DFT16 -> z[16 jj + r]
  if (!(DCTAE_ABLATE & 2)) {
    cf v[16];
    if (on_col) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = zr[S16 * r];
      DFTV<16>::run(v);
    }
    __syncthreads();
    if (on_col) {
      cf* zw = reinterpret_cast<cf*>(zc) + S16 * jj + col;      // zaddr(16 jj + r) = 257 jj + 15 r
#pragma unroll
      for (int r = 0; r < 16; ++r) zw[15 * r] = v[r];
    }
    __syncthreads();
  }
  // ---- pass 2 (Ns = 16): z[jj + 16 r] * W_M^{r jj} -> DFT16 -> in place
  if (!(DCTAE_ABLATE & 4)) {
    cf v[16];
    if (on_col) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = zr[S16 * r];
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        const float2 w = tw_s[r * jj];
        v[r] = cmul_pk(v[r], (cf){w.x, w.y});
      }
      DFTV<16>::run(v);
    }
    __syncthreads();
    if (on_col) {
      cf* zw = reinterpret_cast<cf*>(zc) + 15 * jj + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) zw[S16 * r] = v[r];
    }
    __syncthreads();
  }
  // ---- Makhoul post-processing: k = jj + 16 i; A = Z[k], B = conj Z[M - k] (Z[0] at k = 0, M)
  cf wv[M16 + 1];
  if (on_col && !(DCTAE_ABLATE & 8)) {
    // Z[M - k]: zaddr = 257 (15 - i) + 15 (16 - jj) (jj >= 1), 257 (16 - i) (jj = 0)
    const cf* zb = reinterpret_cast<const cf*>(zc) + (jj == 0 ? S16 : 15 * (16 - jj)) + col;
    const float4* ps = post4 + jj;
#pragma unroll
    for (int i = 0; i < M16; ++i) {
      const cf A = zr[S16 * i];
      cf Bc;
      if (i == 0) Bc = jj == 0 ? A : zb[S16 * 15];
      else Bc = zb[S16 * (15 - i)];
      const float4 ab = ps[16 * i];
      const cf al = (cf){ab.x, ab.y}, be = (cf){ab.z, ab.w};
      const cf s1 = add_conj(A, Bc), d1 = sub_conj(A, Bc);   // A + B, A - B with B = conj Z[M - k]
      wv[i] = fma_iw(d1, be, fma_x(d1, be, fma_iw(s1, al, mul_x(s1, al))));
    }
    if (jj == 0) {   // k = M
      const cf A = zr[0];
      const float4 ab = post4[M];
      const cf s1 = add_conj(A, A), d1 = sub_conj(A, A);
      wv[M16] = fma_iw(d1, (cf){ab.z, ab.w}, fma_x(d1, (cf){ab.z, ab.w}, cmul_pk(s1, (cf){ab.x, ab.y})));
    }
  }
  __syncthreads();
  const int Kh = d.Kh;
  float* X = reinterpret_cast<float*>(zc);
  if (on_col && !(DCTAE_ABLATE & 8)) {
    float* xo = X + jj * KS + col;                             // X[k], k = jj + 16 i
    float* xn = X + (N - jj - 16 * (M16 - 1)) * KS + col;      // X[N - k], from the lowest row
#pragma unroll
    for (int i = 0; i < M16; ++i) {
      const int k = jj + 16 * i;
      if (k < Kh) xo[16 * KS * i] = wv[i].x;
      if (k >= 1 && N - k < Kh) xn[16 * KS * (M16 - 1 - i)] = -wv[i].y;
    }
    if (jj == 0 && M < Kh) X[M * KS + col] = wv[M16].x;
  }
  __syncthreads();
  // ---- token epilogue: tile (h, strip) of channel c, one 16-lane group per tile, row jl
  if (DCTAE_ABLATE & 16) return;
  cols5_epilogue<THR>(d, c, strip, reinterpret_cast<const f2v*>(zc), sbias, thr_r, ep, sk);
}


template <bool THR, bool NTL>
__device__ __forceinline__ void cols5_item(const ImgDesc& d, int c, int strip, const float* __restrict__ T,
                                           float2* zc, const float4* post4, const float2* tw_s, float* sbias,
                                           const EncParams& ep, const TokenSinks& sk) {
  float2 thr_r[2][7];
  cols5_thresholds<THR>(d, c, strip, ep, thr_r, sbias);
  f2v va[7], vb[7];
  cols5_load<NTL>(d, c, strip, T, va, vb);
  cols5_stage(zc, va, vb);
  __syncthreads();
  cols5_compute<THR>(d, c, strip, zc, post4, tw_s, sbias, thr_r, ep, sk);
}

template <bool THR>
__global__ __launch_bounds__(256) void k_fft_cols5(const ImgDesc* __restrict__ imgs, const int4* __restrict__ blocks,
                                                   const float* __restrict__ ws, const float2* __restrict__ tw,
                                                   const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  constexpr int M = 256;
  __shared__ Cols5Lds L;
  __shared__ float4 post4[M + 1];
  __shared__ float2 tw_s[M];
  __shared__ float sbias[32];
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int i = threadIdx.x; i < M + 1; i += 256) post4[i] = p4[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  const int4 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  cols5_item<THR, false>(d, jb.y, jb.z, ws + d.ws_t, L.z, post4, tw_s, sbias, ep, sk);
}

// ---------------------------------------------------------------------------
// cols, several images per block (N = 512): block b owns ONE (channel, tile
// column) item t and IPB consecutive images: the LDS tables and the item's
// LFQ thresholds (2.4 MB per image over all items) are loaded once per IPB
// images, and with PF the next image's T slice is loaded into registers while
// the current one is transformed.  The image loop is fully unrolled: as a
// run-time loop the compiler's allocation of the same body needs ~180 VGPRs
// (82 straight-line).  Items are dealt so that the 8 XCD groups (b % 8) own
// contiguous runs of tile columns: the 56-byte row slices of neighbouring
// items share L2 lines on one XCD.
// ---------------------------------------------------------------------------
template <bool THR, int IPB, bool PF>
__global__ __launch_bounds__(256) void k_fft_cols6(const ImgDesc* __restrict__ imgs, const int* __restrict__ list,
                                                   int n_list, int n_items, int qw,
                                                   const float* __restrict__ ws, const float2* __restrict__ tw,
                                                   const float2* __restrict__ post, EncParams ep, TokenSinks sk) {
  constexpr int M = 256;
  __shared__ Cols5Lds L;
  __shared__ float4 post4[M + 1];
  __shared__ float2 tw_s[M];
  __shared__ float sbias[32];
  const int per_x = (n_items + 7) / 8;
  const int b = blockIdx.x, slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, g = slot / per_x;
  const int k0 = g * IPB;
  if (t >= n_items || k0 >= n_list) return;
  const int c = t / qw, strip = t - c * qw;
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int i = threadIdx.x; i < M + 1; i += 256) post4[i] = p4[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = tw[i];
  float2 thr_r[2][7];
  cols5_thresholds<THR>(imgs[list[k0]], c, strip, ep, thr_r, sbias);
  f2v va[7], vb[7];
  if (PF) {
    const ImgDesc d0 = imgs[list[k0]];
    cols5_load<false>(d0, c, strip, ws + d0.ws_t, va, vb);
  }
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int k = k0 + u;
    if (k < n_list) {
      const ImgDesc dk = imgs[list[k]];
      if (!PF) cols5_load<false>(dk, c, strip, ws + dk.ws_t, va, vb);
      cols5_stage(L.z, va, vb);
      __syncthreads();
      if (PF && u + 1 < IPB && k + 1 < n_list) {
        const ImgDesc dn = imgs[list[k + 1]];
        cols5_load<false>(dn, c, strip, ws + dn.ws_t, va, vb);   // in flight during the transform
      }
      cols5_compute<THR>(dk, c, strip, L.z, post4, tw_s, sbias, thr_r, ep, sk);
      __syncthreads();
    }
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
__device__ __forceinline__ constexpr int z7addr(int m) { return 16 * (m ^ ((m >> 3) & 1)); }

__device__ __forceinline__ int cols7_j2(int w, int g) {
  // wave 0: 0, 8, 1, 15;  wave w > 0: 2w, 16 - 2w, 2w + 1, 15 - 2w
  const int a = (g & 2) ? 2 * w + 1 : 2 * w;
  const int base = (w == 0 && g < 2) ? (g ? 8 : 0) : ((g & 1) ? (g & 2 ? 15 - 2 * w : 16 - 2 * w) : a);
  return base;
}

__device__ __forceinline__ float partner_row(float x, bool even_row) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(even_row ? r[1] : r[0]);
}

// X aliases z (one more barrier, 37 KB instead of 62 KB: 4 workgroups per CU)
union Cols7Lds {
  float2 z[256 * 16];
  float X[448 * 14];
};

template <bool NTL>
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
  constexpr int aux = NTL ? 2 : 0;   // slc: streamed once
  if (DCTAE_ABLATE & 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) va[r] = vb[r] = (float)(lo + r);
    return;
  }
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

// Makhoul post of cols7 for one lane: v = Z[j2 + 16 i]; writes X[k], X[N - k]
// (Kh = 448: X[N - k] kept for k > 64) and X[M] (j2 = 0).  W0: wave 0, whose
// rows 0 and 1 (j2 = 0, 8) pair with themselves.
template <bool W0>
__device__ __forceinline__ void cols7_post(const cf (&v)[16], int j2, int g, int col, const float4* post4,
                                           float* Xs) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14;
  const bool on_col = col < KS;
  const bool self = W0 && g < 2;
  float* xa = Xs + j2 * KS + col;                        // X[j2 + 16 i] at + 224 i
  float* xb = Xs + (N - j2 - 16 * 15) * KS + col;        // X[N - j2 - 16 i] at + 224 (15 - i)
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
    if (on_col) {
      xa[224 * i] = W.x;
      if (i > 4 || (i == 4 && j2 > 0)) xb[224 * (15 - i)] = -W.y;
    }
  }
  if (W0 && j2 == 0 && on_col) {   // k = M (< Kh): A = B = Z[0]
    const cf A = v[0];
    const float4 ab = post4[M];
    const cf s1 = add_conj(A, A), d1 = sub_conj(A, A);
    const cf W = fma_iw(d1, (cf){ab.z, ab.w}, fma_x(d1, (cf){ab.z, ab.w}, cmul_pk(s1, (cf){ab.x, ab.y})));
    Xs[M * KS + col] = W.x;
  }
}

template <bool THR>
__device__ __forceinline__ void cols7_compute(const ImgDesc& d, int c, int strip, Cols7Lds& L, const float (&va)[16],
                                              const float (&vb)[16], const float4* post4, const float2* tw_s,
                                              const float* sbias, const float2 (&thr_r)[2][7], const EncParams& ep,
                                              const TokenSinks& sk) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14, M16 = 16;
  const int tid = opaque_tid();
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), g = (tid >> 4) & 3, col = tid & 15;
  const bool on_col = col < KS;
  cf* z = reinterpret_cast<cf*>(L.z);
  (void)d;
  // ---- pass 1 (Ns = 1): j1 = tid >> 4
  {
    const int j1 = tid >> 4;
    cf v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = (cf){va[r], vb[r]};
    DFTV<16>::run(v);
    if (on_col) {
      cf* zw = z + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) zw[z7addr(16 * j1 + r)] = v[r];
    }
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
  // ---- Makhoul post: k = j2 + 16 i; A = Z[k], B = conj Z[M - k]
  //      j2 >= 1: Z[M - k] = partner row's v[15 - i] (lane ^ 16, ds_swizzle);
  //      j2 = 0: own v[(16 - i) & 15];  j2 = 8: own v[15 - i]  (wave 0, rows 0 and 1)
  //      kept rows: Kh = 448 (H = 512): X[k] always, X[N - k] for k > 64
  if (DCTAE_ABLATE & 8) {
#pragma unroll
    for (int i = 0; i < 16; ++i) L.X[(j2 * 14 + col + 224 * i) % 6272] = v[i].x + v[i].y;
  } else if (w == 0) cols7_post<true>(v, j2, g, col, post4, L.X);
  else cols7_post<false>(v, j2, g, col, post4, L.X);
  __syncthreads();
  if (DCTAE_ABLATE & 16) return;
  cols5_epilogue<THR>(d, c, strip, reinterpret_cast<const f2v*>(L.X), sbias, thr_r, ep, sk);
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
  cols5_thresholds<THR>(imgs[list[k0]], c, strip, ep, thr_r, sbias);
  float va[16], vb[16];
  {
    const ImgDesc d0 = imgs[list[k0]];
    cols7_load<false>(d0, c, strip, ws + d0.ws_t, va, vb);
  }
  __syncthreads();   // tables
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int k = k0 + u;
    if (k < n_list) {
      const ImgDesc dk = imgs[list[k]];
      if (u > 0 && !PF) cols7_load<false>(dk, c, strip, ws + dk.ws_t, va, vb);
      float na[16], nb[16];
      if (PF && u + 1 < IPB && k + 1 < n_list) {
        const ImgDesc dn = imgs[list[k + 1]];
        cols7_load<false>(dn, c, strip, ws + dn.ws_t, na, nb);   // in flight during the transform
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
  cols4_item<N, R2, KS, THR, false>(d, jb.y, jb.z, ws + d.ws_t, L.z, post_s, tw_s, sbias, ep, sk);
}

// ---------------------------------------------------------------------------
// Fused encode: rows and columns of the same images in ONE persistent launch,
// the intermediate T kept on chip.  Every workgroup reads its XCD id and
// serves that XCD's images q, q + n_xcd, ... (j-th image of the queue =
// image q + n_xcd j); it is a ROW worker or a COLUMN worker for its whole
// life (two loops: each keeps the register allocation of its own body), the
// share of row workers set by rows_pct; worker 0 of an XCD rows, worker 1
// columns.  Items are claimed in order from per-XCD counters:
//   row item (j, s):    rows 16 s .. 16 s + 15 of image j -> T slot j % slots
//   column item (j, s): channel s / qw, tile column s % qw of image j
// Dependences (each on items that are claimed in order and never wait on
// the waiter, so they always drain):
//   column items of j wait for all nr row items of j (rows_done[img] == nr);
//   row items of j wait for all nc column items of j - slots (slot reuse).
// Producer and consumer are on the same XCD by construction (queue =
// XCC_ID), so the hand-off goes through that XCD's L2: producers wait for
// their stores (vmcnt(0)) before one relaxed agent-scope counter add per
// workgroup; consumers poll the counter and read T with non-temporal loads,
// which bypass the (stale-prone) CU L1.  No release fence writes the ring
// back: n_xcd * slots slots of 2.75 MB (512^2) stay in L2 / Infinity Cache.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// The dependence helpers below keep every branch WAVE-uniform (wave 0 of the
// workgroup does the work, the branch tested on readfirstlane(threadIdx.x)):
// a `threadIdx.x == 0` region inside the persistent loop is a divergent
// branch to the compiler, whose CFG structurizer then builds a loop around
// the barriers that does not re-run the claim (a hang on gfx950 / ROCm 7.2).
__device__ __forceinline__ bool is_wave0() { return __builtin_amdgcn_readfirstlane((int)threadIdx.x) == 0; }

// wave 0: spin until *p >= target (bounded; false on time-out); uniform result
__device__ __forceinline__ bool wait_count(const int* p, int target, int limit) {
  for (int n = 0;; ++n) {
    const int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v >= target) return true;
    if (n >= limit) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// one add of 1 from wave 0 (lane 0's term; the other lanes add 0)
__device__ __forceinline__ int wave_add1(int* p) {
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int old = __hip_atomic_fetch_add(p, lane == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(old);
}

// every thread: own stores complete, then one counter add for the workgroup
__device__ __forceinline__ void signal_done(int* p) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (is_wave0()) wave_add1(p);
}

// wait (wave 0 polls) then release the workgroup; err |= 8 on time-out
__device__ __forceinline__ void wait_all(const int* p, int target, int limit, int* err) {
  if (is_wave0()) {
    if (!wait_count(p, target, limit)) atomicOr(err, 8);
  }
  __syncthreads();
  // acquire: invalidate this CU's L1 (a ring slot read before may hold stale
  // lines of its previous image) and keep the item's loads below the wait
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// claim the next item of a counter (block-uniform result)
__device__ __forceinline__ int claim(int* ctr, int* s_slot) {
  if (is_wave0()) *s_slot = wave_add1(ctr);
  __syncthreads();
  const int it = __builtin_amdgcn_readfirstlane(*s_slot);
  __syncthreads();
  return it;
}

template <int N, int R2, bool THR>
__global__ __launch_bounds__(256, 4) void k_enc_fused(FusedParams p_, const ImgDesc* __restrict__ imgs) {
  const FusedArgs& a = p_.a;
  constexpr int M = N / 2;
  union Lds {
    RowsLds<N> r;
    ColsLds<N> c;
    Cols7Lds c7;   // N = 512 column items (cols7)
  };
  __shared__ Lds L;
  __shared__ float4 post4[M + 1];   // (alpha_k, beta_k) pairs
  float2* const post_s = reinterpret_cast<float2*>(post4);
  __shared__ float2 tw_s[M];
  __shared__ float sbias[32];
  __shared__ int s_int;
  const FusedArgs& a0 = a;
  for (int i = threadIdx.x; i < 2 * (M + 1); i += 256) post_s[i] = a0.post[i];
  for (int i = threadIdx.x; i < M; i += 256) tw_s[i] = a0.tw[i];
  const int n_xcd = a0.n_xcd, n_img = a0.n_img, nr = a0.nr, nc = a0.nc, slots = a0.slots;
  int* const sync = a0.sync;
  const int q = n_xcd > 1 ? xcc_id() % n_xcd : 0;
  const int nj = n_img > q ? (n_img - q + n_xcd - 1) / n_xcd : 0;
  int* rows_done = sync + 24;
  int* cols_done = sync + 24 + n_img;
  // one claim sequence per XCD: R(0) .. R(look - 1), then [C(j), R(j + look)] per image j
  const int look = min(a0.look, nj);
  const int per = nr + nc;
  const int n_full = nj - look;
  const int head = look * nr;
  const int total = head + n_full * per + look * nc;
  uint64_t prof_w = 0, prof_r = 0, prof_c = 0, n_r = 0, n_c = 0;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  for (;;) {
    const int it = claim(sync + q, &s_int);
    if (it >= total) break;
    bool row;
    int j, sub;
    if (it < head) {
      row = true;
      j = it / nr;
      sub = it - j * nr;
    } else {
      int u = it - head;
      if (u < n_full * per) {
        const int blk = u / per, off = u - blk * per;
        row = off >= nc;
        j = row ? blk + look : blk;
        sub = row ? off - nc : off;
      } else {
        u -= n_full * per;
        row = false;
        j = n_full + u / nc;
        sub = u - (j - n_full) * nc;
      }
    }
    const int img = q + n_xcd * j;
    const ImgDesc d = imgs[img];
    float* T = a.ring + (int64_t)(q * slots + j % slots) * a.slot_floats;
    if (row) {
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      if (j >= slots && !(a.debug & 1))   // the slot's previous image: all its columns read
        wait_all(cols_done + img - n_xcd * slots, nc, a.spin_limit, a.err);
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      const ColorMats& cm = p_.cm;
      rows2_item<N, 16, R2, false, true>(d, 16 * sub, a.rgb, T, L.r, post_s, tw_s, cm);
      signal_done(rows_done + img);
      if (a.prof) {
        prof_w += t1 - t0;
        prof_r += __builtin_amdgcn_s_memtime() - t1;
        ++n_r;
      }
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      if (!(a.debug & 1)) wait_all(rows_done + img, nr, a.spin_limit, a.err);
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      const int qw = a.qw;
      const int c = sub / qw, strip = sub - c * qw;
      const EncParams& ep = p_.ep;
      const TokenSinks& sk = p_.sk;
      if constexpr (N == 512) {
        float2 thr_r[2][7];
        cols5_thresholds<THR>(d, c, strip, ep, thr_r, sbias);
        float va[16], vb[16];
        cols7_load<true>(d, c, strip, T, va, vb);
        cols7_compute<THR>(d, c, strip, L.c7, va, vb, post4, tw_s, sbias, thr_r, ep, sk);
      } else {
        cols4_item<N, R2, 14, THR, true, DCTAE_THR_AT>(d, c, strip, T, L.c.z, post_s, tw_s, sbias, ep, sk);
      }
      signal_done(cols_done + img);
      if (a.prof) {
        prof_w += t1 - t0;
        prof_c += __builtin_amdgcn_s_memtime() - t1;
        ++n_c;
      }
    }
  }
  if (a.prof && is_wave0()) {   // per-XCD totals: wait, row work, column work (s_memtime ticks), items
    const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if (lane == 0) {
      unsigned long long* pr = a.prof + 8 * q;
      atomicAdd(pr + 0, (unsigned long long)prof_w);
      atomicAdd(pr + 1, (unsigned long long)prof_r);
      atomicAdd(pr + 2, (unsigned long long)prof_c);
      atomicAdd(pr + 3, (unsigned long long)n_r);
      atomicAdd(pr + 4, (unsigned long long)n_c);
      atomicAdd(pr + 5, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
      atomicAdd(pr + 6, 1ull);
    }
  }
}

int fused_rows_per_item() { return 16; }

void launch_enc_fused(int spec, bool thr, int grid, const FusedArgs& a, const ColorMats& cm, const EncParams& ep,
                      const TokenSinks& sk, hipStream_t s) {
  if (a.n_img <= 0 || grid <= 0) return;
  FusedParams fp{a, cm, ep, sk};
#define DCTAE_FUSED(NN, RR, T) hipLaunchKernelGGL((k_enc_fused<NN, RR, T>), dim3(grid), dim3(256), 0, s, fp, a.imgs)
  if (spec == 1 && thr) DCTAE_FUSED(512, 16, true);
  else if (spec == 1) DCTAE_FUSED(512, 16, false);
  else if (spec == 2 && thr) DCTAE_FUSED(224, 7, true);
  else if (spec == 2) DCTAE_FUSED(224, 7, false);
#undef DCTAE_FUSED
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

int fft_spec_rows_per_block(int spec) { return spec ? 16 : 0; }

void launch_fft_rows_spec(int spec, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                          const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s, int prefetch) {
  if (n_blocks <= 0) return;
  if (spec == 1) {
    if (prefetch)
      hipLaunchKernelGGL((k_fft_rows2<512, 16, 16, true>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
    else
      hipLaunchKernelGGL((k_fft_rows2<512, 16, 16, false>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
  } else if (spec == 2) {
    hipLaunchKernelGGL((k_fft_rows2<224, 16, 7, false>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
  }
}

void launch_fft_cols_spec(int spec, const ImgDesc* imgs, const int4* blocks, int n_blocks, const float* ws,
                          const float2* tw, const float2* post, const EncParams& ep, const TokenSinks& sk,
                          hipStream_t s, int kernel, int layout, const int* cols6_list, int cols6_n, int cols6_qw,
                          int cols6_ipb, int cols6_pf) {
  if (n_blocks <= 0) return;
  if (kernel == 7 && layout == 0 && spec == 1 && cols6_list && cols6_n > 0) {
    const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
    const int n_items = 3 * cols6_qw;
    const int per_x = (n_items + 7) / 8;
    const int ipb = cols6_ipb;
    const int grid = 8 * per_x * ((cols6_n + ipb - 1) / ipb);
#define DCTAE_COLS7(T, I, P)                                                                                  \
  hipLaunchKernelGGL((k_fft_cols7<T, I, P>), dim3(grid), dim3(256), 0, s, imgs, cols6_list, cols6_n, n_items, \
                     cols6_qw, ws, tw, post, ep, sk)
    if (thr && ipb == 2 && cols6_pf) DCTAE_COLS7(true, 2, true);
    else if (thr && ipb == 2) DCTAE_COLS7(true, 2, false);
    else if (thr && ipb == 4 && cols6_pf) DCTAE_COLS7(true, 4, true);
    else if (thr && ipb == 4) DCTAE_COLS7(true, 4, false);
    else if (ipb == 2) DCTAE_COLS7(false, 2, false);
    else DCTAE_COLS7(false, 4, false);
#undef DCTAE_COLS7
    return;
  }
  if (kernel == 6 && layout == 0 && spec == 1 && cols6_list && cols6_n > 0) {
    const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
    const int n_items = 3 * cols6_qw;
    const int per_x = (n_items + 7) / 8;
    const int ipb = cols6_ipb;
    const int grid = 8 * per_x * ((cols6_n + ipb - 1) / ipb);
#define DCTAE_COLS6(T, I, P)                                                                                  \
  hipLaunchKernelGGL((k_fft_cols6<T, I, P>), dim3(grid), dim3(256), 0, s, imgs, cols6_list, cols6_n, n_items, \
                     cols6_qw, ws, tw, post, ep, sk)
    if (thr && ipb == 2 && cols6_pf) DCTAE_COLS6(true, 2, true);
    else if (thr && ipb == 2) DCTAE_COLS6(true, 2, false);
    else if (thr && ipb == 4 && cols6_pf) DCTAE_COLS6(true, 4, true);
    else if (thr && ipb == 4) DCTAE_COLS6(true, 4, false);
    else if (ipb == 2) DCTAE_COLS6(false, 2, false);
    else DCTAE_COLS6(false, 4, false);
#undef DCTAE_COLS6
    return;
  }
  if ((kernel == 5 || kernel == 6 || kernel == 7) && layout == 0 && spec == 1) {
    const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
    if (thr)
      hipLaunchKernelGGL((k_fft_cols5<true>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk);
    else
      hipLaunchKernelGGL((k_fft_cols5<false>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk);
    return;
  }
  if (kernel >= 4 && (layout == 0 || layout == 3)) {
    // thresholds path: codes (+ raw) only; every image's qh within the 32 tile rows the kernel walks
    const bool thr = ep.median && ep.thr && !sk.norm && ep.maxph <= 32 && ep.cb_dim == 14 && ep.ncb == 14;
#define DCTAE_COLS4(NN, RR, T)                                                                                  \
  hipLaunchKernelGGL((k_fft_cols4<NN, RR, 14, T>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk)
    if (spec == 1 && thr) DCTAE_COLS4(512, 16, true);
    else if (spec == 1) DCTAE_COLS4(512, 16, false);
    else if (spec == 2 && thr) DCTAE_COLS4(224, 7, true);
    else if (spec == 2) DCTAE_COLS4(224, 7, false);
#undef DCTAE_COLS4
    return;
  }
  if (spec == 1)
    hipLaunchKernelGGL((k_fft_cols2<512, 16, 16, 14>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk);
  else if (spec == 2)
    hipLaunchKernelGGL((k_fft_cols2<224, 16, 7, 14>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, tw, post, ep, sk);
}

}  // namespace dctae
