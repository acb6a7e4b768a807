// Bluestein DCT-II for the lengths Makhoul's plans do not cover (odd N, or
// N/2 with a prime factor above 7).  The reference's dct (torch_dct, reference
// util.py:333-338) is FFT-based for every N; here every N in [32, 1024] gets an
// O(N log N) transform instead of the O(N^2) MFMA GEMM.
//
// Per job: two real sequences of length N, each in Makhoul order
// v[n] = x[2n], v[N-1-n] = x[2n+1], packed as z = v1 + i v2.  With the chirp
// c[n] = e^{-i pi n^2 / N}:
//   Z[k] = c[k] * sum_n (z[n] c[n]) conj c[k-n]           (Bluestein)
//        = c[k] * IFFT_L( FFT_L(z c) * Bhat )[k],          Bhat = FFT_L(conj c) / L
// (L = power of two >= 2N - 1, so the cyclic convolution does not wrap), and
//   A = Z[k], B = conj Z[(N-k) mod N], e_k = s_k / 2 * e^{-i pi k / (2N)}:
//   X1[k] = Re(e_k (A + B)),  X2[k] = Im(e_k (A - B))      (k < kept count)
// where s_k is the orthonormal scale.  The inverse FFT is the forward one on
// conjugated data; the conjugation and the Bhat product are fused into the
// forward transform's last pass, the chirps into the first pass and the post.
//
// Layout: one block = 3 G jobs of L points each (G = 128 / (L / 16)), 384
// threads, 16 points per thread; the FFT runs in place in LDS (radix-16
// Stockham passes, register-held, a barrier between a pass's reads and its
// writes), one float2 of padding per 16 so the stride-16 writes of the first
// pass spread over the banks.  LDS = 3 G (L + L/16) * 8 B = 51 KiB for every L:
// three blocks (18 waves) per CU.
//   rows: job = (row pair, channel); RGB -> IPT (util.py:70-82) fused in the
//         load; output T[c][y][kx], kx < Kw (the layout the column kernels read)
//   cols: job = (column pair) of one channel of T; output Y[c][ky][kx], ky < Kh,
//         then k_tile_epilogue as on the GEMM path.
// Tables (host, float64 -> fp32; dctae_api.hip): W_L^m (m < L), c[n], e_k
// (n, k < N), Bhat (L).
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_launch.h"

namespace dctae {

namespace {

__device__ __forceinline__ int bsp(int i) { return i + (i >> 4); }
__device__ __forceinline__ float2 conj2(float2 a) { return make_float2(a.x, -a.y); }

template <int L>
struct Bs {
  // points per thread: 32 for L <= 1024 (a job inside one wave, its passes
  // synchronised by the wave alone; measured 25-30 % faster than 16 points
  // with block barriers); 16 at L = 2048 (two waves per job, block barriers:
  // 32 points need 256 VGPRs there and measured 17 % slower)
  static constexpr int E = L == 2048 ? 16 : 32;
  static constexpr int TPJ = L / E;     // threads per job
  static constexpr int G = 2048 / L;    // sequence pairs per block and channel (rows)
  static constexpr int JOBS = 3 * G;
  static constexpr int NT = JOBS * TPJ; // 192 (L <= 1024) or 384 (L = 2048)
  static constexpr int LP = L + L / 16; // padded job length (float2)
  static constexpr int R3 = L / 256;    // radix of the last pass (1 = none)
};

struct BsTabs {
  const float2* tw;     // W_L^m
  const float2* chirp;  // c[n]
  const float2* bhat;   // FFT_L(conj c) / L
  const float2* ep;     // e_k
};

__device__ __forceinline__ BsTabs bs_tabs(const FftPlan& p, const float2* tabs) {
  return BsTabs{tabs + p.bs_tw_off, tabs + p.bs_chirp_off, tabs + p.bs_bhat_off, tabs + p.bs_post_off};
}

// an opaque copy of a thread index: the per-item table addresses derive from
// it, so they are not hoisted out of the item loop (hoisted, the 64-bit
// addresses of every table load would all be live across the loop)
__device__ __forceinline__ int bs_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// The thread's twiddles of the passes with NS > 1, loaded once per kernel and
// shared by both transforms: tw[q R + r] = W_{NS R}^{r k1(q)}
template <int L, int R, int NS>
__device__ __forceinline__ void bs_twiddles(float2 (&tw)[32], int tt, const BsTabs& t) {
  constexpr int TPJ = Bs<L>::TPJ, Q = Bs<L>::E / R;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int k1 = (tt + TPJ * q) & (NS - 1);
    tw[q * R] = make_float2(1.f, 0.f);
#pragma unroll
    for (int r = 1; r < R; ++r) tw[q * R + r] = t.tw[r * k1 * (L / (NS * R))];
  }
}

// One in-place Stockham pass (radix R, NS = product of the earlier radices) of
// the job at buf; each of the TPJ threads owns 16 / R items.  CHIRP_IN: the
// inputs are z[n] c[n] (buf is zero at n >= N); BHAT_OUT: the outputs are
// replaced by conj(X Bhat), the input of the inverse transform.  Table loads
// are issued before the pass's barrier so their latency overlaps it.
// A job's lanes are all in one wave, so a pass needs no block barrier: its
// reads precede its writes in the wave's in-order LDS stream, and the writes
// precede the next pass's reads (bs_wave_sync keeps the compiler from moving
// LDS accesses across the pass boundary).
template <int L>
__device__ __forceinline__ void bs_wave_sync() {
  if constexpr (Bs<L>::TPJ > 64) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// IN = 1: the first transform's inputs z[n] c[n] (buf is zero at n >= N);
// IN = 2: the second transform's inputs conj(Zhat[n] Bhat[n]) (the spectrum
// product and the conjugation of the inverse, applied as the data is read)
template <int L, int R, int NS, int IN>
__device__ __forceinline__ void bs_pass(float2* __restrict__ buf2, int tt, const BsTabs& t, int N,
                                        const float2 (&tw)[32]) {
  constexpr int TPJ = Bs<L>::TPJ, Q = Bs<L>::E / R, S = L / R;
  // packed (re, im) pairs: complex adds are one v_pk_add_f32, products two packed FMAs
  cf* buf = reinterpret_cast<cf*>(buf2);
  cf v[32];
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int n = tt + TPJ * q + r * S;
      cf x = buf[bsp(n)];
      // no n < N predicate here (the compiler sank the loads into the branch:
      // 16 serialised load -> wait round trips): buf is zero at n >= N
      if (IN == 1) {
        const float2 c = t.chirp[n < N ? n : N - 1];
        x = cmul_pk(x, (cf){c.x, c.y});
      } else if (IN == 2) {
        const float2 b = t.bhat[n];
        x = cmul_pk(x, (cf){b.x, b.y});
        x.y = -x.y;
      }
      v[q * R + r] = x;
    }
  bs_wave_sync<L>();
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int j = tt + TPJ * q;
    const int k1 = j & (NS - 1);
    cf* w = v + q * R;
    if (NS > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) w[r] = cmul_pk(w[r], (cf){tw[q * R + r].x, tw[q * R + r].y});
    }
    DFTV<R>::run(w);
    const int base = (j - k1) * R + k1;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[bsp(base + r * NS)] = w[r];
  }
  bs_wave_sync<L>();
}

// the thread's twiddles of passes 2 and 3, preloaded once per block at 16
// points per thread (loading them per pass measured 14 % slower there); at
// 32 points per thread they are loaded per pass (preloaded: 128 VGPRs)
template <int L>
struct BsTw {
  static constexpr bool kPre = Bs<L>::E == 16;
  float2 t2[kPre ? 32 : 1], t3[kPre ? 32 : 1];
  __device__ __forceinline__ void load(int tt, const BsTabs& t) {
    if constexpr (kPre) {
      bs_twiddles<L, 16, 16>(t2, tt, t);
      if constexpr (Bs<L>::R3 > 1) bs_twiddles<L, Bs<L>::R3, 256>(t3, tt, t);
    }
  }
};

// FFT_L of the job in place; FIRST: chirp on the way in; second: Bhat product
// and conjugation on the way in
template <int L, bool FIRST>
__device__ __forceinline__ void bs_fft(float2* buf, int tt, const BsTabs& t, int N, const BsTw<L>& w) {
  constexpr int R3 = Bs<L>::R3;
  if constexpr (BsTw<L>::kPre) {
    bs_pass<L, 16, 1, FIRST ? 1 : 2>(buf, tt, t, N, w.t2);
    bs_pass<L, 16, 16, 0>(buf, tt, t, N, w.t2);
    if constexpr (R3 > 1) bs_pass<L, R3, 256, 0>(buf, tt, t, N, w.t3);
  } else {
    float2 tw[32];
    bs_pass<L, 16, 1, FIRST ? 1 : 2>(buf, tt, t, N, tw);
    bs_twiddles<L, 16, 16>(tw, tt, t);
    if constexpr (R3 > 1) {
      bs_pass<L, 16, 16, 0>(buf, tt, t, N, tw);
      bs_twiddles<L, R3, 256>(tw, tt, t);
      bs_pass<L, R3, 256, 0>(buf, tt, t, N, tw);
    } else {
      bs_pass<L, 16, 16, 0>(buf, tt, t, N, tw);
    }
  }
}

// (X1[k], X2[k]) of the job whose buffer holds U = FFT(conj(FFT(z c) Bhat)):
// Z = c * conj U
// (kb = (N - k) mod N, ck = c[k], cb = c[kb], e = e_k)
__device__ __forceinline__ float2 bs_out(const float2* buf, int k, int kb, float2 ck, float2 cb, float2 e) {
  const float2 A = cmul(ck, conj2(buf[bsp(k)]));
  const float2 B = conj2(cmul(cb, conj2(buf[bsp(kb)])));
  const float2 s = cadd(A, B), d = csub(A, B);
  return make_float2(fmaf(e.x, s.x, -e.y * s.y), fmaf(e.x, d.y, e.y * d.x));
}

// zero the jobs' buffers at n in [N, L) (the transform's zero padding)
template <int L>
__device__ __forceinline__ void bs_zero_tail(float2* lds, int N, int tid) {
  using S = Bs<L>;
  for (int e = tid; e < S::JOBS * L; e += S::NT) {
    const int jj = e / L, n = e & (L - 1);
    if (n >= N) lds[jj * S::LP + bsp(n)] = make_float2(0.f, 0.f);
  }
}

__device__ __forceinline__ int makhoul_pos(int x, int N) { return (x & 1) ? (N - 1 - (x >> 1)) : (x >> 1); }

// items (row groups / column groups) per block: with more than one, the
// image's descriptor, plan and twiddles are loaded once per block and the
// next item's inputs while the current item is transformed.  Measured: 8
// items per block ran 13 % slower than 1 (the prefetch buffers and the
// loop-carried tables took the kernel to 210 VGPRs, one block per CU), so one
// item per block; the loop stays for the shape of the code.
constexpr int kBsItems = 1;

// rows: block = kBsItems groups of 2G rows of one image from y0; per group the
// jobs (row pair g, channel c)
template <int L>
__global__ __launch_bounds__(Bs<L>::NT) void k_bs_rows(const ImgDesc* __restrict__ imgs, const FftPlan* __restrict__ plans,
                                                 const int2* __restrict__ blocks, const float* __restrict__ rgb,
                                                 float* __restrict__ ws, const float2* __restrict__ tabs, ColorMats cm,
                                                 int ablate) {
  using S = Bs<L>;
  constexpr int PXI = (L / 2 + S::NT - 1) / S::NT, NR = 2 * S::G;
  constexpr int KI = ((L / 2 < 448 ? L / 2 : 448) + S::NT - 1) / S::NT;
  __shared__ float2 lds[S::JOBS * S::LP];
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const BsTabs t = bs_tabs(plans[d.plan_w], tabs);
  const int N = d.W, Kw = d.Kw, H = d.H, tid0 = threadIdx.x;
  const int64_t hw = (int64_t)H * N;
  const float* src = rgb + d.rgb_off;
  float* lf = reinterpret_cast<float*>(lds);
  const float gam = 0.430000007152557373046875f;
  const int job = tid0 / S::TPJ;
  BsTw<L> tw;
  tw.load(tid0 - job * S::TPJ, t);
  float rgbv[NR * PXI][3];
  auto load_rgb = [&](int yb, int tid) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int i = 0; i < PXI; ++i) {
        const int px = tid + S::NT * i, y = yb + r;
        const bool ok = px < N && y < H;
        const int64_t o = ok ? (int64_t)y * N + px : 0;
        rgbv[r * PXI + i][0] = ok ? src[o] : 0.f;
        rgbv[r * PXI + i][1] = ok ? src[hw + o] : 0.f;
        rgbv[r * PXI + i][2] = ok ? src[2 * hw + o] : 0.f;
      }
  };
  load_rgb(jb.y, tid0);
  float2* buf = lds + job * S::LP;
#pragma unroll 1
  for (int it = 0; it < kBsItems; ++it) {
    const int yb = jb.y + NR * it;
    if (yb >= H) break;
    const BsTabs& ti = t;
    const int tid = bs_opaque(tid0), tt = tid - job * S::TPJ;
    bs_zero_tail<L>(lds, N, tid);
    if (!(ablate & 1)) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int i = 0; i < PXI; ++i) {
          const int px = tid + S::NT * i;
          if (px >= N) continue;
          const float R_ = rgbv[r * PXI + i][0], G_ = rgbv[r * PXI + i][1], B_ = rgbv[r * PXI + i][2];
          const float l0 = signed_pow_fast(mat3_row(cm.rgb2lms, 0, R_, G_, B_), gam);
          const float l1 = signed_pow_fast(mat3_row(cm.rgb2lms, 1, R_, G_, B_), gam);
          const float l2 = signed_pow_fast(mat3_row(cm.rgb2lms, 2, R_, G_, B_), gam);
          // job 3g + c, row pair member r & 1 -> re / im (rows past H: RGB 0 -> IPT 0)
          float* o = lf + 2 * (3 * (r >> 1)) * S::LP + 2 * bsp(makhoul_pos(px, N)) + (r & 1);
          o[0] = mat3_row(cm.lms2ipt, 0, l0, l1, l2);
          o[2 * S::LP] = mat3_row(cm.lms2ipt, 1, l0, l1, l2);
          o[4 * S::LP] = mat3_row(cm.lms2ipt, 2, l0, l1, l2);
        }
    }
    if (it + 1 < kBsItems && yb + NR < H) load_rgb(yb + NR, tid);
    __syncthreads();
    if (!(ablate & 2)) {
      bs_fft<L, true>(buf, tt, ti, N, tw);
      bs_fft<L, false>(buf, tt, ti, N, tw);
    }
    __syncthreads();   // the post reads every wave's jobs
    if (!(ablate & 4)) {
      // post: the thread's kept coefficients k for all jobs of the group
#pragma unroll
      for (int i = 0; i < KI; ++i) {
        const int k = tid + S::NT * i;
        if (k >= Kw) continue;
        const int kb = k ? N - k : 0;
        const float2 ck = ti.chirp[k], cb = ti.chirp[kb], ce = ti.ep[k];
#pragma unroll
        for (int jj = 0; jj < S::JOBS; ++jj) {
          const int g = jj / 3, c = jj - 3 * g, y = yb + 2 * g;
          if (y >= H) continue;
          const float2 X = bs_out(lds + jj * S::LP, k, kb, ck, cb, ce);
          float* trow = ws + d.ws_t + ((int64_t)c * H + y) * Kw + k;
          trow[0] = X.x;
          if (y + 1 < H) trow[Kw] = X.y;
        }
      }
    }
    __syncthreads();
  }
}

// cols: block = kBsItems groups of NC = 2 JOBS columns of channel c of T from
// kx0; per group the jobs are column pairs
template <int L>
__global__ __launch_bounds__(Bs<L>::NT) void k_bs_cols(const ImgDesc* __restrict__ imgs, const FftPlan* __restrict__ plans,
                                                 const int4* __restrict__ blocks, float* __restrict__ ws,
                                                 const float2* __restrict__ tabs, int ablate) {
  using S = Bs<L>;
  constexpr int NC = 2 * S::JOBS;
  // N * NC <= (L / 2) * 6 * 128 * 16 / L = 16 * NT: sixteen loads per thread
  constexpr int EI = (L / 2 * NC + S::NT - 1) / S::NT;
  constexpr int KPR = S::NT / S::JOBS;
  constexpr int KR = ((L / 2 < 448 ? L / 2 : 448) + KPR - 1) / KPR;
  __shared__ float2 lds[S::JOBS * S::LP];
  const int4 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const BsTabs t = bs_tabs(plans[d.plan_h], tabs);
  const int N = d.H, c = jb.y, Kw = d.Kw, Kh = d.Kh, tid0 = threadIdx.x;
  const float* T = ws + d.ws_t + (int64_t)c * N * Kw;
  float* Y = ws + d.ws_y + (int64_t)c * Kh * Kw;
  float* lf = reinterpret_cast<float*>(lds);
  const int job = tid0 / S::TPJ;
  BsTw<L> tw;
  tw.load(tid0 - job * S::TPJ, t);
  float tv[EI];
  auto load_t = [&](int kxb, int tid) {
#pragma unroll
    for (int i = 0; i < EI; ++i) {
      const int e = tid + S::NT * i, y = e / NC, kx = kxb + (e - y * NC);
      tv[i] = (y < N && kx < Kw) ? T[(int64_t)y * Kw + kx] : 0.f;
    }
  };
  load_t(jb.z, tid0);
  float2* buf = lds + job * S::LP;
#pragma unroll 1
  for (int it = 0; it < kBsItems; ++it) {
    const int kxb = jb.z + NC * it;
    if (kxb >= Kw) break;
    const BsTabs& ti = t;
    const int tid = bs_opaque(tid0), tt = tid - job * S::TPJ, kk = tid / S::JOBS, jj = tid - kk * S::JOBS;
    bs_zero_tail<L>(lds, N, tid);
    if (!(ablate & 1)) {
#pragma unroll
      for (int i = 0; i < EI; ++i) {
        const int e = tid + S::NT * i, y = e / NC, cc = e - y * NC;
        if (y < N) lf[2 * (cc >> 1) * S::LP + 2 * bsp(makhoul_pos(y, N)) + (cc & 1)] = tv[i];
      }
    }
    if (it + 1 < kBsItems && kxb + NC < Kw) load_t(kxb + NC, tid);
    __syncthreads();
    if (!(ablate & 2)) {
      bs_fft<L, true>(buf, tt, ti, N, tw);
      bs_fft<L, false>(buf, tt, ti, N, tw);
    }
    __syncthreads();   // the post reads every wave's jobs
    const int kx = kxb + 2 * jj;
    if (!(ablate & 4) && kx < Kw) {
      // post: thread = (coefficient row kk + KPR i, column pair jj)
#pragma unroll
      for (int i = 0; i < KR; ++i) {
        const int k = kk + KPR * i;
        if (k >= Kh) continue;
        const int kb = k ? N - k : 0;
        const float2 X = bs_out(lds + jj * S::LP, k, kb, ti.chirp[k], ti.chirp[kb], ti.ep[k]);
        float* yp = Y + (int64_t)k * Kw + kx;
        yp[0] = X.x;
        if (kx + 1 < Kw) yp[1] = X.y;
      }
    }
    __syncthreads();
  }
}

}  // namespace

int bs_rows_per_block(int L) { return kBsItems * 2 * (2048 / L); }
int bs_cols_per_block(int L) { return kBsItems * 2 * 3 * (2048 / L); }

void launch_bs_rows(int L, const ImgDesc* imgs, const FftPlan* plans, const int2* blocks, int n_blocks,
                    const float* rgb, float* ws, const float2* tabs, const ColorMats& cm, hipStream_t s, int ablate) {
  if (n_blocks <= 0) return;
  switch (L) {
    case 256: hipLaunchKernelGGL(k_bs_rows<256>, dim3(n_blocks), dim3(Bs<256>::NT), 0, s, imgs, plans, blocks, rgb, ws, tabs, cm, ablate); break;
    case 512: hipLaunchKernelGGL(k_bs_rows<512>, dim3(n_blocks), dim3(Bs<512>::NT), 0, s, imgs, plans, blocks, rgb, ws, tabs, cm, ablate); break;
    case 1024: hipLaunchKernelGGL(k_bs_rows<1024>, dim3(n_blocks), dim3(Bs<1024>::NT), 0, s, imgs, plans, blocks, rgb, ws, tabs, cm, ablate); break;
    case 2048: hipLaunchKernelGGL(k_bs_rows<2048>, dim3(n_blocks), dim3(Bs<2048>::NT), 0, s, imgs, plans, blocks, rgb, ws, tabs, cm, ablate); break;
    default: break;
  }
}

void launch_bs_cols(int L, const ImgDesc* imgs, const FftPlan* plans, const int4* blocks, int n_blocks, float* ws,
                    const float2* tabs, hipStream_t s, int ablate) {
  if (n_blocks <= 0) return;
  switch (L) {
    case 256: hipLaunchKernelGGL(k_bs_cols<256>, dim3(n_blocks), dim3(Bs<256>::NT), 0, s, imgs, plans, blocks, ws, tabs, ablate); break;
    case 512: hipLaunchKernelGGL(k_bs_cols<512>, dim3(n_blocks), dim3(Bs<512>::NT), 0, s, imgs, plans, blocks, ws, tabs, ablate); break;
    case 1024: hipLaunchKernelGGL(k_bs_cols<1024>, dim3(n_blocks), dim3(Bs<1024>::NT), 0, s, imgs, plans, blocks, ws, tabs, ablate); break;
    case 2048: hipLaunchKernelGGL(k_bs_cols<2048>, dim3(n_blocks), dim3(Bs<2048>::NT), 0, s, imgs, plans, blocks, ws, tabs, ablate); break;
    default: break;
  }
}

}  // namespace dctae
