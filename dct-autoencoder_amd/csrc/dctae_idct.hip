// Decode on the FFT path: the inverse of dctae_fft2.hip's encode, for the
// specialised square sizes (N = 512; rows also N = 224).
//
//   codes -> (+-1, inverse PatchNorm) -> spectrum corner Y (3, Kh, Kw)
//         -> DCT-III along y (column kernel)  -> U (3, H, Kw)  [row-major, like T]
//         -> DCT-III along x (row kernel) -> IPT -> RGB (3, H, W)
//
// The orthonormal DCT-III of length N (torch_dct.idct(norm='ortho'),
// util.py:337-338 <- FE:149) through one N/2-point complex FFT, the inverse of
// Makhoul's encode post-processing:
//   A_k = Ys[k] - i Ys[N-k],  B_k = Ys[M+k] - i Ys[M-k]   (Ys[N] = 0, Ys[0] *= sqrt 2)
//   Z_k = a_k A_k + b_k B_k,  k < M = N/2,
//   a_k = g (1 + i e^{2 pi i k/N}) e^{i pi k/(2N)} / 2,  b_k = g (1 - i e^{2 pi i k/N}) e^{i pi (k+M)/(2N)} / 2,
//   g = sqrt(N/2) / M;  z = sum_k Z_k e^{+2 pi i m k/M}  (computed as conj(FFT(conj Z)));
//   x[4m] = Re z[m], x[4m+2] = Im z[m] (m < M/2);  x[2N-1-4m] = Re z[m], x[2N-3-4m] = Im z[m] (above).
// The tables hold conj(a_k), conj(b_k) (float4 per k), so the kernels build
// conj Z_k = conj(a) (Ys[k] + i Ys[N-k]) + conj(b) (Ys[M+k] + i Ys[M-k]).
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_launch.h"
#include "dctae_rows512.h"

namespace dctae {

namespace {

__device__ __forceinline__ constexpr int ipad16(int m) { return m + (m >> 4); }
__device__ __forceinline__ constexpr int izaddr(int m) { return 15 * (m & 15) + 257 * (m >> 4); }

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int itid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

// conj Z_k from the four real inputs
__device__ __forceinline__ cf pre_z(float yk, float ynk, float ymk, float ymk2, float4 ab) {
#pragma clang fp contract(fast)
  const cf A = (cf){yk, ynk}, B = (cf){ymk, ymk2};
  return cmulv(A, (cf){ab.x, ab.y}) + cmulv(B, (cf){ab.z, ab.w});
}

}  // namespace

// ---------------------------------------------------------------------------
// token map: map[img][c][w][h] = packed slot r * S + j of the token (or -1),
// item-major (a column block's 32 tiles h are contiguous).  The inverse of the
// encode's sort/pack: FE:607-656 revert_patching assigns token (c, h, w) to
// image[c, h, w] in packed order, so of two tokens at one place the later slot
// wins (atomicMax: deterministic, where plain stores would race; +0.03 ms per
// 1024 images).  Same argument checks as k_scatter_tokens.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dec_map_token(int64_t t, int64_t id, int64_t c, int64_t h, int64_t w,
                                              const ImgDesc* __restrict__ imgs, const DecodeArgs& a,
                                              int32_t* __restrict__ map) {
  const int64_t r = t / a.S;
  if (id < 0 || id >= a.lut_w) {
    atomicOr(a.err, 2);
    return;
  }
  const int im = a.lut[r * a.lut_w + id];
  if (im < 0) {
    atomicOr(a.err, 2);
    return;
  }
  const int qh = imgs[im].qh, qw = imgs[im].qw;
  if (c < 0 || c >= 3 || h < 0 || h >= qh || w < 0 || w >= qw) {
    atomicOr(a.err, 4);
    return;
  }
  atomicMax(map + (((int64_t)im * 3 + c) * a.maxpw + w) * a.maxph + h, (int32_t)t);
}

// four consecutive tokens per thread: ids / channels as two 16-byte loads,
// positions as four, key_pad as one 4-byte load, for the first 4 n4 tokens
// (n4 = 0 unless the tensors are 16-byte aligned); the rest token by token
__global__ void k_dec_map(int64_t n_tok, int64_t n4, const ImgDesc* __restrict__ imgs, DecodeArgs a,
                          int32_t* __restrict__ map) {
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t0 = 4 * q;
    const uint32_t kp = *reinterpret_cast<const uint32_t*>(a.key_pad + t0);
    if (kp == 0x01010101u) continue;
    const i64x2* ip = reinterpret_cast<const i64x2*>(a.ids + t0);
    const i64x2* cp = reinterpret_cast<const i64x2*>(a.ch + t0);
    const i64x2* pp = reinterpret_cast<const i64x2*>(a.pos + 2 * t0);
    const i64x2 i01 = ip[0], i23 = ip[1], c01 = cp[0], c23 = cp[1];
    const i64x2 p0 = pp[0], p1 = pp[1], p2 = pp[2], p3 = pp[3];
    if (!(kp & 0xffu)) dec_map_token(t0, i01.x, c01.x, p0.x, p0.y, imgs, a, map);
    if (!(kp & 0xff00u)) dec_map_token(t0 + 1, i01.y, c01.y, p1.x, p1.y, imgs, a, map);
    if (!(kp & 0xff0000u)) dec_map_token(t0 + 2, i23.x, c23.x, p2.x, p2.y, imgs, a, map);
    if (!(kp & 0xff000000u)) dec_map_token(t0 + 3, i23.y, c23.y, p3.x, p3.y, imgs, a, map);
  }
  for (int64_t t = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tok;
       t += (int64_t)gridDim.x * blockDim.x)
    if (!a.key_pad[t]) dec_map_token(t, a.ids[t], a.ch[t], a.pos[2 * t], a.pos[2 * t + 1], imgs, a, map);
}

void launch_dec_map(int64_t n_tok, const ImgDesc* imgs, const DecodeArgs& a, int32_t* map, hipStream_t s) {
  const bool al = ((uintptr_t)a.ids | (uintptr_t)a.ch | (uintptr_t)a.pos) % 16 == 0 && (uintptr_t)a.key_pad % 4 == 0;
  const int64_t n4 = al ? n_tok / 4 : 0;
  const int gx = (int)std::min<int64_t>((std::max<int64_t>(n4, n_tok - 4 * n4) + 255) / 256, 8192);
  if (gx > 0) hipLaunchKernelGGL(k_dec_map, dim3(gx), dim3(256), 0, s, n_tok, n4, imgs, a, map);
}

// ---------------------------------------------------------------------------
// columns (N = H = 512, P = 14): one block = (image, channel, tile column).
//   1. tokens of the tile column -> X[ky][col] (float, natural rows, zero rows
//      for ky >= Kh and for tokens not present);
//   2. conj Z_k for k = jj + 16 i (lane jj of column col) into registers;
//   3. complex z (zaddr layout, as the encode's cols5) -> radix-16 x 2 FFT;
//   4. z[m] -> x[y] (natural rows) -> U[c][y][14 strip + col] (56-byte rows).
// ---------------------------------------------------------------------------
// X row y lives at row xrow(y) = y ^ ((y >> 4) & 3): the FFT output scatter
// (rows 4 m, 4 m + 2 for m = jj + 16 r over the 16 lanes jj of a column)
// then hits 16 distinct bank pairs instead of 4 (4-way -> conflict-free; the
// other X accesses stay within 2-way: 305 vs 672 extra LDS cycles per item by
// the bank rule of MI355X_MICROARCH.md, SQ_LDS_BANK_CONFLICT 91.5 M per launch
// before; the kernel time did not move: it is latency-bound).  Rows
// 448 .. 511 map onto themselves (the zero fill is unchanged).
#ifdef DCTAE_NO_XROW
__device__ __forceinline__ int xrow(int y) { return y; }
#else
__device__ __forceinline__ int xrow(int y) { return y ^ ((y >> 4) & 3); }
#endif

struct IColsLds {
  union {
    float x[512 * 14];
    float2 z[izaddr(255) + 14];
  };
};

// tokens of one (image, channel, tile column) -> X[ky][col] in LDS (natural
// rows through xrow, zero rows for tiles absent from the batch): thread
// (g16, jl) expands tile rows h = g16 + 16 r, element row jl, from the
// token's code (LFQ bit -> +-scale -> inverse PatchNorm: vt) or its patch.
// Three stages, so k_idct_cols512b can keep the next image's in flight:
// icols_map (packed slots of the two tiles, FE:639-643's winner), icols_codes
// (the element row's code of each; a dependent load), icols_expand.
struct IcTok {
  int32_t sl[2];     // packed slot of tile g16 + 16 r, -1 = absent
  int32_t code[2];   // its code for element row jl (use_codes)
};

__device__ __forceinline__ void icols_map(int img, const ImgDesc& d, int c, int strip, const int32_t* __restrict__ map,
                                          const DecodeArgs& a, IcTok& t) {
  const int g16 = itid() >> 4;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int h = g16 + 16 * r;
    t.sl[r] = map[(((int64_t)img * 3 + c) * a.maxpw + strip) * a.maxph + (h < d.qh ? h : 0)];
    if (h >= d.qh) t.sl[r] = -1;
  }
}

__device__ __forceinline__ void icols_codes(const DecodeArgs& a, IcTok& t) {
  constexpr int KS = 14;
  const int jl = itid() & 15;
  if (a.use_codes != 1) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {   // unconditional loads; the low word of the int64 code (lfq.py:117 .int())
    const int64_t s0 = t.sl[r] >= 0 ? t.sl[r] : 0;
    t.code[r] = reinterpret_cast<const int32_t*>(a.codes)[2 * (s0 * a.ncb + (jl < KS ? jl : 0))];
  }
}

// zero_tail: also zero rows 448 .. 511 (read by k_idct_cols512 only)
__device__ __forceinline__ void icols_expand(const IcTok& t, const DecodeArgs& a, const float2 (&vt)[2][14], float* x,
                                             bool zero_tail) {
  constexpr int N = 512, KS = 14, PP = KS * KS;
  const int tid = itid();
#if defined(DCTAE_PROFILING) && defined(DCTAE_IC_ABL)
  if (DCTAE_IC_ABL & 1) {   // profiling ablation: no token loads / expansion (wrong output)
    for (int e = tid; e < N * KS; e += 256) x[e] = 0.001f * (e & 63);
    return;
  }
#endif
  const int g16 = tid >> 4, jl = tid & 15;
  float pv[2][KS];
  if (a.use_codes != 1) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t s0 = t.sl[r] >= 0 ? t.sl[r] : 0;   // unconditional loads
      const float* pt = a.patches + s0 * PP + (jl < KS ? jl : 0) * KS;
#pragma unroll
      for (int p = 0; p < KS; ++p) pv[r][p] = pt[p];
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int h = g16 + 16 * r;
    if (jl < KS) {
      f2v* xr = reinterpret_cast<f2v*>(x + xrow(KS * h + jl) * KS);
#pragma unroll
      for (int p = 0; p < KS / 2; ++p) {
        float v0, v1;
        if (a.use_codes == 2) {
          // PatchNorm-space tokens (dctae_decode_normed): the inverse with this
          // thread's (median, std) pair, pn_inverse's fp32 ops
          v0 = __fadd_rn(__fmul_rn(pv[r][2 * p], vt[r][2 * p].y), vt[r][2 * p].x);
          v1 = __fadd_rn(__fmul_rn(pv[r][2 * p + 1], vt[r][2 * p + 1].y), vt[r][2 * p + 1].x);
        } else if (a.use_codes) {
          // bit select by masks: a ?: on the pair lets the compiler select
          // the address instead and move vt to scratch
          const uint32_t m0 = 0u - ((uint32_t)(t.code[r] >> (KS - 1 - 2 * p)) & 1u);
          const uint32_t m1 = 0u - ((uint32_t)(t.code[r] >> (KS - 2 - 2 * p)) & 1u);
          v0 = __uint_as_float((__float_as_uint(vt[r][2 * p].x) & m0) | (__float_as_uint(vt[r][2 * p].y) & ~m0));
          v1 = __uint_as_float((__float_as_uint(vt[r][2 * p + 1].x) & m1) | (__float_as_uint(vt[r][2 * p + 1].y) & ~m1));
        } else {
          v0 = pv[r][2 * p];
          v1 = pv[r][2 * p + 1];
        }
        xr[p] = t.sl[r] >= 0 ? (f2v){v0, v1} : (f2v){0.0f, 0.0f};
      }
    }
  }
  // rows 448 .. 511 (beyond Kh = 448 when qh = 32): zero
  if (zero_tail)
    for (int e = tid; e < (N - KS * 32) * KS; e += 256) x[KS * 32 * KS + e] = 0.0f;
}

__device__ __forceinline__ void icols_fill_x(int img, const ImgDesc& d, int c, int strip,
                                             const int32_t* __restrict__ map, const DecodeArgs& a,
                                             const float2 (&vt)[2][14], float* x, bool zero_tail) {
  IcTok t;
  icols_map(img, d, c, strip, map, a, t);
  icols_codes(a, t);
  icols_expand(t, a, vt, x, zero_tail);
}

// image-independent values of this thread's two tile rows (h = g16 + 16 r,
// element row jl) of a (channel, strip) item: inverse PatchNorm of y = +scale
// (code bit 1, .x) and y = -scale (bit 0, .y), lfq.py:105-134 -> patchnorm.py:167-177
__device__ __forceinline__ void icols_vt(int c, int strip, const DecodeArgs& a, float2 (&vt)[2][14]) {
  constexpr int KS = 14, PP = KS * KS;
  const int tid = itid();
  const int g16 = tid >> 4, jl = tid & 15;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int h = min(g16 + 16 * r, a.maxph - 1);
    const int64_t tab = (((int64_t)c * a.maxph + h) * a.maxpw + strip) * PP + (jl < KS ? jl : 0) * KS;
    if (a.use_codes == 2) {   // (median, b sqrt2 + eps) of pn_inverse
#pragma unroll
      for (int p = 0; p < KS; ++p)
        vt[r][p] = make_float2(a.median[tab + p], __fadd_rn(__fmul_rn(a.b[tab + p], 1.41421353816986083984375f), a.eps));
    } else if (a.use_codes) {
      const float yp = __fsub_rn(__fmul_rn(1.0f, a.scale * 2.0f), a.scale);
      const float yn = __fsub_rn(__fmul_rn(0.0f, a.scale * 2.0f), a.scale);
#pragma unroll
      for (int p = 0; p < KS; ++p) {
        const float m = a.median[tab + p], bb = a.b[tab + p];
        vt[r][p] = make_float2(pn_inverse(yp, m, bb, a.eps), pn_inverse(yn, m, bb, a.eps));
      }
    }
  }
}

// one (image, channel, tile column) of the column pass; vt[r][p] = the
// (code bit 1, code bit 0) values of this thread's tile row r, element p
// (inverse PatchNorm of +-scale, image-independent: loaded once per block)
__device__ __forceinline__ void idct_col_image(int img, const ImgDesc& d, int c, int strip, float* __restrict__ ws,
                                               const int32_t* __restrict__ map, const DecodeArgs& a,
                                               const float2 (&vt)[2][14], IColsLds& L, const float4* pre_s,
                                               const float2* tw_s) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256, KS = 14, S16 = 257;
  const int tid = itid();
  // ---- 1. tokens -> X rows 14 h + jl (tile h = g16 + 16 r)
  icols_fill_x(img, d, c, strip, map, a, vt, L.x, true);
  __syncthreads();
  // lanes of columns 14 / 15 (tid >= 224) redo column 13: same reads, same
  // values, same stores (no divergent branches)
  const int jj = tid & 15, col = min(tid >> 4, KS - 1);
  // ---- 2. conj Z_k, k = jj + 16 i
  cf zk[16];
  {
    const float* xc = L.x + col;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = jj + 16 * i;
      // xrow(M + y) = M + xrow(y) for y < M: rows k / M + k and M - k / N - k
      // are M * KS floats apart -> one ds_read2st64_b32 per pair
      const float* pk = xc + xrow(k) * KS;
      const float* pm = xc + xrow(M - k) * KS;   // k = 0: row M (its N - k partner is not read)
      float yk = pk[0];
      const float ymk = pk[M * KS], ymk2 = pm[0];
      const float ynk = k == 0 ? 0.0f : pm[M * KS];
      if (k == 0) yk *= 1.41421356237309515f;
      zk[i] = pre_z(yk, ynk, ymk, ymk2, pre_s[k]);
    }
  }
  // ---- 3. forward FFT of conj Z (radix 16 x 16, Stockham).  Pass 1's item
  // jj reads z[jj + 16 r] = this lane's zk[r]: it runs on the registers
  // (no LDS round trip); its outputs go to z[16 jj + r] for pass 2.
  DFTV<16>::run(zk);
  __syncthreads();   // every wave's X reads (step 2) before z (aliased on X) is written
  const cf* zr = reinterpret_cast<const cf*>(L.z) + 15 * jj + col;   // z[jj + 16 r]
  {
    cf* zw = reinterpret_cast<cf*>(L.z) + S16 * jj + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) zw[15 * r] = zk[r];
  }
  __syncthreads();
  {
    cf v[16];
    {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = zr[S16 * r];
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        const float2 w = tw_s[r * jj];
        v[r] = cmulv(v[r], (cf){w.x, w.y});
      }
      DFTV<16>::run(v);
    }
    __syncthreads();
    // ---- 4. w[jj + 16 r] -> x rows (natural), z = conj w
    {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = jj + 16 * r;
        const int ya = m < M / 2 ? 4 * m : 2 * N - 1 - 4 * m;
        const int yb = m < M / 2 ? ya + 2 : ya - 2;
        L.x[xrow(ya) * KS + col] = v[r].x;
        L.x[xrow(yb) * KS + col] = -v[r].y;
      }
    }
    __syncthreads();
  }
  // ---- 5. U[c][y][14 strip + 2p, +1] for rows y = y0 + 32 k
#if defined(DCTAE_PROFILING) && defined(DCTAE_IC_ABL)
  if (DCTAE_IC_ABL & 2) {   // profiling ablation: no U stores (wrong output)
    __syncthreads();
    return;
  }
#endif
  if (tid < 32 * (KS / 2)) {
    const int y0 = tid / (KS / 2), p = tid - y0 * (KS / 2);
    f2v* dst = reinterpret_cast<f2v*>(ws + d.ws_t + ((int64_t)c * d.H + y0) * d.Kw + strip * KS) + p;
    const int64_t rstep = (int64_t)16 * d.Kw;
    const f2v* src = reinterpret_cast<const f2v*>(L.x) + p;
#pragma unroll
    for (int k = 0; k < N / 32; ++k) dst[k * rstep] = src[xrow(y0 + 32 * k) * (KS / 2)];
  }
  __syncthreads();
}

// block = (channel c, tile column strip) item x IPB consecutive images (the
// image loop unrolled: straight-line register allocation); items dealt so the
// 8 XCD groups (b % 8) own contiguous runs of tile columns
template <int IPB>
__global__ __launch_bounds__(256) void k_idct_cols512(const ImgDesc* __restrict__ imgs, int n_img, int n_items, int qw,
                                                      float* __restrict__ ws, const int32_t* __restrict__ map,
                                                      const float2* __restrict__ tw, const float4* __restrict__ pre,
                                                      DecodeArgs a) {
  constexpr int M = 256, KS = 14;
  __shared__ IColsLds L;
  __shared__ float4 pre_s[M];
  __shared__ float2 tw_s[M];
  const int per_x = (n_items + 7) / 8;
  const int b = blockIdx.x, slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, g = slot / per_x;
  const int i0 = g * IPB;
  if (t >= n_items || i0 >= n_img) return;
  const int c = t / qw, strip = t - c * qw;
  for (int i = threadIdx.x; i < M; i += 256) {
    pre_s[i] = pre[i];
    tw_s[i] = tw[i];
  }
  float2 vt[2][KS];
  icols_vt(c, strip, a, vt);
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int img = i0 + u;
    if (img < n_img) idct_col_image(img, imgs[img], c, strip, ws, map, a, vt, L, pre_s, tw_s);
  }
}

// ---------------------------------------------------------------------------
// rows: one wave = one image row, 3 channels; 16 rows per block.
//   U[c][y][kx] (kx < Kw, zero beyond) -> conj Z_k -> FFT -> x[px] -> IPT -> RGB
// ---------------------------------------------------------------------------
template <int N, int R2>
__global__ __launch_bounds__(256) void k_idct_rows2(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                    const float* __restrict__ ws, float* __restrict__ rgb,
                                                    const float2* __restrict__ tw, const float4* __restrict__ pre,
                                                    ColorMats cm) {
#pragma clang fp contract(fast)
  constexpr int R1 = 16;
  constexpr int M = N / 2;
  constexpr int MP = ipad16(M - 1) + 2;
  constexpr int B1 = M / R1, B2 = M / R2;
  constexpr int PX = (N + 63) / 64;
  constexpr int KI = (M + 63) / 64;
  constexpr int RPW = 4;
  static_assert(R1 * R2 == M && 3 * B1 <= 64 && 3 * B2 <= 64, "plan shape");
  __shared__ float2 zs[4][3][MP];
  __shared__ float4 pre_s[M];
  __shared__ float2 tw_s[M];
  for (int i = threadIdx.x; i < M; i += 256) {
    pre_s[i] = pre[i];
    tw_s[i] = tw[i];
  }
  __syncthreads();
  const int tid = itid();
  const int wave = tid >> 6, lane = tid & 63;
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  float2(*z)[MP] = zs[wave];
  const int H = d.H, Kw = d.Kw;
  const int64_t hw = (int64_t)H * N;
  const float inv_gamma = 2.3255813121795654296875f;   // fp32(1/0.43), util.py:93
  // x[px] = sign * (re or im of w[m]) at float offset xo[i] of the channel buffer
  int xo[PX];
  float xs[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int px = lane + 64 * i;
    int m, im;
    if ((px & 1) == 0) {
      m = px >> 2;
      im = (px & 2) ? 1 : 0;
    } else {
      const int q = 2 * N - 1 - px;   // 4m or 4m + 2
      m = q >> 2;
      im = (q & 2) ? 1 : 0;
    }
    xo[i] = 2 * ipad16(m) + im;
    xs[i] = im ? -1.0f : 1.0f;
  }
#pragma unroll 1
  for (int rr = 0, y = jb.y + wave; rr < RPW && y < H; ++rr, y += 4) {
    // ---- stage the 3 input rows (zero beyond Kw) in the channel buffers
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* src = ws + d.ws_t + ((int64_t)c * H + y) * Kw;
      float* zf = reinterpret_cast<float*>(z[c]);
      // unconditional (clamped) loads: a load under `kx < Kw` becomes a branch
      // with its own vmcnt(0) wait, serialising the row's HBM latencies
      float lv[PX];
#pragma unroll
      for (int i = 0; i < PX; ++i) lv[i] = src[min(lane + 64 * i, Kw - 1)];
#pragma unroll
      for (int i = 0; i < PX; ++i) {
        const int kx = lane + 64 * i;
        if (kx < N) zf[kx] = kx < Kw ? lv[i] : 0.0f;
      }
    }
    // ---- conj Z_k per channel (all reads of a channel before its writes)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float* zf = reinterpret_cast<float*>(z[c]);
      cf zk[KI];
#pragma unroll
      for (int i = 0; i < KI; ++i) {
        const int k = lane + 64 * i;
        if (k < M) {
          float yk = zf[k];
          const float ynk = k == 0 ? 0.0f : zf[N - k];
          if (k == 0) yk *= 1.41421356237309515f;
          zk[i] = pre_z(yk, ynk, zf[M + k], zf[M - k], pre_s[k]);
        }
      }
#pragma unroll
      for (int i = 0; i < KI; ++i) {
        const int k = lane + 64 * i;
        if (k < M) z[c][ipad16(k)] = make_float2(zk[i].x, zk[i].y);
      }
    }
    // ---- pass 1: radix 16, Ns = 1
    if (lane < 3 * B1) {
      const int c = lane / B1, j = lane - c * B1;
      cf v[R1];
#pragma unroll
      for (int r = 0; r < R1; ++r) {
        const float2 t = z[c][ipad16(j + r * B1)];
        v[r] = (cf){t.x, t.y};
      }
      DFTV<R1>::run(v);
#pragma unroll
      for (int r = 0; r < R1; ++r) z[c][ipad16(j * R1 + r)] = make_float2(v[r].x, v[r].y);
    }
    // ---- pass 2: radix R2, Ns = R1
    if (lane < 3 * B2) {
      const int c = lane / B2, j = lane - c * B2;
      cf v[R2];
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        const float2 t = z[c][ipad16(j + r * B2)];
        v[r] = (cf){t.x, t.y};
      }
#pragma unroll
      for (int r = 1; r < R2; ++r) {
        const float2 w = tw_s[r * j];
        v[r] = cmulv(v[r], (cf){w.x, w.y});
      }
      DFTV<R2>::run(v);
#pragma unroll
      for (int r = 0; r < R2; ++r) z[c][ipad16(j + r * R1)] = make_float2(v[r].x, v[r].y);
    }
    // ---- x -> IPT -> RGB (util.py:85-97)
    const float* z0 = reinterpret_cast<const float*>(z[0]);
    const float* z1 = reinterpret_cast<const float*>(z[1]);
    const float* z2 = reinterpret_cast<const float*>(z[2]);
    float* dst = rgb + d.rgb_off + (int64_t)y * N;
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int px = lane + 64 * i;
      if (px < N) {
        const float i0 = xs[i] * z0[xo[i]], i1 = xs[i] * z1[xo[i]], i2 = xs[i] * z2[xo[i]];
        const float l0 = signed_pow_fast(mat3_row(cm.ipt2lms, 0, i0, i1, i2), inv_gamma);
        const float l1 = signed_pow_fast(mat3_row(cm.ipt2lms, 1, i0, i1, i2), inv_gamma);
        const float l2 = signed_pow_fast(mat3_row(cm.ipt2lms, 2, i0, i1, i2), inv_gamma);
        dst[px] = mat3_row(cm.lms2rgb, 0, l0, l1, l2);
        dst[hw + px] = mat3_row(cm.lms2rgb, 1, l0, l1, l2);
        dst[2 * hw + px] = mat3_row(cm.lms2rgb, 2, l0, l1, l2);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_idct_cols512b: the column DCT-III of 512 x 512 images at 32 x 32 kept
// tiles with the encode's register-resident FFT (fft256_group, dctae_rows512.h)
// and U written straight from registers in the band layout U'[c][y / 4][kx][4]
// (u4_index: band16 by default, rows 4 m .. 4 m + 3 of one column = one
// float4, natural order), read by k_idct_rows512<448, true>.  Block = (channel,
// tile strip) x IPB images, one 16-lane group per column (groups 14 / 15
// repeat column 13 and store the same values), XCD-dealt like k_cols512b.
// Per image: tokens -> X (LDS, icols_fill_x) | barrier | lane j of column col
// builds conj Z[j + 16 r] (its pass-1 inputs) from X | barrier (X aliases the
// transpose regions) | fft256_group with the identity butterfly order: lane j
// holds W[j + 16 i] and the mirror lane W[255 - j - 16 i], so rows 4 m + (0,
// 1, 2, 3) of m = j + 16 i are (Re W[m], -Im W[255 - m], -Im W[m], Re W[255 - m])
// (dctae_idct.hip header) -- eight 16-byte stores per lane.  Three block
// barriers per image against k_idct_cols512's six, no LDS round trip for U.
// ---------------------------------------------------------------------------
struct ICols512bLds {
  union {
    float x[448 * 14];            // Y[ky][col] of the strip, rows through xrow (25,088 B)
    cf xch[16][kXchStridePk];     // per group transpose region (34,816 B)
  } u;
  float2 tw2[16][16];
  float4 pre[256];                // (conj a_k, conj b_k)
};                                // 40,960 B: 4 blocks per CU

#ifndef DCTAE_IC5B_WPE
#define DCTAE_IC5B_WPE 0
#endif
// 1: the token map entries two images ahead, the codes one image ahead (issued
// right after the expansion); 0: map one ahead, codes after the FFT
#ifndef DCTAE_IC5B_AHEAD2
#define DCTAE_IC5B_AHEAD2 1
#endif
template <int IPB>
__global__ __launch_bounds__(256)
#if DCTAE_IC5B_WPE
__attribute__((amdgpu_waves_per_eu(DCTAE_IC5B_WPE)))
#endif
void k_idct_cols512b(const ImgDesc* __restrict__ imgs, int n_img,
                                                       float* __restrict__ ws, const int32_t* __restrict__ map,
                                                       const float2* __restrict__ tw, const float4* __restrict__ pre,
                                                       DecodeArgs a) {
#pragma clang fp contract(fast)
  constexpr int M = 256, KS = 14, KW = 448, per_x = 12;   // 96 items = 3 channels x 32 strips, 12 per XCD lane
  constexpr int ustep = 16 * KW * 16;   // bytes between band4 = m and m + 16 (both layouts)
  __shared__ ICols512bLds L;
  const int b = blockIdx.x, slot = b >> 3;
  const int t = (b & 7) * per_x + slot % per_x, i0 = (slot / per_x) * IPB;
  if (i0 >= n_img) return;
  const int c = t >> 5, strip = t & 31;
  const int tid = itid();
  L.tw2[tid >> 4][tid & 15] = tw[(tid >> 4) * (tid & 15)];
  L.pre[tid] = pre[tid];
  float2 vt[2][KS];
  icols_vt(c, strip, a, vt);
  const int G = tid >> 4, j = tid & 15;
  const int col = min(G, KS - 1);
  const int uo = u4_index(j, KS * strip + col) * 16;   // band4 = j + 16 i at + i * ustep
  // the tokens of image u + 1 in flight during image u: its map entries are
  // loaded right after image u's expansion, its codes (dependent on them)
  // after image u's FFT, before image u's U stores
  IcTok tk, tm;   // this image's map entries + codes; the next image's map entries
  icols_map(i0, imgs[i0], c, strip, map, a, tk);
  icols_codes(a, tk);
#if DCTAE_IC5B_AHEAD2
  if (IPB > 1) {
    const int i1 = min(i0 + 1, n_img - 1);
    icols_map(i1, imgs[i1], c, strip, map, a, tm);
  }
#endif
#pragma unroll
  for (int u = 0; u < IPB; ++u) {
    const int img = i0 + u;
    if (img >= n_img) break;   // block-uniform
    const ImgDesc d = imgs[img];
    __syncthreads();   // tables (u = 0) / the previous image's transposes (x aliases xch)
    icols_expand(tk, a, vt, L.u.x, false);
    IcTok tn;
#if DCTAE_IC5B_AHEAD2
    // the next image's codes (its map entries arrived during this image's
    // predecessor) and the map entries of the one after, all in flight
    // through this image's transform and stores (unconditional: past the end
    // of the list the last image reloads itself)
    tn = tm;
    if (u + 1 < IPB) icols_codes(a, tn);
    const int img_n2 = min(img + 2, n_img - 1);
    if (u + 2 < IPB) icols_map(img_n2, imgs[img_n2], c, strip, map, a, tm);
#else
    const int img_n = min(img + 1, n_img - 1);   // unconditional (the last image reloads itself)
    if (u + 1 < IPB) icols_map(img_n, imgs[img_n], c, strip, map, a, tn);
#endif
    __syncthreads();
    // conj Z_k, k = j + 16 i (Ys[M + k] = 0 for i >= 12, Ys[N - k] = 0 for k <= 64)
    cf v[16];
    {
      const float* xc = L.u.x + col;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = j + 16 * i;
        const float* pk = xc + xrow(k) * KS;
        const float* pm = xc + xrow(M - k) * KS;   // k = 0: row M
        float yk = pk[0];
        if (i == 0) yk = j == 0 ? yk * 1.41421356237309515f : yk;
        const float ymk2 = pm[0];
        const float ymk = i < 12 ? pk[M * KS] : 0.0f;   // xrow(M + y) = M + xrow(y)
        float ynk = 0.0f;
        if (i >= 4) {
          ynk = pm[M * KS];                              // row N - k (i = 4, j = 0: row 448, dropped)
          if (i == 4) ynk = j == 0 ? 0.0f : ynk;
        }
        v[i] = pre_z(yk, ynk, ymk, ymk2, L.pre[k]);
      }
    }
    __syncthreads();   // every group's X reads before the transposes
    fft256_group(v, L.u.xch[G], j, j, L.tw2);
#if !DCTAE_IC5B_AHEAD2
    if (u + 1 < IPB) icols_codes(a, tn);
#endif
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(ws + d.ws_t + (int64_t)c * 512 * KW, 0, 512 * KW * 4,
                                                        0x00020000);
#if defined(DCTAE_PROFILING) && defined(DCTAE_IC_ABL)
    // profiling ablation: no U' stores (wrong output; a never-true test keeps the transform live)
    if ((DCTAE_IC_ABL & 4) && v[0].x != 1234.5f) {
      if (u + 1 < IPB) tk = tn;
      continue;
    }
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float px = mirror16(v[15 - i].x), py = mirror16(v[15 - i].y);
      __builtin_amdgcn_raw_buffer_store_b128(
          (v4u){__float_as_uint(v[i].x), __float_as_uint(-py), __float_as_uint(-v[i].y), __float_as_uint(px)}, rsrc,
          uo, i * ustep, DCTAE_U_ST_AUX);
    }
    if (u + 1 < IPB) tk = tn;
  }
}

#ifndef DCTAE_IC5B_IPB
#define DCTAE_IC5B_IPB 12   // images per block (same-box A/Bs, decode 1024 x 512^2: 4 1.98, 6 1.93, 8 1.925 / 1.960, 12 1.910 / 1.945, 16 2.19 ms)
#endif
void launch_idct_cols512b(const ImgDesc* imgs, int n_img, float* ws, const int32_t* map, const float2* tw,
                          const float4* pre, const DecodeArgs& a, hipStream_t s) {
  constexpr int IPB = DCTAE_IC5B_IPB;
  const int grid = 8 * 12 * ((n_img + IPB - 1) / IPB);
  if (n_img > 0)
    hipLaunchKernelGGL((k_idct_cols512b<IPB>), dim3(grid), dim3(256), 0, s, imgs, n_img, ws, map, tw, pre, a);
}

void launch_idct_cols512(const ImgDesc* imgs, int n_img, int qw, float* ws, const int32_t* map, const float2* tw,
                         const float4* pre, const DecodeArgs& a, hipStream_t s) {
  constexpr int IPB = 2;
  const int n_items = 3 * qw, per_x = (n_items + 7) / 8;
  const int grid = 8 * per_x * ((n_img + IPB - 1) / IPB);
  if (n_img > 0)
    hipLaunchKernelGGL((k_idct_cols512<IPB>), dim3(grid), dim3(256), 0, s, imgs, n_img, n_items, qw, ws, map, tw,
                       pre, a);
}

void launch_idct_rows_spec(int spec, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* ws,
                           float* rgb, const float2* tw, const float4* pre, const ColorMats& cm, hipStream_t s) {
  if (n_blocks <= 0) return;
  if (spec == 1)
    hipLaunchKernelGGL((k_idct_rows2<512, 16>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, rgb, tw, pre, cm);
  else if (spec == 2)
    hipLaunchKernelGGL((k_idct_rows2<224, 7>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, rgb, tw, pre, cm);
}

}  // namespace dctae
