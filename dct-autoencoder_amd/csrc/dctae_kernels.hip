// HIP kernels (gfx950 / CDNA4) for the dct-autoencoder feature-extraction
// hot path.  Host-side planning and the C ABI live in dctae_api.hip.
//
// Numerics notes (see DESIGN.md "Bit-exactness"):
//  * compiled with -ffp-contract=off: every a*b+c below is two roundings
//    unless written as fmaf() on purpose (only in DCT/colour arithmetic, which
//    is compared with a tolerance);
//  * PatchNorm / LFQ / score arithmetic uses __fmul_rn/__fadd_rn/__fdiv_rn
//    in the reference's op order so it is bit-exact given identical inputs.
#include "dctae_internal.h"
#include "dctae_launch.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <rocprim/block/block_radix_sort.hpp>
#include "dctae_device.h"

namespace dctae {


// ---------------------------------------------------------------------------
// synthetic images (same hash as oracle/rng.py)
// ---------------------------------------------------------------------------

__global__ void k_synth(uint64_t seed, int64_t first, int64_t per_img, int32_t n_img, float* out) {
  const int img = blockIdx.y;
  const uint64_t key = splitmix64(splitmix64(seed) ^ (uint64_t)(first + img));
  float* o = out + (int64_t)img * per_img;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < per_img;
       e += (int64_t)gridDim.x * blockDim.x) {
    uint64_t u = splitmix64(key + (uint64_t)e);
    o[e] = (float)(u >> 40) * 5.9604644775390625e-08f;  // 2^-24
  }
}

void launch_synth(uint64_t seed, int64_t first, int32_t n_img, int32_t H, int32_t W, float* out,
                  hipStream_t s) {
  int64_t per = 3ll * H * W;
  int gx = (int)std::min<int64_t>((per + 255) / 256, 2048);
  hipLaunchKernelGGL(k_synth, dim3(gx, n_img), dim3(256), 0, s, seed, first, per, n_img, out);
}

// ---------------------------------------------------------------------------
// colour transforms (reference util.py:70-97)
// ---------------------------------------------------------------------------

// IPT of the images whose rows run through the GEMM DCT, written folded for
// the even / odd halves of the transform.  Along x (every such image): row y
// holds u[x] = p[x] + p[W-1-x] at x < ceil(W/2) (u = p at the middle of an
// odd W) and v[x] = p[x] - p[W-1-x] at ceil(W/2) + x, x < floor(W/2).  Along
// y (images whose columns also run through the GEMM): row m < floor(H/2)
// holds p[m] + p[H-1-m] and row H-1-m holds p[m] - p[H-1-m]; the row DCT is
// linear per row, so the row GEMM then yields T already folded for the
// column GEMM.  One thread per group of up to 4 mirrored pixels.
// Blocks from a host list of (image, first group): kRgbGroups groups per
// block (a grid over every image x the largest image's groups spent most of its
// blocks exiting on the ragged config 4), kRgbGpt groups per thread (thread t
// takes groups t + 256 k): every group's 12 loads are issued before any
// colour math, so a thread keeps up to 48 loads in flight (one group per
// thread, 256 groups per block, measured 1.55 ms on config 4).
constexpr int kRgbGpt = 4;
constexpr int kRgbGroups = 256 * kRgbGpt;

// |max| of a 256-thread block's values in uint order (|x| bits: NaN above Inf
// above finite) into *dst: one atomic per block (one per wave serialised
// thousands of atomics on one address per image: +0.25 ms on config 4).
// Every thread of the block must call it.
__device__ __forceinline__ void block_amax(uint32_t m, uint32_t* dst) {
  __shared__ uint32_t part[4];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max(part[0], part[1]), max(part[2], part[3]));
    if (m != 0u) atomicMax(dst, m);
  }
}

// cache policy of k_rgb_to_ipt's RGB loads / folded IPT stores: A/B switches,
// both off (nontemporal measured slower on config 4, round 5: rgb_to_ipt
// 1.41 -> 1.63 ms with NT loads, 1.93 ms with NT stores)
#ifndef DCTAE_IPT_ST_NT
#define DCTAE_IPT_ST_NT 0
#endif
#ifndef DCTAE_RGB_LD_NT
#define DCTAE_RGB_LD_NT 0
#endif
__device__ __forceinline__ void ipt_store(float* p, float v) {
  if (DCTAE_IPT_ST_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ float rgb_load(const float* p) {
  if (DCTAE_RGB_LD_NT) return __builtin_nontemporal_load(p);
  return *p;
}

__global__ __launch_bounds__(256) void k_rgb_to_ipt(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                    const float* __restrict__ rgb, float* __restrict__ ws,
                                                    ColorMats cm, uint32_t* __restrict__ amax) {
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const int W = d.W, H = d.H;
  const int64_t hw = (int64_t)H * W;
  const int Wh = (W + 1) / 2;
  const bool yfold = d.plan_h < 0;
  const int Hh = yfold ? (H + 1) / 2 : H;
  const int n_groups = Hh * Wh;   // < 2^31: the ABI's int32 image sides
  const float* src = rgb + d.rgb_off;
  float* dst = ws + d.ws_p;
  const float gam = 0.430000007152557373046875f;
  // pixel q of group k: 0 = (y, x), 1 = (y, x2), 2 = (y2, x), 3 = (y2, x2); absent
  // mirrors (middle column / row, no y-fold) re-read pixel 0 and are not stored
  float px[kRgbGpt][4][3];
  int yk[kRgbGpt], xk[kRgbGpt];
#pragma unroll
  for (int k = 0; k < kRgbGpt; ++k) {
    const int e = min(jb.y + (int)threadIdx.x + 256 * k, n_groups - 1);
    const int y = e / Wh, x = e - y * Wh;
    yk[k] = y;
    xk[k] = x;
    const int x2 = W - 1 - x, y2 = yfold ? H - 1 - y : y;
    const int64_t o[4] = {(int64_t)y * W + x, (int64_t)y * W + x2, (int64_t)y2 * W + x, (int64_t)y2 * W + x2};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < 3; ++c) px[k][q][c] = rgb_load(src + c * hw + o[q]);
  }
  uint32_t mx = 0;   // |max| of the values written (k_gemm_h2's operand scale)
#pragma unroll
  for (int k = 0; k < kRgbGpt; ++k) {
    const int e = jb.y + (int)threadIdx.x + 256 * k;
    if (e >= n_groups || e >= jb.y + kRgbGroups) break;
    const int y = yk[k], x = xk[k], x2 = W - 1 - x, y2 = H - 1 - y;
    const bool xp = x2 != x, yp = yfold && y2 != y;
    float p[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // util.py:70-82
      const float r = px[k][q][0], g = px[k][q][1], b = px[k][q][2];
      const float l0 = signed_pow_fast(mat3_row(cm.rgb2lms, 0, r, g, b), gam);
      const float l1 = signed_pow_fast(mat3_row(cm.rgb2lms, 1, r, g, b), gam);
      const float l2 = signed_pow_fast(mat3_row(cm.rgb2lms, 2, r, g, b), gam);
#pragma unroll
      for (int c = 0; c < 3; ++c) p[q][c] = mat3_row(cm.lms2ipt, c, l0, l1, l2);
    }
    // y-fold (rows y / y2: sum / difference), then the x-fold of each row's pair
    float a[3], b[3], c2[3], d2[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float pb = xp ? p[1][c] : 0.0f, pd = xp ? p[3][c] : 0.0f;
      a[c] = yp ? p[0][c] + p[2][c] : p[0][c];
      b[c] = yp ? pb + pd : pb;
      c2[c] = p[0][c] - p[2][c];
      d2[c] = pb - pd;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float* ro = dst + c * hw + (int64_t)y * W;
      const float u0 = xp ? a[c] + b[c] : a[c], v0 = a[c] - b[c];
      const float u1 = xp ? c2[c] + d2[c] : c2[c], v1 = c2[c] - d2[c];
      ipt_store(ro + x, u0);
      if (xp) ipt_store(ro + Wh + x, v0);
      if (yp) {
        float* r2 = dst + c * hw + (int64_t)y2 * W;
        ipt_store(r2 + x, u1);
        if (xp) ipt_store(r2 + Wh + x, v1);
      }
      mx = max(mx, __float_as_uint(u0) & 0x7fffffffu);
      if (xp) mx = max(mx, __float_as_uint(v0) & 0x7fffffffu);
      if (yp) mx = max(mx, __float_as_uint(u1) & 0x7fffffffu);
      if (yp && xp) mx = max(mx, __float_as_uint(v1) & 0x7fffffffu);
    }
  }
  if (amax) block_amax(mx, amax + 2 * jb.x);
}

// T (3, H, Kw) of the images whose columns run through the GEMM DCT but rows
// through the FFT, folded in place along y: T[m] <- T[m] + T[H-1-m],
// T[H-1-m] <- T[m] - T[H-1-m] for m < floor(H/2) (middle row of an odd H kept).
// Launched over the listed images only (grid.y = list entries): on the
// ragged config 4 a grid over every image spent 0.23 ms exiting blocks.
__global__ void k_fold_t(const ImgDesc* __restrict__ imgs, const int32_t* __restrict__ list, float* __restrict__ ws,
                         uint32_t* __restrict__ amax) {
  const ImgDesc d = imgs[list[blockIdx.y]];
  if (d.plan_h >= 0 || d.plan_w < 0) return;  // GEMM rows: folded by k_rgb_to_ipt
  const int Hh = (d.H + 1) / 2;                // the middle row of an odd H is kept (its |max| counts)
  const int64_t n = (int64_t)Hh * d.Kw;
  float* t = ws + d.ws_t;
  uint32_t mx = 0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < 3 * n; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e / n);
    const int64_t r = e - c * n;
    const int64_t m = r / d.Kw, kx = r - m * d.Kw;
    float* p0 = t + (int64_t)c * d.H * d.Kw + m * d.Kw + kx;
    float* p1 = t + (int64_t)c * d.H * d.Kw + (d.H - 1 - m) * d.Kw + kx;
    const float a = *p0;
    if (p1 == p0) {
      mx = max(mx, __float_as_uint(a) & 0x7fffffffu);
      continue;
    }
    const float b = *p1;
    *p0 = a + b;
    *p1 = a - b;
    mx = max(mx, max(__float_as_uint(a + b), __float_as_uint(a - b)) & 0x7fffffffu);
  }
  if (amax) block_amax(mx, amax + 2 * list[blockIdx.y] + 1);
}

void launch_fold_t(const ImgDesc* imgs, const int32_t* list, int n_list, int64_t max_hw, float* ws, uint32_t* amax,
                   hipStream_t s) {
  if (n_list <= 0) return;
  // up to 64 blocks per image (grid-stride): each block ends in one atomic on its image's |max|
  int gx = (int)std::min<int64_t>((3 * max_hw / 2 + 255) / 256, 64);
  hipLaunchKernelGGL(k_fold_t, dim3(std::max(gx, 1), n_list), dim3(256), 0, s, imgs, list, ws, amax);
}

int rgb_to_ipt_groups_per_block() { return kRgbGroups; }

void launch_rgb_to_ipt(const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                       const ColorMats& cm, uint32_t* amax, hipStream_t s) {
  if (n_blocks > 0) hipLaunchKernelGGL(k_rgb_to_ipt, dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, cm, amax);
}

// ipt (3,H,W) in place -> rgb written to out (3,H,W)
__global__ void k_ipt_to_rgb(const ImgDesc* __restrict__ imgs, const float* __restrict__ ws,
                             float* __restrict__ out, ColorMats cm) {
  const ImgDesc d = imgs[blockIdx.y];
  const int64_t hw = (int64_t)d.H * d.W;
  const float* src = ws + d.ws_p;
  float* dst = out + d.rgb_off;
  const float inv_gamma = 2.3255813121795654296875f;  // fp32(1/0.43)
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < hw;
       e += (int64_t)gridDim.x * blockDim.x) {
    float i0 = src[e], i1 = src[hw + e], i2 = src[2 * hw + e];
    float l0 = signed_pow(mat3_row(cm.ipt2lms, 0, i0, i1, i2), inv_gamma);
    float l1 = signed_pow(mat3_row(cm.ipt2lms, 1, i0, i1, i2), inv_gamma);
    float l2 = signed_pow(mat3_row(cm.ipt2lms, 2, i0, i1, i2), inv_gamma);
    dst[e] = mat3_row(cm.lms2rgb, 0, l0, l1, l2);
    dst[hw + e] = mat3_row(cm.lms2rgb, 1, l0, l1, l2);
    dst[2 * hw + e] = mat3_row(cm.lms2rgb, 2, l0, l1, l2);
  }
}

void launch_ipt_to_rgb(const ImgDesc* imgs, int n_img, int64_t max_hw, const float* ws, float* out,
                       const ColorMats& cm, hipStream_t s) {
  int gx = (int)std::min<int64_t>((max_hw + 255) / 256, 1024);
  hipLaunchKernelGGL(k_ipt_to_rgb, dim3(gx, n_img), dim3(256), 0, s, imgs, ws, out, cm);
}

// colour transform of a contiguous batch of (3, H, W) images, out of place:
// dir 0 = rgb_to_ipt (util.py:70-82), dir 1 = ipt_to_rgb (util.py:85-97).
// The standalone FE._transform_image_in / _out entry points (dctae_dct2).
__global__ void k_color(const float* __restrict__ x, float* __restrict__ y, int64_t hw, int n_img, int dir,
                        ColorMats cm) {
  const int64_t n = hw * n_img;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / hw, p = e - i * hw;
    const float* s = x + 3 * hw * i + p;
    float* d = y + 3 * hw * i + p;
    const float a = s[0], b = s[hw], c = s[2 * hw];
    if (dir == 0) {
      const float l0 = signed_pow_fast(mat3_row(cm.rgb2lms, 0, a, b, c), 0.430000007152557373046875f);
      const float l1 = signed_pow_fast(mat3_row(cm.rgb2lms, 1, a, b, c), 0.430000007152557373046875f);
      const float l2 = signed_pow_fast(mat3_row(cm.rgb2lms, 2, a, b, c), 0.430000007152557373046875f);
      d[0] = mat3_row(cm.lms2ipt, 0, l0, l1, l2);
      d[hw] = mat3_row(cm.lms2ipt, 1, l0, l1, l2);
      d[2 * hw] = mat3_row(cm.lms2ipt, 2, l0, l1, l2);
    } else {
      const float inv_gamma = 2.3255813121795654296875f;  // fp32(1/0.43)
      const float l0 = signed_pow(mat3_row(cm.ipt2lms, 0, a, b, c), inv_gamma);
      const float l1 = signed_pow(mat3_row(cm.ipt2lms, 1, a, b, c), inv_gamma);
      const float l2 = signed_pow(mat3_row(cm.ipt2lms, 2, a, b, c), inv_gamma);
      d[0] = mat3_row(cm.lms2rgb, 0, l0, l1, l2);
      d[hw] = mat3_row(cm.lms2rgb, 1, l0, l1, l2);
      d[2 * hw] = mat3_row(cm.lms2rgb, 2, l0, l1, l2);
    }
  }
}

// rgb_to_ipt of an fp16 / bf16 image the way the reference runs it in the
// input dtype (FE:135 calls util.rgb_to_ipt before x.float()): the matrices
// rounded to the dtype (Trgb2lms.to(x.dtype), Mipt.to(x.dtype)), each einsum
// accumulated in fp32 and rounded once (torch CPU einsum), the exponent 0.43
// rounded to the dtype and |x|**g computed in fp32 then rounded (torch CPU
// pow of a half / bfloat16 tensor), util.py:56-82.  x holds the dtype's values
// exactly as fp32; y: the dtype-rounded IPT values as fp32.
template <int LOWP>   // 2: fp16, 3: bf16
__device__ __forceinline__ float round_lowp(float v) {
  if (LOWP == 2) return __half2float(__float2half_rn(v));
  return __bfloat162float(__float2bfloat16(v));
}

template <int LOWP>
__global__ void k_color_lowp(const float* __restrict__ x, float* __restrict__ y, int64_t hw, int n_img, ColorMats cm) {
  float m1[9], m2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    m1[i] = round_lowp<LOWP>(cm.rgb2lms[i]);
    m2[i] = round_lowp<LOWP>(cm.lms2ipt[i]);
  }
  const float g = round_lowp<LOWP>(0.430000007152557373046875f);
  const int64_t n = hw * n_img;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / hw, p = e - i * hw;
    const float* s = x + 3 * hw * i + p;
    float* d = y + 3 * hw * i + p;
    const float a = s[0], b = s[hw], c = s[2 * hw];
    float l[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      // fp32 products of dtype values are exact; sum in j order, one rounding
      const float v = round_lowp<LOWP>(__fadd_rn(__fadd_rn(__fmul_rn(m1[3 * r], a), __fmul_rn(m1[3 * r + 1], b)),
                                                 __fmul_rn(m1[3 * r + 2], c)));
      const float pw = round_lowp<LOWP>(powf(fabsf(v), g));
      l[r] = v < 0.0f ? -pw : pw;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
      d[r * hw] = round_lowp<LOWP>(__fadd_rn(__fadd_rn(__fmul_rn(m2[3 * r], l[0]), __fmul_rn(m2[3 * r + 1], l[1])),
                                             __fmul_rn(m2[3 * r + 2], l[2])));
  }
}

void launch_color(const float* x, float* y, int64_t hw, int n_img, int dir, const ColorMats& cm, hipStream_t s) {
  const int64_t n = hw * n_img;
  const int g = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (dir == 2)
    hipLaunchKernelGGL(k_color_lowp<2>, dim3(std::max(g, 1)), dim3(256), 0, s, x, y, hw, n_img, cm);
  else if (dir == 3)
    hipLaunchKernelGGL(k_color_lowp<3>, dim3(std::max(g, 1)), dim3(256), 0, s, x, y, hw, n_img, cm);
  else
    hipLaunchKernelGGL(k_color, dim3(std::max(g, 1)), dim3(256), 0, s, x, y, hw, n_img, dir, cm);
}

// ---------------------------------------------------------------------------
// generic batched strided fp32 GEMM on MFMA (v_mfma_f32_32x32x2_f32)
//   O[c][m][n] = sum_k A[c][m][k] * B[c][n][k]
// 64x64 output tile per workgroup, 4 waves (2x2) of 32x32, K chunks of 32.
// Used for the DCT of sizes without an FFT plan and for the decode IDCT.
// ---------------------------------------------------------------------------

constexpr int GT = 64;      // tile edge
constexpr int GK = 32;      // k chunk
constexpr int GLD = GK + 4; // LDS row stride (floats), keeps float4 alignment

// SH: which operand all channels share, known at compile time — 1: B (the DCT
// matrix of a row transform), 2: A (of a column transform), 0: read from the
// problem's strides.  Only the unshared operand is staged per channel (LDS
// 37 KB instead of 55 KB at NC = 3), and the per-lane offsets are 32-bit on a
// uniform per-channel base: the 64-bit address arithmetic of 48 loads had
// taken the kernel to 256 VGPRs with spills (2 waves / SIMD).
template <int NC, int SH>
__global__ __launch_bounds__(256, 2) void k_gemm_f32(const GemmProblem* __restrict__ probs,
                                                  const TileRef* __restrict__ tiles) {
  constexpr int NA = SH == 2 ? 1 : NC, NB = SH == 1 ? 1 : NC;
  __shared__ __attribute__((aligned(16))) float As[NA][GT * GLD];
  __shared__ __attribute__((aligned(16))) float Bs[NB][GT * GLD];
  const TileRef tr = tiles[blockIdx.x];
  if (tr.problem < 0) return;   // padding of an XCD-dealt list
  const GemmProblem p = probs[tr.problem];
  const int tm = tr.tile / p.tiles_n, tn = tr.tile % p.tiles_n;
  const int m0 = tm * GT, n0 = tn * GT;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int half = lane >> 5, l32 = lane & 31;
  const bool a_shared = SH == 2 ? true : SH == 1 ? false : (p.sAc == 0);
  const bool b_shared = SH == 1 ? true : SH == 2 ? false : (p.sBc == 0);

  floatx16 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;

  // ---- staging: the next K chunk is loaded into registers while the current
  //      one is multiplied (generic strides, zero-filled at the edges)
  constexpr int EPT = (GT * GK) / 256;   // elements per thread and operand tile
  float ra[NA][EPT], rb[NB][EPT];
  const bool akf = (p.sAk == 1), bkf = (p.sBk == 1);
  const int sAm = (int)p.sAm, sAk = (int)p.sAk, sBn = (int)p.sBn, sBk = (int)p.sBk;
  auto load = [&](int k0) {
#pragma unroll
    for (int c = 0; c < NA; ++c) {
      if (c == 0 || !a_shared) {
        const float* A = p.A + (int64_t)c * p.sAc;
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + 256 * i;
          const int mm = akf ? (e >> 5) : (e & 63), kk = akf ? (e & 31) : (e >> 6);
          const int gm = m0 + mm, gk = k0 + kk;
          const bool ok = gm < p.M && gk < p.K;
          ra[c][i] = ok ? A[ok ? gm * sAm + gk * sAk : 0] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      if (c == 0 || !b_shared) {
        const float* B = p.B + (int64_t)c * p.sBc;
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + 256 * i;
          const int nn = bkf ? (e >> 5) : (e & 63), kk = bkf ? (e & 31) : (e >> 6);
          const int gn = n0 + nn, gk = k0 + kk;
          const bool ok = gn < p.N && gk < p.K;
          rb[c][i] = ok ? B[ok ? gn * sBn + gk * sBk : 0] : 0.0f;
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int c = 0; c < NA; ++c) {
      if (c == 0 || !a_shared) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + 256 * i;
          const int mm = akf ? (e >> 5) : (e & 63), kk = akf ? (e & 31) : (e >> 6);
          As[c][mm * GLD + kk] = ra[c][i];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      if (c == 0 || !b_shared) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + 256 * i;
          const int nn = bkf ? (e >> 5) : (e & 63), kk = bkf ? (e & 31) : (e >> 6);
          Bs[c][nn * GLD + kk] = rb[c][i];
        }
      }
    }
  };
  load(0);
  store();
  __syncthreads();
  for (int k0 = 0; k0 < p.K; k0 += GK) {
    const bool more = k0 + GK < p.K;
    if (more) load(k0 + GK);
    // ---- MFMA: lane half h takes k = 8g + 4h + s in step s of group g
#pragma unroll
    for (int g = 0; g < GK / 8; ++g) {
      const int kofs = 8 * g + 4 * half;
      float4 a4[NC], b4[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ca = (NA == 1 || a_shared) ? 0 : c, cb = (NB == 1 || b_shared) ? 0 : c;
        a4[c] = *reinterpret_cast<const float4*>(&As[ca][(wm * 32 + l32) * GLD + kofs]);
        b4[c] = *reinterpret_cast<const float4*>(&Bs[cb][(wn * 32 + l32) * GLD + kofs]);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[c].x, b4[c].x, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[c].y, b4[c].y, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[c].z, b4[c].z, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[c].w, b4[c].w, acc[c], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  // ---- store: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float* O = p.O + (int64_t)c * p.sOc;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = (r & 3) + 8 * (r >> 2) + 4 * half;
      int gm = m0 + wm * 32 + row, gn = n0 + wn * 32 + l32;
      if (gm < p.M && gn < p.N) O[(int64_t)gm * p.sOm + (int64_t)gn * p.sOn] = acc[c][r];
    }
  }
}

int gemm_share(const GemmProblem& g) {
  if (g.C > 1 && g.sBc == 0 && g.sAc != 0) return 1;
  if (g.C > 1 && g.sAc == 0 && g.sBc != 0) return 2;
  return 0;
}

void launch_gemm(int nc, const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share) {
  if (n_tiles <= 0) return;
  if (nc == 3 && share == 1)
    hipLaunchKernelGGL((k_gemm_f32<3, 1>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else if (nc == 3 && share == 2)
    hipLaunchKernelGGL((k_gemm_f32<3, 2>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else if (nc == 3)
    hipLaunchKernelGGL((k_gemm_f32<3, 0>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
  else
    hipLaunchKernelGGL((k_gemm_f32<1, 0>), dim3(n_tiles), dim3(256), 0, s, probs, tiles);
}

// ---------------------------------------------------------------------------
// tile epilogue: spectrum corner Y (3,Kh,Kw) -> per token (flat order
// f = (h*qw+w)*3 + c): importance score (FE:401-416), LFQ codes of the
// PatchNorm'd token (patchnorm.py:157-165, lfq.py:174-187), optional raw /
// normalised token copies.  One 16-lane group per token, lane j = tile row j.
// ---------------------------------------------------------------------------


// dense path: Y from workspace.  grid (ceil(Tmax/64), n_img), 256 threads:
// each block handles 64 tokens (16 per pass, 4 passes).
__global__ __launch_bounds__(256) void k_tile_epilogue(const ImgDesc* __restrict__ imgs,
                                                       const float* __restrict__ ws, EncParams ep,
                                                       TokenSinks sk) {
  __shared__ uint16_t rowbits[16 * kMaxP];
  const ImgDesc d = imgs[blockIdx.y];
  if (d.plan_h >= 0 && !(d.bs & 2)) return;  // columns on the Makhoul FFT kernels (epilogue fused there)
  const int g16 = threadIdx.x >> 4, j = threadIdx.x & 15;
  const float* Y = ws + d.ws_y;
  for (int pass = 0; pass < 4; ++pass) {
    const int f = blockIdx.x * 64 + pass * 16 + g16;
    if (f >= d.T) break;  // uniform per group; groups past T idle
    const int c = f % ep.C, s = f / ep.C, h = s / d.qw, w = s % d.qw;
    float vals[kMaxP];
    if (j < ep.P) {
      const float* row = Y + ((int64_t)c * d.Kh + (int64_t)ep.P * h + j) * d.Kw;
      for (int p2 = 0; p2 < ep.P; ++p2) vals[p2] = row[col_of_kx(d, ep.P * w + p2)];
    }
    token_epilogue(ep, c, h, w, j, g16, vals, d.tok_off + f, sk, rowbits);
  }
}

// patch size fixed at compile time: one block per (tile row h, channel c) of
// an image stages the P spectrum rows it covers (contiguous in Y) through LDS
// with coalesced loads, then one 16-lane group per tile runs
// token_epilogue_p on its row held in registers.
#ifndef DCTAE_TEPI_ROWS
#define DCTAE_TEPI_ROWS 1
#endif
#ifndef DCTAE_TEPI_LIST
#define DCTAE_TEPI_LIST 1   // 0: the grid over every image x 3 max_patch_h (A/B)
#endif
// list (nullable): the (local image, 3 h + c) blocks of the images with Y in the
// workspace, built on the host (grid = list length): a grid over every image x
// 3 max_patch_h spent most of its blocks exiting on ragged batches
template <int P>
__global__ __launch_bounds__(256) void k_tile_epilogue_p(const ImgDesc* __restrict__ imgs,
                                                         const float* __restrict__ ws, EncParams ep,
                                                         TokenSinks sk, const int2* __restrict__ list) {
  extern __shared__ float ys[];
  const int2 jb = list ? list[blockIdx.x] : make_int2((int)blockIdx.y, (int)blockIdx.x);
  const ImgDesc d = imgs[jb.x];
  if (d.plan_h >= 0 && !(d.bs & 2)) return;
  const int c = jb.y % 3, h = jb.y / 3;
  if (h >= d.qh) return;
  const int Kw = d.Kw, ld = Kw + 1;
  const float* Y = ws + d.ws_y + ((int64_t)c * d.Kh + (int64_t)P * h) * Kw;
#if DCTAE_TEPI_ROWS
  // the tile row's P rows column chunk by column chunk: P independent loads per
  // thread in flight, no per-element division (the flat loop's e / Kw cost
  // ~20 VALU per element and serialised its loads)
  for (int x0 = 0; x0 < Kw; x0 += 256) {
    const int x = x0 + (int)threadIdx.x;
    const bool on = x < Kw;
    float a[P];
#pragma unroll
    for (int r = 0; r < P; ++r) a[r] = Y[(int64_t)r * Kw + (on ? x : 0)];
    if (on) {
      const int kx = kx_of_col(d, x);   // parity-planar Y (tperm) back to natural columns
#pragma unroll
      for (int r = 0; r < P; ++r) ys[r * ld + kx] = a[r];
    }
  }
#else
  for (int e = threadIdx.x; e < P * Kw; e += 256) {
    const int r = e / Kw;
    ys[r * ld + kx_of_col(d, e - r * Kw)] = Y[e];
  }
#endif
  __syncthreads();
  const int g16 = threadIdx.x >> 4, j = threadIdx.x & 15;
  const int jr = j < P ? j : 0;
  for (int w = g16; w < d.qw; w += 16) {
    float vals[P];
#pragma unroll
    for (int p2 = 0; p2 < P; ++p2) vals[p2] = ys[jr * ld + P * w + p2];
    token_epilogue_p<P>(ep, c, h, w, j, vals, d.tok_off + (int64_t)(h * d.qw + w) * 3 + c, sk);
  }
}

void launch_tile_epilogue(const ImgDesc* imgs, int n_img, int max_T, const float* ws,
                          const EncParams& ep, const TokenSinks& sk, hipStream_t s, const int2* list, int n_list) {
  if (ep.P == 14 && ep.C == 3 && 14 * (14 * ep.maxpw + 1) * sizeof(float) <= 64 * 1024) {
    const size_t lds = (size_t)14 * (14 * ep.maxpw + 1) * sizeof(float);
    if (list && DCTAE_TEPI_LIST) {
      if (n_list > 0)
        hipLaunchKernelGGL(k_tile_epilogue_p<14>, dim3(n_list), dim3(256), lds, s, imgs, ws, ep, sk, list);
    } else {
      hipLaunchKernelGGL(k_tile_epilogue_p<14>, dim3(3 * ep.maxph, n_img), dim3(256), lds, s, imgs, ws, ep, sk,
                         (const int2*)nullptr);
    }
  } else
    hipLaunchKernelGGL(k_tile_epilogue, dim3((max_T + 63) / 64, n_img), dim3(256), 0, s, imgs, ws, ep, sk);
}

// ---------------------------------------------------------------------------
// per-image sort (score desc, flat index asc) + scatter into packed rows
// (FE:418-445 gather, FE:515-605 concatenation).  One block per image.
// ---------------------------------------------------------------------------


__global__ __launch_bounds__(1024) void k_sort_pack(const ImgDesc* __restrict__ imgs, int np2,
                                                    EncParams ep, TokenSinks st, PackSinks out) {
  extern __shared__ uint64_t keys[];
  const ImgDesc d = imgs[blockIdx.x];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < np2; i += nt) {
    uint64_t k = 0;
    if (i < d.T)
      k = ((uint64_t)float_key(st.scores[d.tok_off + stage_pos(d, i)]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
    keys[i] = k;
  }
  // bitonic sort, descending
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < (np2 >> 1); t += nt) {
        int i = 2 * t - (t & (stride - 1));
        int jx = i + stride;
        uint64_t a = keys[i], b = keys[jx];
        bool desc = (i & size) == 0;
        if (desc ? (a < b) : (a > b)) {
          keys[i] = b;
          keys[jx] = a;
        }
      }
    }
  }
  __syncthreads();
  const int S = ep.S, PP = ep.P * ep.P, C = ep.C;
  const int64_t base = (int64_t)d.row * S + d.col;
  for (int t = tid; t < d.k; t += nt) {
    const uint32_t f = 0xFFFFFFFFu - (uint32_t)(keys[t] & 0xFFFFFFFFu);
    const int c = f % C, s = f / C, h = s / d.qw, w = s % d.qw;
    const int64_t o = base + t;
    out.pos[2 * o] = h;
    out.pos[2 * o + 1] = w;
    out.ch[o] = c;
    out.ids[o] = d.local_id;
    if (out.key_pad) out.key_pad[o] = 0;
    if (out.scores) out.scores[o] = st.scores[d.tok_off + stage_pos(d, f)];
  }
  if (out.codes) {
    const int ncb = ep.ncb;
    for (int e = tid; e < d.k * ncb; e += nt) {
      const int t = e / ncb, q = e % ncb;
      const uint32_t f = stage_pos(d, 0xFFFFFFFFu - (uint32_t)(keys[t] & 0xFFFFFFFFu));
      out.codes[(base + t) * ncb + q] = (int64_t)lfq_index_bits(st.codes[(d.tok_off + f) * ncb + q], ep.code_pos,
                                                                ep.code_neg);
    }
  }
  if (out.patches || out.raw) {
    for (int64_t e = tid; e < (int64_t)d.k * PP; e += nt) {
      const int t = (int)(e / PP), q = (int)(e % PP);
      const uint32_t f = stage_pos(d, 0xFFFFFFFFu - (uint32_t)(keys[t] & 0xFFFFFFFFu));
      if (out.patches) out.patches[(base + t) * PP + q] = st.norm[(d.tok_off + f) * PP + q];
      if (out.raw) out.raw[(base + t) * PP + q] = st.raw[(d.tok_off + f) * PP + q];
    }
  }
}

// packed-order copy of the staged tokens (PP floats each) of one image:
// 16-byte pieces when PP % 4 == 0 and every base is 16-byte aligned (196 =
// 49 x 4 at P = 14), 32-bit index math (k * PP <= 3072 * 196)
__device__ __forceinline__ void gather_tokens(const ImgDesc& d, const uint16_t* order, int64_t base, int PP,
                                              const TokenSinks& st, const PackSinks& out, int tid, int nt) {
  const bool vec = (PP & 3) == 0 && ((reinterpret_cast<uintptr_t>(out.patches) | reinterpret_cast<uintptr_t>(out.raw) |
                                      reinterpret_cast<uintptr_t>(st.norm) | reinterpret_cast<uintptr_t>(st.raw)) & 15) == 0;
  if (vec) {
    const uint32_t P4 = (uint32_t)PP >> 2, n = (uint32_t)d.k * P4;
    for (uint32_t e = tid; e < n; e += nt) {
      const uint32_t t = e / P4, q = e - t * P4;
      const int64_t src = (d.tok_off + order[t]) * P4 + q, dst = (base + t) * P4 + q;
      if (out.patches) reinterpret_cast<float4*>(out.patches)[dst] = reinterpret_cast<const float4*>(st.norm)[src];
      if (out.raw) reinterpret_cast<float4*>(out.raw)[dst] = reinterpret_cast<const float4*>(st.raw)[src];
    }
    return;
  }
  const uint32_t n = (uint32_t)d.k * (uint32_t)PP;
  for (uint32_t e = tid; e < n; e += nt) {
    const uint32_t t = e / (uint32_t)PP, q = e - t * (uint32_t)PP;
    const int64_t src = (d.tok_off + order[t]) * PP + q, dst = (base + t) * PP + q;
    if (out.patches) out.patches[dst] = st.norm[src];
    if (out.raw) out.raw[dst] = st.raw[src];
  }
}

// Same contract with rocPRIM's block radix sort (LSD, stable): 32-bit score
// keys sorted descending, flat indices as values; stability keeps equal
// scores in ascending index order = the (score desc, index asc) order above.
// Tokens per image <= 512 x 6 = 3072 (max_patch 32 x 32, 3 channels); the
// 256 x 3 instance covers 224^2 images (768 tokens).
typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
typedef unsigned v2u32s __attribute__((ext_vector_type(2)));

template <int kSortBS, int kSortIPT>
__global__ __launch_bounds__(kSortBS) void k_sort_pack2(const ImgDesc* __restrict__ imgs, EncParams ep,
                                                        TokenSinks st, PackSinks out) {
  using Sort = rocprim::block_radix_sort<uint32_t, kSortBS, kSortIPT, uint32_t>;
  __shared__ typename Sort::storage_type tmp;
  __shared__ uint16_t order[kSortBS * kSortIPT];   // flat token index f of rank t
  __shared__ uint16_t spos[kSortBS * kSortIPT];    // its staging position (stage_pos)
  const int tid = threadIdx.x;
  const ImgDesc d = imgs[blockIdx.x];
  uint32_t keys[kSortIPT], vals[kSortIPT];
  {
    // all six score loads in flight at once (unconditional: past-the-end lanes
    // read 0 through the descriptor's num_records)
    const auto krs = __builtin_amdgcn_make_buffer_rsrc(st.scores + d.tok_off, 0, d.T * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < kSortIPT; ++i) {
      const int idx = tid * kSortIPT + i;   // blocked: input order = index order (stability -> index asc)
      keys[i] = __builtin_amdgcn_raw_buffer_load_b32(krs, idx < d.T ? stage_pos(d, idx) * 4 : 0x7ffffff0, 0, 0);
      vals[i] = (uint32_t)idx;
    }
#pragma unroll
    for (int i = 0; i < kSortIPT; ++i) keys[i] = (int)vals[i] < d.T ? float_key(__uint_as_float(keys[i])) : 0u;
  }
  Sort().sort_desc_to_striped(keys, vals, tmp);
#pragma unroll
  for (int i = 0; i < kSortIPT; ++i) {
    const int rank = tid + kSortBS * i;
    if (rank < d.k) {
      order[rank] = (uint16_t)vals[i];
      spos[rank] = (uint16_t)stage_pos(d, (int)vals[i]);
    }
  }
  __syncthreads();
  const int S = ep.S, PP = ep.P * ep.P, C = ep.C;
  const int64_t base = (int64_t)d.row * S + d.col;
  for (int t = tid; t < d.k; t += kSortBS) {
    const uint32_t f = order[t];
    const int c = f % C, s = f / C, h = s / d.qw, w = s % d.qw;
    const int64_t o = base + t;
#ifdef DCTAE_SORT_META_NT
    __builtin_nontemporal_store((v2i64){(long long)h, (long long)w}, reinterpret_cast<v2i64*>(out.pos + 2 * o));
    __builtin_nontemporal_store((long long)c, reinterpret_cast<long long*>(out.ch + o));
    __builtin_nontemporal_store((long long)d.local_id, reinterpret_cast<long long*>(out.ids + o));
#else
    *reinterpret_cast<longlong2*>(out.pos + 2 * o) = make_longlong2(h, w);
    out.ch[o] = c;
    out.ids[o] = d.local_id;
#endif
    if (out.key_pad) out.key_pad[o] = 0;
    if (out.scores) out.scores[o] = st.scores[d.tok_off + spos[t]];
  }
  if (out.codes && ep.ncb == 14) {
    // two codes per lane: one u32 of the u16 staging -> one 16-byte int64 pair
    // (coalesced).  kCU gathers in flight per lane before any is used (one
    // gather + wait per iteration exposed the load latency 42 times per lane),
    // buffer descriptors on the image's staging / packed span (32-bit offsets;
    // past-the-end lanes clipped by num_records)
    constexpr int kCU = 14;
    const uint32_t pos2 = ep.code_pos | (ep.code_pos << 16), neg2 = ep.code_neg | (ep.code_neg << 16);
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(st.codes + d.tok_off * 14, 0, d.T * 28, 0x00020000);
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(out.codes + base * 14, 0, d.k * 112, 0x00020000);
    const int n = d.k * 7;
    for (int e0 = tid; e0 < n; e0 += kSortBS * kCU) {
      uint32_t v[kCU];
#pragma unroll
      for (int u = 0; u < kCU; ++u) {
        const int e = e0 + kSortBS * u;
        const int t = min(e / 7, d.k - 1), q = e - (e / 7) * 7;
        v[u] = __builtin_amdgcn_raw_buffer_load_b32(srs, (spos[t] * 7 + q) * 4, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kCU; ++u) {
        const int e = e0 + kSortBS * u;
        const uint32_t c2 = (uint32_t)lfq_index_bits(v[u], pos2, neg2);
        // write-once outputs: nontemporal stores (their lines leave the L2 /
        // Infinity Cache early instead of being written back under the next
        // step's row kernel: sort 0.146 -> 0.143 ms, next rows 1.13 -> 1.11 ms)
        __builtin_amdgcn_raw_buffer_store_b128((v4u32){c2 & 0xFFFFu, 0u, c2 >> 16, 0u}, drs,
                                               e < n ? e * 16 : 0x7ffffff0, 0, 2);
      }
    }
  } else if (out.codes) {
    // any ncb: one u16 -> one int64 per lane, kCU gathers in flight (as above)
    constexpr int kCU = 16;
    const int ncb = ep.ncb, n = d.k * ncb;
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(st.codes + d.tok_off * ncb, 0, d.T * ncb * 2, 0x00020000);
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(out.codes + base * ncb, 0, n * 8, 0x00020000);
    for (int e0 = tid; e0 < n; e0 += kSortBS * kCU) {
      uint32_t v[kCU];
#pragma unroll
      for (int u = 0; u < kCU; ++u) {
        const int e = e0 + kSortBS * u;
        const int t = min(e / ncb, d.k - 1), q = e - (e / ncb) * ncb;
        v[u] = __builtin_amdgcn_raw_buffer_load_b16(srs, (spos[t] * ncb + q) * 2, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kCU; ++u) {
        const int e = e0 + kSortBS * u;
        const uint32_t cv = (uint32_t)lfq_index_bits(v[u], ep.code_pos, ep.code_neg);
        __builtin_amdgcn_raw_buffer_store_b64((v2u32s){cv, 0u}, drs, e < n ? e * 8 : 0x7ffffff0, 0, 2);
      }
    }
  }
  if (out.patches || out.raw) gather_tokens(d, spos, base, PP, st, out, tid, kSortBS);
}

void launch_sort_pack(const ImgDesc* imgs, int n_img, int np2, const EncParams& ep, const TokenSinks& st,
                      const PackSinks& out, hipStream_t s, int kernel, int max_T) {
  // 224^2 images (768 tokens): a quarter-size block (a full one sorted 3072
  // padded keys per image)
  if (kernel == 2 && max_T <= 256 * 3)
    hipLaunchKernelGGL((k_sort_pack2<256, 3>), dim3(n_img), dim3(256), 0, s, imgs, ep, st, out);
  else if (kernel == 2 && max_T <= 512 * 6)
    hipLaunchKernelGGL((k_sort_pack2<512, 6>), dim3(n_img), dim3(512), 0, s, imgs, ep, st, out);
  else
    hipLaunchKernelGGL(k_sort_pack, dim3(n_img), dim3(1024), (size_t)np2 * 8, s, imgs, np2, ep, st, out);
}

// pad positions j >= row_len[r] of each packed row: the reference pads
// patches with zeros (util.py:149-164), ids/pos/ch with 0 and then runs
// PatchNorm/LFQ on them like on any token (c = h = w = 0).
__global__ void k_pad_fill(const int32_t* __restrict__ row_len, int n_rows, EncParams ep, uint8_t* key_pad,
                           PackSinks out) {
  // the pad token (zeros at c = h = w = 0) normalises and quantises the same
  // at every pad position: its patch and codes once per block, in LDS
  __shared__ float pp[kMaxP * kMaxP];
  __shared__ int64_t pcode[kMaxCodebooks];
  const int r = blockIdx.y;
  const int S = ep.S, PP = ep.P * ep.P;
  const int len = row_len[r];
  if ((int)(blockIdx.x * blockDim.x) + (int)blockDim.x <= len) {   // no pads in this block's span
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < S; j += gridDim.x * blockDim.x)
      key_pad[(int64_t)r * S + j] = 0;
    if (gridDim.x * blockDim.x >= (unsigned)S) return;
  }
  if (out.patches || out.codes) {
    for (int e = threadIdx.x; e < PP; e += blockDim.x)
      pp[e] = pn_forward(0.0f, ep.median[e], ep.b[e], ep.eps, ep.min_val, ep.max_val);
    __syncthreads();
    if (out.codes)
      for (int q = threadIdx.x; q < ep.ncb; q += blockDim.x) {
        uint32_t code = 0;
        for (int dd = 0; dd < ep.cb_dim; ++dd) code |= (pp[q * ep.cb_dim + dd] > 0.0f ? 1u : 0u) << (ep.cb_dim - 1 - dd);
        pcode[q] = (int64_t)lfq_index_bits(code, ep.code_pos, ep.code_neg);
      }
    __syncthreads();
  }
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < S; j += gridDim.x * blockDim.x) {
    const int64_t o = (int64_t)r * S + j;
    key_pad[o] = (j >= len) ? 1 : 0;
    if (j < len) continue;
    out.pos[2 * o] = 0;
    out.pos[2 * o + 1] = 0;
    out.ch[o] = 0;
    out.ids[o] = 0;
    if (out.scores) out.scores[o] = 0.0f;
    if (out.raw)
      for (int e = 0; e < PP; ++e) out.raw[o * PP + e] = 0.0f;
    if (out.patches)
      for (int e = 0; e < PP; ++e) out.patches[o * PP + e] = pp[e];
    if (out.codes)
      for (int q = 0; q < ep.ncb; ++q) out.codes[o * ep.ncb + q] = pcode[q];
  }
}

void launch_pad_fill(const int32_t* row_len, int n_rows, const EncParams& ep, uint8_t* key_pad,
                     const PackSinks& out, hipStream_t s) {
  int gx = (ep.S + 255) / 256;
  hipLaunchKernelGGL(k_pad_fill, dim3(gx, n_rows), dim3(256), 0, s, row_len, n_rows, ep, key_pad, out);
}

// ---------------------------------------------------------------------------
// standalone elementwise ops on packed tokens
// ---------------------------------------------------------------------------

__global__ void k_norm(const float* __restrict__ x, const int64_t* __restrict__ ch,
                       const int64_t* __restrict__ pos, int64_t n, int PP, int maxph, int maxpw,
                       const float* __restrict__ med, const float* __restrict__ b, float eps, float lo,
                       float hi, int inverse, float* __restrict__ y, int* __restrict__ err) {
  const int64_t total = n * PP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / PP;
    const int q = (int)(e % PP);
    const int64_t c = ch[t], h = pos[2 * t], w = pos[2 * t + 1];
    if (c < 0 || c >= 3 || h < 0 || h >= maxph || w < 0 || w >= maxpw) {
      // the reference raises IndexError on out-of-range table indices
      atomicOr(err, 1);
      y[e] = __int_as_float(0x7fc00000);
      continue;
    }
    const int64_t tab = ((c * maxph + h) * maxpw + w) * PP + q;
    y[e] = inverse ? pn_inverse(x[e], med[tab], b[tab], eps) : pn_forward(x[e], med[tab], b[tab], eps, lo, hi);
  }
}

void launch_norm(const float* x, const int64_t* ch, const int64_t* pos, int64_t n, int PP, int maxph,
                 int maxpw, const float* med, const float* b, float eps, float lo, float hi, int inverse,
                 float* y, int* err, hipStream_t s) {
  int64_t total = n * PP;
  int gx = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (gx <= 0) return;
  hipLaunchKernelGGL(k_norm, dim3(gx), dim3(256), 0, s, x, ch, pos, n, PP, maxph, maxpw, med, b, eps, lo, hi,
                     inverse, y, err);
}

// LFQ forward: one thread per (token, codebook)
__global__ void k_lfq_forward(const float* __restrict__ x, int64_t n, int cb_dim, int ncb, float scale,
                              uint64_t code_pos, uint64_t code_neg, float* __restrict__ q, int64_t* __restrict__ idx) {
  const int64_t total = n * ncb;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float* xi = x + e * cb_dim;
    int64_t code = 0;
    for (int d = 0; d < cb_dim; ++d) {
      const bool pos = xi[d] > 0.0f;  // lfq.py:175 (NaN -> False)
      code += pos ? ((int64_t)1 << (cb_dim - 1 - d)) : 0;
      if (q) q[e * cb_dim + d] = pos ? scale : -scale;
    }
    idx[e] = (int64_t)lfq_index_bits((uint64_t)code, code_pos, code_neg);   // lfq.py:187 (quantized > 0)
  }
}

void launch_lfq_forward(const float* x, int64_t n, int cb_dim, int ncb, float scale, float* q, int64_t* idx,
                        hipStream_t s) {
  int64_t total = n * ncb;
  int gx = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (gx <= 0) return;
  uint64_t pos, neg;
  lfq_index_masks(scale, cb_dim, &pos, &neg);
  hipLaunchKernelGGL(k_lfq_forward, dim3(gx), dim3(256), 0, s, x, n, cb_dim, ncb, scale, pos, neg, q, idx);
}

// LFQ.indices_to_codes: bits * scale * 2 - scale
__global__ void k_lfq_codes(const int64_t* __restrict__ idx, int64_t n, int cb_dim, int ncb, float scale,
                            float* __restrict__ out) {
  const int64_t total = n * ncb * cb_dim;
  const float s2 = scale * 2.0f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / cb_dim;
    const int d = (int)(e % cb_dim);
    const int32_t v = (int32_t)idx[t];  // lfq.py:117 indices.int()
    const float bit = ((v & (1 << (cb_dim - 1 - d))) != 0) ? 1.0f : 0.0f;
    out[e] = __fsub_rn(__fmul_rn(bit, s2), scale);
  }
}

void launch_lfq_codes(const int64_t* idx, int64_t n, int cb_dim, int ncb, float scale, float* out, hipStream_t s) {
  int64_t total = n * ncb * cb_dim;
  int gx = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (gx <= 0) return;
  hipLaunchKernelGGL(k_lfq_codes, dim3(gx), dim3(256), 0, s, idx, n, cb_dim, ncb, scale, out);
}

// ---------------------------------------------------------------------------
// decode: scatter tokens of packed rows into per-image spectrum corners
// (FE:607-656 revert_patching), optionally dequantising LFQ codes
// (lfq.py:105-134) and inverting PatchNorm (patchnorm.py:167-177) on the fly.
// ---------------------------------------------------------------------------


// Two tokens at one image place (c, h, w): FE:639-643 assigns them in packed
// order, so the later slot wins.  map (k_dec_map, atomicMax) holds that slot
// per place; only its elements are stored (plain stores of every duplicate
// would race and make the result depend on the schedule).
__global__ void k_scatter_tokens(int64_t n_tok, const ImgDesc* __restrict__ imgs, float* __restrict__ ws,
                                 DecodeArgs a, const int32_t* __restrict__ map) {
  const int PP = a.P * a.P;
  const int64_t total = n_tok * PP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / PP;
    const int q = (int)(e % PP);
    if (a.key_pad[t]) continue;
    const int64_t r = t / a.S;
    const int64_t id = a.ids[t];
    if (id < 0 || id >= a.lut_w) { atomicOr(a.err, 2); continue; }
    const int im = a.lut[r * a.lut_w + id];
    if (im < 0) { atomicOr(a.err, 2); continue; }
    const ImgDesc d = imgs[im];
    const int64_t c = a.ch[t], h = a.pos[2 * t], w = a.pos[2 * t + 1];
    if (c < 0 || c >= 3 || h < 0 || h >= d.qh || w < 0 || w >= d.qw) { atomicOr(a.err, 4); continue; }
    if (map[(((int64_t)im * 3 + c) * a.maxpw + w) * a.maxph + h] != (int32_t)t) continue;   // a later slot wins
    float v;
    if (a.use_codes) {
      const int cbi = q / a.cb_dim, dd = q % a.cb_dim;
      const int32_t code = (int32_t)a.codes[t * a.ncb + cbi];
      const float bit = ((code & (1 << (a.cb_dim - 1 - dd))) != 0) ? 1.0f : 0.0f;
      const float y = __fsub_rn(__fmul_rn(bit, a.scale * 2.0f), a.scale);
      const int64_t tab = ((c * a.maxph + h) * a.maxpw + w) * PP + q;
      v = pn_inverse(y, a.median[tab], a.b[tab], a.eps);
    } else {
      v = a.patches[e];
    }
    const int p1 = q / a.P, p2 = q % a.P;
    ws[d.ws_y + (c * d.Kh + (int64_t)a.P * h + p1) * d.Kw + (int64_t)a.P * w + p2] = v;
  }
}

void launch_scatter_tokens(int64_t n_tok, const ImgDesc* imgs, float* ws, const DecodeArgs& a, const int32_t* map,
                           hipStream_t s) {
  int64_t total = n_tok * a.P * a.P;
  int gx = (int)std::min<int64_t>((total + 255) / 256, 16384);
  if (gx <= 0) return;
  hipLaunchKernelGGL(k_scatter_tokens, dim3(gx), dim3(256), 0, s, n_tok, imgs, ws, a, map);
}

}  // namespace dctae
