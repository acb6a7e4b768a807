// Decode row pass for images 512 pixels wide with Kw = 448 (the config-3
// round trip): U[c][y][kx] (kx < 448, zero beyond) -> orthonormal DCT-III of
// every row (torch_dct.idct, util.py:337-338 <- FE:149) -> IPT -> RGB
// (util.py:85-97), the mirror image of the row item of k_rows512pk (dctae_rows512.h).
//
// Inverse Makhoul (dctae_idct.hip's header): conj Z_k = conj(a_k) (Ys[k] +
// i Ys[N-k]) + conj(b_k) (Ys[M+k] + i Ys[M-k]), k < M = 256; W = FFT_256(conj Z)
// (two radix-16 Stockham passes); x[4m] = Re W[m], x[4m+2] = -Im W[m] (m < 128),
// x[1023-4m] = Re W[m], x[1021-4m] = -Im W[m] (m >= 128).
//
// One 16-lane row group of a wave owns one image row (all 3 channels); lane j
// is pass-1 butterfly j, whose inputs are conj Z[j + 16 r]:
//  * lane j loads Ys[j + 16 r] and Ys[256 + j + 16 r] (16 lanes x 4 B = 64 B
//    contiguous per load); Ys[M - k] and Ys[N - k] of k = j + 16 r are the same
//    two arrays of lane 16 - j at index 15 - r: DPP row_mirror + row_ror (lane
//    0 pairs with itself one index on: it takes the previous iteration's move);
//  * pass 1 in registers -> ONE LDS transpose -> pass 2: lane j holds W[j + 16 r];
//  * output pixels 64 b + 4 j .. + 3 of block b: (Re W[b], -Im W'[15-b],
//    -Im W[b], Re W'[15-b]) with W' the mirror lane's: 16-byte stores.
#include "dctae_device.h"
#include "dctae_fft_common.h"
#include "dctae_launch.h"
#include "dctae_rows512.h"

namespace dctae {

namespace {

__device__ __forceinline__ float imirror16(float x) {   // lane l <- lane 15 - l of its 16-lane row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xf, 0xf, false));
}
__device__ __forceinline__ float iror16(float x) {      // lane l <- lane l - 1 (mod 16)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x121, 0xf, 0xf, false));
}

constexpr int kIXchStride = 528;   // the two row groups of a half-wave on opposite bank halves

struct IRows512Lds {
  float xch[4][4][kIXchStride];   // [wave][row group][re 256 | im 256 | pad]
  float2 tw2[16][16];             // W_256^{r s}
  float4 pre[256];                // (conj a_k, conj b_k)
};

}  // namespace

// BAND: U in the band layout U'[c][y / 4][kx][4] of k_idct_cols512b (element
// (y, kx) at u4_index(y / 4, kx) * 4 + y % 4); otherwise row-major
// U[c][y][kx] (k_idct_cols512)
template <int KW, bool BAND>
__global__ __launch_bounds__(256) void k_idct_rows512(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                      const float* __restrict__ ws, float* __restrict__ rgb,
                                                      const float2* __restrict__ tw, const float4* __restrict__ pre,
                                                      ColorMats cm) {
#pragma clang fp contract(fast)
  constexpr int N = 512, M = 256;
  constexpr int NB = (KW - M + 15) / 16;   // Ys[256 + j + 16 r] can be nonzero for r < NB (12 at KW = 448)
  static_assert(KW == 448, "kept width of a 512-wide image at max_patch_w >= 32");
  __shared__ IRows512Lds L;
  const int tid = threadIdx.x;
  {
    const int r = tid >> 4, s = tid & 15;
    L.tw2[r][s] = tw[r * s];
    L.pre[tid] = pre[tid];
  }
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  const int wv = tid >> 6, g = (tid >> 4) & 3, j = tid & 15;
  const int y = jb.y + 4 * wv + g;
  const int H = d.H;
  const int yl = min(y, H - 1);   // rows past H compute a duplicate and store nothing
  const int64_t cstride = (int64_t)H * KW;
  // ---- loads: A[c][r] = Ys[j + 16 r], B[c][r] = Ys[256 + j + 16 r] (r < NB)
  float A[3][16], B[3][NB];
  if constexpr (BAND) {
    // the wave's four rows are one band4 of U': lane (g, j) loads the float4
    // (rows 4 bnd .. + 3) of column kx = j + 16 (4 q + g); the 4 x 4 cross-row
    // transpose (xpose4_rows) then leaves row g's values of the columns
    // j + 16 (4 q + k), k = 0..3, in the lane (1 KB per wave load at layout 0)
    static_assert(NB % 4 == 0, "B in whole transposes");
    const int bnd = (jb.y >> 2) + wv;
    const float* ub = ws + d.ws_t;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int q = 0; q < 4 + NB / 4; ++q) {
        const int kx = j + 16 * (4 * q + g);   // q >= 4: B[4 (q - 4) + k] = Ys[M + j + 16 (4 (q - 4) + k)]
#if DCTAE_U_LD_NT
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f fv = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(ub + c * cstride + (int64_t)u4_index(bnd, kx) * 4));
        const float4 f = make_float4(fv.x, fv.y, fv.z, fv.w);
#else
        const float4 f = *reinterpret_cast<const float4*>(ub + c * cstride + (int64_t)u4_index(bnd, kx) * 4);
#endif
        float r4[4] = {f.x, f.y, f.z, f.w};
        xpose4_rows(r4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (q < 4) A[c][4 * q + k] = r4[k];
          else B[c][4 * (q - 4) + k] = r4[k];
        }
      }
    }
  } else {
    const float* src = ws + d.ws_t + (int64_t)yl * KW + j;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int r = 0; r < 16; ++r) A[c][r] = src[c * cstride + 16 * r];
#pragma unroll
      for (int r = 0; r < NB; ++r) B[c][r] = src[c * cstride + M + 16 * r];
    }
  }
  __syncthreads();   // tables

  float* xre = L.xch[wv][g];
  float* xim = L.xch[wv][g] + 256;
  const bool lane0 = (j == 0);
  float4 X[3][8];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    auto bv = [&](int t) { return t < NB ? B[c][t] : 0.0f; };
    // ---- conj Z_k, k = j + 16 r; partner arrays of lane 16 - j at index 15 - r
    float re[16], im[16];
    float pa = iror16(imirror16(A[c][15])), pb = iror16(imirror16(bv(15)));   // D_0
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // D_r: every lane runs both moves (a DPP source lane must be active);
      // lane 0 takes D_{r-1} = its own index 16 - r (r >= 1)
      const float da = iror16(imirror16(A[c][15 - r])), db = iror16(imirror16(bv(15 - r)));
      float ymk2 = lane0 ? pa : da;   // Ys[M - k]
      float ynk = lane0 ? pb : db;    // Ys[N - k]
      if (r == 0) {                   // lane 0, k = 0: Ys[M] = own B[0], Ys[N] = 0
        ymk2 = lane0 ? B[c][0] : ymk2;
        ynk = lane0 ? 0.0f : ynk;
      }
      pa = da;
      pb = db;
      float yk = A[c][r];
      if (r == 0) yk = lane0 ? yk * 1.41421356237309515f : yk;
      const float ymk = bv(r);        // Ys[M + k]
      const float4 ab = L.pre[j + 16 * r];
      // conj Z = conj(a) (yk + i ynk) + conj(b) (ymk + i ymk2)
      re[r] = ab.x * yk - ab.y * ynk + ab.z * ymk - ab.w * ymk2;
      im[r] = ab.x * ynk + ab.y * yk + ab.z * ymk2 + ab.w * ymk;
    }
    // ---- pass 1 (Ns = 1): DFT16 in registers
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
    // ---- W[j + 16 r] -> pixels 64 b + 4 j .. + 3
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const float mr = imirror16(re[15 - b]), mi = imirror16(im[15 - b]);
      X[c][b] = make_float4(re[b], -mi, -im[b], mr);
    }
  }
  // ---- IPT -> LMS -> RGB (util.py:85-97), 16-byte stores
  if (y >= H) return;
  const float inv_gamma = 2.3255813121795654296875f;   // fp32(1/0.43), util.py:93
  const int64_t hw = (int64_t)H * N;
  float* dst = rgb + d.rgb_off + (int64_t)y * N + 4 * j;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const float* i0 = reinterpret_cast<const float*>(&X[0][b]);
    const float* i1 = reinterpret_cast<const float*>(&X[1][b]);
    const float* i2 = reinterpret_cast<const float*>(&X[2][b]);
    float o[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float l0 = signed_pow_fast(mat3_row(cm.ipt2lms, 0, i0[e], i1[e], i2[e]), inv_gamma);
      const float l1 = signed_pow_fast(mat3_row(cm.ipt2lms, 1, i0[e], i1[e], i2[e]), inv_gamma);
      const float l2 = signed_pow_fast(mat3_row(cm.ipt2lms, 2, i0[e], i1[e], i2[e]), inv_gamma);
      o[0][e] = mat3_row(cm.lms2rgb, 0, l0, l1, l2);
      o[1][e] = mat3_row(cm.lms2rgb, 1, l0, l1, l2);
      o[2][e] = mat3_row(cm.lms2rgb, 2, l0, l1, l2);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#ifdef DCTAE_DEC_NT
      typedef float v4f __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store((v4f){o[c][0], o[c][1], o[c][2], o[c][3]}, reinterpret_cast<v4f*>(dst + c * hw + 64 * b));
#else
      *reinterpret_cast<float4*>(dst + c * hw + 64 * b) = make_float4(o[c][0], o[c][1], o[c][2], o[c][3]);
#endif
    }
  }
}

void launch_idct_rows512(bool band, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* ws, float* rgb,
                         const float2* tw, const float4* pre, const ColorMats& cm, hipStream_t s) {
  if (n_blocks <= 0) return;
  if (band)
    hipLaunchKernelGGL((k_idct_rows512<448, true>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, rgb, tw, pre, cm);
  else
    hipLaunchKernelGGL((k_idct_rows512<448, false>), dim3(n_blocks), dim3(256), 0, s, imgs, blocks, ws, rgb, tw, pre,
                       cm);
}

}  // namespace dctae
