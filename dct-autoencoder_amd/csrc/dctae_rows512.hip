// k_rows512: the row pass of 512-wide images as its own launch (the
// two-kernel encode; the item body and its design notes: dctae_rows512.h).
#include "dctae_launch.h"
#include "dctae_rows512.h"

namespace dctae {

namespace {

struct Rows512Lds {
  Rows512Xch x;
  Rows512Tab t;
};

}  // namespace

// blocks[i] = (image, first row); ablate (profiling builds only, else 0):
// bit 0 drops every T store, bit 1 replaces the RGB loads
template <int KW>
#ifndef DCTAE_ROWS_MINB
#define DCTAE_ROWS_MINB 1
#endif
__global__ __launch_bounds__(256, DCTAE_ROWS_MINB) void k_rows512(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                const float* __restrict__ rgb, float* __restrict__ ws,
                                                const float2* __restrict__ tw, const float2* __restrict__ post,
                                                ColorMats cm, int ablate) {
  static_assert(KW == 448, "kept width of a 512-wide image at max_patch_w >= 32");
  __shared__ Rows512Lds L;
  rows512_tables(L.t, tw, post);
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  __syncthreads();   // tables
  const uint32_t plane_bytes = (ablate & 1) ? 0u : (uint32_t)(d.H * KW * 4);
#ifdef DCTAE_PROFILING
  if (ablate & 2) {
    rows512_item<2>(L.x, L.t, rgb + d.rgb_off, d.H, jb.y, ws + d.ws_t, plane_bytes, cm);
    return;
  }
#endif
  rows512_item<0>(L.x, L.t, rgb + d.rgb_off, d.H, jb.y, ws + d.ws_t, plane_bytes, cm);
}

// rows_kernel 4: the packed-f32 item (dctae_rows512.h rows512_item_pk)
#ifdef DCTAE_PK_WPE   // experiment switch (waves per SIMD); default: the compiler's choice (3)
#define DCTAE_PK_ATTR __attribute__((amdgpu_waves_per_eu(DCTAE_PK_WPE)))
#else
#define DCTAE_PK_ATTR
#endif
__global__ __launch_bounds__(256) DCTAE_PK_ATTR void k_rows512pk(const ImgDesc* __restrict__ imgs, const int2* __restrict__ blocks,
                                                   const float* __restrict__ rgb, float* __restrict__ ws,
                                                   const float2* __restrict__ tw, const float2* __restrict__ post,
                                                   ColorMats cm) {
  __shared__ Rows512XchPk x;
  __shared__ Rows512Tab t;
  rows512_tables(t, tw, post);
  const int2 jb = blocks[blockIdx.x];
  const ImgDesc d = imgs[jb.x];
  __syncthreads();   // tables
  rows512_item_pk(x, t, rgb + d.rgb_off, d.H, jb.y, ws + d.ws_t, (uint32_t)(d.H * 448 * 4), cm);
}

// rows_p1: the row pass + the column FFT's pass 1 (dctae_rows512.h
// rows512_p1_item); blocks[i] = (image, j1), 512 threads
__global__ __launch_bounds__(512) void k_rows512p1(const ImgDesc* __restrict__ imgs, int n_img,
                                                   const float* __restrict__ rgb, float* __restrict__ ws,
                                                   const float2* __restrict__ tw, const float2* __restrict__ post,
                                                   ColorMats cm) {
  __shared__ Rows512P1Lds L;
  rows512_p1_tables(L.t, tw, post);
  const int i = blockIdx.x >> 4, j1 = blockIdx.x & 15;
  if (i >= n_img) return;   // never: grid = 16 x n_img
  const ImgDesc d = imgs[i];
  __syncthreads();   // tables
  rows512_p1_item(L, rgb + d.rgb_off, j1, reinterpret_cast<float2*>(ws + d.ws_t), cm);
}

void launch_rows512p1(const ImgDesc* imgs, int n_img, const float* rgb, float* ws, const float2* tw,
                      const float2* post, const ColorMats& cm, hipStream_t s) {
  if (n_img <= 0) return;
  hipLaunchKernelGGL(k_rows512p1, dim3(16 * n_img), dim3(512), 0, s, imgs, n_img, rgb, ws, tw, post, cm);
}

void launch_rows512(const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                    const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s, int ablate, bool packed) {
  if (n_blocks <= 0) return;
  if (packed && !ablate)
    hipLaunchKernelGGL(k_rows512pk, dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
  else
    hipLaunchKernelGGL(k_rows512<448>, dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm, ablate);
}

}  // namespace dctae
