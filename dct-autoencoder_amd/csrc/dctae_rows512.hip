// k_rows512pk: the row pass of 512-wide images as its own launch (the
// two-kernel encode; the item body and its design notes: dctae_rows512.h).
#include "dctae_launch.h"
#include "dctae_rows512.h"

namespace dctae {

// blocks[i] = (image, first row of a 16-row item)
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
  // the two store layouts as separate bodies (one runtime branch inside the
  // channel loop costs ~80 VGPRs: 2 waves / SIMD instead of 3)
  if (d.tband)
    rows512_item_pk<true>(x, t, rgb + d.rgb_off, d.H, jb.y, ws + d.ws_t, (uint32_t)(d.H * 448 * 4), cm);
  else
    rows512_item_pk<false>(x, t, rgb + d.rgb_off, d.H, jb.y, ws + d.ws_t, (uint32_t)(d.H * 448 * 4), cm);
}

void launch_rows512(const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                    const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s) {
  if (n_blocks <= 0) return;
  hipLaunchKernelGGL(k_rows512pk, dim3(n_blocks), dim3(256), 0, s, imgs, blocks, rgb, ws, tw, post, cm);
}

}  // namespace dctae
