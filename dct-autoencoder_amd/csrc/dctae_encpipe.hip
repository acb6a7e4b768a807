// k_enc_pipe: the 512^2 encode as a software pipeline over image chunks, one
// launch per step.  Launch L runs the row items of chunk L beside the column
// items of chunk L - 1 (SURVEY §7 hard part 2; reference util.py:333-334:
// dct_2d = the row DCT, then the column DCT of its result).
//
// Why: the two-kernel encode writes T (2.75 MB per image) to HBM and reads it
// back (58 % of the encode's traffic), and each kernel alone leaves half of
// the machine idle -- the row pass is HBM-bound (RGB in, T out), the column
// pass VALU / LDS-bound.  Here T lives in a ring of two chunk slots (2 x C
// images, C x 5.5 MB) small enough for the 256 MB Infinity Cache, so the
// columns of chunk L - 1 read T written one launch earlier (the launch
// boundary is the only ordering: no flags, no spin waits), and the two kinds
// of work share every CU.
//
// Block b of a launch: unit u = b / 8, XCD lane x = b % 8 (the dispatcher
// deals consecutive blocks to the 8 XCDs).  Units are row units (8 row items)
// or column units (8 column blocks), spread evenly over the launch
// (Bresenham), so the XCD lane of a column block is its position in the
// cols7 grid mod 8 -- the (image, channel) items of one XCD read neighbouring
// T strips through that XCD's L2, exactly as k_fft_cols7 lays them out.
//   row item rb (of chunk L): image L C + rb / 32, rows 16 (rb % 32) .. + 15
//     (rows512_item_pk / rows512_item, dctae_rows512.h);
//   column block cb (of chunk L - 1): the k_fft_cols7<thr, IPB = 2> block
//     (dctae_spec512.h): item t = x 12 + (cb / 8) % 12 = (channel, tile
//     column), images 2 g, 2 g + 1 of the chunk, g = (cb / 8) / 12.
// Codes only, on the exact LFQ thresholds (the cols7 THR epilogue); the sort /
// pack runs after the last launch as in the two-kernel path.
#include "dctae_launch.h"
#include "dctae_rows512.h"
#include "dctae_spec512.h"

namespace dctae {

namespace {

constexpr int kKW = 448, kH = 512;
constexpr int64_t kTFloats = 3ll * kH * kKW;   // one image's T
constexpr int kPerX = 12;                      // cols7 items per XCD lane: 96 / 8

struct PipeRows {
  Rows512XchPk xpk;
  Rows512Tab t;
};
struct PipeRowsScalar {
  Rows512Xch x;
  Rows512Tab t;
};
struct PipeCols {
  Cols7Lds L;
  float4 post4[257];
  float2 tw_s[256];
  float sbias[32];
};
union PipeLds {
  PipeRows r;
  PipeRowsScalar rs;
  PipeCols c;
};

}  // namespace

template <bool PK>
__global__ __launch_bounds__(256) void k_enc_pipe(const ImgDesc* __restrict__ imgs, int n_img, int C, int L,
                                                  const float* __restrict__ rgb, float* __restrict__ tring,
                                                  const float2* __restrict__ tw, const float2* __restrict__ post,
                                                  ColorMats cm, EncParams ep, TokenSinks sk, int ru, int cu) {
  __shared__ PipeLds U;
  const int unit = blockIdx.x >> 3, x = blockIdx.x & 7;
  const int64_t tot = ru + cu;
  const int rbefore = (int)(((int64_t)unit * ru) / tot);
  const bool is_row = (int)(((int64_t)(unit + 1) * ru) / tot) > rbefore;
  if (is_row) {
    const int rb = rbefore * 8 + x;
    const int li = rb >> 5, i = L * C + li;
    if (i >= n_img) return;   // never: ru = 4 x (images of chunk L)
    const ImgDesc d = imgs[i];
    float* T = tring + (int64_t)((L & 1) * C + li) * kTFloats;
    if (PK) {
      rows512_tables(U.r.t, tw, post);
      __syncthreads();
      rows512_item_pk(U.r.xpk, U.r.t, rgb + d.rgb_off, kH, (rb & 31) * 16, T, (uint32_t)(kH * kKW * 4), cm);
    } else {
      rows512_tables(U.rs.t, tw, post);
      __syncthreads();
      rows512_item<0>(U.rs.x, U.rs.t, rgb + d.rgb_off, kH, (rb & 31) * 16, T, (uint32_t)(kH * kKW * 4), cm);
    }
    return;
  }
  // column block of chunk L - 1
  constexpr int M = 256;
  const int cb = (unit - rbefore) * 8 + x;
  const int slot = cb >> 3;
  const int t = x * kPerX + slot % kPerX, g = slot / kPerX;
  const int base = (L - 1) * C;
  const int nl = min(C, n_img - base);
  const int k0 = 2 * g;
  if (k0 >= nl) return;
  const int c = t >> 5, strip = t & 31;
  PipeCols& P = U.c;
  const float4* p4 = reinterpret_cast<const float4*>(post);
  for (int e = threadIdx.x; e < M + 1; e += 256) P.post4[e] = p4[e];
  for (int e = threadIdx.x; e < M; e += 256) P.tw_s[e] = tw[e];
  const float* Tb = tring + (int64_t)(((L - 1) & 1) * C) * kTFloats;
  float2 thr_r[2][7];
  cols_thresholds<true>(imgs[base + k0], c, strip, ep, thr_r, P.sbias);
  float va[16], vb[16];
  cols7_load(imgs[base + k0], c, strip, Tb + (int64_t)k0 * kTFloats, va, vb);
  __syncthreads();   // tables
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = k0 + u;
    if (k < nl) {
      const ImgDesc dk = imgs[base + k];
      float na[16], nb[16];
      if (u == 0 && k + 1 < nl)
        cols7_load(imgs[base + k + 1], c, strip, Tb + (int64_t)(k + 1) * kTFloats, na, nb);   // in flight
      cols7_compute<true>(dk, c, strip, P.L, va, vb, P.post4, P.tw_s, P.sbias, thr_r, ep, sk);
      __syncthreads();
      if (u == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          va[r] = na[r];
          vb[r] = nb[r];
        }
      }
    }
  }
}

size_t enc_pipe_ring_bytes(int C) { return (size_t)2 * C * kTFloats * sizeof(float); }

// imgs: n_img 512 x 512 images with qh = qw = 32 in one staging (tok_off);
// tring: enc_pipe_ring_bytes(C); ep must carry the exact LFQ thresholds.
void launch_enc_pipe(const ImgDesc* imgs, int n_img, int C, const float* rgb, float* tring, const float2* tw,
                     const float2* post, const ColorMats& cm, const EncParams& ep, const TokenSinks& sk, bool packed,
                     hipStream_t s) {
  if (n_img <= 0 || C <= 0) return;
  const int nch = (n_img + C - 1) / C;
  for (int L = 0; L <= nch; ++L) {
    const int n_rows = L < nch ? std::min(C, n_img - L * C) : 0;
    const int n_cols = L >= 1 ? std::min(C, n_img - (L - 1) * C) : 0;
    const int ru = 4 * n_rows, cu = kPerX * ((n_cols + 1) / 2);
    const int grid = 8 * (ru + cu);
    if (packed)
      hipLaunchKernelGGL(k_enc_pipe<true>, dim3(grid), dim3(256), 0, s, imgs, n_img, C, L, rgb, tring, tw, post, cm,
                         ep, sk, ru, cu);
    else
      hipLaunchKernelGGL(k_enc_pipe<false>, dim3(grid), dim3(256), 0, s, imgs, n_img, C, L, rgb, tring, tw, post, cm,
                         ep, sk, ru, cu);
  }
}

}  // namespace dctae
