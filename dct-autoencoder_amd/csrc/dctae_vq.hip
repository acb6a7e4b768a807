// VectorQuantize inference (reference dct_autoencoder/vector_quantize.py)
// as the model builds it (modeling_dct_autoencoder.py:76-77): euclidean codebook
// shared by all heads, codebook_dim 16, affine parameters, eval mode.
//
//   xp = x W_in^T + b_in                                  (MFMA GEMM, k_gemm_f32)
//   batch mean / biased variance of the valid vectors      (k_vq_stats1/2, fp64 sums)
//   EMA of the batch statistics, transformed codebook     (k_vq_codebook)
//       e' = (e - cm) * (sqrt(max(bv,1e-5)) / sqrt(max(cv,1e-5))) + bm,  y2 = |e'|^2
//   per vector: argmax_j -sqrt((|x|^2 + y2_j) + (-2 x.e'_j)),  first index on ties,
//   NaN (negative radicand) first                          (k_vq_assign, codebook in LDS)
//   quantize = e'[j] -> (b n (h d)), out = q W_out^T + b_out, where(mask, out, x)
#include "dctae_device.h"
#include "dctae_launch.h"

namespace dctae {

namespace {
constexpr int VD = 16;   // codebook_dim of the model configuration
}

// bias add over rows (+ optional mask select against the original input)
__global__ void k_vq_bias(float* __restrict__ y, const float* __restrict__ bias, int64_t n, int cols,
                          const uint8_t* __restrict__ mask, const float* __restrict__ orig) {
  const int64_t total = n * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / cols;
    const int c = (int)(e - t * cols);
    float v = y[e];
    if (bias) v = __fadd_rn(v, bias[c]);
    if (mask && !mask[t]) v = orig[e];          // vector_quantize.py:1044-1048
    y[e] = v;
  }
}

// pass 1: sum over valid vectors (tok, h) of xp[tok][16 h + d]; acc[16] = count
__global__ __launch_bounds__(256) void k_vq_stats1(const float* __restrict__ xp, const uint8_t* __restrict__ mask,
                                                   int64_t n_tok, int heads, double* __restrict__ acc) {
  __shared__ double part[256 / VD][VD + 1];
  const int d = threadIdx.x & (VD - 1), r = threadIdx.x >> 4;   // 16 vectors per block step
  double s = 0.0, cnt = 0.0;
  const int64_t nv = n_tok * heads;
  for (int64_t v = (int64_t)blockIdx.x * (256 / VD) + r; v < nv; v += (int64_t)gridDim.x * (256 / VD)) {
    const int64_t t = v / heads;
    if (mask && !mask[t]) continue;
    s += (double)xp[v * VD + d];
    cnt += 1.0;
  }
  part[r][d] = s;
  if (d == 0) part[r][VD] = cnt;
  __syncthreads();
  if (threadIdx.x <= VD) {
    double a = 0.0;
    for (int i = 0; i < 256 / VD; ++i) a += part[i][threadIdx.x];
    atomicAdd(acc + threadIdx.x, a);
  }
}

// pass 2: sum of squared deviations from the batch mean (two-pass variance)
__global__ __launch_bounds__(256) void k_vq_stats2(const float* __restrict__ xp, const uint8_t* __restrict__ mask,
                                                   int64_t n_tok, int heads, double* __restrict__ acc) {
  __shared__ double part[256 / VD][VD];
  const int d = threadIdx.x & (VD - 1), r = threadIdx.x >> 4;
  const double mean = acc[d] / acc[VD];
  double s = 0.0;
  const int64_t nv = n_tok * heads;
  for (int64_t v = (int64_t)blockIdx.x * (256 / VD) + r; v < nv; v += (int64_t)gridDim.x * (256 / VD)) {
    const int64_t t = v / heads;
    if (mask && !mask[t]) continue;
    const double x = (double)xp[v * VD + d] - mean;
    s += x * x;
  }
  part[r][d] = s;
  __syncthreads();
  if (threadIdx.x < VD) {
    double a = 0.0;
    for (int i = 0; i < 256 / VD; ++i) a += part[i][threadIdx.x];
    atomicAdd(acc + VD + 1 + threadIdx.x, a);
  }
}

// EMA update of the batch statistics (vector_quantize.py:330-343, 353-359) and
// the transformed codebook e' + |e'|^2 (vector_quantize.py:456-460)
__global__ __launch_bounds__(256) void k_vq_codebook(const double* __restrict__ acc, float* __restrict__ bm,
                                                     float* __restrict__ bv, int32_t* __restrict__ init,
                                                     float decay, int affine, const float* __restrict__ embed,
                                                     const float* __restrict__ cm, const float* __restrict__ cv,
                                                     int C, float* __restrict__ et, float* __restrict__ y2) {
  __shared__ float sm[VD], sr[VD];
  if (threadIdx.x < VD) {
    const int d = threadIdx.x;
    float mean = 0.0f, var = 0.0f;
    if (affine) {
      const double n = acc[VD];
      mean = n > 0 ? (float)(acc[d] / n) : __int_as_float(0x7fc00000);       // empty batch: torch.mean -> NaN
      var = n > 0 ? (float)(acc[VD + 1 + d] / n) : __int_as_float(0x7fc00000);
    }
    // every block computes the same values; block 0 publishes the new state
    float m2, v2;
    if (!affine) {
      m2 = 0.0f;
      v2 = 1.0f;
    } else if (*init == 0) {
      m2 = mean;
      v2 = var;
    } else {
      m2 = __fadd_rn(__fmul_rn(bm[d], decay), __fmul_rn(mean, __fsub_rn(1.0f, decay)));
      v2 = __fadd_rn(__fmul_rn(bv[d], decay), __fmul_rn(var, __fsub_rn(1.0f, decay)));
    }
    sm[d] = m2;
    // ratio batch_std / codebook_std
    sr[d] = affine ? __fdiv_rn(__fsqrt_rn(fmaxf(v2, 1e-5f)), __fsqrt_rn(fmaxf(cv[d], 1e-5f))) : 1.0f;
  }
  __syncthreads();
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < C; j += gridDim.x * blockDim.x) {
    float s = 0.0f;
    float e[VD];
#pragma unroll
    for (int d = 0; d < VD; ++d) {
      const float x = embed[(int64_t)j * VD + d];
      e[d] = affine ? __fadd_rn(__fmul_rn(__fsub_rn(x, cm[d]), sr[d]), sm[d]) : x;
      et[(int64_t)j * VD + d] = e[d];
    }
#pragma unroll
    for (int d = 0; d < VD; ++d) s = __fadd_rn(s, __fmul_rn(e[d], e[d]));
    y2[j] = s;
  }
}

// publishes the EMA'd statistics (one block, after k_vq_codebook consumed the old ones)
__global__ void k_vq_publish(const double* __restrict__ acc, float* __restrict__ bm, float* __restrict__ bv,
                             int32_t* __restrict__ init, float decay) {
  const int d = threadIdx.x;
  if (d >= VD) return;
  const double n = acc[VD];
  const float mean = n > 0 ? (float)(acc[d] / n) : __int_as_float(0x7fc00000);
  const float var = n > 0 ? (float)(acc[VD + 1 + d] / n) : __int_as_float(0x7fc00000);
  if (*init == 0) {
    bm[d] = mean;
    bv[d] = var;
  } else {
    bm[d] = __fadd_rn(__fmul_rn(bm[d], decay), __fmul_rn(mean, __fsub_rn(1.0f, decay)));
    bv[d] = __fadd_rn(__fmul_rn(bv[d], decay), __fmul_rn(var, __fsub_rn(1.0f, decay)));
  }
  __syncthreads();
  if (d == 0) *init = 1;
}

// nearest code per vector (tok, h): thread = vector; the transformed codebook
// streamed through LDS in chunks (all lanes read the same code: broadcast)
constexpr int kVqChunk = 512;
__global__ __launch_bounds__(256) void k_vq_assign(const float* __restrict__ xp, int64_t nv, int heads,
                                                   const float* __restrict__ et, const float* __restrict__ y2, int C,
                                                   float* __restrict__ xq, int64_t* __restrict__ ind) {
  __shared__ float4 es[kVqChunk][VD / 4];
  __shared__ float ys[kVqChunk];
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = v < nv;
  float x[VD];
  float x2 = 0.0f;
#pragma unroll
  for (int d = 0; d < VD; ++d) x[d] = live ? xp[v * VD + d] : 0.0f;
#pragma unroll
  for (int d = 0; d < VD; ++d) x2 = __fadd_rn(x2, __fmul_rn(x[d], x[d]));
  float dbest = __int_as_float(0x7f800000), sbest = dbest;
  int jbest = 0;
  bool nan_best = false;
  for (int j0 = 0; j0 < C; j0 += kVqChunk) {
    const int nc = min(kVqChunk, C - j0);
    __syncthreads();
    for (int i = threadIdx.x; i < nc * (VD / 4); i += blockDim.x)
      es[i / (VD / 4)][i % (VD / 4)] = reinterpret_cast<const float4*>(et + (int64_t)j0 * VD)[i];
    for (int i = threadIdx.x; i < nc; i += blockDim.x) ys[i] = y2[j0 + i];
    __syncthreads();
    for (int jj = 0; jj < nc; ++jj) {
      float dot = 0.0f;
#pragma unroll
      for (int q = 0; q < VD / 4; ++q) {
        const float4 e = es[jj][q];
        dot = fmaf(x[4 * q], e.x, dot);
        dot = fmaf(x[4 * q + 1], e.y, dot);
        dot = fmaf(x[4 * q + 2], e.z, dot);
        dot = fmaf(x[4 * q + 3], e.w, dot);
      }
      // (x2 + y2) + (-2 x.e), vector_quantize.py:29-33
      const float dd = __fadd_rn(__fadd_rn(x2, ys[jj]), __fmul_rn(dot, -2.0f));
      if (nan_best) continue;
      if (dd < 0.0f) {           // sqrt -> NaN: argmax picks the first NaN
        nan_best = true;
        jbest = j0 + jj;
        continue;
      }
      if (dd <= dbest) {         // sqrt is monotone: only then can sqrt(dd) beat sqrt(dbest)
        const float s = __fsqrt_rn(dd);
        if (s < sbest) {
          sbest = s;
          dbest = dd;
          jbest = j0 + jj;
        }
      }
    }
  }
  if (!live) return;
  ind[v] = jbest;
#pragma unroll
  for (int d = 0; d < VD; ++d) xq[v * VD + d] = et[(int64_t)jbest * VD + d];
}

// get_codes_from_indices (vector_quantize.py:820-841): raw codebook rows
__global__ void k_vq_codes(const int64_t* __restrict__ ind, int64_t nv, const float* __restrict__ embed, int C,
                           float* __restrict__ out, int* err) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nv * VD; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = e / VD;
    const int d = (int)(e - v * VD);
    const int64_t j = ind[v];
    if (j < 0 || j >= C) {
      atomicOr(err, 16);   // dctae_check_device_errors: IndexError
      out[e] = __int_as_float(0x7fc00000);
      continue;
    }
    out[e] = embed[j * VD + d];
  }
}

void launch_vq_bias(float* y, const float* bias, int64_t n, int cols, const uint8_t* mask, const float* orig,
                    hipStream_t s) {
  const int gx = (int)std::min<int64_t>((n * cols + 255) / 256, 8192);
  if (gx > 0) hipLaunchKernelGGL(k_vq_bias, dim3(gx), dim3(256), 0, s, y, bias, n, cols, mask, orig);
}

void launch_vq_stats(const float* xp, const uint8_t* mask, int64_t n_tok, int heads, double* acc, hipStream_t s) {
  const int64_t nv = n_tok * heads;
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((nv + 15) / 16, 2048));
  hipLaunchKernelGGL(k_vq_stats1, dim3(gx), dim3(256), 0, s, xp, mask, n_tok, heads, acc);
  hipLaunchKernelGGL(k_vq_stats2, dim3(gx), dim3(256), 0, s, xp, mask, n_tok, heads, acc);
}

void launch_vq_codebook(const double* acc, float* bm, float* bv, int32_t* init, float decay, int affine,
                        const float* embed, const float* cm, const float* cv, int C, float* et, float* y2,
                        hipStream_t s) {
  const int gx = std::max(1, std::min((C + 255) / 256, 256));
  hipLaunchKernelGGL(k_vq_codebook, dim3(gx), dim3(256), 0, s, acc, bm, bv, init, decay, affine, embed, cm, cv, C,
                     et, y2);
  if (affine) hipLaunchKernelGGL(k_vq_publish, dim3(1), dim3(64), 0, s, acc, bm, bv, init, decay);
}

void launch_vq_assign(const float* xp, int64_t nv, int heads, const float* et, const float* y2, int C, float* xq,
                      int64_t* ind, hipStream_t s) {
  const int64_t gx = (nv + 255) / 256;
  if (gx > 0) hipLaunchKernelGGL(k_vq_assign, dim3((unsigned)gx), dim3(256), 0, s, xp, nv, heads, et, y2, C, xq, ind);
}

void launch_vq_codes(const int64_t* ind, int64_t nv, const float* embed, int C, float* out, int* err, hipStream_t s) {
  const int gx = (int)std::min<int64_t>((nv * VD + 255) / 256, 8192);
  if (gx > 0) hipLaunchKernelGGL(k_vq_codes, dim3(gx), dim3(256), 0, s, ind, nv, embed, C, out, err);
}

}  // namespace dctae
