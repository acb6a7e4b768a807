// Probe: is the 512-point column FFT's DFT16 pass cheaper on the (idle) MFMA
// pipe than on the VALU?  (offload part of k_cols512b's
// transform to MFMA.)  Three kernels do the same work -- 64 complex 16-point
// DFTs per wave per iteration, the amount one fft256_group pass does for the
// wave's 4 columns -- and report SIMD cycles per DFT16:
//   valu : DFTV<16> on packed fp32 in registers (the shipped code path);
//   f32  : the DFT16 matrix (complex 16 x 16 = real 32 x 32) times the 64
//          vectors (32 x 64 real) on v_mfma_f32_32x32x2_f32 (fp32 exact);
//   bf16 : the same product on v_mfma_f32_32x32x16_bf16 with both operands
//          split into three bf16 pieces and six products (the fp32-level
//          scheme of dctae_gemm_x3.hip), the data split on the VALU per pass.
// The MFMA arms leave out the operand re-layout a real pass would need (the
// FFT holds one butterfly's 16 values per lane; MFMA operands hold one element
// of 64 different vectors per lane): a lower bound on their cost.
//   hipcc -O3 --offload-arch=gfx950 -I dct-autoencoder_amd/csrc tools/probe/dft16_mfma.hip -o tools/probe/dft16_mfma
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "dctae_fft_common.h"

using namespace dctae;

typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

constexpr int kWaves = 8;   // per block (2 per SIMD)

__global__ __launch_bounds__(64 * kWaves) void k_valu(float* out, int iters) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  cf v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = (cf){0.001f * (t & 127) + r, 0.002f * r};
  for (int it = 0; it < iters; ++it) {
    DFTV<16>::run(v);   // 64 DFT16 per wave (one per lane)
    __builtin_amdgcn_sched_barrier(0);
  }
  cf acc = v[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) acc += v[r];
  out[t] = acc.x + acc.y;
}

__global__ __launch_bounds__(64 * kWaves) void k_f32(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  // A = F (32 x 32 real): per k step (K = 2) one value per lane: A[lane % 32][2 ks + lane / 32]
  float a[16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) a[ks] = 0.01f * ((lane * 7 + ks) & 31);
  // B = 64 vectors (32 x 64 real, two 32-column tiles): B[2 ks + lane / 32][n0 + lane % 32]
  float b[2][16];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) b[nt][ks] = 0.001f * ((lane + ks + nt) & 63);
  f16v c0 = {}, c1 = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks], b[0][ks], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks], b[1][ks], c1, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  out[threadIdx.x + blockIdx.x * blockDim.x] = s;
}

__device__ __forceinline__ void split3(const float (&x)[8], bf8v& h0, bf8v& h1, bf8v& h2) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 p0 = (__bf16)x[e];
    const float r1 = x[e] - (float)p0;
    const __bf16 p1 = (__bf16)r1;
    const float r2 = r1 - (float)p1;
    h0[e] = p0;
    h1[e] = p1;
    h2[e] = (__bf16)r2;
  }
}

__global__ __launch_bounds__(64 * kWaves) void k_bf16x6(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  // A = F pre-split (constant): per k step (K = 16) 8 bf16 per lane and piece
  bf8v a[2][3];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = 0.01f * ((lane * 7 + ks * 8 + e) & 31) + 1e-4f * e;
    split3(x, a[ks][0], a[ks][1], a[ks][2]);
  }
  // B = data, fp32 (8 per lane per k step and tile), split every pass
  float b[2][2][8];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) b[nt][ks][e] = 0.001f * ((lane + ks + nt + e) & 63) + 1e-5f * e;
  f16v c0 = {}, c1 = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf8v p[2][3];
      split3(b[0][ks], p[0][0], p[0][1], p[0][2]);
      split3(b[1][ks], p[1][0], p[1][1], p[1][2]);
      // the six products with piece orders summing to <= 2
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        f16v& c = nt ? c1 : c0;
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], p[nt][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], p[nt][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1], p[nt][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1], p[nt][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], p[nt][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][2], p[nt][0], c, 0, 0, 0);
      }
    }
    // the next pass's data: fold the accumulators back (keeps the split live)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b[0][0][e] += 1e-7f * c0[e];
      b[1][1][e] += 1e-7f * c1[e + 8];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  out[threadIdx.x + blockIdx.x * blockDim.x] = s;
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

int main() {
  int dev = 0, cus = 0, clk_khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
  const int blocks = cus * 2;   // 16 waves per CU = 4 per SIMD
  const int threads = 64 * kWaves;
  float* out;
  CK(hipMalloc(&out, sizeof(float) * blocks * threads));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 2000;
  const double waves = (double)blocks * kWaves;
  const double dft16 = waves * 64.0 * iters;   // 64 DFT16 per wave per iteration
  const double simd_cycles = (double)cus * 4 * (clk_khz * 1e3);   // per second
  printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"iters\": %d, \"waves\": %.0f", cus, clk_khz / 1e3, iters, waves);
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {   // first run warms up
      CK(hipEventRecord(e0));
      if (k == 0) hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(threads), 0, 0, out, iters);
      if (k == 1) hipLaunchKernelGGL(k_f32, dim3(blocks), dim3(threads), 0, 0, out, iters);
      if (k == 2) hipLaunchKernelGGL(k_bf16x6, dim3(blocks), dim3(threads), 0, 0, out, iters);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const char* nm = k == 0 ? "valu_dftv16" : (k == 1 ? "mfma_f32_32x32x2" : "mfma_bf16x6_32x32x16");
    printf(", \"%s\": {\"ms\": %.3f, \"simd_cycles_per_dft16\": %.3f, \"gdft16_per_s\": %.1f}", nm, ms,
           simd_cycles * ms / 1e3 / dft16, dft16 / (ms / 1e3) / 1e9);
  }
  printf("}\n");
  return 0;
}
