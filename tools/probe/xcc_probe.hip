// Probe: which XCC / CU each workgroup of a 768 x 256 grid lands on
// (HW_REG_XCC_ID, HW_REG_HW_ID).  hipcc --offload-arch=gfx950 -o xcc_probe xcc_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void k_probe(unsigned* out) {
  __shared__ float pad[11000];   // ~44 KB of LDS, like the persistent encode
  unsigned xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  pad[threadIdx.x] = (float)xcc;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hwid + (unsigned)pad[5] * 0u;
  }
}

int main() {
  const int n = 768;
  unsigned* d;
  hipMalloc(&d, 2 * n * sizeof(unsigned));
  hipLaunchKernelGGL(k_probe, dim3(n), dim3(256), 0, 0, d);
  std::vector<unsigned> h(2 * n);
  hipMemcpy(h.data(), d, 2 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
  std::map<unsigned, int> byxcc, byx7;
  std::map<std::pair<unsigned, unsigned>, int> cu;
  for (int i = 0; i < n; ++i) {
    byxcc[h[2 * i]]++;
    byx7[h[2 * i] & 7]++;
    const unsigned hw = h[2 * i + 1];
    const unsigned cu_id = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cu[{h[2 * i], (se << 8) | (sh << 4) | cu_id}]++;
  }
  printf("raw XCC_ID values:");
  for (auto& kv : byxcc) printf(" %u:%d", kv.first, kv.second);
  printf("\nXCC_ID & 7:");
  for (auto& kv : byx7) printf(" %u:%d", kv.first, kv.second);
  printf("\ndistinct (xcc, se/sh/cu) slots: %zu\n", cu.size());
  printf("first 24 blocks xcc:");
  for (int i = 0; i < 24; ++i) printf(" %u", h[2 * i]);
  printf("\n");
  return 0;
}
