// PatchNorm training-mode statistics (reference patchnorm.py:101-155) on gfx950.
//
// One training step of the reference, for a packed batch of tokens:
//   batch_n[c,h,w]        = #non-pad tokens in cell (c,h,w)            (scatter_add_3d, :112-119)
//   batch_median[cell,:]  = torch.median(tokens of the cell, 0)        (lower median, :121-130)
//   median <- (median*n + batch_median*batch_n) / clamp(n+batch_n, 1)  (:135-138)
//   batch_b[cell,:]       = sum_{tokens in order} |x - median| / clamp(batch_n, 1)   (:140-144)
//   b      <- (b*n + batch_b*batch_n) / clamp(n+batch_n, 1)           (:146-148)
//   n      <- n + batch_n                                              (:150)
// Bit-exact with the reference's fp32 CPU ops: the per-cell token lists keep
// batch order (the scatter_add_ accumulation order) and every op is rounded
// separately (-ffp-contract=off, __f*_rn).
#include "dctae_device.h"
#include "dctae_launch.h"

namespace dctae {

// cell id of every token (-1 for padding / out of range) and per-cell counts
__global__ void k_stats_cells(const int64_t* __restrict__ ch, const int64_t* __restrict__ pos,
                              const uint8_t* __restrict__ key_pad, int64_t n_tok, int C, int mh, int mw,
                              int32_t* __restrict__ cell, int32_t* __restrict__ count, int* __restrict__ err) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tok; t += (int64_t)gridDim.x * blockDim.x) {
    int32_t id = -1;
    if (!key_pad || !key_pad[t]) {
      const int64_t c = ch[t], h = pos[2 * t], w = pos[2 * t + 1];
      if (c < 0 || c >= C || h < 0 || h >= mh || w < 0 || w >= mw) {
        atomicOr(err, 1);
      } else {
        id = (int32_t)((c * mh + h) * mw + w);
        atomicAdd(&count[id], 1);
      }
    }
    cell[t] = id;
  }
}

// exclusive scan of the cell counts (single block)
__global__ void k_stats_scan(const int32_t* __restrict__ count, int n_cells, int32_t* __restrict__ start) {
  __shared__ int32_t part[1024];
  const int tid = threadIdx.x;
  const int per = (n_cells + 1023) / 1024;
  int32_t s = 0;
  for (int i = 0; i < per; ++i) {
    const int c = tid * per + i;
    if (c < n_cells) s += count[c];
  }
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int32_t v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int32_t run = part[tid] - s;
  for (int i = 0; i < per; ++i) {
    const int c = tid * per + i;
    if (c < n_cells) {
      start[c] = run;
      run += count[c];
    }
  }
}

// stable per-cell token lists: one wave per cell scans the tokens in batch
// order with a ballot, so list order == batch order (the reference's
// scatter_add_ accumulation order)
__global__ __launch_bounds__(256) void k_stats_lists(const int32_t* __restrict__ cell, int64_t n_tok, int n_cells,
                                                     const int32_t* __restrict__ start,
                                                     const int32_t* __restrict__ count, int32_t* __restrict__ list) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= n_cells) return;
  if (count[wave] == 0) return;
  int32_t out = start[wave];
  for (int64_t base = 0; base < n_tok; base += 64) {
    const int64_t t = base + lane;
    const bool hit = t < n_tok && cell[t] == wave;
    const uint64_t m = __ballot(hit);
    if (hit) list[out + __popcll(m & ((1ull << lane) - 1))] = (int32_t)t;
    out += __popcll(m);
  }
}

// per (cell, element): lower median of the cell's values (torch.median:
// sorted position (cnt-1)/2; NaN if the column holds a NaN) and batch_n; zero
// for empty cells.  One block per cell: the cell's values are staged in LDS
// in element chunks and every (element, candidate) pair computes its rank
// #(v_j < v_i) + #(j < i, v_j == v_i) — ranks are unique, so exactly one
// candidate per element writes.
constexpr int kMedianLds = 12288;  // floats of LDS staging (48 KiB)

__global__ __launch_bounds__(256) void k_stats_median(const float* __restrict__ x, int PP,
                                                      const int32_t* __restrict__ start,
                                                      const int32_t* __restrict__ count,
                                                      const int32_t* __restrict__ list,
                                                      float* __restrict__ batch_median, float* __restrict__ batch_n) {
  __shared__ float sv[kMedianLds];
  __shared__ int nanf[256];
  const int cellid = blockIdx.x, tid = threadIdx.x;
  const int cnt = count[cellid], s0 = start[cellid];
  float* out = batch_median + (int64_t)cellid * PP;
  if (tid == 0) batch_n[cellid] = (float)cnt;
  if (cnt == 0) {
    for (int e = tid; e < PP; e += blockDim.x) out[e] = 0.0f;
    return;
  }
  const int want = (cnt - 1) / 2;
  // more tokens in the cell than LDS holds: same selection, values read from global memory
  const bool staged = cnt <= kMedianLds;
  const int E = staged ? min(min(PP, 256), kMedianLds / cnt) : min(PP, 256);
  for (int e0 = 0; e0 < PP; e0 += E) {
    const int Ec = min(E, PP - e0);
    for (int e = tid; e < Ec; e += blockDim.x) nanf[e] = 0;
    __syncthreads();
    for (int q = tid; q < cnt * Ec; q += blockDim.x) {
      const int i = q / Ec, e = q - i * Ec;
      const float v = x[(int64_t)list[s0 + i] * PP + e0 + e];
      if (staged) sv[q] = v;
      if (isnan(v)) nanf[e] = 1;
    }
    __syncthreads();
    for (int q = tid; q < cnt * Ec; q += blockDim.x) {
      const int i = q / Ec, e = q - i * Ec;
      if (nanf[e]) {
        if (i == 0) out[e0 + e] = __int_as_float(0x7fc00000);
        continue;
      }
      int rank = 0;
      if (staged) {
        const float vi = sv[q];
        for (int j = 0; j < cnt; ++j) {
          const float vj = sv[j * Ec + e];
          rank += (vj < vi) || (vj == vi && j < i);
        }
        if (rank == want) out[e0 + e] = vi;
      } else {
        const float vi = x[(int64_t)list[s0 + i] * PP + e0 + e];
        for (int j = 0; j < cnt; ++j) {
          const float vj = x[(int64_t)list[s0 + j] * PP + e0 + e];
          rank += (vj < vi) || (vj == vi && j < i);
        }
        if (rank == want) out[e0 + e] = vi;
      }
    }
    __syncthreads();
  }
}

// sum over the cell's tokens, in batch order, of |x - median| / clamp(batch_n, 1)
__global__ void k_stats_batch_b(const float* __restrict__ x, int PP, const int32_t* __restrict__ start,
                                const int32_t* __restrict__ count, const int32_t* __restrict__ list,
                                const float* __restrict__ median, float* __restrict__ batch_b) {
  const int cellid = blockIdx.x;
  const int cnt = count[cellid], s0 = start[cellid];
  for (int e = threadIdx.x; e < PP; e += blockDim.x) {
    const float m = median[(int64_t)cellid * PP + e];
    float acc = 0.0f;
    for (int i = 0; i < cnt; ++i) acc = __fadd_rn(acc, fabsf(__fsub_rn(x[(int64_t)list[s0 + i] * PP + e], m)));
    batch_b[(int64_t)cellid * PP + e] = __fdiv_rn(acc, fmaxf((float)cnt, 1.0f));
  }
}

// running merge t <- (t*n + s*bn) / clamp(n + bn, 1) per element (+ n update)
__global__ void k_stats_merge(float* __restrict__ t, const float* __restrict__ s, const float* __restrict__ n,
                              const float* __restrict__ bn, int n_cells, int PP) {
  const int64_t total = (int64_t)n_cells * PP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cidx = e / PP;
    const float nn = n[cidx], bb = bn[cidx];
    const float den = fmaxf(__fadd_rn(nn, bb), 1.0f);
    t[e] = __fdiv_rn(__fadd_rn(__fmul_rn(t[e], nn), __fmul_rn(s[e], bb)), den);
  }
}

__global__ void k_stats_add(float* __restrict__ n, const float* __restrict__ bn, int n_cells) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_cells; i += gridDim.x * blockDim.x)
    n[i] = __fadd_rn(n[i], bn[i]);
}

// patchnorm.py:153-155: training forward returns the raw patches, pads zeroed
__global__ void k_zero_pads(const float* __restrict__ x, const uint8_t* __restrict__ key_pad, int64_t n_tok, int PP,
                            float* __restrict__ y) {
  const int64_t total = n_tok * PP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x)
    y[e] = key_pad[e / PP] ? 0.0f : x[e];
}

static int grid_for(int64_t n, int cap = 8192) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap)); }

void launch_stats_lists(const int64_t* ch, const int64_t* pos, const uint8_t* key_pad, int64_t n_tok, int C, int mh,
                        int mw, int32_t* cell, int32_t* count, int32_t* start, int32_t* list, int* err, hipStream_t s) {
  const int n_cells = C * mh * mw;
  hipMemsetAsync(count, 0, sizeof(int32_t) * n_cells, s);
  hipLaunchKernelGGL(k_stats_cells, dim3(grid_for(n_tok)), dim3(256), 0, s, ch, pos, key_pad, n_tok, C, mh, mw, cell,
                     count, err);
  hipLaunchKernelGGL(k_stats_scan, dim3(1), dim3(1024), 0, s, count, n_cells, start);
  hipLaunchKernelGGL(k_stats_lists, dim3((n_cells * 64 + 255) / 256), dim3(256), 0, s, cell, n_tok, n_cells, start,
                     count, list);
}

void launch_stats_median(const float* x, int PP, int n_cells, const int32_t* start, const int32_t* count,
                         const int32_t* list, float* batch_median, float* batch_n, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_median, dim3(n_cells), dim3(256), 0, s, x, PP, start, count, list, batch_median, batch_n);
}

void launch_stats_batch_b(const float* x, int PP, int n_cells, const int32_t* start, const int32_t* count,
                          const int32_t* list, const float* median, float* batch_b, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_batch_b, dim3(n_cells), dim3(256), 0, s, x, PP, start, count, list, median, batch_b);
}

void launch_stats_merge(float* t, const float* src, const float* n, const float* bn, int n_cells, int PP,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_stats_merge, dim3(grid_for((int64_t)n_cells * PP)), dim3(256), 0, s, t, src, n, bn, n_cells, PP);
}

void launch_stats_add(float* n, const float* bn, int n_cells, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_add, dim3(grid_for(n_cells)), dim3(256), 0, s, n, bn, n_cells);
}

void launch_zero_pads(const float* x, const uint8_t* key_pad, int64_t n_tok, int PP, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_zero_pads, dim3(grid_for(n_tok * PP)), dim3(256), 0, s, x, key_pad, n_tok, PP, y);
}

}  // namespace dctae
