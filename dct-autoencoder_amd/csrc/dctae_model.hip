// DCTAutoencoder transformer forward: the kernels under the
// CLIPEncoder encoder / decoder around the LFQ bottleneck
// (modeling_dct_autoencoder.py; transformers==4.35.2 CLIPEncoderLayer).
//
//   k_linear<EPI>   y = x W^T (+ bias) on v_mfma_f32_32x32x16_bf16: 128 x 128
//                   tiles, BK = 64, 4 waves of 64 x 64, operands staged by
//                   global_load_lds into two XOR-swizzled LDS buffers (tile
//                   k+1 in flight during tile k); epilogues: f32 store, bf16
//                   store, bf16 quick_gelu, f32 residual add (in place)
//   k_attention     flash attention, d_head = 64: S^T = K Q^T so the softmax
//                   probabilities come out of the MFMA already in B-operand
//                   layout for O^T = V^T P^T (keys permuted consistently in
//                   V^T); online softmax in fp32; the reference's attention
//                   "mask" is ADDED (+1.0 where id_i == id_j and key j is a
//                   pad, FE:580-584 -> modeling:131-133), computed from the
//                   row's image ids and key_pad_mask (no S x S tensor)
//   k_layernorm     one wave per token row, fp32 statistics, bf16 out
//   k_ln_pos        embedding LayerNorm (eps 1e-4) + encoder position terms
//   k_pos_add       decoder position terms (in place)
//   k_to_bf16       fp32 -> bf16 with zero K padding
//   k_lfq_codes     LFQ.forward eval (lfq.py:164-212): sign, MSB-first codes,
//                   +-1 features (bf16 for project_out, or f32)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dctae_model.h"
#include "dctae_internal.h"

namespace dctae {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint16_t f2bf(float f) {   // round to nearest even (v_cvt_pk_bf16_f32)
  const __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// ---------------------------------------------------------------------------
// linear: 128 x 128 tile, BK = 64, 4 waves of 64 x 64 (2 x 2 MFMA 32x32x16
// blocks), A and W tiles staged global -> LDS with global_load_lds_dwordx4
// (async, no VGPR staging) into two LDS buffers: tile k+1 is in flight while
// tile k is multiplied.  One wave-instruction writes 1 KB = 8 rows x 64 bf16
// lane-linearly; the XOR swizzle is applied to the global source address:
// 16-byte segment s of row r holds k-segment s ^ g(r), g(r) = (r >> 1) & 7,
// so every ds_read_b128 lane group (16 rows, one k-segment) covers the 16
// slots of a 256-byte bank row: conflict-free fragment reads.
// ---------------------------------------------------------------------------
constexpr int LBM = 128, LBN = 128, LBK = 64;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int lswz(int row, int kseg) { return row * LBK + ((kseg ^ ((row >> 1) & 7)) << 3); }

// epilogue of a wave's 64 x 64 block at (mb, nb): acc[i][j][v] = C[row =
// 8 (v / 4) + 4 (lane / 32) + v % 4][col = lane % 32] of 32 x 32 block (i, j)
template <int EPI>
__device__ __forceinline__ void lin_epilogue(const LinearArgs& a, const f32x16 (&acc)[2][2], int64_t mb, int nb, int fr,
                                             int fh) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = nb + j * 32 + fr;
    if (n >= a.N) continue;
    const float bias = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t m = mb + i * 32 + 8 * (v >> 2) + 4 * fh + (v & 3);
        if (m >= a.M) continue;
        float y = acc[i][j][v] + bias;
        if (EPI == LIN_F32) {
          reinterpret_cast<float*>(a.out)[m * a.ldo + n] = y;
        } else if (EPI == LIN_BF16) {
          reinterpret_cast<__bf16*>(a.out)[m * a.ldo + n] = (__bf16)y;   // v_cvt_pk_bf16_f32 (RNE)
        } else if (EPI == LIN_BF16_QGELU) {
          // quick_gelu x * sigmoid(1.702 x) with the hardware exp2 / reciprocal
          // (~1 ulp each; the result is rounded to bf16 right after)
          y = y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.45546696228f * y));   // 1.702 log2(e)
          reinterpret_cast<__bf16*>(a.out)[m * a.ldo + n] = (__bf16)y;
        } else {   // LIN_F32_RESIDUAL
          float* o = reinterpret_cast<float*>(a.out) + m * a.ldo + n;
          *o = *o + y;
        }
      }
  }
}

// tile id -> (M tile, N tile), grouped raster: runs of LGM M tiles per N tile
// column, so the ~64 tiles an XCD holds at once cover about 8 x 8 tiles and
// their A rows and W rows (a few MB) stay in that XCD's L2 (a row-major order
// streams all of W through L2 for every M row: 40 % L2 hit rate measured)
constexpr int LGM = 8;
__device__ __forceinline__ void lin_tile(int t, int ntm, int ntn, int& tm, int& tn) {
  const int per = LGM * ntn, g = t / per, r = t - g * per;
  const int first = g * LGM, gm = min(ntm - first, LGM);
  tm = first + r % gm;
  tn = r / gm;
}

template <int EPI>
__global__ __launch_bounds__(256) void k_linear(LinearArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t L[2 * (LBM + LBN) * LBK];   // [buf][A 128 rows | W 128 rows][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: workgroup b runs on XCD b % 8; give each XCD a contiguous
  // range of tile ids, row-major over (M tile, N tile), so an XCD's blocks share
  // their A rows through its L2 (A is then read from HBM once, not once per XCD)
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  const int ntn = (a.N + LBN - 1) / LBN, ntm = (int)((a.M + LBM - 1) / LBM);
  int tm, tn;
  lin_tile(wgid, ntm, ntn, tm, tn);
  const int64_t m0 = (int64_t)tm * LBM;
  const int n0 = tn * LBN;
  // this lane's glds sources: wave-instruction j covers rows 8 (4 wave + j) + lane / 8, slot lane % 8
  const uint16_t* srcA[4];
  const uint16_t* srcW[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wave + j) + (lane >> 3), slot = lane & 7;
    const int kseg = slot ^ ((row >> 1) & 7);
    srcA[j] = a.x + min<int64_t>(m0 + row, a.M - 1) * a.ldx + kseg * 8;
    srcW[j] = a.w + (int64_t)min(n0 + row, a.Nw - 1) * a.ldw + kseg * 8;
  }
  auto stage = [&](int buf, int k0) {
    uint16_t* base = L + buf * (LBM + LBN) * LBK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + k0), (lds_ptr_t)(base + 8 * (4 * wave + j) * LBK), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(srcW[j] + k0), (lds_ptr_t)(base + (LBM + 8 * (4 * wave + j)) * LBK),
                                       16, 0, 0);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.0f;
  const int nk = a.K / LBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 31, fh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * LBK);
    const uint16_t* As = L + (kt & 1) * (LBM + LBN) * LBK;
    const uint16_t* Ws = As + LBM * LBK;
#pragma unroll
    for (int kk = 0; kk < LBK / 16; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + lswz(wm * 64 + i * 32 + fr, 2 * kk + fh));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Ws + lswz(wn * 64 + j * 32 + fr, 2 * kk + fh));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile kt + 1 landed
    __syncthreads();                                    // ... for every wave; tile kt's buffer free
  }
  // vectorised epilogue: each wave's 64 x 64 block goes through LDS (the last
  // loop barrier freed the operand buffers) and leaves as 16-byte row
  // segments (the accumulator layout alone gives 32 x 2- or 4-byte columns)
  constexpr int VEC = (EPI == LIN_BF16 || EPI == LIN_BF16_QGELU) ? 8 : 4;   // elements per 16 bytes
  const bool vec_ok = n0 + LBN <= a.N && a.ldo % VEC == 0 && (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
  if (!vec_ok) {
    lin_epilogue<EPI>(a, acc, m0 + wm * 64, n0 + wn * 64, fr, fh);
    return;
  }
  float* Cs = reinterpret_cast<float*>(L) + wave * 64 * 64;   // [64 rows][64 cols], 4 x 16 KB = the 64 KB of L
  const int64_t mb = m0 + wm * 64;
  const int nb = n0 + wn * 64;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float bias = a.bias ? a.bias[nb + j * 32 + fr] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        float y = acc[i][j][v] + bias;
        if (EPI == LIN_BF16_QGELU)
          y = y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.45546696228f * y));   // quick_gelu
        Cs[(i * 32 + 8 * (v >> 2) + 4 * fh + (v & 3)) * 64 + j * 32 + fr] = y;   // 32 lanes: one row, 32 banks
      }
  }
  if (VEC == 8) {   // bf16: 8 lanes per 128-byte row, 8 rows per pass
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int r = it * 8 + (lane >> 3), c8 = (lane & 7) * 8;
      const float4 lo = *reinterpret_cast<const float4*>(Cs + r * 64 + c8);
      const float4 hi = *reinterpret_cast<const float4*>(Cs + r * 64 + c8 + 4);
      uint4 pk;
      pk.x = (uint32_t)f2bf(lo.x) | ((uint32_t)f2bf(lo.y) << 16);
      pk.y = (uint32_t)f2bf(lo.z) | ((uint32_t)f2bf(lo.w) << 16);
      pk.z = (uint32_t)f2bf(hi.x) | ((uint32_t)f2bf(hi.y) << 16);
      pk.w = (uint32_t)f2bf(hi.z) | ((uint32_t)f2bf(hi.w) << 16);
      if (mb + r < a.M) *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out) + (mb + r) * a.ldo + nb + c8) = pk;
    }
  } else {   // f32 (plain or residual): 16 lanes per 256-byte row, 4 rows per pass
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = it * 4 + (lane >> 4), c4 = (lane & 15) * 4;
      float4 y = *reinterpret_cast<const float4*>(Cs + r * 64 + c4);
      if (mb + r < a.M) {
        float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + (mb + r) * a.ldo + nb + c4);
        if (EPI == LIN_F32_RESIDUAL) {
          const float4 x = *o;
          y.x += x.x;
          y.y += x.y;
          y.z += x.z;
          y.w += x.w;
        }
        *o = y;
      }
    }
  }
}

void launch_linear(const LinearArgs& a, int epi, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  const dim3 grid((unsigned)(((a.N + LBN - 1) / LBN) * ((a.M + LBM - 1) / LBM)));
  switch (epi) {
    case LIN_F32: hipLaunchKernelGGL(k_linear<LIN_F32>, grid, dim3(256), 0, s, a); break;
    case LIN_BF16: hipLaunchKernelGGL(k_linear<LIN_BF16>, grid, dim3(256), 0, s, a); break;
    case LIN_BF16_QGELU: hipLaunchKernelGGL(k_linear<LIN_BF16_QGELU>, grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(k_linear<LIN_F32_RESIDUAL>, grid, dim3(256), 0, s, a); break;
  }
}

// ---------------------------------------------------------------------------
// attention (d_head = 64): block = (row b, head h, 256 queries), wave = 32
// queries.  Per 64-key block: K (64 x 64) and V^T (64 x 64) staged in LDS.
//   S^T tile t (keys 32 t .., 32 queries) = sum_kk mfma(A = K[keys][d kk],
//   B = Q^T[d kk][queries]):  lane l holds keys 32 t + 8 (v/4) + 4 (l/32) + v%4
//   of query l % 32.
//   O^T (64 d x 32 q) += mfma(A = V^T[d][keys], B = P^T[keys][q]) over 4 key
//   steps; key step kk covers, for lane half h, the keys
//   32 (kk/2) + 8 (2 (kk%2) + e/4) + 4 h + e%4, e < 8 — exactly the S^T values
//   the lane already holds, so P needs no shuffle; V^T is read with the same
//   key order (two 8-byte LDS reads per fragment).
// ---------------------------------------------------------------------------
// LDS row strides (bf16): K / O rows 72 (ds_read_b128 fragment reads: rows r
// land on 16-byte slots 9 r mod 16, conflict-free); V rows 96 (the transposed
// ds_read_b64_tr_b16 reads: rows kb + q at banks 48 q mod 64 plus the 8-bank
// column groups tile the 64 banks; at 72 they were 2-way)
constexpr int AQ = 256, AK = 64, AD = 64, ASTR = 72, AVS = 96, ATH = 4 * AQ / 2;   // ATH threads: one wave per 32 queries

__global__ __launch_bounds__(ATH) void k_attention(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[AK * ASTR];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[AK * AVS];   // row-major; read transposed (ds_read_b64_tr_b16)
  __shared__ __attribute__((aligned(16))) int32_t kid[AK];   // key image id, or -1 for a non-pad key (no bias)
  __shared__ __attribute__((aligned(16))) uint16_t Os[AQ * ASTR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = a.S, D = a.heads * AD;
  const int q0 = blockIdx.x * AQ, h = blockIdx.y, b = blockIdx.z;
  const int64_t rowbase = (int64_t)b * S;
  const int64_t ld = 3ll * D;
  const uint16_t* qkv = a.qkv;
  // this lane's query and its Q fragments (B operand: Q[q][d kk*16 + 8 (l/32) ..])
  const int ql = q0 + wave * 32 + (lane & 31);
  const int qc = min(ql, S - 1);
  bf16x8 qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    qf[kk] = *reinterpret_cast<const bf16x8*>(qkv + (rowbase + qc) * ld + h * AD + kk * 16 + (lane >> 5) * 8);
  const int32_t my_id = (int32_t)a.ids[rowbase + qc];
  const float sc = a.scale * 1.4426950408889634f;   // logits in log2 units
  const float bias2 = 1.4426950408889634f;           // +1.0 bias in log2 units
  f32x16 o[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) o[t][v] = 0.0f;
  float mrun = -INFINITY, lsum = 0.0f;
  for (int k0 = 0; k0 < S; k0 += AK) {
    __syncthreads();   // previous block's K / V reads done
    // stage K and V rows: 64 keys x 64 d, 16 B per load (two per thread each)
#pragma unroll
    for (int j = 0; j < AK * 8 / ATH; ++j) {
      const int idx = tid + ATH * j, key = idx >> 3, seg = idx & 7;
      const int kg = min(k0 + key, S - 1);
      const uint16_t* src = qkv + (rowbase + kg) * ld + h * AD + seg * 8;
      const uint4 kv = *reinterpret_cast<const uint4*>(src + D);
      const uint4 vv = *reinterpret_cast<const uint4*>(src + 2 * D);
      *reinterpret_cast<uint4*>(Ks + key * ASTR + seg * 8) = kv;
      *reinterpret_cast<uint4*>(Vs + key * AVS + seg * 8) = vv;
    }
    bool pad = false;
    if (tid < AK) {
      const int kg = k0 + tid;
      pad = kg < S && a.key_pad[rowbase + kg];
      kid[tid] = pad ? (int32_t)a.ids[rowbase + kg] : -1;
    }
    const bool any_pad = __syncthreads_or(pad);   // block-uniform: the +1 bias only ever hits pad keys
    // S^T tiles
    f32x16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int v = 0; v < 16; ++v) st[t][v] = 0.0f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (t * 32 + (lane & 31)) * ASTR + kk * 16 + (lane >> 5) * 8);
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], st[t], 0, 0, 0);
      }
    }
    // scale + bias, block max over the 64 keys of this query (lanes l and l ^ 32).
    // Without pad keys in the block the logits stay unscaled (sce = sc) and the
    // scale is applied inside the exponent's FMA; with pad keys they are scaled
    // and biased here (sce = 1).
    float bm = -INFINITY;
    float sce = sc;
    if (any_pad) {
      sce = 1.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const int4 ki = *reinterpret_cast<const int4*>(kid + t * 32 + 8 * q4 + 4 * (lane >> 5));
          st[t][4 * q4 + 0] = st[t][4 * q4 + 0] * sc + (ki.x == my_id ? bias2 : 0.0f);
          st[t][4 * q4 + 1] = st[t][4 * q4 + 1] * sc + (ki.y == my_id ? bias2 : 0.0f);
          st[t][4 * q4 + 2] = st[t][4 * q4 + 2] * sc + (ki.z == my_id ? bias2 : 0.0f);
          st[t][4 * q4 + 3] = st[t][4 * q4 + 3] * sc + (ki.w == my_id ? bias2 : 0.0f);
        }
    }
    if (k0 + AK > S) {   // last, partial key block
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          if (k0 + t * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3) >= S) st[t][v] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) bm = fmaxf(bm, st[t][v]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(bm), __float_as_uint(bm), false, false);
      bm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sce;
    }
    // lazy rescale: the reference max moves only when the block max exceeds it
    // by more than 8 (log2 units), so p = 2^(s - m) <= 2^8 stays exact in fp32
    // and in range for bf16; O and the sum always share the same m, so the
    // normalised result is unchanged.  The O rescale (AGPR round trip) runs
    // only when some lane moved its max.
    if (bm > mrun + 8.0f) {
      const float alpha = __builtin_amdgcn_exp2f(mrun - bm);   // 0 on the first block (mrun = -inf)
      mrun = bm;
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) o[t][v] *= alpha;
    }
    const float nm = -mrun;
    // P (bf16) in B-operand order: key step kk = (tile kk / 2, quarters 2 (kk % 2), +1)
    bf16x8 pf[4];
    float ls2[2] = {0.0f, 0.0f};   // two partial sums (pairs for packed adds)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int t = kk >> 1, v0 = 8 * (kk & 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // raw v_exp_f32: exp2f's denormal-range fix-up (5 VALU ops per call)
        // is not needed (results below 2^-126 are negligible probabilities)
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(st[t][v0 + e], sce, nm));
        ls2[e & 1] += p;
        pf[kk][e] = (__bf16)p;
      }
    }
    lsum += ls2[0] + ls2[1];
    // O^T += V^T P^T; the A fragment V^T[d = 32 dt + lane % 32][keys kb + (0..3), kb + 8 + (0..3)] comes
    // from the row-major V tile by two transposed reads: lane 4q + p of each 16-lane group addresses key
    // row kb + q, columns 4p .. 4p + 3 of the group's 16 d columns, and receives its own column
    typedef short s4 __attribute__((ext_vector_type(4)));
    const int gq = (lane & 15) >> 2, gp = lane & 3, gx = (lane >> 4) & 1;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int kb = 32 * (kk >> 1) + 8 * (2 * (kk & 1)) + 4 * (lane >> 5);
        const uint16_t* vr = Vs + (kb + gq) * AVS + 32 * dt + 16 * gx + 4 * gp;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)vr);
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(vr + 8 * AVS));
        bf16x8 vf;
        short* vsh = reinterpret_cast<short*>(&vf);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vsh[e] = lo[e];
          vsh[4 + e] = hi[e];
        }
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kk], o[dt], 0, 0, 0);
      }
  }
  // normalise: the query's sum is split over lanes l and l ^ 32
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
    lsum = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = 1.0f / lsum;
  // O^T[d = 32 dt + 8 (v/4) + 4 (l/32) + v%4][query l%32] -> Os[query][d] -> coalesced rows
  const int qr = wave * 32 + (lane & 31);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int d = 32 * dt + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
      Os[qr * ASTR + d] = f2bf(o[dt][v] * inv);
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < AQ * 8 / ATH; ++j) {
    const int idx = tid + ATH * j, r = idx >> 3, seg = idx & 7;
    if (q0 + r < S)
      *reinterpret_cast<uint4*>(a.out + (rowbase + q0 + r) * (int64_t)a.ldo + h * AD + seg * 8) =
          *reinterpret_cast<const uint4*>(Os + r * ASTR + seg * 8);
  }
}

void launch_attention(const AttnArgs& a, hipStream_t s) {
  if (a.R <= 0 || a.S <= 0) return;
  hipLaunchKernelGGL(k_attention, dim3((a.S + AQ - 1) / AQ, a.heads, a.R), dim3(ATH), 0, s, a);
}

// ---------------------------------------------------------------------------
// LayerNorm (torch semantics: biased variance, eps inside the sqrt), one wave
// per token row; D % 64 == 0, D <= 64 * 64.
// ---------------------------------------------------------------------------
template <int PER>
__device__ __forceinline__ void ln_row(const float* x, const float* g, const float* bt, float eps, int D,
                                       float (&y)[PER]) {
  const int lane = threadIdx.x & 63;
  float v[PER];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < D ? x[c] : 0.0f;
    s += v[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)D;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const float dv = c < D ? v[i] - mean : 0.0f;
    q += dv * dv;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / (float)D + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    y[i] = c < D ? (v[i] - mean) * rstd * g[c] + bt[c] : 0.0f;
  }
}

template <int PER>
__global__ __launch_bounds__(256) void k_layernorm(LnArgs a) {
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int lane = threadIdx.x & 63;
  float y[PER];
  ln_row<PER>(a.x + m * a.ldx, a.gamma, a.beta, a.eps, a.D, y);
  if (a.out_f32) {   // + position terms (embedding), f32 out
    const int64_t c = a.ch[m], ph = a.pos[2 * m], pw = a.pos[2 * m + 1];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int cc = lane + 64 * i;
      if (cc < a.D)
        a.out_f32[m * a.ldo + cc] = y[i] + a.pos_h[ph * a.D + cc] + a.pos_w[pw * a.D + cc] + a.pos_c[c * a.D + cc];
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int cc = lane + 64 * i;
      if (cc < a.D) a.out_bf16[m * a.ldo + cc] = f2bf(y[i]);
    }
  }
}

// LayerNorm -> bf16 for D % 256 == 0 with 16-byte row accesses: lane l holds
// columns 4 (l + 64 i) .. +3 (float4 loads, 8-byte bf16x4 stores; the scalar
// kernel moves 2 bytes per lane per store)
template <int P4>
__global__ __launch_bounds__(256) void k_layernorm_v(LnArgs a) {
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int lane = threadIdx.x & 63;
  const float4* x4 = reinterpret_cast<const float4*>(a.x + m * a.ldx);
  float4 v[P4];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < P4; ++i) {
    v[i] = x4[lane + 64 * i];
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)a.D;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < P4; ++i) {
    const float d0 = v[i].x - mean, d1 = v[i].y - mean, d2 = v[i].z - mean, d3 = v[i].w - mean;
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / (float)a.D + a.eps);
  const float4* g4 = reinterpret_cast<const float4*>(a.gamma);
  const float4* b4 = reinterpret_cast<const float4*>(a.beta);
  uint2* o2 = reinterpret_cast<uint2*>(a.out_bf16 + m * a.ldo);
#pragma unroll
  for (int i = 0; i < P4; ++i) {
    const int c4 = lane + 64 * i;
    const float4 g = g4[c4], b = b4[c4];
    uint2 pk;
    pk.x = (uint32_t)f2bf((v[i].x - mean) * rstd * g.x + b.x) | ((uint32_t)f2bf((v[i].y - mean) * rstd * g.y + b.y) << 16);
    pk.y = (uint32_t)f2bf((v[i].z - mean) * rstd * g.z + b.z) | ((uint32_t)f2bf((v[i].w - mean) * rstd * g.w + b.w) << 16);
    o2[c4] = pk;
  }
}

void launch_layernorm(const LnArgs& a, hipStream_t s) {
  if (a.M <= 0) return;
  const unsigned grid = (unsigned)((a.M + 3) / 4);
  const bool vec = !a.out_f32 && a.D % 256 == 0 && a.D <= 4096 && a.ldx % 4 == 0 && a.ldo % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(a.x) | reinterpret_cast<uintptr_t>(a.gamma) |
                     reinterpret_cast<uintptr_t>(a.beta)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.out_bf16) & 7) == 0;
  if (vec) {
    const int p4 = a.D / 256;
    if (p4 == 1) hipLaunchKernelGGL(k_layernorm_v<1>, dim3(grid), dim3(256), 0, s, a);
    else if (p4 == 2) hipLaunchKernelGGL(k_layernorm_v<2>, dim3(grid), dim3(256), 0, s, a);
    else if (p4 == 4) hipLaunchKernelGGL(k_layernorm_v<4>, dim3(grid), dim3(256), 0, s, a);
    else if (p4 == 8) hipLaunchKernelGGL(k_layernorm_v<8>, dim3(grid), dim3(256), 0, s, a);
    else if (p4 == 16) hipLaunchKernelGGL(k_layernorm_v<16>, dim3(grid), dim3(256), 0, s, a);
    else goto scalar;
    return;
  }
scalar:
  const int per = (a.D + 63) / 64;
  if (per <= 2) hipLaunchKernelGGL(k_layernorm<2>, dim3(grid), dim3(256), 0, s, a);
  else if (per <= 4) hipLaunchKernelGGL(k_layernorm<4>, dim3(grid), dim3(256), 0, s, a);
  else if (per <= 8) hipLaunchKernelGGL(k_layernorm<8>, dim3(grid), dim3(256), 0, s, a);
  else if (per <= 16) hipLaunchKernelGGL(k_layernorm<16>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_layernorm<64>, dim3(grid), dim3(256), 0, s, a);
}

// x[m] += pos_h[h] + pos_w[w] + pos_c[c]   (decoder position embedding, modeling:88-93)
__global__ void k_pos_add(PosArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.M * a.D) return;
  const int64_t m = i / a.D;
  const int cc = (int)(i - m * a.D);
  const int64_t c = a.ch[m], ph = a.pos[2 * m], pw = a.pos[2 * m + 1];
  a.x[m * a.ldx + cc] += a.pos_h[ph * a.D + cc] + a.pos_w[pw * a.D + cc] + a.pos_c[c * a.D + cc];
}

void launch_pos_add(const PosArgs& a, hipStream_t s) {
  const int64_t n = a.M * a.D;
  if (n > 0) hipLaunchKernelGGL(k_pos_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

// fp32 (M, K) -> bf16 (M, Kp), zero columns K .. Kp
__global__ void k_to_bf16(const float* x, int64_t ldx, int64_t M, int K, int Kp, uint16_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * Kp) return;
  const int64_t m = i / Kp;
  const int k = (int)(i - m * Kp);
  out[i] = k < K ? f2bf(x[m * ldx + k]) : (uint16_t)0;
}

void launch_to_bf16(const float* x, int64_t ldx, int64_t M, int K, int Kp, uint16_t* out, hipStream_t s) {
  const int64_t n = M * Kp;
  if (n > 0) hipLaunchKernelGGL(k_to_bf16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, M, K, Kp, out);
}

// LFQ eval on (M, ncb * cbd) features: codes (M, ncb) int64 MSB-first
// (lfq.py:87, 187), +-1 features into q_bf16 (M, ldq; zero pad to ldq) or q_f32
__global__ void k_lfq_codes(LfqArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.M * a.ncb) return;
  const int64_t m = i / a.ncb;
  const int j = (int)(i - m * a.ncb);
  const float* x = a.x + m * a.ldx + j * a.cbd;
  int64_t code = 0;
  for (int d = 0; d < a.cbd; ++d) {
    const bool pos = x[d] > 0.0f;
    code |= (int64_t)(pos ? 1 : 0) << (a.cbd - 1 - d);
    const float q = pos ? a.scale : -a.scale;
    if (a.q_bf16) a.q_bf16[m * a.ldq + j * a.cbd + d] = f2bf(q);
    if (a.q_f32) a.q_f32[m * a.ldq + j * a.cbd + d] = q;
  }
  // lfq.py:187: the index bit of the quantized value (any codebook_scale sign)
  a.codes[i] = (int64_t)lfq_index_bits((uint64_t)code, a.scale > 0.0f ? ~0ull : 0ull, -a.scale > 0.0f ? ~0ull : 0ull) &
               ((1ll << a.cbd) - 1);
  if (a.q_bf16 && j == a.ncb - 1)
    for (int k = a.ncb * a.cbd; k < a.ldq; ++k) a.q_bf16[m * a.ldq + k] = 0;
}

void launch_lfq_codes(const LfqArgs& a, hipStream_t s) {
  const int64_t n = a.M * a.ncb;
  if (n > 0) hipLaunchKernelGGL(k_lfq_codes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
}

}  // namespace dctae
