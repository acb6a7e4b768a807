// Device helpers shared by the HIP translation units.
#pragma once
#include "dctae_internal.h"

namespace dctae {

// Lanes of one wave handing data to each other through LDS: orders the
// earlier phase's LDS stores before the later phase's loads for the compiler
// (the hardware runs the wave's instructions in order).  Costs no instructions.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef float floatx16 __attribute__((ext_vector_type(16)));


__device__ __forceinline__ float mat3_row(const float* m, int i, float a, float b, float c) {
  // lms/ipt channel mix (reference util.py:46-47 einsum "i j, ... j h w")
  return fmaf(m[3 * i + 2], c, fmaf(m[3 * i + 1], b, m[3 * i + 0] * a));
}

__device__ __forceinline__ float signed_pow(float x, float p) {
  // util.py:76-78: y = |x|**p ; y[x<0] = -y
  float y = powf(fabsf(x), p);
  return x < 0.0f ? -y : y;
}

// |x|^p through the hardware log2/exp2 (v_log_f32 / v_exp_f32, ~2 ulp):
// the encode colour transform is compared with a tolerance (SURVEY §7 hard
// part 7), and generic powf costs ~10x the instructions.
__device__ __forceinline__ float signed_pow_fast(float x, float p) {
  const float y = __builtin_amdgcn_exp2f(p * __builtin_amdgcn_logf(fabsf(x)));
  return x < 0.0f ? -y : y;
}

// NaN-propagating max (torch.amax semantics)
__device__ __forceinline__ float nanmax(float a, float b) {
  return (a != a || a > b) ? a : ((b != b) ? b : (a > b ? a : b));
}

// nanmax over each 16-lane row of the wave, every lane gets its row's value:
// DPP row rotations by 8, 4, 2, 1 (VALU only; __shfl_xor is an LDS permute)
__device__ __forceinline__ float row16_nanmax(float a) {
  a = nanmax(a, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x128, 0xf, 0xf, false)));
  a = nanmax(a, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x124, 0xf, 0xf, false)));
  a = nanmax(a, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x122, 0xf, 0xf, false)));
  return nanmax(a, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), 0x121, 0xf, 0xf, false)));
}

// order-preserving float -> uint32 key; every NaN sorts above +inf
// (torch.sort(descending=True) puts NaN first).
__device__ __forceinline__ uint32_t float_key(float f) {
  if (f != f) return 0xFFFFFFFFu;
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// PatchNorm eval for one element, reference op order (patchnorm.py:157-163):
//   std = b * 2**0.5 + eps ; y = (x - m) / std ; clamp(min, max)
__device__ __forceinline__ float pn_forward(float x, float m, float b, float eps, float lo, float hi) {
  float sd = __fadd_rn(__fmul_rn(b, 1.41421353816986083984375f), eps);
  float y = __fdiv_rn(__fsub_rn(x, m), sd);
  // torch.clamp_ propagates NaN
  return (y != y) ? y : fminf(fmaxf(y, lo), hi);
}

// PatchNorm.inverse_norm (patchnorm.py:167-177): y * std + m, two roundings.
__device__ __forceinline__ float pn_inverse(float y, float m, float b, float eps) {
  float sd = __fadd_rn(__fmul_rn(b, 1.41421353816986083984375f), eps);
  return __fadd_rn(__fmul_rn(y, sd), m);
}

// one token, called by all 16 lanes of a group; vals[p2] = Y[P*h + j][P*w + p2]
__device__ inline void token_epilogue(const EncParams& ep, int c, int h, int w, int j, int g16,
                               const float* vals, int64_t tok, TokenSinks sk, uint16_t* rowbits) {
  const int P = ep.P, PP = P * P;
  float amax = 0.0f;
  uint32_t bits = 0;
  const bool lane_on = j < P;
  if (lane_on) {
    const int64_t tab = ((((int64_t)c * ep.maxph + h) * ep.maxpw) + w) * PP + (int64_t)j * P;
    for (int p2 = 0; p2 < P; ++p2) {
      float v = vals[p2];
      amax = nanmax(amax, fabsf(v));
      if (sk.raw) sk.raw[tok * PP + j * P + p2] = v;
      if (ep.median) {
        if (sk.norm || !ep.thr) {
          float y = pn_forward(v, ep.median[tab + p2], ep.b[tab + p2], ep.eps, ep.min_val, ep.max_val);
          if (y > 0.0f) bits |= 1u << p2;
          if (sk.norm) sk.norm[tok * PP + j * P + p2] = y;
        } else if (v >= ep.thr[tab + p2]) {
          // thr = smallest fp32 x with PatchNorm(x) > 0 (k_norm_thresholds): same bit, one compare
          bits |= 1u << p2;
        }
      }
    }
  }
  // group max over the 16 lanes (xor shuffles stay inside the group)
  amax = row16_nanmax(amax);
  if (j == 0) {
    // score = amax*mw + (-(h+w))/ci[c]      (FE:409-416, fp32 ops)
    float s = __fadd_rn(__fmul_rn(amax, ep.mw), __fdiv_rn(-(float)(h + w), ep.ci[c]));
    sk.scores[tok] = s;
  }
  if (ep.median && sk.codes) {
    if (lane_on) rowbits[g16 * kMaxP + j] = (uint16_t)bits;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int q = j; q < ep.ncb; q += 16) {
      uint32_t code = 0;
      for (int d = 0; d < ep.cb_dim; ++d) {
        int e = q * ep.cb_dim + d;
        uint32_t bit = (rowbits[g16 * kMaxP + e / P] >> (e % P)) & 1u;
        code |= bit << (ep.cb_dim - 1 - d);
      }
      sk.codes[tok * ep.ncb + q] = (uint16_t)code;
    }
    __builtin_amdgcn_wave_barrier();
  }
}


// token_epilogue specialised for a compile-time patch size with one LFQ
// codebook per tile row (codebook_dim == P): lane j's code is its row's sign
// bits in MSB-first order (lfq.py:187), i.e. a bit reversal — no exchange.
// vals: this lane's row, thr: thresholds row (nullable -> PatchNorm values).
// ny (optional): receives this lane's PatchNorm values (computed, not stored).
template <int P>
__device__ __forceinline__ void token_epilogue_p(const EncParams& ep, int c, int h, int w, int j,
                                                 const float* vals, int64_t tok, TokenSinks sk, float* ny = nullptr) {
  constexpr int PP = P * P;
  float amax = 0.0f;
  uint32_t bits = 0;
  if (j < P) {
    const int64_t tab = ((((int64_t)c * ep.maxph + h) * ep.maxpw) + w) * PP + (int64_t)j * P;
#pragma unroll
    for (int p2 = 0; p2 < P; ++p2) amax = nanmax(amax, fabsf(vals[p2]));
    if (sk.raw) {
#pragma unroll
      for (int p2 = 0; p2 < P; ++p2) sk.raw[tok * PP + j * P + p2] = vals[p2];
    }
    if (ep.median) {
      if (sk.norm || ny || !ep.thr) {
        float med[P], bb[P];
        if ((P & 1) == 0) {   // tab is even: 8-byte table loads
          const float2* m2 = reinterpret_cast<const float2*>(ep.median + tab);
          const float2* b2 = reinterpret_cast<const float2*>(ep.b + tab);
#pragma unroll
          for (int p = 0; p < P / 2; ++p) {
            const float2 mv = m2[p], bv = b2[p];
            med[2 * p] = mv.x, med[2 * p + 1] = mv.y, bb[2 * p] = bv.x, bb[2 * p + 1] = bv.y;
          }
        } else {
#pragma unroll
          for (int p2 = 0; p2 < P; ++p2) med[p2] = ep.median[tab + p2], bb[p2] = ep.b[tab + p2];
        }
#pragma unroll
        for (int p2 = 0; p2 < P; ++p2) {
          const float y = pn_forward(vals[p2], med[p2], bb[p2], ep.eps, ep.min_val, ep.max_val);
          bits |= (y > 0.0f ? 1u : 0u) << p2;
          if (sk.norm) sk.norm[tok * PP + j * P + p2] = y;
          if (ny) ny[p2] = y;
        }
      } else if ((P & 1) == 0) {
        const float2* t2 = reinterpret_cast<const float2*>(ep.thr + tab);
#pragma unroll
        for (int p = 0; p < P / 2; ++p) {
          const float2 t = t2[p];
          bits |= (vals[2 * p] >= t.x ? 1u : 0u) << (2 * p);
          bits |= (vals[2 * p + 1] >= t.y ? 1u : 0u) << (2 * p + 1);
        }
      } else {
#pragma unroll
        for (int p2 = 0; p2 < P; ++p2) bits |= (vals[p2] >= ep.thr[tab + p2] ? 1u : 0u) << p2;
      }
    }
  }
  amax = row16_nanmax(amax);
  if (j == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(amax, ep.mw), __fdiv_rn(-(float)(h + w), ep.ci[c]));
  if (ep.median && sk.codes) {
    if (ep.cb_dim == P && ep.ncb == P) {
      if (j < P) sk.codes[tok * P + j] = (uint16_t)(__builtin_bitreverse32(bits) >> (32 - P));
    } else {
      // other LFQ groupings: gather the group's row bits, cut the flat
      // (row-major) sign-bit string into codebook_dim-bit codes, MSB first
      uint32_t rb[P];
      const int base = (int)(threadIdx.x & 63) & ~15;
#pragma unroll
      for (int r = 0; r < P; ++r) rb[r] = (uint32_t)__shfl((int)bits, base + r, 64);
      for (int q = j; q < ep.ncb; q += 16) {
        uint32_t code = 0;
        for (int d = 0; d < ep.cb_dim; ++d) {
          const int e = q * ep.cb_dim + d;
          code |= ((rb[e / P] >> (e % P)) & 1u) << (ep.cb_dim - 1 - d);
        }
        sk.codes[tok * ep.ncb + q] = (uint16_t)code;
      }
    }
  }
}

// token_epilogue_p with the thresholds already in registers (thr[p] covers
// elements 2p, 2p+1 of this lane's row); codes-only path.
template <int P>
__device__ __forceinline__ void token_epilogue_thr(const EncParams& ep, int c, int h, int w, int j, const float* vals,
                                                   const float2* thr, int64_t tok, TokenSinks sk) {
  constexpr int PP = P * P;
  float amax = 0.0f;
  uint32_t bits = 0;
  if (j < P) {
#pragma unroll
    for (int p = 0; p < P / 2; ++p) {
      amax = nanmax(amax, fabsf(vals[2 * p]));
      amax = nanmax(amax, fabsf(vals[2 * p + 1]));
      bits |= (vals[2 * p] >= thr[p].x ? 1u : 0u) << (2 * p);
      bits |= (vals[2 * p + 1] >= thr[p].y ? 1u : 0u) << (2 * p + 1);
    }
    if (sk.raw) {
#pragma unroll
      for (int p2 = 0; p2 < P; ++p2) sk.raw[tok * PP + j * P + p2] = vals[p2];
    }
  }
  amax = row16_nanmax(amax);
  if (j == 0) sk.scores[tok] = __fadd_rn(__fmul_rn(amax, ep.mw), __fdiv_rn(-(float)(h + w), ep.ci[c]));
  if (sk.codes && j < P) sk.codes[tok * P + j] = (uint16_t)(__builtin_bitreverse32(bits) >> (32 - P));
}

}  // namespace dctae
