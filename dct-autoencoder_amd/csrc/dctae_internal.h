// Internal structures shared by the HIP kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dctae {

constexpr int kMaxP = 16;          // patch_size upper bound of the fused kernels
constexpr int kMaxCodebooks = 256; // num_codebooks upper bound (P*P / codebook_dim)

// Colour matrices (row-major 3x3, fp32 bits as the reference builds them).
struct ColorMats {
  float rgb2lms[9];
  float lms2ipt[9];
  float ipt2lms[9];
  float lms2rgb[9];
};

// Per-image plan entry (device resident).
struct ImgDesc {
  int64_t rgb_off;   // element offset of the (3,H,W) image in the input buffer
  int64_t ws_p;      // workspace offsets (floats): ipt image (3,H,W)
  int64_t ws_t;      //   row-pass output  Tt (3, Kw, H)
  int64_t ws_y;      //   spectrum corner   Y (3, Kh, Kw)
  int64_t tok_off;   // first flat token of this image in token staging
  int32_t H, W;
  int32_t ph, pw;    // uncapped patch grid  (H/P, W/P)
  int32_t qh, qw;    // capped patch grid    min(ph, max_patch_h) ...
  int32_t Kh, Kw;    // kept spectrum corner P*qh, P*qw
  int32_t T;         // tokens = C*qh*qw
  int32_t row, col, k, local_id;  // packing
  int32_t plan_w, plan_h;         // FFT plan index for rows (length W) / cols (length H); -1 = GEMM
  int32_t bs;        // bit 0: rows, bit 1: columns on the Bluestein kernels (columns: Y + k_tile_epilogue)
  int32_t tband;     // bit 0: the row pass writes T in the band layout T' (512 x 512 on k_rows512pk + k_cols512b);
                     // bit 1: item-major token staging (stage_pos), packed encodes of band images only (qh = qw = 32)
  int32_t tperm;     // rows AND columns on the GEMM DCT: T and Y hold their kx columns parity-planar, column
                     // n' = kx / 2 for even kx, ceil(Kw / 2) + kx / 2 for odd kx (each parity problem of the row
                     // GEMM then stores whole lines; kx_of_col maps back in the tile epilogue)
};

// tperm images: spectrum column kx of the parity-planar column n'
__host__ __device__ inline int kx_of_col(const ImgDesc& d, int n) {
  if (!d.tperm) return n;
  const int ne = (d.Kw + 1) >> 1;
  return n < ne ? 2 * n : 2 * (n - ne) + 1;
}
// ... and the column n' of spectrum column kx
__host__ __device__ inline int col_of_kx(const ImgDesc& d, int kx) {
  if (!d.tperm) return kx;
  return (kx & 1) ? ((d.Kw + 1) >> 1) + (kx >> 1) : (kx >> 1);
}

// Token staging position of flat token f = (h qw + w) 3 + c (FE:374-380 order,
// the sort's tie order): flat, or with tband bit 1 item-major (c qw + w) qh + h,
// so the 32 tokens of one column-kernel item (channel c, tile strip w) are
// contiguous staging (full cache lines from one workgroup instead of 28-byte
// pieces shared by the three channels' items on three XCDs).  C = 3.
__host__ __device__ inline int stage_pos(const ImgDesc& d, int f) {
  if (!(d.tband & 2)) return f;
  // band images have qh = qw = 32 (512 x 512 at max_patch 32 x 32): no runtime division
  const int c = f % 3, s = f / 3, h = s >> 5, w = s & 31;
  return ((c << 5) + w) * 32 + h;
}

// Generic batched strided fp32 GEMM problem:
//   O[c][m][n] = sum_k A[c][m][k] * B[c][n][k]     (c < C)
struct GemmProblem {
  const float* A;
  const float* B;
  float* O;
  int64_t sAc, sAm, sAk;
  int64_t sBc, sBn, sBk;
  int64_t sOc, sOm, sOn;
  int32_t M, N, K, C;
  int32_t tiles_n;   // ceil(N / tile_n)
  int32_t tile_m, tile_n;   // 64 x 64 (k_gemm_f32); k_gemm_x3: 128 along the shared operand
  // k_gemm_x3 only: the shared operand (B when only B is shared, else A)
  // pre-split into three bf16 planes [3][Rp][xs_ld] (Rp = rows rounded up to
  // 128, xs_ld = K rounded up to 32, zero padded); null = split in the kernel
  int32_t xs_ld;
  int32_t pad2;
  const uint16_t* Xs;
  int64_t xs_plane;  // Rp * xs_ld
  // k_gemm_h2 (encode DCT GEMMs, option gemm_h2): the shared operand as two
  // fp16 planes of the matrix scaled by 2^xh_exp [2][Rp][xs_ld]; amax = the
  // |max| bits (uint order of |x|) of the per-channel operand, written by the
  // kernel that produced it (k_rgb_to_ipt, k_fold_t, the row GEMM's omax);
  // omax (nullable) receives the |max| bits of this GEMM's outputs
  const uint16_t* Xh;
  const uint32_t* amax;
  uint32_t* omax;
  int32_t xh_exp;
  int32_t pad3;
};

// FFT-DCT plan for one length N (M = N/2 point complex FFT), dctae_fft.hip
struct FftPlan {
  int32_t N, M, npass, rows_per_block;
  int32_t radix[8];
  int32_t spec;  // compile-time specialised kernel id (dctae_fft2.hip), 0 = generic
  // odd N: M = N complex points of the real Makhoul sequence (imaginary parts
  // zero), X_k = Re(w_k Z_k) with w_k = s_k e^{-i pi k / (2N)} at post[2 k]
  int32_t odd;
  int64_t tw_off;    // float2 offset of W_M^k (k < M) in the FFT table buffer
  int64_t post_off;  // float2 offset of (alpha_k, beta_k), k = 0..M
  int64_t ipre_off;  // float2 offset of the DCT-III pre-processing table (conj a_k, conj b_k), k < M (dctae_idct.hip)
  // Bluestein plans (kind 1, dctae_bluestein.hip): any N in [32, 1024], L = 2^ceil(log2(2N - 1)) >= 256
  int32_t kind, bs_L;
  int64_t bs_tw_off;     // W_L^m, m < L
  int64_t bs_chirp_off;  // c[n] = e^{-i pi n^2 / N}, n < N
  int64_t bs_bhat_off;   // FFT_L(conj c) / L
  int64_t bs_post_off;   // e_k = s_k / 2 e^{-i pi k / (2N)}, k < N
};

struct TileRef {
  int32_t problem;
  int32_t tile;  // tm * tiles_n + tn
};

struct EncParams {
  int32_t P, C, maxph, maxpw, S;
  float ci[3];
  float mw;
  // PatchNorm (nullable median => no norm/codes)
  const float* median;
  const float* b;
  const float* thr;   // optional LFQ-bit thresholds (k_norm_thresholds), same shape
  float eps, min_val, max_val;
  // LFQ
  int32_t cb_dim, ncb;
  float scale;
  // index rule masks (lfq_index_bits): the staged u16 codes hold the raw sign
  // bits x > 0; the packing kernels map them (code_pos/code_neg: cb_dim bits)
  uint32_t code_pos, code_neg;
};

// The reference's LFQ index bit (lfq.py:174-187) is taken from the QUANTIZED
// value: q = where(x > 0, +s, -s), bit = q > 0.  With b = (x > 0) (NaN -> 0):
// bit = b ? (s > 0) : (-s > 0), i.e. b for s > 0, !b for s < 0 (NaN x -> 1),
// 0 for s == 0.  pos / neg = all-ones masks of the cb_dim code bits when
// s > 0 / -s > 0 (fp32 s, as the reference's ones_like(x) * s), else 0.
__host__ __device__ inline uint64_t lfq_index_bits(uint64_t b, uint64_t pos, uint64_t neg) {
  return (b & pos) | (~b & neg);
}
inline void lfq_index_masks(float s, int cb_dim, uint64_t* pos, uint64_t* neg) {
  const uint64_t full = cb_dim >= 64 ? ~0ull : ((1ull << cb_dim) - 1ull);
  *pos = s > 0.0f ? full : 0ull;
  *neg = -s > 0.0f ? full : 0ull;
}

struct TokenSinks {
  uint16_t* codes;   // (T, ncb) or null
  float* scores;     // (T)
  float* raw;        // (T, P*P) or null
  float* norm;       // (T, P*P) or null
};

struct PackSinks {
  int64_t* codes;     // (R,S,ncb)
  int64_t* pos;       // (R,S,2)
  int64_t* ch;        // (R,S)
  int64_t* ids;       // (R,S)
  float* patches;     // (R,S,PP) gathered from norm staging
  float* raw;         // (R,S,PP) gathered from raw staging
  float* scores;      // (R,S)
  uint8_t* key_pad;   // (R,S): k_sort_pack* write 0 at their tokens (k_pad_fill writes the rows' pads)
};

struct DecodeArgs {
  const int64_t* ids;       // (R,S)
  const uint8_t* key_pad;   // (R,S)
  const int64_t* pos;       // (R,S,2)
  const int64_t* ch;        // (R,S)
  const int64_t* codes;     // (R,S,ncb) when use_codes
  const float* patches;     // (R,S,PP) otherwise
  const int32_t* lut;       // (R, lut_w) row-local id -> image index (-1 = none)
  int32_t lut_w, S, P, use_codes;   // use_codes: 1 = codes, 0 = patches, 2 = PatchNorm-space patches (FFT path)
  int32_t cb_dim, ncb;
  float scale;
  const float* median;
  const float* b;
  float eps;
  int32_t maxph, maxpw;
  int* err;
};

}  // namespace dctae
