// Host-side launch wrappers of the kernels in dctae_kernels.hip / dctae_fft.hip.
#pragma once
#include <algorithm>
#include <cstring>
#include <vector>

#include "dctae_internal.h"

namespace dctae {

void launch_synth(uint64_t seed, int64_t first, int32_t n_img, int32_t H, int32_t W, float* out, hipStream_t s);
int rgb_to_ipt_groups_per_block();
// amax (nullable): per job-local image, [2 i] receives the |max| bits of the folded IPT (k_gemm_h2)
void launch_rgb_to_ipt(const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                       const ColorMats& cm, uint32_t* amax, hipStream_t s);
void launch_ipt_to_rgb(const ImgDesc* imgs, int n_img, int64_t max_hw, const float* ws, float* out,
                       const ColorMats& cm, hipStream_t s);
void launch_color(const float* x, float* y, int64_t hw, int n_img, int dir, const ColorMats& cm, hipStream_t s);
// amax (nullable): [2 i + 1] receives the |max| bits of the folded T (k_gemm_h2)
void launch_fold_t(const ImgDesc* imgs, const int32_t* list, int n_list, int64_t max_hw, float* ws, uint32_t* amax,
                   hipStream_t s);
// share: 1 = B shared by the channels (row transforms), 2 = A shared (column
// transforms), 0 = from each problem's strides; must hold for every problem the
// tiles reference (gemm_share of one of them)
int gemm_share(const GemmProblem& g);
void launch_gemm(int nc, const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share = 0);
// the same GEMM on the bf16 MFMA with three-piece operand splits (fp32 accuracy, k_gemm_x3)
void launch_gemm_x3(int nc, const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share = 0);
// three bf16 planes [3][Rp][Kp] of a row-major fp32 matrix (GemmProblem::Xs)
void split_matrix_x3(const float* m, int R, int K, std::vector<uint16_t>& out, int* Rp, int* Kp);
// the encode's DCT GEMMs on fp16 MFMAs, two-piece scaled operands (k_gemm_h2; 3 channels, share 1 or 2)
// colour transform + folds + row GEMM of the tperm images (k_rows_fused), or
// the fix-up of the images it flagged; tiles = (even-parity row problem, block
// of row pairs), the odd parity's problem next to it
int fused_pairs_per_block();
int fused_max_n();
void launch_rows_fused(const GemmProblem* probs, const TileRef* tiles, int n_tiles, const ImgDesc* imgs,
                       const float* rgb, const ColorMats& cm, uint32_t* amax, int* flags, int n_img, hipStream_t s,
                       bool fixup);
// share 1 (the encode's row GEMM: A k-contiguous, sAm > 0): dma = k_gemm_h2r
// share 2 (the encode's column GEMM: B = T, sBn = 1): dma_cols = k_gemm_h2c
void launch_gemm_h2(const GemmProblem* probs, const TileRef* tiles, int n_tiles, hipStream_t s, int share, bool dma,
                    bool dma_cols);
void split_matrix_h2(const float* m, int R, int K, std::vector<uint16_t>& out, int* Rp, int* Kp, int* e_out);
void launch_tile_epilogue(const ImgDesc* imgs, int n_img, int max_T, const float* ws, const EncParams& ep,
                          const TokenSinks& sk, hipStream_t s, const int2* list = nullptr, int n_list = 0);
void launch_sort_pack(const ImgDesc* imgs, int n_img, int np2, const EncParams& ep, const TokenSinks& st,
                      const PackSinks& out, hipStream_t s, int kernel = 1, int max_T = 1 << 30);
void launch_pad_fill(const int32_t* row_len, int n_rows, const EncParams& ep, uint8_t* key_pad,
                     const PackSinks& out, hipStream_t s);
void launch_norm(const float* x, const int64_t* ch, const int64_t* pos, int64_t n, int PP, int maxph, int maxpw,
                 const float* med, const float* b, float eps, float lo, float hi, int inverse, float* y, int* err,
                 hipStream_t s);
void launch_lfq_forward(const float* x, int64_t n, int cb_dim, int ncb, float scale, float* q, int64_t* idx,
                        hipStream_t s);
void launch_lfq_codes(const int64_t* idx, int64_t n, int cb_dim, int ncb, float scale, float* out, hipStream_t s);
// dctae_lfq_proj.hip: LFQ with projections, fused project_in + sign + pack / codes + project_out
// wsp: scratch of lfq_proj_scratch_bytes(out features, in features) for the pre-split weight
size_t lfq_proj_scratch_bytes(int N, int K);
void launch_lfq_project_in(const float* x, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                           float scale, int64_t* idx, uint16_t* wsp, hipStream_t s, float x_bound = 0.f,
                           bool ws = false);
void launch_lfq_project_in16(const float* x, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                             uint16_t* idx, uint16_t* wsp, hipStream_t s,
                             float x_bound = 0.f, bool ws = false);
void launch_lfq_project_out(const int64_t* idx, int64_t n, int D, const float* w, const float* b, int cd, int ncb,
                            float scale, float* out, uint16_t* wsp, hipStream_t s, const int64_t* ch = nullptr,
                            const int64_t* pos = nullptr, const float* med = nullptr, const float* nb = nullptr,
                            float eps = 0.f, int maxph = 0, int maxpw = 0, int* err = nullptr, bool h2 = true,
                            bool ws = false);
// dctae_lfq_ws.hip: the W-stationary form of the two (fp16 pieces; 192 < K <= 208, 192 < N <= 224)
bool lfq_ws_fits(int mode, int K, int N, int cd, int ncb);
void launch_lfq_ws(int mode, hipStream_t s, const float* x, const int64_t* idx_in, int64_t n, int K, int N,
                   const float* bias, int cd, int ncb, float scale, int64_t* idx_out, float* out, uint16_t* idx16,
                   const int64_t* ch, const int64_t* pos, const float* med, const float* nb, float eps, int maxph,
                   int maxpw, int* err, const uint16_t* wsp, int NPw, int Kp, float a_scale);
// VectorQuantize inference (dctae_vq.hip)
void launch_vq_bias(float* y, const float* bias, int64_t n, int cols, const uint8_t* mask, const float* orig,
                    hipStream_t s);
void launch_vq_stats(const float* xp, const uint8_t* mask, int64_t n_tok, int heads, double* acc, hipStream_t s);
void launch_vq_codebook(const double* acc, float* bm, float* bv, int32_t* init, float decay, int affine,
                        const float* embed, const float* cm, const float* cv, int C, float* et, float* y2,
                        hipStream_t s);
void launch_vq_assign(const float* xp, int64_t nv, int heads, const float* et, const float* y2, int C, float* xq,
                      int64_t* ind, hipStream_t s);
void launch_vq_codes(const int64_t* ind, int64_t nv, const float* embed, int C, float* out, int* err, hipStream_t s);
void launch_scatter_tokens(int64_t n_tok, const ImgDesc* imgs, float* ws, const DecodeArgs& a, const int32_t* map,
                           hipStream_t s);

// PatchNorm training statistics (dctae_stats.hip)
void launch_stats_lists(const int64_t* ch, const int64_t* pos, const uint8_t* key_pad, int64_t n_tok, int C, int mh,
                        int mw, int32_t* cell, int32_t* count, int32_t* start, int32_t* list, int* err, hipStream_t s);
void launch_stats_median(const float* x, int PP, int n_cells, const int32_t* start, const int32_t* count,
                         const int32_t* list, float* batch_median, float* batch_n, hipStream_t s);
void launch_stats_batch_b(const float* x, int PP, int n_cells, const int32_t* start, const int32_t* count,
                          const int32_t* list, const float* median, float* batch_b, hipStream_t s);
void launch_stats_merge(float* t, const float* src, const float* n, const float* bn, int n_cells, int PP,
                        hipStream_t s);
void launch_stats_add(float* n, const float* bn, int n_cells, hipStream_t s);
void launch_zero_pads(const float* x, const uint8_t* key_pad, int64_t n_tok, int PP, float* y, hipStream_t s);

size_t fft_kernel_setup(int device);
void launch_fft_rows(const ImgDesc* imgs, const FftPlan* plans, const int2* blocks, int n_blocks, size_t lds,
                     const float* rgb, float* ws, const float2* tabs, const ColorMats& cm, hipStream_t s);
void launch_fft_cols(const ImgDesc* imgs, const FftPlan* plans, const int4* blocks, int n_blocks, size_t lds,
                     const float* ws, const float2* tabs, const EncParams& ep, const TokenSinks& sk, hipStream_t s);
void launch_norm_thresholds(const float* med, const float* b, int64_t n, float eps, float lo, float hi, float* thr,
                            int* bad, hipStream_t s);

int fft_spec_id(int N, const int* radix, int npass, int P);
int fft_spec_rows_per_block(int spec);
void launch_fft_rows_spec(int spec, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                          const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s);
void launch_fft_cols_spec(int spec, const ImgDesc* imgs, const int4* blocks, int n_blocks, const float* ws,
                          const float2* tw, const float2* post, const EncParams& ep, const TokenSinks& sk,
                          hipStream_t s, const int* list, int n_list, int qw);

// decode on the FFT path (dctae_idct.hip)
void launch_dec_map(int64_t n_tok, const ImgDesc* imgs, const DecodeArgs& a, int32_t* map, hipStream_t s);
void launch_idct_cols512b(const ImgDesc* imgs, int n_img, float* ws, const int32_t* map, const float2* tw,
                          const float4* pre, const DecodeArgs& a, hipStream_t s);
void launch_idct_cols512(const ImgDesc* imgs, int n_img, int qw, float* ws, const int32_t* map, const float2* tw,
                         const float4* pre, const DecodeArgs& a, hipStream_t s);
void launch_idct_rows_spec(int spec, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* ws,
                           float* rgb, const float2* tw, const float4* pre, const ColorMats& cm, hipStream_t s);

void launch_idct_rows512(bool band, const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* ws, float* rgb,
                         const float2* tw, const float4* pre, const ColorMats& cm, hipStream_t s);
void launch_rows512(const ImgDesc* imgs, const int2* blocks, int n_blocks, const float* rgb, float* ws,
                    const float2* tw, const float2* post, const ColorMats& cm, hipStream_t s);

int cols7_grid(int n_list, int qw, int ipb);
// band-layout column pass of 512 x 512 images (k_cols512b; the rows wrote T' with band = 1)
void launch_cols512b(const ImgDesc* imgs, const int* list, int n_list, const float* ws, const float2* tw,
                     const float2* post, const EncParams& ep, const TokenSinks& sk, hipStream_t s,
                     bool wide = false);

// Bluestein DCT for lengths without a Makhoul plan (dctae_bluestein.hip)
int bs_rows_per_block(int L);
int bs_cols_per_block(int L);
void launch_bs_rows(int L, const ImgDesc* imgs, const FftPlan* plans, const int2* blocks, int n_blocks,
                    const float* rgb, float* ws, const float2* tabs, const ColorMats& cm, hipStream_t s,
                    int ablate = 0);
void launch_bs_cols(int L, const ImgDesc* imgs, const FftPlan* plans, const int4* blocks, int n_blocks, float* ws,
                    const float2* tabs, hipStream_t s, int ablate = 0);

}  // namespace dctae
