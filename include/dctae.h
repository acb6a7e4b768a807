/*
 * dctae.h — C ABI of libdctae.so, the MI355X (gfx950) implementation of the
 * dct-autoencoder feature-extraction hot path:
 *
 *   RGB -> IPT -> global orthonormal DCT-II -> 14x14 spectral tiles ->
 *   importance order -> packing -> PatchNorm -> LFQ codes          (encode)
 *   LFQ codes -> +-1 -> inverse PatchNorm -> unpatch -> DCT-III -> RGB (decode)
 *
 * The reference (theAdamColton/dct-autoencoder) has no native boundary: its
 * operator API is the Python class surface.  Each entry point below states
 * the reference function(s) it replaces (paths relative to the reference
 * repo; FE = dct_autoencoder/feature_extraction_dct_autoencoder.py).  The
 * Python layer in dct-autoencoder_amd/ mirrors the reference classes and is
 * the only intended caller; INTEGRATION.md shows the ctypes binding.
 *
 * Conventions
 *  - Every pointer argument named *_dev is HIP device memory owned by the
 *    caller; the library never frees or retains it past the call.
 *  - All work is enqueued on `stream` (a hipStream_t, passed as void*; NULL =
 *    legacy default stream).  The library never synchronises the host, except
 *    when it must grow its internal workspace or upload a new plan.
 *  - Every call returns 0 on success and a negative DCTAE_E* code on error;
 *    dctae_last_error(ctx) describes the last error of that context.
 *  - One context per device per host thread (not re-entrant).
 *  - Integer outputs that the reference returns as torch.long are int64.
 */
#ifndef DCTAE_H
#define DCTAE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCTAE_OK 0
#define DCTAE_EINVAL (-1)   /* bad argument / shape (reference: AssertionError) */
#define DCTAE_EHIP (-2)     /* HIP runtime error */
#define DCTAE_ENOMEM (-3)   /* workspace allocation failed */
#define DCTAE_EUNSUP (-4)   /* unsupported configuration */

#define DCTAE_ABI_VERSION 1

typedef struct dctae_ctx dctae_ctx;

/* DCTAutoencoderFeatureExtractor.__init__ arguments (FE:108-127). */
typedef struct {
  int32_t channels;               /* must be 3 (IPT colour transform, util.py:70-97) */
  int32_t patch_size;             /* P, 2..16 (reference configs use 14) */
  int32_t max_patch_h;            /* 32 */
  int32_t max_patch_w;            /* 32 */
  int32_t max_seq_len;            /* S */
  float channel_importances[3];   /* (8, 1, 1) */
  float magnitude_weight;         /* patch_sample_magnitude_weight, 0.1 */
} dctae_fe_cfg;

/* Frozen/eval PatchNorm state (patchnorm.py:32-78): tables of shape
 * (channels, max_patch_h, max_patch_w, P*P), fp32, device. */
typedef struct {
  const float* median_dev;
  const float* b_dev;
  float eps;        /* 1e-6 */
  float min_val;    /* -6 */
  float max_val;    /*  6 */
  /* optional (NULL): LFQ-bit thresholds from dctae_norm_thresholds; when
   * set, codes-only encodes compare x >= thr instead of normalising */
  const float* thr_dev;
} dctae_norm;

/* LFQ without projections (lfq.py:35-96): codebook_dim * num_codebooks must
 * equal the token dim (P*P); codebook_dim <= 16. */
typedef struct {
  int32_t codebook_dim;   /* log2(codebook_size) */
  int32_t num_codebooks;
  float codebook_scale;   /* 1.0 */
} dctae_lfq;

/* Images: `n_img` fp32 RGB images of shape (3, H_i, W_i), contiguous, at
 * element offsets img_off[i] of rgb_dev (host arrays). */
typedef struct {
  const float* rgb_dev;
  const int64_t* img_off;   /* host, n_img */
  const int32_t* hw;        /* host, 2*n_img: H0,W0,H1,W1,... */
  int32_t n_img;
} dctae_images;

/* Packing of images into rows of length S (host arrays, n_img entries each),
 * produced by the host mirror of FE._group_patches_by_max_seq_len /
 * _batch_groups (FE:454-605): image i occupies row[i], positions
 * [col[i], col[i]+k[i]) and has image id local_id[i] inside its row.
 * row_len (host, n_rows) = tokens used in each row (key_pad_mask = j >= len). */
typedef struct {
  const int32_t* row;
  const int32_t* col;
  const int32_t* k;
  const int32_t* local_id;
  const int32_t* row_len;
  int32_t n_rows;
} dctae_packing;

/* Packed DCTPatches fields (dct_patches.py:6-51), device, rows x S. */
typedef struct {
  int64_t* codes_dev;        /* (R, S, num_codebooks) LFQ indices (lfq.py:187) */
  int64_t* positions_dev;    /* (R, S, 2)  patch_positions [h, w]            */
  int64_t* channels_dev;     /* (R, S)     patch_channels                    */
  int64_t* image_ids_dev;    /* (R, S)     batched_image_ids                 */
  uint8_t* key_pad_dev;      /* (R, S)     key_pad_mask (True = padding)     */
  float* patches_dev;        /* (R, S, P*P) optional (NULL): PatchNorm output */
  float* raw_patches_dev;    /* (R, S, P*P) optional (NULL): DCT tokens       */
  float* scores_dev;         /* (R, S)     optional (NULL): importance score  */
} dctae_packed_out;

int dctae_abi_version(void);
int dctae_ctx_create(int device, dctae_ctx** out);
int dctae_ctx_destroy(dctae_ctx* ctx);
const char* dctae_last_error(dctae_ctx* ctx);

/* Colour matrices (row-major 3x3 fp32) used by the IPT transforms; the
 * Python layer passes the reference's exact fp32 values (util.py:40-41, 91:
 * Trgb2lms = MHPE @ MsRGB, Tlms2rgb = Trgb2lms.inverse(), Mipt, Mipt.inverse()).
 * Defaults are the same matrices computed in float64 and rounded. */
int dctae_set_color_matrices(dctae_ctx* ctx, const float* rgb2lms, const float* lms2ipt,
                             const float* ipt2lms, const float* lms2rgb);

/* Fused encode: FE.preprocess for every image (FE:154-177: rgb_to_ipt,
 * dct2, _crop_image, _patch_image) + FE._batch_groups (FE:515-605) +
 * PatchNorm.forward eval (patchnorm.py:157-165) + LFQ.forward eval
 * (lfq.py:136-227).  Token order inside an image: score desc, flat index asc.
 * norm may be NULL (then codes_dev must be NULL: only tokens/metadata). */
int dctae_encode(dctae_ctx* ctx, const dctae_fe_cfg* cfg, const dctae_images* imgs,
                 const dctae_packing* pack, const dctae_norm* norm, const dctae_lfq* lfq,
                 const dctae_packed_out* out, void* stream);

/* Spectrum tokens of each image in flat order f = (h*qw + w)*3 + c, plus the
 * importance scores (FE:364-416) — the part of FE.preprocess before sorting.
 * tokens_dev: (sum_i T_i, P*P) fp32; scores_dev: (sum_i T_i); tok_off (host,
 * n_img): first token row of each image. */
int dctae_spectrum_tokens(dctae_ctx* ctx, const dctae_fe_cfg* cfg, const dctae_images* imgs,
                          const int64_t* tok_off, float* tokens_dev, float* scores_dev, void* stream);

/* FE._transform_image_in / _transform_image_out (FE:129-152) on n_img
 * contiguous (3, H, W) fp32 images: direction 0 = dct2(rgb_to_ipt(x)),
 * direction 1 = ipt_to_rgb(idct2(x)); color = 0 skips the colour transform
 * (util.dct2 / util.idct2 alone, util.py:333-338); forward only: color = 2 / 3
 * runs rgb_to_ipt in fp16 / bf16 arithmetic, as the reference does for an
 * input of that dtype (FE:135 transforms before x.float()), x then holding
 * the dtype's values as fp32.  Orthonormal DCT-II / III
 * over the whole H x W (no crop).  x_dev and y_dev must not alias. */
int dctae_dct2(dctae_ctx* ctx, const float* x_dev, int32_t n_img, int32_t H, int32_t W, int32_t direction,
               int32_t color, float* y_dev, void* stream);

/* FE._patch_image (FE:364-452) of one cropped spectrum x (3, H, W), H and W
 * multiples of patch_size: 14x14 tiles of the kept corner (max_patch_h/w),
 * importance scores, order (score desc, flat index asc), top k.  Outputs:
 * patches (k, P*P) fp32, positions (k, 2) int64 [h, w], channels (k) int64,
 * scores (k) fp32 (nullable). */
int dctae_patch_spectrum(dctae_ctx* ctx, const dctae_fe_cfg* cfg, const float* x_dev, int32_t H, int32_t W,
                         int32_t k, float* patches_dev, int64_t* positions_dev, int64_t* channels_dev,
                         float* scores_dev, void* stream);

/* PatchNorm.forward, eval/frozen (patchnorm.py:157-165) on n tokens of dim
 * P*P with their channel / position (int64 device arrays). Pad tokens are
 * normalised like the reference does (with c=h=w=0). */
int dctae_norm_forward(dctae_ctx* ctx, const dctae_norm* norm, int32_t P, int32_t max_patch_h,
                       int32_t max_patch_w, const float* x_dev, const int64_t* channels_dev,
                       const int64_t* positions_dev, int64_t n, float* y_dev, void* stream);

/* PatchNorm.inverse_norm (patchnorm.py:167-177): y*std + median, no FMA. */
int dctae_norm_inverse(dctae_ctx* ctx, const dctae_norm* norm, int32_t P, int32_t max_patch_h,
                       int32_t max_patch_w, const float* y_dev, const int64_t* channels_dev,
                       const int64_t* positions_dev, int64_t n, float* x_dev, void* stream);

/* PatchNorm training statistics of one packed batch of n_tok tokens
 * (patchnorm.py:101-130; replaces the reference's scatter_add_3d + per-cell
 * torch.median loop).  key_pad_dev (n_tok bytes, nullable) marks padding.
 * batch_n_dev: (C*mh*mw) fp32 token counts; batch_median_dev: (C*mh*mw, P*P)
 * lower median per cell (0 for empty cells).  Bit-exact with the reference. */
int dctae_norm_batch_stats(dctae_ctx* ctx, int32_t P, int32_t C, int32_t max_patch_h, int32_t max_patch_w,
                           const float* x_dev, const int64_t* channels_dev, const int64_t* positions_dev,
                           const uint8_t* key_pad_dev, int64_t n_tok, float* batch_n_dev,
                           float* batch_median_dev, void* stream);

/* Mean absolute deviation of the batch around the (already merged) running
 * median (patchnorm.py:140-144): batch_b = sum_{tokens, batch order}
 * |x - median| / clamp(batch_n, 1). */
int dctae_norm_batch_mad(dctae_ctx* ctx, int32_t P, int32_t C, int32_t max_patch_h, int32_t max_patch_w,
                         const float* x_dev, const int64_t* channels_dev, const int64_t* positions_dev,
                         const uint8_t* key_pad_dev, int64_t n_tok, const float* median_dev, float* batch_b_dev,
                         void* stream);

/* Running merge (patchnorm.py:135-138 / 146-148): per cell,
 * table <- (table*n + batch*batch_n) / clamp(n + batch_n, 1); then, if
 * n_update, n <- n + batch_n (patchnorm.py:150). */
int dctae_norm_merge(dctae_ctx* ctx, int32_t n_cells, int32_t PP, float* table_dev, const float* batch_dev,
                     float* n_dev, const float* batch_n_dev, int32_t n_update, void* stream);

/* One PatchNorm training forward (patchnorm.py:101-155, not frozen):
 * updates norm->median_dev, norm->b_dev and n_dev (C*mh*mw) in place;
 * y_dev (nullable) = x with padding rows zeroed. */
int dctae_norm_train_step(dctae_ctx* ctx, const dctae_norm* norm, float* n_dev, int32_t P, int32_t C,
                          int32_t max_patch_h, int32_t max_patch_w, const float* x_dev, const int64_t* channels_dev,
                          const int64_t* positions_dev, const uint8_t* key_pad_dev, int64_t n_tok, float* y_dev,
                          void* stream);

/* LFQ.forward eval (lfq.py:136-227): quantized (n, dim) = +-scale (nullable)
 * and indices (n, num_codebooks) int64. */
int dctae_lfq_forward(dctae_ctx* ctx, const dctae_lfq* lfq, const float* x_dev, int64_t n,
                      float* quantized_dev, int64_t* indices_dev, void* stream);

/* LFQ.indices_to_codes (lfq.py:105-134), project_out = identity. */
int dctae_lfq_indices_to_codes(dctae_ctx* ctx, const dctae_lfq* lfq, const int64_t* indices_dev,
                               int64_t n, float* codes_dev, void* stream);

/* dctae_encode for an LFQ with projections (lfq.py:54-62; conf/patch14-l.json:
 * 196 -> 16 x 13): the column epilogues stage the PatchNorm output, the fused
 * project_in + sign + pack kernel (below) turns the staged tokens into staged
 * codes, and the sort / pack writes them like dctae_encode's.  w_in (ncb*cd,
 * P*P) / b_in (ncb*cd, nullable) fp32 as nn.Linear stores them.  codebook_dim
 * <= 16, ncb*cd <= 256; rows without padding (every packed row full, e.g. the
 * fixed-geometry BatchEncoder), else DCTAE_EUNSUP. */
int dctae_encode_lfq_proj(dctae_ctx* ctx, const dctae_fe_cfg* cfg, const dctae_images* imgs,
                          const dctae_packing* pack, const dctae_norm* norm, const dctae_lfq* lfq,
                          const float* w_in_dev, const float* b_in_dev, const dctae_packed_out* out, void* stream);

/* LFQ with projections (lfq.py:54-62, dim != codebook_dim * num_codebooks),
 * encode direction: LFQ.forward's indices (lfq.py:164 project_in, :175-187
 * sign + packing) in one fused MFMA kernel: x (n, dim) fp32, w_in (ncb*cd,
 * dim) and b_in (ncb*cd, nullable) as nn.Linear stores them -> indices (n,
 * ncb) int64.  dim % 4 == 0, ncb*cd <= 256, cd <= 31; 16-byte aligned x / w. */
int dctae_lfq_project_in(dctae_ctx* ctx, const dctae_lfq* lfq, const float* x_dev, int64_t n, int32_t dim,
                         const float* w_in_dev, const float* b_in_dev, int64_t* indices_dev, void* stream);

/* The same for an x the caller bounds, |x| <= x_bound (NaN aside), e.g. the
 * PatchNorm output (clamped to [min_val, max_val], patchnorm.py:163) that
 * DCTAutoencoderFeatureExtractor.encode_batch projects: the operand then
 * scales exactly into the fp16 range and the projection runs on the fp16
 * two-piece MFMA kernels -- the ones dctae_encode_lfq_proj uses on its staged
 * tokens, so both give the same codes (option "gemm_h2" 0: the split-bf16
 * kernel of dctae_lfq_project_in).  x_bound > 0 and finite. */
int dctae_lfq_project_in_bounded(dctae_ctx* ctx, const dctae_lfq* lfq, const float* x_dev, int64_t n, int32_t dim,
                                 const float* w_in_dev, const float* b_in_dev, float x_bound, int64_t* indices_dev,
                                 void* stream);

/* Decode direction: LFQ.indices_to_codes with project_out (lfq.py:105-127):
 * indices (n, ncb) -> +-scale codes -> out (n, dim) = codes w_out^T + b_out,
 * w_out (dim, ncb*cd), b_out (dim, nullable).  dim <= 256, ncb*cd % 4 == 0,
 * ncb <= 32, cd <= 31. */
int dctae_lfq_project_out(dctae_ctx* ctx, const dctae_lfq* lfq, const int64_t* indices_dev, int64_t n, int32_t dim,
                          const float* w_out_dev, const float* b_out_dev, float* out_dev, void* stream);

/* The same with PatchNorm.inverse_norm (patchnorm.py:167-177) fused into the
 * epilogue: out = inverse_norm(codes w_out^T + b_out) at each token's
 * (channel, h, w) table row; dim = P*P.  Out-of-range table indices write NaN
 * and set the device error flag (dctae_check_device_errors), like
 * dctae_norm_inverse. */
int dctae_lfq_project_out_inverse_norm(dctae_ctx* ctx, const dctae_lfq* lfq, const int64_t* indices_dev, int64_t n,
                                       int32_t dim, const float* w_out_dev, const float* b_out_dev,
                                       const dctae_norm* norm, int32_t max_patch_h, int32_t max_patch_w,
                                       const int64_t* channels_dev, const int64_t* positions_dev, float* out_dev,
                                       void* stream);

/* VectorQuantize (vector_quantize.py:675-1050) as the model builds it
 * (modeling_dct_autoencoder.py:76-77): euclidean codebook shared by the
 * heads, codebook_dim 16, kmeans-initialised, affine codebook parameters,
 * eval (inference) mode.  Weights are fp32 device tensors with torch's
 * layouts; w_in/b_in/w_out/b_out are NULL when dim == heads * codebook_dim
 * (project_in/out = Identity, vector_quantize.py:727-728).  The batch affine
 * statistics are state the forward updates even in eval
 * (vector_quantize.py:353-359): batch_mean/batch_variance (codebook_dim
 * floats each) and *batch_initted_dev (0 until the first forward). */
typedef struct {
  int32_t dim;
  int32_t heads;
  int32_t codebook_dim;     /* 16 */
  int32_t codebook_size;
  int32_t affine;           /* affine_param (the model sets True) */
  float affine_decay;       /* affine_param_batch_decay, 0.99 */
  const float* w_in_dev;    /* (heads*codebook_dim, dim) */
  const float* b_in_dev;    /* (heads*codebook_dim) */
  const float* w_out_dev;   /* (dim, heads*codebook_dim) */
  const float* b_out_dev;   /* (dim) */
  const float* embed_dev;   /* _codebook.embed (1, codebook_size, codebook_dim) */
  const float* codebook_mean_dev;      /* (codebook_dim) */
  const float* codebook_variance_dev;  /* (codebook_dim) */
  float* batch_mean_dev;               /* in/out state (codebook_dim) */
  float* batch_variance_dev;           /* in/out state (codebook_dim) */
  int32_t* batch_initted_dev;          /* in/out state: 0 -> first forward sets the statistics */
} dctae_vq;

/* VectorQuantize.forward, eval (vector_quantize.py:855-1050): x (n_tok, dim)
 * fp32 (the reference's (b, n, dim) flattened), optional mask (n_tok) u8
 * (NULL = all valid).  Writes quantize (n_tok, dim) = where(mask,
 * project_out(codes), x) (nullable) and indices (n_tok, heads) int64
 * ('b n h').  Updates the batch statistics in place. */
int dctae_vq_forward(dctae_ctx* ctx, const dctae_vq* vq, const float* x_dev, const uint8_t* mask_dev,
                     int64_t n_tok, float* quantize_dev, int64_t* indices_dev, void* stream);

/* VectorQuantize.get_codes_from_indices (vector_quantize.py:820-841), shared
 * codebook: the raw codebook rows, (n, heads * codebook_dim) for indices
 * (n, heads).  Out-of-range indices raise (DCTAE_EINVAL via
 * dctae_check_device_errors) like the reference's IndexError. */
int dctae_vq_codes_from_indices(dctae_ctx* ctx, const dctae_vq* vq, const int64_t* indices_dev, int64_t n,
                                float* codes_dev, void* stream);

/* VectorQuantize.get_output_from_indices (vector_quantize.py:833-836):
 * project_out(get_codes_from_indices(indices)), (n, dim). */
int dctae_vq_output_from_indices(dctae_ctx* ctx, const dctae_vq* vq, const int64_t* indices_dev, int64_t n,
                                 float* out_dev, void* stream);

/* Decode of a packed batch back to RGB: FE.postprocess (FE:289-310) =
 * revert_patching (FE:607-656) -> zero pad to (3,H,W) -> idct2 -> ipt_to_rgb.
 * With codes_dev != NULL the tokens are first LFQ.indices_to_codes
 * (lfq.py:105-134) then PatchNorm.inverse_norm (patchnorm.py:167-177), i.e.
 * DCTAutoencoder.decode_from_codes + inv_normalize_ without the transformer;
 * with codes_dev == NULL the (un-normalised) patches_dev are used as is.
 * Images are enumerated row by row and, inside a row, by ascending image id
 * (FE:628 image_ids.unique()).  img_lut (host, n_rows x lut_w) maps
 * (row, image id) -> image index (or -1); out_hw / out_off / patch_hw (host,
 * per image) give the original size, the output element offset in rgb_dev
 * and the (uncapped) patch_sizes. */
int dctae_decode(dctae_ctx* ctx, const dctae_fe_cfg* cfg, int32_t n_rows, const int32_t* img_lut,
                 int32_t lut_w, int32_t n_img, const int32_t* out_hw, const int64_t* out_off,
                 const int32_t* patch_hw, const int64_t* image_ids_dev, const uint8_t* key_pad_dev,
                 const int64_t* positions_dev, const int64_t* channels_dev, const dctae_norm* norm,
                 const dctae_lfq* lfq, const int64_t* codes_dev, const float* patches_dev,
                 float* rgb_dev, void* stream);

/* dctae_decode of PatchNorm-space patches (PatchNorm outputs, e.g. the LFQ
 * project_out of codes, lfq.py:126-134 / dctae_lfq_project_out): the
 * PatchNorm.inverse_norm (patchnorm.py:167-177) runs inside the decode --
 * on 512 x 512 images in the FFT column kernel with the tile's (median, std)
 * rows held per block (the same fp32 ops as dctae_norm_inverse, so the result
 * equals dctae_norm_inverse followed by dctae_decode bit for bit), on other
 * geometries as dctae_norm_inverse into the context's staging buffer first.
 * Replaces inv_normalize_ (modeling_dct_autoencoder.py:122-127) + the
 * processor's postprocess (FE:289-310) after LFQ.indices_to_codes with
 * projections (the codes path: dctae_decode with codes_dev). */
int dctae_decode_normed(dctae_ctx* ctx, const dctae_fe_cfg* cfg, int32_t n_rows, const int32_t* img_lut,
                        int32_t lut_w, int32_t n_img, const int32_t* out_hw, const int64_t* out_off,
                        const int32_t* patch_hw, const int64_t* image_ids_dev, const uint8_t* key_pad_dev,
                        const int64_t* positions_dev, const int64_t* channels_dev, const dctae_norm* norm,
                        const float* normed_patches_dev, float* rgb_dev, void* stream);

/* thr[e] = the smallest fp32 x with PatchNorm(x)[e] > 0, for the n table
 * elements (patchnorm.py:157-165 is monotone in x for a positive std), so
 * that the LFQ bit of a token element is exactly (x >= thr[e]); NaN = never.
 * Synchronises `stream`. */
int dctae_norm_thresholds(dctae_ctx* ctx, const dctae_norm* norm, int64_t n, float* thr_dev,
                          void* stream);

/* Route lengths with an FFT plan through the FFT-DCT kernels (default 1);
 * 0 forces the MFMA GEMM DCT for every size (A/B and parity testing). */
int dctae_set_fft(dctae_ctx* ctx, int enable);

/* Target workspace bytes per chunk of FFT-path images (default: unlimited,
 * one chunk; smaller chunks keep the row-pass output Infinity-Cache resident
 * but measured slower on MI355X because of the extra launch boundaries). */
int dctae_set_chunk_bytes(dctae_ctx* ctx, int64_t bytes);

/* Tuning / test knobs.  Each one selects between kernels that the library
 * also runs by default for other shapes, so every setting gives outputs
 * within the parity tolerances of DESIGN.md section 6 (bit-identical packing
 * metadata; tokens within 1e-6 x max|Y|; codes equal outside the guard band):
 * "fft" (0/1), "fft_spec" (0/1: compile-time specialised FFT kernels),
 * "bluestein" (0/1, default 0: sides in [32, 1024] without a Makhoul plan on
 * the Bluestein FFT instead of the MFMA GEMM; measured slower at these
 * sizes), "chunk_bytes", "workspace_limit" (bytes),
 * "rows_kernel" (4, default: k_rows512pk for 512-wide rows; 2: the general
 * compile-time plan kernel k_fft_rows2, which serves max_patch_w < 32),
 * "cols512b" (1, default: 512 x 512 images at max_patch 32 x 32 pass the
 * row-pass output in the band16 layout T'[c][y/16][kx][16] from k_rows512pk
 * to k_cols512b; 0: row-major T and k_fft_cols7), "sort_overlap" (0,
 * default / 1: a batch of >= 64 such images runs its column pass in two
 * halves and the first half's sort / pack on a context-owned side stream
 * beside the second half; the caller's stream waits for it, outputs
 * bit-identical),
 * "sort_kernel" (2, default: rocPRIM radix for <= 3072 tokens per image; 1:
 * the bitonic kernel that serves larger images), "fft_decode" (0/1),
 * "xcd_order" (0/1), "dec_rows_kernel" (3 / 2), "dec_cols_kernel" (2,
 * default: k_idct_cols512b writing the band-layout U for k_idct_rows512; 1:
 * k_idct_cols512, row-major U), "gemm_x3" (1, default: the DCT GEMMs on the
 * split-bf16 MFMA kernel k_gemm_x3, fp32-level accuracy; 0: the fp32 MFMA
 * kernel), "gemm_h2" (1, default: the encode's DCT GEMMs and the fused LFQ
 * projections on fp16 MFMAs with two-piece operands scaled by powers of two
 * (k_gemm_h2 / k_lfq_proj_h2: tokens within 5e-7 x max|Y|); 0: split-bf16),
 * "halves" (0, default / 1: a batch of >= 32 images of one size whose rows
 * and columns each run one compile-time plan kernel, e.g. 224 x 224, runs its
 * first half's columns and sort / pack on the side stream beside the second
 * half's rows and columns; outputs bit-identical; measured slower),
 * "cols_wide" (0, default / 1: the codes-only column pass of 512 x 512 band
 * images on k_cols512w, two tile strips per 7-wave block; bit-identical;
 * measured slower), "lfq_ws" (1, default: the fp16 LFQ projections of the
 * conf/patch14-l.json shapes (196 -> 208 project_in, 208 -> 196 project_out)
 * on the W-stationary kernel k_lfq_ws; 0: k_lfq_proj_h2), "fft_odd" (0,
 * default / 1: odd 7-smooth sides N <= 256 on the generic FFT kernels in the
 * real-FFT form, M = N; tokens within 2e-6 x max|Y| of the oracle; measured
 * slower than the MFMA GEMM DCT on the ragged batch; needs "fft_generic"),
 * "fft_generic" (0, default / 1: 7-smooth sides without a compile-time
 * kernel -- every N but 512 and 224 -- on the generic LDS Stockham FFT
 * kernels instead of the MFMA GEMM DCT; measured slower on every shape tried),
 * "tperm" (1, default: images with both passes on the GEMM DCT keep their
 * row-pass output T and spectrum Y parity-planar, so each parity problem of
 * the row GEMM stores whole lines; 0: interleaved columns; outputs
 * bit-identical), "rows_fused" (1, default: images whose rows and columns
 * both run on the GEMM DCT take the colour transform, both folds and both
 * parities' row GEMM in one pass, k_rows_fused, its fp16 pieces at a fixed
 * scale; an image whose folded IPT leaves that scale's range, or is not
 * finite, is redone at the per-image scale -- bit-identical to 0 then, and for
 * [0, 1] RGB, where the two scales coincide; 0: k_rgb_to_ipt + the row GEMM),
 * "cols_dma" (1, default: the encode's column GEMM on k_gemm_h2c, the matrix
 * and T streamed into a two-stage LDS ring by buffer_load ... lds; 0:
 * k_gemm_h2's register staging; outputs bit-identical),
 * "gemm_dma" (1, default: the encode's row GEMM on
 * k_gemm_h2r, both operands streamed into a two-stage LDS ring by
 * buffer_load ... lds; 0: k_gemm_h2's register staging; outputs
 * bit-identical), "ws_poison" (0, default; 1: a debug check that fills the
 * workspace and staging buffers with NaN bits before every call that sizes
 * them, so a read of a word the call did not write shows in its outputs;
 * also set by the environment variable DCTAE_WS_POISON=1 at context
 * creation; slow).  Profiling builds only (make PROFILING=1; the shipped
 * library returns DCTAE_EUNSUP): "bs_ablate", "t_alias", "gate" (these write
 * wrong outputs on purpose). */
int dctae_set_option(dctae_ctx* ctx, const char* key, int64_t value);

/* Raise (return DCTAE_EINVAL) if a previous kernel of this context saw an
 * out-of-range channel / position / image id (the reference raises
 * IndexError there).  Synchronises `stream`. */
int dctae_check_device_errors(dctae_ctx* ctx, void* stream);

/* Counter-based synthetic RGB images (same hash as oracle/rng.py):
 * value(seed, first_index + i, e) for i < n_img, images of (3, H, W)
 * contiguous. */
int dctae_synth_images(dctae_ctx* ctx, uint64_t seed, int64_t first_index, int32_t n_img,
                       int32_t H, int32_t W, float* rgb_dev, void* stream);

/* Per-kernel device timing for benchmarks.  While enabled, every kernel the
 * library launches is bracketed by a pair of HIP events on its stream (no
 * host synchronisation).  dctae_timing_collect synchronises those events and
 * accumulates elapsed time per kernel name; dctae_timing_get(idx) then reads
 * entry idx (returns DCTAE_EINVAL past the last one); dctae_timing_reset
 * clears the totals. */
int dctae_set_timing(dctae_ctx* ctx, int enable);
int dctae_timing_collect(dctae_ctx* ctx);
int dctae_timing_get(dctae_ctx* ctx, int idx, const char** name, double* total_ms, int64_t* launches);
int dctae_timing_reset(dctae_ctx* ctx);

/* Workspace cap in bytes for the chunked encode/decode (default 8 GiB). */
int dctae_set_workspace_limit(dctae_ctx* ctx, int64_t bytes);

/* ---- DCTAutoencoder transformer forward -----------------
 * Operator-level entry points under the host mirror of
 * modeling_dct_autoencoder.py (dct_autoencoder_amd/model.py): the CLIPEncoder
 * (transformers==4.35.2 CLIPEncoderLayer) encoder / decoder around LFQ.
 * bf16 tensors are uint16_t bit patterns; the caller owns every buffer.
 * Linear: K % 64 == 0 (zero-padded), x / w rows 16-byte aligned (ld % 8 == 0). */
#define DCTAE_LIN_F32 0           /* out f32 = x W^T + b */
#define DCTAE_LIN_BF16 1          /* out bf16 = x W^T + b */
#define DCTAE_LIN_BF16_QGELU 2    /* out bf16 = quick_gelu(x W^T + b)          (CLIPMLP fc1 + act) */
#define DCTAE_LIN_F32_RESIDUAL 3  /* out f32 += x W^T + b (in place)          (residual adds) */

/* nn.Linear (x (M, K) . W (N, K)^T + bias): q/k/v/out_proj, fc1/fc2
 * (CLIPAttention / CLIPMLP), to_patch_embedding[0] (modeling:57), LFQ
 * project_in / project_out (lfq.py:61-62), proj_out[1] (modeling:76).
 * w_rows >= N rows are allocated (padding rows are never stored). */
int dctae_model_linear(dctae_ctx* ctx, int64_t M, int32_t N, int32_t K, const uint16_t* x_dev, int64_t ldx,
                       const uint16_t* w_dev, int32_t w_rows, int64_t ldw, const float* bias_dev, int32_t epilogue,
                       void* out_dev, int64_t ldo, void* stream);

/* CLIPAttention core (softmax(q k^T / sqrt(64) + attn_mask) v) for R packed
 * rows of S tokens, head_dim 64: qkv (R*S, 3*heads*64) bf16 = [q | k | v];
 * attn_mask is DCTPatches.attn_mask, (id_i == id_j) & key_pad_mask_j
 * (FE:580-584), ADDED as +1.0 like transformers 4.35.2 (modeling:131-133),
 * derived here from ids (R, S) int64 and key_pad (R, S) u8.  out (R*S, ldo)
 * bf16, head h at columns 64 h. */
int dctae_model_attention(dctae_ctx* ctx, int32_t R, int32_t S, int32_t heads, int32_t head_dim,
                          const uint16_t* qkv_dev, const int64_t* ids_dev, const uint8_t* key_pad_dev,
                          uint16_t* out_dev, int64_t ldo, void* stream);

/* LayerNorm over D (torch semantics) of f32 rows -> bf16 (layer_norm1/2). */
int dctae_model_layernorm(dctae_ctx* ctx, int64_t M, int32_t D, const float* x_dev, int64_t ldx,
                          const float* gamma_dev, const float* beta_dev, float eps, uint16_t* out_dev, int64_t ldo,
                          void* stream);

/* to_patch_embedding[1] LayerNorm (eps 1e-4) + encoder position embedding
 * (modeling:57-60, 98-108) -> f32 residual stream. */
int dctae_model_embed_norm(dctae_ctx* ctx, int64_t M, int32_t D, const float* x_dev, int64_t ldx,
                           const float* gamma_dev, const float* beta_dev, float eps, const float* pos_h_dev,
                           const float* pos_w_dev, const float* pos_c_dev, const int64_t* ch_dev,
                           const int64_t* pos_dev, float* out_dev, int64_t ldo, void* stream);

/* x += pos_h[h] + pos_w[w] + pos_c[c] (decoder position embedding, modeling:79-93). */
int dctae_model_pos_add(dctae_ctx* ctx, int64_t M, int32_t D, float* x_dev, int64_t ldx, const float* pos_h_dev,
                        const float* pos_w_dev, const float* pos_c_dev, const int64_t* ch_dev,
                        const int64_t* pos_dev, void* stream);

/* f32 (M, K) -> bf16 (M, Kp), columns K .. Kp zero. */
int dctae_model_to_bf16(dctae_ctx* ctx, int64_t M, int32_t K, const float* x_dev, int64_t ldx, int32_t Kp,
                        uint16_t* out_dev, void* stream);

/* LFQ.forward eval on projected features (lfq.py:164-212): x (M, ncb*cbd)
 * f32 -> codes (M, ncb) int64 MSB-first, +-scale features into q_bf16
 * (M, ldq; zero-padded) and/or q_f32 (M, ldq). */
int dctae_model_lfq(dctae_ctx* ctx, int64_t M, int32_t ncb, int32_t cbd, float scale, const float* x_dev,
                    int64_t ldx, int64_t* codes_dev, uint16_t* q_bf16_dev, float* q_f32_dev, int64_t ldq,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DCTAE_H */
