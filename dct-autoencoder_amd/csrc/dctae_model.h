// Device-side argument blocks of the DCTAutoencoder transformer kernels
// (dctae_model.hip); the C ABI is in include/dctae.h (dctae_model_*).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dctae {

enum { LIN_F32 = 0, LIN_BF16 = 1, LIN_BF16_QGELU = 2, LIN_F32_RESIDUAL = 3 };

struct LinearArgs {
  const uint16_t* x;   // (M, ldx) bf16, K-contiguous, K % 64 == 0 valid columns
  const uint16_t* w;   // (Nw, ldw) bf16 (nn.Linear weight layout), K columns
  const float* bias;   // (N) or null
  void* out;           // (M, ldo) f32 or bf16 per epilogue
  int64_t M, ldx, ldw, ldo;
  int32_t N, Nw, K;
};

struct AttnArgs {
  const uint16_t* qkv;     // (R * S, 3 * heads * 64) bf16: q | k | v
  const int64_t* ids;      // (R, S) batched_image_ids
  const uint8_t* key_pad;  // (R, S) key_pad_mask (True = pad)
  uint16_t* out;           // (R * S, ldo) bf16, head h at columns 64 h
  int32_t R, S, heads, ldo;
  float scale;             // d_head ** -0.5
};

struct LnArgs {
  const float* x;
  const float* gamma;
  const float* beta;
  uint16_t* out_bf16;      // LayerNorm -> bf16, or
  float* out_f32;          // LayerNorm + position terms -> f32 (embedding)
  const float* pos_h;      // (max_patch_h, D)
  const float* pos_w;      // (max_patch_w, D)
  const float* pos_c;      // (C, D)
  const int64_t* ch;       // (M)
  const int64_t* pos;      // (M, 2)
  int64_t M, ldx, ldo;
  int32_t D;
  float eps;
};

struct PosArgs {
  float* x;
  const float* pos_h;
  const float* pos_w;
  const float* pos_c;
  const int64_t* ch;
  const int64_t* pos;
  int64_t M, ldx;
  int32_t D;
};

struct LfqArgs {
  const float* x;     // (M, ldx): ncb * cbd features
  int64_t* codes;     // (M, ncb)
  uint16_t* q_bf16;   // (M, ldq) or null
  float* q_f32;       // (M, ldq) or null
  int64_t M, ldx, ldq;
  int32_t ncb, cbd;
  float scale;
};

void launch_linear(const LinearArgs& a, int epi, hipStream_t s);
void launch_attention(const AttnArgs& a, hipStream_t s);
void launch_layernorm(const LnArgs& a, hipStream_t s);
void launch_pos_add(const PosArgs& a, hipStream_t s);
void launch_to_bf16(const float* x, int64_t ldx, int64_t M, int K, int Kp, uint16_t* out, hipStream_t s);
void launch_lfq_codes(const LfqArgs& a, hipStream_t s);

}  // namespace dctae
