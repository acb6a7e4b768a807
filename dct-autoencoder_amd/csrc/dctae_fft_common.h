// FFT codelets shared by dctae_fft.hip (generic plans) and dctae_fft2.hip
// (compile-time specialised plans): forward DFTs of size 2, 3, 4, 5, 7, 8, 16
// on float2 registers, natural order in and out.
#pragma once
#include "dctae_device.h"

namespace dctae {

__device__ constexpr float kCos3[3] = {1.0f, -0.5f, -0.5f};
__device__ constexpr float kSin3[3] = {0.0f, 8.660254038e-01f, -8.660254038e-01f};
__device__ constexpr float kCos5[5] = {1.0f, 3.090169944e-01f, -8.090169944e-01f, -8.090169944e-01f, 3.090169944e-01f};
__device__ constexpr float kSin5[5] = {0.0f, 9.510565163e-01f, 5.877852523e-01f, -5.877852523e-01f, -9.510565163e-01f};
__device__ constexpr float kCos7[7] = {1.0f, 6.234898019e-01f, -2.225209340e-01f, -9.009688679e-01f,
                                       -9.009688679e-01f, -2.225209340e-01f, 6.234898019e-01f};
__device__ constexpr float kSin7[7] = {0.0f, 7.818314825e-01f, 9.749279122e-01f, 4.338837391e-01f,
                                       -4.338837391e-01f, -9.749279122e-01f, -7.818314825e-01f};
__device__ constexpr float kCos16[16] = {1.0f, 9.238795325e-01f, 7.071067812e-01f, 3.826834324e-01f, 0.0f,
                                         -3.826834324e-01f, -7.071067812e-01f, -9.238795325e-01f, -1.0f,
                                         -9.238795325e-01f, -7.071067812e-01f, -3.826834324e-01f, 0.0f,
                                         3.826834324e-01f, 7.071067812e-01f, 9.238795325e-01f};
__device__ constexpr float kSin16[16] = {0.0f, 3.826834324e-01f, 7.071067812e-01f, 9.238795325e-01f, 1.0f,
                                         9.238795325e-01f, 7.071067812e-01f, 3.826834324e-01f, 0.0f,
                                         -3.826834324e-01f, -7.071067812e-01f, -9.238795325e-01f, -1.0f,
                                         -9.238795325e-01f, -7.071067812e-01f, -3.826834324e-01f};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // -i * a

// forward DFT codelets, natural order in and out: V[k] = sum_n v[n] e^{-2 pi i nk/R}
template <int R>
struct DFT;

template <>
struct DFT<2> {
  static __device__ __forceinline__ void run(float2* v) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};

template <>
struct DFT<4> {
  static __device__ __forceinline__ void run(float2* v) {
    float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    float2 t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
  }
};

template <>
struct DFT<8> {
  static __device__ __forceinline__ void run(float2* v) {
    float2 e[4] = {v[0], v[2], v[4], v[6]};
    float2 o[4] = {v[1], v[3], v[5], v[7]};
    DFT<4>::run(e);
    DFT<4>::run(o);
    const float c = 7.071067812e-01f;
    float2 w1 = make_float2(c * (o[1].x + o[1].y), c * (o[1].y - o[1].x));    // o1 * (c - ic)
    float2 w2 = mul_mi(o[2]);                                                  // o2 * -i
    float2 w3 = make_float2(c * (o[3].y - o[3].x), -c * (o[3].x + o[3].y));   // o3 * (-c - ic)
    v[0] = cadd(e[0], o[0]);
    v[4] = csub(e[0], o[0]);
    v[1] = cadd(e[1], w1);
    v[5] = csub(e[1], w1);
    v[2] = cadd(e[2], w2);
    v[6] = csub(e[2], w2);
    v[3] = cadd(e[3], w3);
    v[7] = csub(e[3], w3);
  }
};

template <>
struct DFT<16> {
  static __device__ __forceinline__ void run(float2* v) {
    float2 a[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
      for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[4 * n1 + n2];
      DFT<4>::run(a[n2]);
    }
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
      for (int k1 = 1; k1 < 4; ++k1) {
        const int m = n2 * k1;
        a[n2][k1] = cmul(a[n2][k1], make_float2(kCos16[m], -kSin16[m]));
      }
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      float2 b[4] = {a[0][k1], a[1][k1], a[2][k1], a[3][k1]};
      DFT<4>::run(b);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = b[k2];
    }
  }
};

template <int R>
__device__ __forceinline__ void dft_odd(float2* v, const float* C, const float* S) {
  constexpr int H = (R - 1) / 2;
  float2 s[H], d[H];
  float2 x0 = v[0], sum = v[0];
#pragma unroll
  for (int n = 1; n <= H; ++n) {
    s[n - 1] = cadd(v[n], v[R - n]);
    d[n - 1] = csub(v[n], v[R - n]);
    sum = cadd(sum, s[n - 1]);
  }
  float2 out[R];
  out[0] = sum;
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    float re = x0.x, im = x0.y, re2 = 0.0f, im2 = 0.0f;
#pragma unroll
    for (int n = 1; n <= H; ++n) {
      const int m = (n * k) % R;
      re = fmaf(s[n - 1].x, C[m], re);
      im = fmaf(s[n - 1].y, C[m], im);
      re2 = fmaf(d[n - 1].y, S[m], re2);
      im2 = fmaf(d[n - 1].x, S[m], im2);
    }
    out[k] = make_float2(re + re2, im - im2);
    out[R - k] = make_float2(re - re2, im + im2);
  }
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = out[k];
}

template <>
struct DFT<3> {
  static __device__ __forceinline__ void run(float2* v) { dft_odd<3>(v, kCos3, kSin3); }
};
template <>
struct DFT<5> {
  static __device__ __forceinline__ void run(float2* v) { dft_odd<5>(v, kCos5, kSin5); }
};
template <>
struct DFT<7> {
  static __device__ __forceinline__ void run(float2* v) { dft_odd<7>(v, kCos7, kSin7); }
};

// ---------------------------------------------------------------------------
// The same codelets on a native 2-float vector (re, im): every complex add is
// one v_pk_add_f32 on an aligned register pair and multiplies become
// v_pk_mul / v_pk_fma with op_sel swizzles, instead of scalar ops that the
// SLP vectoriser re-pairs with register moves.  FMA contraction is allowed
// here (the DCT is compared with a tolerance; PatchNorm / LFQ / score code
// lives elsewhere and keeps -ffp-contract=off).
// ---------------------------------------------------------------------------
typedef float cf __attribute__((ext_vector_type(2)));

__device__ __forceinline__ cf cmulv(cf a, cf w) {
#pragma clang fp contract(fast)
  return a.xx * w + a.yy * (cf){-w.y, w.x};
}
__device__ __forceinline__ cf mul_mi_v(cf a) { return (cf){a.y, -a.x}; }  // -i * a

// Packed complex ops with the swizzle / sign folded into VOP3P op_sel and neg
// modifiers (the compiler materialises (a.y, -a.x) with v_mov + v_xor instead).
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ cf add_mi(cf a, cf b) {
  cf d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ cf sub_mi(cf a, cf b) {
  cf d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a + conj(b), a - conj(b)
__device__ __forceinline__ cf add_conj(cf a, cf b) {
  cf d;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ cf sub_conj(cf a, cf b) {
  cf d;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// a.x * w   and   a.y * (i w) + c = (c.x - a.y w.y, c.y + a.y w.x): a * w = fma_iw(a, w, mul_x(a, w))
__device__ __forceinline__ cf mul_x(cf a, cf w) {
  cf d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(d) : "v"(a), "v"(w));
  return d;
}
__device__ __forceinline__ cf fma_x(cf a, cf w, cf c) {   // a.x * w + c
  cf d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}
__device__ __forceinline__ cf fma_iw(cf a, cf w, cf c) {  // a.y * (i w) + c
  cf d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}
__device__ __forceinline__ cf cmul_pk(cf a, cf w) { return fma_iw(a, w, mul_x(a, w)); }

template <int R>
struct DFTV;

template <>
struct DFTV<4> {
  static __device__ __forceinline__ void run(cf* v) {
    const cf t0 = v[0] + v[2], t1 = v[0] - v[2];
    const cf t2 = v[1] + v[3], t3 = v[1] - v[3];
    v[0] = t0 + t2;
    v[2] = t0 - t2;
    v[1] = add_mi(t1, t3);   // t1 + (-i) t3
    v[3] = sub_mi(t1, t3);
  }
};

template <>
struct DFTV<2> {
  static __device__ __forceinline__ void run(cf* v) {
    const cf a = v[0], b = v[1];
    v[0] = a + b;
    v[1] = a - b;
  }
};

template <>
struct DFTV<8> {
  static __device__ __forceinline__ void run(cf* v) {
#pragma clang fp contract(fast)
    cf e[4] = {v[0], v[2], v[4], v[6]};
    cf o[4] = {v[1], v[3], v[5], v[7]};
    DFTV<4>::run(e);
    DFTV<4>::run(o);
    const float c = 7.071067812e-01f;
    const cf w1 = cmulv(o[1], (cf){c, -c});
    const cf w3 = cmulv(o[3], (cf){-c, -c});
    v[0] = e[0] + o[0];
    v[4] = e[0] - o[0];
    v[1] = e[1] + w1;
    v[5] = e[1] - w1;
    v[2] = add_mi(e[2], o[2]);   // e2 + (-i) o2
    v[6] = sub_mi(e[2], o[2]);
    v[3] = e[3] + w3;
    v[7] = e[3] - w3;
  }
};

template <>
struct DFTV<16> {
  static __device__ __forceinline__ void run(cf* v) {
#pragma clang fp contract(fast)
    cf a[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
      for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[4 * n1 + n2];
      DFTV<4>::run(a[n2]);
    }
    // twiddles W16^(n2 k1): m = 4 -> -i (free), m = 2, 6 -> (1 -+ i)/sqrt2 forms
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
      for (int k1 = 1; k1 < 4; ++k1) {
        const int m = n2 * k1;
        if (m != 4) a[n2][k1] = cmulv(a[n2][k1], (cf){kCos16[m], -kSin16[m]});
      }
    // the W16^4 = -i twiddle of a[2][2] is folded into the k1 = 2 column's DFT4:
    // its n = 2 input enters as (-i) a[2][1] (t0/t1 of DFTV<4> with +- (-i) terms)
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      cf b[4] = {a[0][k1], a[1][k1], a[2][k1], a[3][k1]};
      if (k1 == 2) {
        const cf t0 = add_mi(b[0], b[2]), t1 = sub_mi(b[0], b[2]);   // b0 +- (-i) b2
        const cf t2 = b[1] + b[3], t3 = b[1] - b[3];
        b[0] = t0 + t2;
        b[2] = t0 - t2;
        b[1] = add_mi(t1, t3);
        b[3] = sub_mi(t1, t3);
      } else {
        DFTV<4>::run(b);
      }
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = b[k2];
    }
  }
};

template <int R>
__device__ __forceinline__ void dftv_odd(cf* v, const float* C, const float* S) {
#pragma clang fp contract(fast)
  constexpr int H = (R - 1) / 2;
  cf s[H], d[H];
  const cf x0 = v[0];
  cf sum = v[0];
#pragma unroll
  for (int n = 1; n <= H; ++n) {
    s[n - 1] = v[n] + v[R - n];
    d[n - 1] = v[n] - v[R - n];
    sum = sum + s[n - 1];
  }
  cf out[R];
  out[0] = sum;
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    cf a = x0, b = (cf){0.0f, 0.0f};
#pragma unroll
    for (int n = 1; n <= H; ++n) {
      const int m = (n * k) % R;
      a = a + s[n - 1] * C[m];
      b = b + d[n - 1].yx * S[m];      // (d.y S, d.x S)
    }
    out[k] = (cf){a.x + b.x, a.y - b.y};
    out[R - k] = (cf){a.x - b.x, a.y + b.y};
  }
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = out[k];
}

template <>
struct DFTV<7> {
  static __device__ __forceinline__ void run(cf* v) { dftv_odd<7>(v, kCos7, kSin7); }
};

// ---------------------------------------------------------------------------
// Scalar DFT16 on split (re, im) arrays, natural order in and out (4 x 4
// with internal twiddles W16^(n2 k1); the W16^4 = -i twiddle is a rename).
// No packed pairs: the caller's inputs can come from any registers without
// the moves a (re, im) register pair needs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dft4s(float& r0, float& i0, float& r1, float& i1, float& r2, float& i2, float& r3,
                                      float& i3) {
  const float t0r = r0 + r2, t0i = i0 + i2, t1r = r0 - r2, t1i = i0 - i2;
  const float t2r = r1 + r3, t2i = i1 + i3, t3r = r1 - r3, t3i = i1 - i3;
  r0 = t0r + t2r;
  i0 = t0i + t2i;
  r2 = t0r - t2r;
  i2 = t0i - t2i;
  r1 = t1r + t3i;   // t1 + (-i) t3
  i1 = t1i - t3r;
  r3 = t1r - t3i;
  i3 = t1i + t3r;
}

__device__ __forceinline__ void dft16s(float (&re)[16], float (&im)[16]) {
#pragma clang fp contract(fast)
  float ar[4][4], ai[4][4];   // [n2][k1]
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    float x0r = re[n2], x0i = im[n2], x1r = re[4 + n2], x1i = im[4 + n2];
    float x2r = re[8 + n2], x2i = im[8 + n2], x3r = re[12 + n2], x3i = im[12 + n2];
    dft4s(x0r, x0i, x1r, x1i, x2r, x2i, x3r, x3i);
    ar[n2][0] = x0r, ai[n2][0] = x0i, ar[n2][1] = x1r, ai[n2][1] = x1i;
    ar[n2][2] = x2r, ai[n2][2] = x2i, ar[n2][3] = x3r, ai[n2][3] = x3i;
  }
  constexpr float c = 7.071067812e-01f;
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) {
      const int m = n2 * k1;
      const float a = ar[n2][k1], b = ai[n2][k1];
      if (m == 4) {          // -i
        ar[n2][k1] = b;
        ai[n2][k1] = -a;
      } else if (m == 2) {   // (1 - i) / sqrt2
        ar[n2][k1] = c * (a + b);
        ai[n2][k1] = c * (b - a);
      } else if (m == 6) {   // (-1 - i) / sqrt2
        ar[n2][k1] = c * (b - a);
        ai[n2][k1] = -c * (a + b);
      } else {
        const float wr = kCos16[m], wi = -kSin16[m];
        ar[n2][k1] = a * wr - b * wi;
        ai[n2][k1] = a * wi + b * wr;
      }
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float x0r = ar[0][k1], x0i = ai[0][k1], x1r = ar[1][k1], x1i = ai[1][k1];
    float x2r = ar[2][k1], x2i = ai[2][k1], x3r = ar[3][k1], x3i = ai[3][k1];
    dft4s(x0r, x0i, x1r, x1i, x2r, x2i, x3r, x3i);
    re[k1] = x0r, im[k1] = x0i, re[k1 + 4] = x1r, im[k1 + 4] = x1i;
    re[k1 + 8] = x2r, im[k1 + 8] = x2i, re[k1 + 12] = x3r, im[k1 + 12] = x3i;
  }
}

}  // namespace dctae
