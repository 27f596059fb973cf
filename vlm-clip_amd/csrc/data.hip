// Data-movement kernels around the towers: patch im2col and pooled-row gather/scatter.
//
// im2col replaces the stride=kernel Conv2d of CLIPVisionEmbeddings ([HF] modeling_clip.py
// :148-154, :211-212) as a coalesced gather feeding the MFMA GEMM; its output has one zero
// row per image in the CLS slot, so the patch GEMM writes the full [B*(Np+1), D] token
// matrix in place and the patch-weight gradient is one wgrad GEMM over that same buffer.
// Pooling: model_m.py:102,122 take token 0 ([:,0,:]); HF's EOS pooler ([HF] :561-581)
// takes the first EOS (or argmax id when eos_token_id == 2).
#include "common.h"
#include "internal.h"
#include <cmath>
#include <type_traits>

namespace {

template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const float* px, T* X, int B, int C, int Hh, int P, int G,
                                                     int K, int Kp) {
  const int64_t row = blockIdx.y + (int64_t)blockIdx.z * 65535;
  const int Np1 = G * G + 1;
  if (row >= (int64_t)B * Np1) return;
  const int b = (int)(row / Np1), t = (int)(row % Np1);
  for (int k = blockIdx.x * 256 + threadIdx.x; k < Kp; k += gridDim.x * 256) {
    float v = 0.f;
    if (t > 0 && k < K) {
      const int p = t - 1, gy = p / G, gx = p % G;
      const int c = k / (P * P), r = k % (P * P), ky = r / P, kx = r % P;
      v = px[(((int64_t)b * C + c) * Hh + gy * P + ky) * Hh + gx * P + kx];
    }
    X[row * Kp + k] = (T)v;
  }
}

// Vectorised form for P % 8 == 0 (ViT-B/16, B/32): one thread per 8 consecutive k of a token
// row, i.e. 8 consecutive kx of one pixel row: two 16-B loads, one 16-B (bf16) store; a wave
// stores 1 KiB contiguous.  The scalar kernel above remains for other patch sizes (L/14).
template <typename T>
__global__ __launch_bounds__(256) void im2col8_kernel(const float* px, T* X, int64_t rows, int C, int Hh, int P, int G,
                                                      int K, int Kp) {
  const int gpr = Kp >> 3;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = id / gpr;
  if (row >= rows) return;
  const int k = (int)(id - row * gpr) * 8;
  const int Np1 = G * G + 1;
  const int b = (int)(row / Np1), t = (int)(row - (int64_t)b * Np1);
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (t > 0 && k < K) {
    const int p = t - 1, gy = p / G, gx = p - gy * G;
    const int c = k / (P * P), r = k - c * P * P, ky = r / P, kx = r - ky * P;
    const float* src = px + (((int64_t)b * C + c) * Hh + gy * P + ky) * Hh + gx * P + kx;
    const f32x4 a = *(const f32x4*)src, a2 = *(const f32x4*)(src + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = a2[j]; }
  }
  T* dst = X + row * Kp + k;
  store4(dst, v);
  store4(dst + 4, v + 4);
}

// P = 14 (ViT-L/14; K = 588): one thread per (token row, channel, kernel row) -- 14 consecutive pixels of one image
// row in seven 8-B loads, written as 14 consecutive elements of the im2col row in seven pair stores -- and a 43rd
// thread per row zeroing the padded columns K .. Kp.  The scalar kernel moved one element per thread with its index
// divisions (ViT-L/14@336, B = 4096: 6.4 ms).  Even H, 8-B aligned pixels, even Kp (host-checked).
template <typename T>
__global__ __launch_bounds__(256) void im2col14_kernel(const float* px, T* X, int64_t rows, int C, int Hh, int G,
                                                       int K, int Kp) {
  const int per = C * 14 + 1;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = id / per;
  if (row >= rows) return;
  const int w = (int)(id - row * per);
  T* dst = X + row * Kp;
  if (w == C * 14) {
    for (int k = K; k < Kp; k += 2) {
      dst[k] = (T)0.f;
      dst[k + 1] = (T)0.f;
    }
    return;
  }
  const int Np1 = G * G + 1;
  const int b = (int)(row / Np1), t = (int)(row - (int64_t)b * Np1);
  const int c = w / 14, ky = w - c * 14;
  float v[14];
#pragma unroll
  for (int j = 0; j < 14; ++j) v[j] = 0.f;
  if (t > 0) {
    const int p = t - 1, gy = p / G, gx = p - gy * G;
    const float* src = px + (((int64_t)b * C + c) * Hh + gy * 14 + ky) * Hh + gx * 14;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const float2 a = *(const float2*)(src + 2 * j);
      v[2 * j] = a.x;
      v[2 * j + 1] = a.y;
    }
  }
  T* o = dst + c * 196 + ky * 14;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if constexpr (std::is_same<T, float>::value) {
      *(float2*)(o + 2 * j) = make_float2(v[2 * j], v[2 * j + 1]);
    } else {
      *(bf16x2*)(o + 2 * j) = bf16x2{(bf16)v[2 * j], (bf16)v[2 * j + 1]};
    }
  }
}

// The input step fused into patch-embed: decoded uint8 images, channels
// last (what CLIPImageProcessor receives), centre-cropped to G*P, rescaled by 1/255 and
// normalised per channel ([HF] image_processing_clip.py: center_crop, rescale, normalize;
// do_resize stays on the host), written straight as im2col rows.  One thread per (token, ky,
// GW consecutive kx): GW = 8 for P % 8 == 0 (a 24-B read of 8 RGB pixels, three 8-element
// writes, one per channel), GW = 2 for ViT-L/14 (P = 14, whose padded K columns it zeroes).
template <typename T, int GW>
__global__ __launch_bounds__(256) void im2col_u8_kernel(const uint8_t* img, T* X, int64_t rows, int Hin, int Win,
                                                        int y0, int x0, int P, int G, int Kp, float m0, float m1,
                                                        float m2, float r0, float r1, float r2) {
  const int per_row = P * (P / GW);  // (ky, kx-group) pairs per token
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = id / per_row;
  if (row >= rows) return;
  const int q = (int)(id - row * per_row);
  const int ky = q / (P / GW), kx = (q - ky * (P / GW)) * GW;
  const int Np1 = G * G + 1;
  const int b = (int)(row / Np1), t = (int)(row - (int64_t)b * Np1);
  float v[3][GW];
  if (t == 0) {  // CLS slot: zero row (the class embedding is added after the patch GEMM)
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < GW; ++j) v[c][j] = 0.f;
  } else {
    const int p = t - 1, gy = p / G, gx = p - gy * G;
    const int y = y0 + gy * P + ky, x = x0 + gx * P + kx;
    const uint8_t* src = img + (((int64_t)b * Hin + y) * Win + x) * 3;
    const float mean[3] = {m0, m1, m2}, rstd[3] = {r0, r1, r2};
#pragma unroll
    for (int j = 0; j < GW; ++j)
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c][j] = ((float)src[3 * j + c] * (1.0f / 255.0f) - mean[c]) * rstd[c];
  }
  T* dst = X + row * Kp + ky * P + kx;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if constexpr (GW == 8) {
      store4(dst + c * P * P, v[c]);
      store4(dst + c * P * P + 4, v[c] + 4);
    } else {
#pragma unroll
      for (int j = 0; j < GW; ++j) dst[c * P * P + j] = (T)v[c][j];
    }
  }
  if (q == 0)  // padded K (ViT-L/14: 588 -> 640): zero the pad columns once per token row
    for (int k = 3 * P * P; k < Kp; ++k) X[row * Kp + k] = (T)0.f;
}

// idx[b] = pooled token: mode 0 -> 0, mode 1 -> first position with id == eos, mode 2 -> argmax id
__global__ void pool_index_kernel(const int64_t* ids, int B, int S, int64_t eos, int mode, int* idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int best = 0;
  if (mode == 1) {
    for (int s = S - 1; s >= 0; --s)
      if (ids[(int64_t)b * S + s] == eos) best = s;
  } else if (mode == 2) {
    int64_t bv = ids[(int64_t)b * S];
    for (int s = 1; s < S; ++s)
      if (ids[(int64_t)b * S + s] > bv) { bv = ids[(int64_t)b * S + s]; best = s; }
  }
  idx[b] = best;
}

// out[b][:] = src[(b*S + idx[b])][:]  (idx == NULL -> token 0)
template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(const T* src, const int* idx, int B, int S, int D, T* out) {
  const int b = blockIdx.x;
  const int64_t r = (int64_t)b * S + (idx ? idx[b] : 0);
  for (int c = threadIdx.x; c < D; c += 256) out[(int64_t)b * D + c] = src[r * D + c];
}

// dst[(b*S + idx[b])][:] (+)= src[b][:]
template <typename T>
__global__ __launch_bounds__(256) void scatter_rows_kernel(const T* src, const int* idx, int B, int S, int D, T* dst,
                                                           int beta) {
  const int b = blockIdx.x;
  const int64_t r = (int64_t)b * S + (idx ? idx[b] : 0);
  for (int c = threadIdx.x; c < D; c += 256) {
    float v = (float)src[(int64_t)b * D + c];
    if (beta) v += (float)dst[r * D + c];
    dst[r * D + c] = (T)v;
  }
}

// ---- input-step resize: CLIPImageProcessor's shortest-edge resize = PIL Image.resize(BICUBIC)
// (transformers CLIPImageProcessorPil; PIL libImaging/Resample.c, restated in oracle/resize_ref.py
// and bit-exact against PIL): per output coordinate the taps [xmin, xmin + n) and fp64 bicubic
// (a = -0.5) weights stretched by max(in/out, 1), normalised, then fixed point with 22 fraction
// bits; a horizontal 8-bit pass, then a vertical one, each out = clamp((2^21 + sum k*in) >> 22).
// Tables: per output coordinate [xmin, n, k_0 .. k_{ksize-1}] int32.
constexpr int RS_PREC = 22;

__device__ double rs_bicubic(double x) {
#pragma clang fp contract(off)
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0;
  if (x < 2.0) return (((x - 5.0) * x + 8.0) * x - 4.0) * a;
  return 0.0;
}

// one thread per output coordinate; fp64 exactly as PIL's precompute_coeffs (no contraction)
__global__ void resize_coeffs_kernel(int in_size, int out_size, int ksize, int* tab) {
#pragma clang fp contract(off)
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= out_size) return;
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double ss = 1.0 / filterscale;
  const double center = (xx + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  int* t = tab + (int64_t)xx * (2 + ksize);
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += rs_bicubic((x + xmin - center + 0.5) * ss);
  for (int x = 0; x < ksize; ++x) {
    int k = 0;
    if (x < xmax) {
      double w = rs_bicubic((x + xmin - center + 0.5) * ss);
      if (ww != 0.0) w /= ww;
      k = w < 0 ? (int)(-0.5 + w * (double)(1 << RS_PREC)) : (int)(0.5 + w * (double)(1 << RS_PREC));
    }
    t[2 + x] = k;
  }
  t[0] = xmin;
  t[1] = xmax;
}

__device__ __forceinline__ uint8_t rs_clip8(int acc) {
  const int v = acc >> RS_PREC;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// horizontal (HORIZ) or vertical pass over channels-last RGB: one thread per output pixel
template <bool HORIZ>
__global__ __launch_bounds__(256) void resize_pass_kernel(const uint8_t* in, uint8_t* out, int B, int Hin, int Win,
                                                          int Hout, int Wout, const int* tab, int ksize) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)B * Hout * Wout;
  if (i >= total) return;
  const int xo = (int)(i % Wout);
  const int64_t r = i / Wout;
  const int yo = (int)(r % Hout), b = (int)(r / Hout);
  const int* t = tab + (int64_t)(HORIZ ? xo : yo) * (2 + ksize);
  const int lo = t[0], n = t[1];
  int a0 = 1 << (RS_PREC - 1), a1 = a0, a2 = a0;
  const uint8_t* src = HORIZ ? in + (((int64_t)b * Hin + yo) * Win + lo) * 3 : in + (((int64_t)b * Hin + lo) * Win + xo) * 3;
  const int64_t step = HORIZ ? 3 : (int64_t)Win * 3;
  for (int j = 0; j < n; ++j) {
    const int k = t[2 + j];
    a0 += k * (int)src[0];
    a1 += k * (int)src[1];
    a2 += k * (int)src[2];
    src += step;
  }
  uint8_t* dst = out + i * 3;
  dst[0] = rs_clip8(a0);
  dst[1] = rs_clip8(a1);
  dst[2] = rs_clip8(a2);
}

int rs_ksize(int in, int out) {
  const double scale = (double)in / (double)out;
  const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
  return (int)ceil(support) * 2 + 1;
}
int64_t rs_al(int64_t x) { return (x + 255) & ~(int64_t)255; }

}  // namespace

extern "C" int clipmi_im2col(void* stream, int dtype, const float* pixels, void* X, int B, int C, int H, int P, int Kp) {
  CLIPMI_REQUIRE(H % P == 0, "image size must be a multiple of the patch size");
  const int G = H / P, K = C * P * P;
  CLIPMI_REQUIRE(Kp >= K && Kp % 8 == 0, "Kp must be >= C*P*P and a multiple of 8");
  const int64_t rows = (int64_t)B * (G * G + 1);
  if (rows == 0) return CLIPMI_OK;
  if (P % 8 == 0 && H % 4 == 0 && ((uintptr_t)pixels & 15) == 0 && ((uintptr_t)X & 15) == 0) {
    const int64_t n = rows * (Kp / 8);
    const unsigned nb = (unsigned)((n + 255) / 256);
    if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(im2col8_kernel<bf16>, dim3(nb), dim3(256), 0, (hipStream_t)stream, pixels, (bf16*)X, rows, C, H, P, G, K, Kp);
    else hipLaunchKernelGGL(im2col8_kernel<float>, dim3(nb), dim3(256), 0, (hipStream_t)stream, pixels, (float*)X, rows, C, H, P, G, K, Kp);
    CLIPMI_CHECK_LAUNCH();
    return CLIPMI_OK;
  }
  if (P == 14 && H % 2 == 0 && Kp % 2 == 0 && ((uintptr_t)pixels & 7) == 0 && ((uintptr_t)X & 7) == 0) {
    const int64_t n = rows * (C * 14 + 1);
    const unsigned nb = (unsigned)((n + 255) / 256);
    if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(im2col14_kernel<bf16>, dim3(nb), dim3(256), 0, (hipStream_t)stream, pixels, (bf16*)X, rows, C, H, G, K, Kp);
    else hipLaunchKernelGGL(im2col14_kernel<float>, dim3(nb), dim3(256), 0, (hipStream_t)stream, pixels, (float*)X, rows, C, H, G, K, Kp);
    CLIPMI_CHECK_LAUNCH();
    return CLIPMI_OK;
  }
  dim3 g((Kp + 255) / 256 > 4 ? 4 : (Kp + 255) / 256, (unsigned)(rows < 65535 ? rows : 65535),
         (unsigned)((rows + 65534) / 65535));
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(im2col_kernel<bf16>, g, dim3(256), 0, (hipStream_t)stream, pixels, (bf16*)X, B, C, H, P, G, K, Kp);
  else hipLaunchKernelGGL(im2col_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, pixels, (float*)X, B, C, H, P, G, K, Kp);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_im2col_u8(void* stream, int dtype, const uint8_t* images, void* X, int B, int Hin, int Win,
                                int image_size, int P, int Kp, const float* mean, const float* std) {
  CLIPMI_REQUIRE(image_size % P == 0 && P % 2 == 0, "image size must be a multiple of the patch size, P even");
  CLIPMI_REQUIRE(Hin >= image_size && Win >= image_size, "images smaller than the crop (resize them first)");
  CLIPMI_REQUIRE(Kp >= 3 * P * P && (Kp == 3 * P * P || Kp % 8 == 0), "Kp must be 3*P*P or a padded multiple of 8");
  CLIPMI_REQUIRE(mean && std && std[0] != 0.f && std[1] != 0.f && std[2] != 0.f, "mean/std");
  const int G = image_size / P;
  const int64_t rows = (int64_t)B * (G * G + 1);
  if (rows == 0) return CLIPMI_OK;
  const int y0 = (Hin - image_size) / 2, x0 = (Win - image_size) / 2;  // [HF] center_crop offsets
  const int gw = P % 8 == 0 ? 8 : 2;  // 8 pixels (24 B) per thread for P = 16/32, 2 for P = 14
  const int64_t n = rows * P * (P / gw);
  const unsigned nb = (unsigned)((n + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  const float r0 = 1.f / std[0], r1 = 1.f / std[1], r2 = 1.f / std[2];
#define CLIPMI_U8(T, GW) hipLaunchKernelGGL((im2col_u8_kernel<T, GW>), dim3(nb), dim3(256), 0, s, images, (T*)X, rows, \
                                            Hin, Win, y0, x0, P, G, Kp, mean[0], mean[1], mean[2], r0, r1, r2)
  if (dtype == CLIPMI_BF16) {
    if (gw == 8) CLIPMI_U8(bf16, 8); else CLIPMI_U8(bf16, 2);
  } else {
    if (gw == 8) CLIPMI_U8(float, 8); else CLIPMI_U8(float, 2);
  }
#undef CLIPMI_U8
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_pool_index(void* stream, const int64_t* ids, int B, int S, int64_t eos, int mode, int* idx) {
  hipLaunchKernelGGL(pool_index_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, ids, B, S, eos, mode, idx);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_gather_rows(void* stream, int dtype, const void* src, const int* idx, int B, int S, int D, void* out) {
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const bf16*)src, idx, B, S, D, (bf16*)out);
  else hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const float*)src, idx, B, S, D, (float*)out);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_scatter_rows(void* stream, int dtype, const void* src, const int* idx, int B, int S, int D, void* dst, int beta) {
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(scatter_rows_kernel<bf16>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const bf16*)src, idx, B, S, D, (bf16*)dst, beta);
  else hipLaunchKernelGGL(scatter_rows_kernel<float>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const float*)src, idx, B, S, D, (float*)dst, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// ---- input-step resize (see resize_pass_kernel): workspace = the two coefficient tables + the
// horizontally resized intermediate [B, Hin, Wout, 3]
extern "C" int64_t clipmi_resize_u8_ws(int B, int Hin, int Win, int Hout, int Wout) {
  return rs_al((int64_t)Wout * (2 + rs_ksize(Win, Wout)) * 4) + rs_al((int64_t)Hout * (2 + rs_ksize(Hin, Hout)) * 4) +
         rs_al((int64_t)B * Hin * Wout * 3);
}

extern "C" int clipmi_resize_u8(void* stream, const uint8_t* in, int B, int Hin, int Win, uint8_t* out, int Hout,
                                int Wout, void* ws, int64_t ws_bytes) {
  CLIPMI_REQUIRE(B >= 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0, "resize: sizes");
  CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_resize_u8_ws(B, Hin, Win, Hout, Wout), "resize: workspace too small");
  if (B == 0) return CLIPMI_OK;
  hipStream_t s = (hipStream_t)stream;
  const int kw = rs_ksize(Win, Wout), kh = rs_ksize(Hin, Hout);
  int* htab = (int*)ws;
  int* vtab = (int*)((char*)ws + rs_al((int64_t)Wout * (2 + kw) * 4));
  uint8_t* tmp = (uint8_t*)vtab + rs_al((int64_t)Hout * (2 + kh) * 4);
  const bool hz = Wout != Win, vt = Hout != Hin;  // PIL skips a pass whose size does not change
  if (!hz && !vt) {
    CLIPMI_HIP(hipMemcpyAsync(out, in, (size_t)B * Hin * Win * 3, hipMemcpyDeviceToDevice, s));
    return CLIPMI_OK;
  }
  if (hz) {
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3((Wout + 255) / 256), dim3(256), 0, s, Win, Wout, kw, htab);
    const int64_t n = (int64_t)B * Hin * Wout;
    hipLaunchKernelGGL(resize_pass_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in,
                       vt ? tmp : out, B, Hin, Win, Hin, Wout, htab, kw);
  }
  if (vt) {
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3((Hout + 255) / 256), dim3(256), 0, s, Hin, Hout, kh, vtab);
    const int64_t n = (int64_t)B * Hout * Wout;
    hipLaunchKernelGGL(resize_pass_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       hz ? tmp : in, out, B, Hin, Wout, Hout, Wout, vtab, kh);
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
