// 2D max / average pooling on channels-last (NHWC) activations, bf16 or fp32.
// Reference: SubsamplingLayer.java:207-263,341-358; CudnnSubsamplingHelper (MAX / AVERAGE_COUNT_INCLUDE_PADDING).
// Forward: one thread per (n, oh, ow, 8-channel group); MAX stores the in-window argmax as one byte per
// element for the backward. Backward is a GATHER (each input pixel sums the windows that chose it), so
// overlapping windows (3x3/2) need no atomics and results are deterministic.
#include "common.h"

template <typename T, bool MAX>
__global__ __launch_bounds__(256) void pool_fwd(const T* __restrict__ x, T* __restrict__ y, unsigned char* __restrict__ am,
                                                int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh,
                                                int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * OH * OW * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    int cg, ow, oh, n;
    idx_decomp4(t, CG, OW, OH, cg, ow, oh, n);
    float acc[8];
    unsigned char idx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { acc[i] = MAX ? -INFINITY : 0.f; idx[i] = 0; }
    for (int i = 0; i < kh; ++i) {
      const int ih = oh * sh - pt + i;
      if (ih < 0 || ih >= H) continue;
      for (int j = 0; j < kw; ++j) {
        const int iw = ow * sw - pl + j;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        Vec8<T>::load(x + (((long long)n * H + ih) * W + iw) * C + cg * 8, v);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          if (MAX) { if (v[c] > acc[c]) { acc[c] = v[c]; idx[c] = (unsigned char)(i * kw + j); } }
          else acc[c] += v[c];
        }
      }
    }
    if (!MAX) {
      const float inv = 1.f / (float)(kh * kw);
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] *= inv;
    }
    Vec8<T>::store(y + t * 8, acc);
    if (MAX) {
      unsigned long long pk = 0;
#pragma unroll
      for (int c = 0; c < 8; ++c) pk |= ((unsigned long long)idx[c]) << (8 * c);
      *reinterpret_cast<unsigned long long*>(am + t * 8) = pk;
    }
  }
}

template <typename T, bool MAX>
__global__ __launch_bounds__(256) void pool_bwd(const T* __restrict__ dy, const unsigned char* __restrict__ am,
                                                T* __restrict__ dx, int N, int H, int W, int C, int OH, int OW, int kh,
                                                int kw, int sh, int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * H * W * CG;
  const float inv = 1.f / (float)(kh * kw);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    int cg, iw, ih, n;
    idx_decomp4(t, CG, W, H, cg, iw, ih, n);
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    const int hp = ih + pt, wp = iw + pl;
    int oh0 = hp - kh + 1; oh0 = oh0 <= 0 ? 0 : (oh0 + sh - 1) / sh;
    int ow0 = wp - kw + 1; ow0 = ow0 <= 0 ? 0 : (ow0 + sw - 1) / sw;
    const int oh1 = min(hp / sh, OH - 1), ow1 = min(wp / sw, OW - 1);
    for (int oh = oh0; oh <= oh1; ++oh) {
      for (int ow = ow0; ow <= ow1; ++ow) {
        const long long o = (((long long)n * OH + oh) * OW + ow) * C + cg * 8;
        float g[8];
        Vec8<T>::load(dy + o, g);
        if (MAX) {
          const unsigned long long pk = *reinterpret_cast<const unsigned long long*>(am + o);
          const unsigned char me = (unsigned char)((hp - oh * sh) * kw + (wp - ow * sw));
#pragma unroll
          for (int c = 0; c < 8; ++c) if (((pk >> (8 * c)) & 0xff) == me) acc[c] += g[c];
        } else {
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[c] += g[c] * inv;
        }
      }
    }
    Vec8<T>::store(dx + t * 8, acc);
  }
}

static inline int grid_for(long long total) {
  long long g = (total + 255) / 256;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

// mode: 0 max, 1 avg. argmax: N*OH*OW*C bytes (max only).
DL4J_API int dl4j_pool_fwd(int dtype, int mode, const void* x, void* y, unsigned char* argmax, int N, int H, int W, int C,
                           int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl, hipStream_t s) {
  if (C % 8 != 0 || kh * kw > 255) return -1;
  const int g = grid_for((long long)N * OH * OW * (C / 8));
#define PF(T, M) hipLaunchKernelGGL((pool_fwd<T, M>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, argmax, N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl)
  if (dtype == 1) { if (mode == 0) PF(bf16, true); else PF(bf16, false); }
  else if (dtype == 2) { if (mode == 0) PF(f16, true); else PF(f16, false); }
  else { if (mode == 0) PF(float, true); else PF(float, false); }
#undef PF
  return (int)hipGetLastError();
}

DL4J_API int dl4j_pool_bwd(int dtype, int mode, const void* dy, const unsigned char* argmax, void* dx, int N, int H, int W,
                           int C, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl, hipStream_t s) {
  if (C % 8 != 0) return -1;
  const int g = grid_for((long long)N * H * W * (C / 8));
#define PB(T, M) hipLaunchKernelGGL((pool_bwd<T, M>), dim3(g), dim3(256), 0, s, (const T*)dy, argmax, (T*)dx, N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl)
  if (dtype == 1) { if (mode == 0) PB(bf16, true); else PB(bf16, false); }
  else if (dtype == 2) { if (mode == 0) PB(f16, true); else PB(f16, false); }
  else { if (mode == 0) PB(float, true); else PB(float, false); }
#undef PB
  return (int)hipGetLastError();
}
