// LayerNorm forward / backward for gfx950, with the transformer residual add fused in:
//   s = x (+ r);  y = (s - mean(s)) * rstd * gamma + beta,  rstd = 1/sqrt(var(s) + eps)   (biased var)
// One wave per row: 16-byte vector loads (8 elements per lane per chunk), the row held in registers, fp32 stats by
// wave shuffles (exact two-pass: mean, then centred variance), no LDS and no block barriers. Saves mean/rstd
// (fp32, per row) for the backward.
// Backward: dxhat = dy*gamma; ds = rstd*(dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)) (the same gradient flows to
// x and r); dgamma/dbeta column sums are accumulated per block in registers and written as per-block partials,
// reduced by a second small kernel (no atomics: deterministic).
#include "common.h"

template <typename T> struct V8;
template <> struct V8<bf16> {
  static __device__ __forceinline__ void ld(const bf16* p, float* o) { Vec8<bf16>::load(p, o); }
  static __device__ __forceinline__ void st(bf16* p, const float* o) { Vec8<bf16>::store(p, o); }
};
template <> struct V8<f16> {
  static __device__ __forceinline__ void ld(const f16* p, float* o) { Vec8<f16>::load(p, o); }
  static __device__ __forceinline__ void st(f16* p, const float* o) { Vec8<f16>::store(p, o); }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void ld(const float* p, float* o) { Vec8<float>::load(p, o); }
  static __device__ __forceinline__ void st(float* p, const float* o) { Vec8<float>::store(p, o); }
};

// CH = 8-element chunks per lane (N <= 512*CH)
template <typename T, int CH, bool RES>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     T* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long long M, int N, float eps) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = N >> 3;
  float v[CH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      V8<T>::ld(x + row * N + ch * 8, v[c]);
      if (RES) {
        float rr[8];
        V8<T>::ld(r + row * N + ch * 8, rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[c][k] += rr[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[c][k];
    }
  }
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    if (lane + c * 64 < nch) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[c][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float g[8], b[8], o[8];
      Vec8<float>::load(gamma + ch * 8, g);
      Vec8<float>::load(beta + ch * 8, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (v[c][k] - mean) * rstd * g[k] + b[k];
      V8<T>::st(y + row * N + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Each block: 4 waves x RPW rows; per-lane column partials of dgamma/dbeta written to part[blockIdx.x][2][N].
template <typename T, int CH, bool RES, int RPW>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ r, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     T* __restrict__ dx, float* __restrict__ part, long long M, int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = N >> 3;
  float dg[CH][8], db[CH][8], g[CH][8];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[c][k] = db[c][k] = 0.f;
    if (ch < nch) Vec8<float>::load(gamma + ch * 8, g[c]);
  }
  for (int i = 0; i < RPW; ++i) {
    const long long row = ((long long)blockIdx.x * 4 + wave) * RPW + i;
    if (row >= M) break;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[CH][8], d[CH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float xv[8], dv[8];
        V8<T>::ld(x + row * N + ch * 8, xv);
        if (RES) {
          float rr[8];
          V8<T>::ld(r + row * N + ch * 8, rr);
#pragma unroll
          for (int k = 0; k < 8; ++k) xv[k] += rr[k];
        }
        V8<T>::ld(dy + row * N + ch * 8, dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[c][k] = (xv[k] - mean) * rstd;
          d[c][k] = dv[k] * g[c][k];
          s1 += d[c][k];
          s2 += d[c][k] * xh[c][k];
          dg[c][k] += dv[k] * xh[c][k];
          db[c][k] += dv[k];
        }
      }
    }
    const float m1 = wave_sum(s1) / N, m2 = wave_sum(s2) / N;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (d[c][k] - m1 - xh[c][k] * m2);
        V8<T>::st(dx + row * N + ch * 8, o);
      }
    }
  }
  // per-wave partials: part[(blockIdx.x*4 + wave)][0/1][N]
  float* pg = part + ((long long)blockIdx.x * 4 + wave) * 2 * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::store(pg + ch * 8, dg[c]);
      Vec8<float>::store(pg + N + ch * 8, db[c]);
    }
  }
}

// out[0/1][N] = sum over P partial rows. Block = 32 columns x 8 row groups (coalesced 128-byte row reads), the 8
// group sums combined through LDS.
__global__ void __launch_bounds__(256) ln_bwd_reduce(const float* __restrict__ part, int P, int N,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + cl;                          // over the concatenated [dgamma | dbeta] columns
  float s = 0.f;
  if (j < 2 * N) {
    const int which = j / N, col = j - which * N;
    const float* src = part + which * N + col;
    for (int p = rg; p < P; p += 8) s += src[(long long)p * 2 * N];
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < 2 * N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][cl];
    const int which = j / N, col = j - which * N;
    (which == 0 ? dgamma : dbeta)[col] = t;
  }
}

template <typename T, int CH>
static int fwd_l(const void* x, const void* r, const float* g, const float* b, void* y, float* mean, float* rstd,
                 long long M, int N, float eps, hipStream_t s) {
  const dim3 grid((unsigned)((M + 3) / 4));
  if (r)
    hipLaunchKernelGGL((ln_fwd_kernel<T, CH, true>), grid, dim3(256), 0, s, (const T*)x, (const T*)r, g, b, (T*)y,
                       mean, rstd, M, N, eps);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<T, CH, false>), grid, dim3(256), 0, s, (const T*)x, (const T*)nullptr, g, b,
                       (T*)y, mean, rstd, M, N, eps);
  return (int)hipGetLastError();
}

static constexpr int kRPW = 16;

static long long ln_bwd_partials(long long M) { return ((M + 4 * kRPW - 1) / (4 * kRPW)) * 4; }

template <typename T, int CH>
static int bwd_l(const void* dy, const void* x, const void* r, const float* g, const float* mean, const float* rstd,
                 void* dx, float* part, float* dgamma, float* dbeta, long long M, int N, hipStream_t s) {
  const long long blocks = (M + 4 * kRPW - 1) / (4 * kRPW);
  if (r)
    hipLaunchKernelGGL((ln_bwd_kernel<T, CH, true, kRPW>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)x, (const T*)r, g, mean, rstd, (T*)dx, part, M, N);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<T, CH, false, kRPW>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)x, (const T*)nullptr, g, mean, rstd, (T*)dx, part, M, N);
  const int P = (int)(blocks * 4);
  hipLaunchKernelGGL(ln_bwd_reduce, dim3((2 * N + 31) / 32), dim3(256), 0, s, part, P, N, dgamma, dbeta);
  return (int)hipGetLastError();
}

#define LN_CH_DISPATCH(FN, T, ...)                       \
  do {                                                   \
    if (N <= 512) return FN<T, 1>(__VA_ARGS__);          \
    if (N <= 1024) return FN<T, 2>(__VA_ARGS__);         \
    if (N <= 2048) return FN<T, 4>(__VA_ARGS__);         \
    if (N <= 4096) return FN<T, 8>(__VA_ARGS__);         \
    return -1;                                           \
  } while (0)

DL4J_API long long dl4j_ln_partial_rows(long long M) { return ln_bwd_partials(M); }

// dtype 0 fp32, 1 bf16, 2 fp16. r may be null (no residual). Returns -1 when N is unsupported (N % 8 or N > 4096).
DL4J_API int dl4j_ln_fwd(int dtype, const void* x, const void* r, const float* gamma, const float* beta, void* y,
                         float* mean, float* rstd, long long M, int N, float eps, hipStream_t s) {
  if (N % 8 != 0 || N > 4096 || M < 1) return -1;
  if (dtype == 1) LN_CH_DISPATCH(fwd_l, bf16, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
  if (dtype == 2) LN_CH_DISPATCH(fwd_l, f16, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
  LN_CH_DISPATCH(fwd_l, float, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
}

// part: fp32 workspace of dl4j_ln_partial_rows(M) * 2 * N floats.
DL4J_API int dl4j_ln_bwd(int dtype, const void* dy, const void* x, const void* r, const float* gamma,
                         const float* mean, const float* rstd, void* dx, float* part, float* dgamma, float* dbeta,
                         long long M, int N, hipStream_t s) {
  if (N % 8 != 0 || N > 4096 || M < 1) return -1;
  if (dtype == 1) LN_CH_DISPATCH(bwd_l, bf16, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, M, N, s);
  if (dtype == 2) LN_CH_DISPATCH(bwd_l, f16, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, M, N, s);
  LN_CH_DISPATCH(bwd_l, float, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, M, N, s);
}
