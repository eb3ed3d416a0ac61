// Batch normalization for channels-last activations viewed as a row-major [M, C] matrix
// (M = N*H*W, C % 8 == 0), bf16 or fp32 storage, fp32 math. Optional fused ReLU.
//
// Semantics = reference nn/layers/normalization/BatchNormalization.java (biased batch variance, eps added
// before sqrt, running stats: run = decay*run + (1-decay)*stat, running var tracks var+eps).
//
// Forward (training): stats_partial -> finalize (mean, invstd, running stats, per-channel scale/shift)
//                     -> apply (y = x*scale + shift [+relu]).  3 launches, x read twice, y written once.
// Backward:           bwd_partial (sum dy', sum dy'*xhat; dy' = relu-masked dy, mask recomputed from x)
//                     -> bwd_finalize (dgamma, dbeta into the flat gradient) -> bwd_apply.
// Each thread owns 8 consecutive channels (one 16-byte vector); a block covers R = 256/(C/8) rows per
// sweep, so every wave issues fully coalesced dwordx4 loads. Partial sums go to a [nblk, C] fp32
// workspace (no atomics -> bitwise reproducible).
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial(const T* __restrict__ x, long long M, int C,
                                                        long long rows_per_blk, float* __restrict__ part_s1,
                                                        float* __restrict__ part_s2, const float* __restrict__ shiftv) {
  const int T8 = C >> 3;
  const int R = 256 / T8;                       // rows per sweep
  const int cg = threadIdx.x % T8, r0 = threadIdx.x / T8;
  float s1[8], s2[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; sh[i] = shiftv[cg * 8 + i]; }
  const long long rbeg = (long long)blockIdx.x * rows_per_blk;
  long long rend = rbeg + rows_per_blk;
  if (rend > M) rend = M;
  if (r0 < R) {
    for (long long r = rbeg + r0; r < rend; r += R) {
      float v[8];
      Vec8<T>::load(x + r * C + cg * 8, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = v[i] - sh[i]; s1[i] += d; s2[i] += d * d; }
    }
  }
  // reduce the R partials of each channel group through LDS
  __shared__ float red1[2048];
  __shared__ float red2[2048];
  for (int i = 0; i < 8; ++i) {
    red1[threadIdx.x * 8 + i] = (r0 < R) ? s1[i] : 0.f;
    red2[threadIdx.x * 8 + i] = (r0 < R) ? s2[i] : 0.f;
  }
  __syncthreads();
  // thread t < C sums channel t over the R sweeps
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < R; ++rr) { a += red1[(rr * T8 + g) * 8 + k]; b += red2[(rr * T8 + g) * 8 + k]; }
    part_s1[(long long)blockIdx.x * C + c] = a;
    part_s2[(long long)blockIdx.x * C + c] = b;
  }
}

template <typename T>
__global__ void bn_shift_init(const T* __restrict__ x, int C, float* __restrict__ shiftv) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) shiftv[c] = ld1<T>(x + c);  // row 0 as the shift
}

// training=1: reduce partials -> mean/var; update running stats. training=0: use running stats.
__global__ void bn_finalize(const float* __restrict__ part_s1, const float* __restrict__ part_s2, int nblk, int C,
                            long long M, const float* __restrict__ shiftv, const float* __restrict__ gamma,
                            const float* __restrict__ beta, float gconst, float bconst, float* __restrict__ run_mean,
                            float* __restrict__ run_var, float decay, float eps, int training,
                            float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ scale,
                            float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, var;
  if (training) {
    double a = 0.0, b = 0.0;
    for (int i = 0; i < nblk; ++i) { a += part_s1[(long long)i * C + c]; b += part_s2[(long long)i * C + c]; }
    const double m1 = a / (double)M;
    mean = (float)(shiftv[c] + m1);
    double v = b / (double)M - m1 * m1;
    if (v < 0) v = 0;
    var = (float)v + eps;
    run_mean[c] = decay * run_mean[c] + (1.f - decay) * mean;
    run_var[c] = decay * run_var[c] + (1.f - decay) * var;
  } else {
    mean = run_mean[c];
    var = run_var[c];
  }
  const float inv = rsqrtf(var);
  const float g = gamma ? gamma[c] : gconst;
  const float bb = beta ? beta[c] : bconst;
  mean_out[c] = mean;
  invstd_out[c] = inv;
  scale[c] = g * inv;
  shift[c] = bb - mean * g * inv;
}

template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bn_apply(const T* __restrict__ x, T* __restrict__ y, long long M, int C,
                                                const float* __restrict__ scale, const float* __restrict__ shift) {
  const long long nvec = M * (C >> 3);
  const int T8 = C >> 3;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(v % T8);
    float a[8];
    Vec8<T>::load(x + v * 8, a);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = a[i] * scale[cg * 8 + i] + shift[cg * 8 + i];
      a[i] = RELU ? fmaxf(t, 0.f) : t;
    }
    Vec8<T>::store(y + v * 8, a);
  }
}

// ---------------------------------------------------------------------------------------- backward
template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_partial(const T* __restrict__ x, const T* __restrict__ dy, long long M,
                                                      int C, long long rows_per_blk, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, float* __restrict__ part_db,
                                                      float* __restrict__ part_dg) {
  const int T8 = C >> 3;
  const int R = 256 / T8;
  const int cg = threadIdx.x % T8, r0 = threadIdx.x / T8;
  float db[8], dg[8], mu[8], is[8], sc[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    db[i] = 0.f; dg[i] = 0.f;
    mu[i] = mean[cg * 8 + i]; is[i] = invstd[cg * 8 + i];
    sc[i] = scale[cg * 8 + i]; sf[i] = shift[cg * 8 + i];
  }
  const long long rbeg = (long long)blockIdx.x * rows_per_blk;
  long long rend = rbeg + rows_per_blk;
  if (rend > M) rend = M;
  if (r0 < R) {
    for (long long r = rbeg + r0; r < rend; r += R) {
      float xv[8], gv[8];
      Vec8<T>::load(x + r * C + cg * 8, xv);
      Vec8<T>::load(dy + r * C + cg * 8, gv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = gv[i];
        if (RELU) d = (xv[i] * sc[i] + sf[i] > 0.f) ? d : 0.f;
        db[i] += d;
        dg[i] += d * (xv[i] - mu[i]) * is[i];
      }
    }
  }
  __shared__ float red1[2048];
  __shared__ float red2[2048];
  for (int i = 0; i < 8; ++i) {
    red1[threadIdx.x * 8 + i] = (r0 < R) ? db[i] : 0.f;
    red2[threadIdx.x * 8 + i] = (r0 < R) ? dg[i] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < R; ++rr) { a += red1[(rr * T8 + g) * 8 + k]; b += red2[(rr * T8 + g) * 8 + k]; }
    part_db[(long long)blockIdx.x * C + c] = a;
    part_dg[(long long)blockIdx.x * C + c] = b;
  }
}

__global__ void bn_bwd_finalize(const float* __restrict__ part_db, const float* __restrict__ part_dg, int nblk, int C,
                                long long M, float* __restrict__ dbeta, float* __restrict__ dgamma,
                                float* __restrict__ cdb, float* __restrict__ cdg) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
  for (int i = 0; i < nblk; ++i) { a += part_db[(long long)i * C + c]; b += part_dg[(long long)i * C + c]; }
  if (dbeta) dbeta[c] = (float)a;
  if (dgamma) dgamma[c] = (float)b;
  cdb[c] = (float)(a / (double)M);
  cdg[c] = (float)(b / (double)M);
}

template <typename T, bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_apply(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx,
                                                    long long M, int C, const float* __restrict__ mean,
                                                    const float* __restrict__ invstd, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, const float* __restrict__ cdb,
                                                    const float* __restrict__ cdg) {
  const long long nvec = M * (C >> 3);
  const int T8 = C >> 3;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)(v % T8) * 8;
    float xv[8], gv[8];
    Vec8<T>::load(x + v * 8, xv);
    Vec8<T>::load(dy + v * 8, gv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = c0 + i;
      float d = gv[i];
      if (RELU) d = (xv[i] * scale[c] + shift[c] > 0.f) ? d : 0.f;
      const float xh = (xv[i] - mean[c]) * invstd[c];
      // dx = gamma*invstd * (dy' - mean(dy') - xhat*mean(dy'*xhat));  gamma*invstd == scale
      xv[i] = scale[c] * (d - cdb[c] - xh * cdg[c]);
    }
    Vec8<T>::store(dx + v * 8, xv);
  }
}

static inline void bn_grid(long long M, int C, int* nblk, long long* rows_per_blk) {
  const int T8 = C / 8;
  const long long work = M * T8;                  // vector loads
  long long nb = work / (256LL * 32);             // >= 32 vector loads per thread
  if (nb < 1) nb = 1;
  if (nb > 1024) nb = 1024;
  long long rpb = (M + nb - 1) / nb;
  nb = (M + rpb - 1) / rpb;
  *nblk = (int)nb;
  *rows_per_blk = rpb;
}

static inline int apply_grid(long long M, int C) {
  long long nvec = M * (C / 8);
  long long g = (nvec + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

DL4J_API int dl4j_bn_workspace_floats(long long M, int C) {
  int nblk; long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  return 2 * nblk * C + 8 * C;
}

// dtype: 0 fp32, 1 bf16. ws: >= dl4j_bn_workspace_floats floats. ctx_out: 4*C floats (mean, invstd, scale, shift)
DL4J_API int dl4j_bn_fwd(int dtype, const void* x, void* y, long long M, int C, const float* gamma, const float* beta,
                         float gconst, float bconst, float* run_mean, float* run_var, float decay, float eps,
                         int training, int relu, float* ws, float* ctx_out, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256) return -1;
  int nblk; long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* shiftv = p2 + (long long)nblk * C;
  float *mean = ctx_out, *inv = ctx_out + C, *scale = ctx_out + 2 * C, *shift = ctx_out + 3 * C;
  if (training) {
    if (dtype == 1) {
      hipLaunchKernelGGL(bn_shift_init<bf16>, dim3(1), dim3(256), 0, s, (const bf16*)x, C, shiftv);
      hipLaunchKernelGGL(bn_stats_partial<bf16>, dim3(nblk), dim3(256), 0, s, (const bf16*)x, M, C, rpb, p1, p2, shiftv);
    } else {
      hipLaunchKernelGGL(bn_shift_init<float>, dim3(1), dim3(256), 0, s, (const float*)x, C, shiftv);
      hipLaunchKernelGGL(bn_stats_partial<float>, dim3(nblk), dim3(256), 0, s, (const float*)x, M, C, rpb, p1, p2, shiftv);
    }
  }
  hipLaunchKernelGGL(bn_finalize, dim3((C + 255) / 256), dim3(256), 0, s, p1, p2, nblk, C, M, shiftv, gamma, beta, gconst,
                     bconst, run_mean, run_var, decay, eps, training, mean, inv, scale, shift);
  const int ag = apply_grid(M, C);
  if (dtype == 1) {
    if (relu) hipLaunchKernelGGL((bn_apply<bf16, true>), dim3(ag), dim3(256), 0, s, (const bf16*)x, (bf16*)y, M, C, scale, shift);
    else hipLaunchKernelGGL((bn_apply<bf16, false>), dim3(ag), dim3(256), 0, s, (const bf16*)x, (bf16*)y, M, C, scale, shift);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply<float, true>), dim3(ag), dim3(256), 0, s, (const float*)x, (float*)y, M, C, scale, shift);
    else hipLaunchKernelGGL((bn_apply<float, false>), dim3(ag), dim3(256), 0, s, (const float*)x, (float*)y, M, C, scale, shift);
  }
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bn_bwd(int dtype, const void* x, const void* dy, void* dx, long long M, int C, const float* ctx,
                         float* dgamma, float* dbeta, int relu, float* ws, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256) return -1;
  int nblk; long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* cdb = p2 + (long long)nblk * C;
  float* cdg = cdb + C;
  const float *mean = ctx, *inv = ctx + C, *scale = ctx + 2 * C, *shift = ctx + 3 * C;
#define BWD_PART(T, R) hipLaunchKernelGGL((bn_bwd_partial<T, R>), dim3(nblk), dim3(256), 0, s, (const T*)x, (const T*)dy, M, C, rpb, mean, inv, scale, shift, p1, p2)
  if (dtype == 1) { if (relu) BWD_PART(bf16, true); else BWD_PART(bf16, false); }
  else { if (relu) BWD_PART(float, true); else BWD_PART(float, false); }
#undef BWD_PART
  hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + 255) / 256), dim3(256), 0, s, p1, p2, nblk, C, M, dbeta, dgamma, cdb, cdg);
  const int ag = apply_grid(M, C);
#define BWD_APPLY(T, R) hipLaunchKernelGGL((bn_bwd_apply<T, R>), dim3(ag), dim3(256), 0, s, (const T*)x, (const T*)dy, (T*)dx, M, C, mean, inv, scale, shift, cdb, cdg)
  if (dtype == 1) { if (relu) BWD_APPLY(bf16, true); else BWD_APPLY(bf16, false); }
  else { if (relu) BWD_APPLY(float, true); else BWD_APPLY(float, false); }
#undef BWD_APPLY
  return (int)hipGetLastError();
}
