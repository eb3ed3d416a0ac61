// Fused softmax + multi-class cross-entropy (MCXENT / NLL), forward score AND gradient in one pass.
// Reference: LossMCXENT with softmax: grad = softmax(z) - y, score_row = -sum y*log(clip(p, eps, 1-eps))
// (called from BaseOutputLayer.java:82-92,173). One 256-thread block per row: row max and exp-sum by
// wave shuffles + LDS, logits read twice (L2-resident), gradient written once.
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const T* __restrict__ z, const float* __restrict__ y, int V,
                                                           T* __restrict__ grad, float* __restrict__ score,
                                                           float* __restrict__ prob, float log_eps, float log_1m_eps,
                                                           const float* __restrict__ rmask) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  // per-row mask (masked time steps of an RNN output): the row's score and gradient are scaled by it
  const float mr = rmask ? rmask[row] : 1.f;
  const T* zr = z + row * V;
  const float* yr = y + row * V;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < V; j += blockDim.x) m = fmaxf(m, ld1<T>(zr + j));
  m = block_reduce<true>(m, red);
  float s = 0.f;
  for (int j = threadIdx.x; j < V; j += blockDim.x) s += __expf(ld1<T>(zr + j) - m);
  s = block_reduce<false>(s, red);
  const float lse = m + __logf(s);
  const float inv = 1.f / s;
  float sc = 0.f;
  for (int j = threadIdx.x; j < V; j += blockDim.x) {
    const float zj = ld1<T>(zr + j);
    const float p = __expf(zj - m) * inv;
    const float yj = yr[j];
    float lp = zj - lse;
    lp = fminf(fmaxf(lp, log_eps), log_1m_eps);
    sc -= yj * lp;
    st1<T>(grad + row * V + j, (p - yj) * mr);
    if (prob) prob[row * V + j] = p;
  }
  sc = block_reduce<false>(sc, red);
  if (threadIdx.x == 0) score[row] = sc * mr;
}

// Strided variant: logits rows with leading dimension ldz; label row r = t*mb + b (t = r / mb, b = r % mb) read at
// y + b*ys_b + t*ys_t + j*ys_j, so the RNN output layer's [mb, V, T] labels are consumed in place (2-D labels: mb = B,
// ys_t = 0); gradient rows have leading dimension ldg >= V with columns V..ldg-1 written as zeros — the gradient is
// directly a zero-K-padded GEMM operand for dW = hᵀ·g and dx = g·Wᵀ (ops/gemm.py kz_view).
template <typename T>
__global__ __launch_bounds__(256) void softmax_xent_strided(const T* __restrict__ z, int ldz, const float* __restrict__ y,
                                                            long long ys_b, long long ys_t, long long ys_j, int mb,
                                                            int V, T* __restrict__ grad, int ldg,
                                                            float* __restrict__ score, float log_eps,
                                                            float log_1m_eps) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  const T* zr = z + row * ldz;
  const float* yr = y + (row % mb) * ys_b + (row / mb) * ys_t;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < V; j += blockDim.x) m = fmaxf(m, ld1<T>(zr + j));
  m = block_reduce<true>(m, red);
  float s = 0.f;
  for (int j = threadIdx.x; j < V; j += blockDim.x) s += __expf(ld1<T>(zr + j) - m);
  s = block_reduce<false>(s, red);
  const float lse = m + __logf(s);
  const float inv = 1.f / s;
  float sc = 0.f;
  for (int j = threadIdx.x; j < ldg; j += blockDim.x) {
    if (j < V) {
      const float zj = ld1<T>(zr + j);
      const float p = __expf(zj - m) * inv;
      const float yj = yr[j * ys_j];
      float lp = zj - lse;
      lp = fminf(fmaxf(lp, log_eps), log_1m_eps);
      sc -= yj * lp;
      st1<T>(grad + row * ldg + j, p - yj);
    } else {
      st1<T>(grad + row * ldg + j, 0.f);
    }
  }
  sc = block_reduce<false>(sc, red);
  if (threadIdx.x == 0) score[row] = sc;
}

DL4J_API int dl4j_softmax_xent_strided(int dtype, const void* z, int ldz, const float* y, long long ys_b,
                                       long long ys_t, long long ys_j, int mb, int B, int V, void* grad, int ldg,
                                       float* score, float clip_eps, hipStream_t s) {
  if (B <= 0) return 0;
  if (mb <= 0 || ldz < V || ldg < V) return -1;
  const float le = clip_eps > 0.f ? logf(clip_eps) : -INFINITY;
  const float l1 = clip_eps > 0.f ? log1pf(-clip_eps) : 0.f;
#define SXS(T) hipLaunchKernelGGL(softmax_xent_strided<T>, dim3(B), dim3(256), 0, s, (const T*)z, ldz, y, ys_b, ys_t, \
                                  ys_j, mb, V, (T*)grad, ldg, score, le, l1)
  if (dtype == 1) SXS(bf16);
  else if (dtype == 2) SXS(f16);
  else if (dtype == 0) SXS(float);
  else return -1;
#undef SXS
  return (int)hipGetLastError();
}

static int softmax_xent_launch(int dtype, const void* z, const float* y, int B, int V, void* grad, float* score,
                               float* prob, float clip_eps, const float* rmask, hipStream_t s) {
  const float le = clip_eps > 0.f ? logf(clip_eps) : -INFINITY;
  const float l1 = clip_eps > 0.f ? log1pf(-clip_eps) : 0.f;
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_xent_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)z, y, V, (bf16*)grad, score,
                       prob, le, l1, rmask);
  else if (dtype == 2)
    hipLaunchKernelGGL(softmax_xent_kernel<f16>, dim3(B), dim3(256), 0, s, (const f16*)z, y, V, (f16*)grad, score,
                       prob, le, l1, rmask);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)z, y, V, (float*)grad, score,
                       prob, le, l1, rmask);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_softmax_xent(int dtype, const void* z, const float* y, int B, int V, void* grad, float* score,
                               float* prob, float clip_eps, hipStream_t s) {
  return softmax_xent_launch(dtype, z, y, B, V, grad, score, prob, clip_eps, nullptr, s);
}

// rmask: fp32 [B] per-row mask (RNN output time-step masks as [T*mb] rows)
DL4J_API int dl4j_softmax_xent_masked(int dtype, const void* z, const float* y, int B, int V, void* grad, float* score,
                                      const float* rmask, float clip_eps, hipStream_t s) {
  if (!rmask) return -1;
  return softmax_xent_launch(dtype, z, y, B, V, grad, score, nullptr, clip_eps, rmask, s);
}

// ------------------------------------------------------------------------------------------------ score scalar
// out[0] = (sum_{i<n} s[i] + add) * scale + (reg ? reg[0] * reg_scale : 0), one 256-thread block, fixed summation
// order (bitwise reproducible). The training score on the device without library reduce / elementwise kernels:
// per-example losses -> minibatch score (BaseOutputLayer.computeScore: (sum + l1 + l2) / minibatch), and the
// updater's per-block regularisation partials folded into it. out may alias reg.
__global__ __launch_bounds__(256) void score_reduce(const float* __restrict__ s, long long n, float add, float scale,
                                                    const float* reg, float reg_scale, float* out) {
  __shared__ float red[256];
  float acc = 0.f;
  for (long long i = threadIdx.x; i < n; i += 256) acc += s[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float r = reg ? reg[0] * reg_scale : 0.f;
    out[0] = (red[0] + add) * scale + r;
  }
}

DL4J_API int dl4j_score_reduce(const float* s, long long n, float add, float scale, const float* reg, float reg_scale,
                               float* out, hipStream_t st) {
  hipLaunchKernelGGL(score_reduce, dim3(1), dim3(256), 0, st, s, n, add, scale, reg, reg_scale, out);
  return (int)hipGetLastError();
}
