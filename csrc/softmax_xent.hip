// Fused softmax + multi-class cross-entropy (MCXENT / NLL), forward score AND gradient in one pass.
// Reference: LossMCXENT with softmax: grad = softmax(z) - y, score_row = -sum y*log(clip(p, eps, 1-eps))
// (called from BaseOutputLayer.java:82-92,173). One 256-thread block per row: row max and exp-sum by
// wave shuffles + LDS, logits read twice (L2-resident), gradient written once.
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const T* __restrict__ z, const float* __restrict__ y, int V,
                                                           T* __restrict__ grad, float* __restrict__ score,
                                                           float* __restrict__ prob, float log_eps, float log_1m_eps) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
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
    st1<T>(grad + row * V + j, p - yj);
    if (prob) prob[row * V + j] = p;
  }
  sc = block_reduce<false>(sc, red);
  if (threadIdx.x == 0) score[row] = sc;
}

DL4J_API int dl4j_softmax_xent(int dtype, const void* z, const float* y, int B, int V, void* grad, float* score,
                               float* prob, float clip_eps, hipStream_t s) {
  const float le = clip_eps > 0.f ? logf(clip_eps) : -INFINITY;
  const float l1 = clip_eps > 0.f ? log1pf(-clip_eps) : 0.f;
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_xent_kernel<bf16>, dim3(B), dim3(256), 0, s, (const bf16*)z, y, V, (bf16*)grad, score,
                       prob, le, l1);
  else if (dtype == 2)
    hipLaunchKernelGGL(softmax_xent_kernel<f16>, dim3(B), dim3(256), 0, s, (const f16*)z, y, V, (f16*)grad, score,
                       prob, le, l1);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)z, y, V, (float*)grad, score,
                       prob, le, l1);
  return (int)hipGetLastError();
}
