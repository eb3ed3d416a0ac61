// Fused elementwise activation kernels for the transformer FFN: exact (erf) GELU forward and its backward
// dz = dy * (Phi(z) + z * phi(z)), bf16/fp32 I/O with fp32 math, 8 elements (16 B for bf16) per thread per step.
// Replaces the 5-6 separate fp32 elementwise launches (+ bf16<->fp32 copies) of an unfused backward.
#include "common.h"

__device__ __forceinline__ float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_d(float z) {
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.3989422804014327f * __expf(-0.5f * z * z);
}

template <typename T, bool BWD>
__global__ void __launch_bounds__(256) gelu_kernel(const T* __restrict__ z, const T* __restrict__ dy,
                                                   T* __restrict__ out, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float a[8], o[8];
    Vec8<T>::load(z + i * 8, a);
    if (BWD) {
      float g[8];
      Vec8<T>::load(dy + i * 8, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = g[k] * gelu_d(a[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = gelu_f(a[k]);
    }
    Vec8<T>::store(out + i * 8, o);
  }
}

template <typename T>
static int gelu_l(const void* z, const void* dy, void* out, long long n, hipStream_t s) {
  const long long n8 = n / 8;
  long long blocks = (n8 + 255) / 256;
  blocks = blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks);
  if (dy)
    hipLaunchKernelGGL((gelu_kernel<T, true>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)z, (const T*)dy,
                       (T*)out, n8);
  else
    hipLaunchKernelGGL((gelu_kernel<T, false>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)z, (const T*)nullptr,
                       (T*)out, n8);
  return (int)hipGetLastError();
}

// dy == null: out = gelu(z); else out = dy * gelu'(z). n % 8 == 0 and 16-byte aligned buffers (else -1).
DL4J_API int dl4j_gelu(int dtype, const void* z, const void* dy, void* out, long long n, hipStream_t s) {
  if (n % 8 != 0 || (reinterpret_cast<uintptr_t>(z) & 15) || (reinterpret_cast<uintptr_t>(out) & 15) ||
      (dy && (reinterpret_cast<uintptr_t>(dy) & 15)))
    return -1;
  if (dtype == 1) return gelu_l<bf16>(z, dy, out, n, s);
  if (dtype == 2) return gelu_l<f16>(z, dy, out, n, s);
  if (dtype == 0) return gelu_l<float>(z, dy, out, n, s);
  return -1;
}
