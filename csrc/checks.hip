// Numerical panic checks (ND4J OpExecutioner.ProfilingMode NAN_PANIC / INF_PANIC / ANY_PANIC parity,
// SURVEY §5.1-5.2; reference enables them via Nd4j.getExecutioner().setProfilingMode, CORET:BaseDL4JTest.java:11-16).
// One launch counts NaN and ±Inf elements over a LIST of device arrays (a layer's output + its gradient views):
// 16-byte vector loads, per-wave ballot popcounts, one atomic pair per wave. The host reads the two counters only
// when a panic mode is on, so the training hot path never pays for it.
#include "common.h"

struct CheckSeg {
  const void* ptr;
  long long n;
  int dtype;          // 0 fp32, 1 bf16
  int pad;
};

__device__ __forceinline__ void classify(float v, unsigned& nan_c, unsigned& inf_c) {
  nan_c += (v != v);
  inf_c += (fabsf(v) == INFINITY);
}

__global__ void __launch_bounds__(256) nonfinite_kernel(const CheckSeg* __restrict__ segs, int nseg,
                                                        unsigned long long* __restrict__ counts) {
  const CheckSeg sg = segs[blockIdx.y];
  unsigned nan_c = 0, inf_c = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (sg.dtype == 0) {
    const float* p = reinterpret_cast<const float*>(sg.ptr);
    const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
    const long long nv = al ? sg.n / 4 : 0;
    for (long long i = tid; i < nv; i += stride) {
      const f32x4 v = reinterpret_cast<const f32x4*>(p)[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) classify(v.v[k], nan_c, inf_c);
    }
    for (long long i = nv * 4 + tid; i < sg.n; i += stride) classify(p[i], nan_c, inf_c);
  } else {
    const u16* p = reinterpret_cast<const u16*>(sg.ptr);
    const bool al = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
    const long long nv = al ? sg.n / 8 : 0;
    for (long long i = tid; i < nv; i += stride) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(p)[i];
#pragma unroll
      for (int k = 0; k < 8; ++k) classify(bf2f(v.v[k]), nan_c, inf_c);
    }
    for (long long i = nv * 8 + tid; i < sg.n; i += stride) classify(bf2f(p[i]), nan_c, inf_c);
  }
  // wave totals, one atomic pair per wave
  float a = (float)nan_c, b = (float)inf_c;
  a = wave_sum(a);
  b = wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    if (a > 0.f) atomicAdd(counts + 2 * blockIdx.y, (unsigned long long)a);
    if (b > 0.f) atomicAdd(counts + 2 * blockIdx.y + 1, (unsigned long long)b);
  }
}

// segs: host array of nseg {ptr, n, dtype}; seg_dev: device scratch of nseg CheckSeg; counts: device [nseg][2]
// (zeroed here). Asynchronous on stream s.
DL4J_API int dl4j_nonfinite_count(const void* segs, int nseg, void* seg_dev, unsigned long long* counts,
                                  long long max_n, hipStream_t s) {
  if (nseg <= 0) return 0;
  hipError_t e = hipMemcpyAsync(seg_dev, segs, sizeof(CheckSeg) * nseg, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return (int)e;
  e = hipMemsetAsync(counts, 0, sizeof(unsigned long long) * 2 * nseg, s);
  if (e != hipSuccess) return (int)e;
  long long blocks = (max_n / 8 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)blocks, nseg), dim3(256), 0, s,
                     reinterpret_cast<const CheckSeg*>(seg_dev), nseg, counts);
  return (int)hipGetLastError();
}
