// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of deeplearning4j_amd.
// Wave size is 64 on CDNA; everything here is written for that.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DL4J_API extern "C" __attribute__((visibility("default")))

typedef __hip_bfloat16 bf16;
typedef unsigned short u16;

// 8 x bf16 = 16 bytes: the coalescing sweet spot (one dwordx4 per lane).
struct __attribute__((aligned(16))) bf16x8 { u16 v[8]; };
struct __attribute__((aligned(16))) f32x4 { float v[4]; };

__device__ __forceinline__ float bf2f(u16 u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  bf16 b = __float2bfloat16(f);           // lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return *reinterpret_cast<u16*>(&b);
}

// Load / store 8 consecutive elements as float, for bf16 or fp32 storage.
template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* o) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = bf2f(v.v[i]);
  }
  static __device__ __forceinline__ void store(bf16* p, const float* o) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v.v[i] = f2bf(o[i]);
    *reinterpret_cast<bf16x8*>(p) = v;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* o) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a.v[i]; o[i + 4] = b.v[i]; }
  }
  static __device__ __forceinline__ void store(float* p, const float* o) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a.v[i] = o[i]; b.v[i] = o[i + 4]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};

// Raw 8-element vectors kept packed in registers until used (half the VGPRs of the unpacked floats for 16-bit T):
// RawVec8<T>::load issues the 16-byte (fp32: 2 x 16-byte) load, ::get unpacks element i.
template <typename T> struct RawVec8;
template <> struct RawVec8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ float get(int i) const { return i < 4 ? a.v[i] : b.v[i - 4]; }
};
template <> struct RawVec8<bf16> {
  uint4 q;
  __device__ __forceinline__ void load(const bf16* p) { q = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ float get(int i) const {
    const unsigned w = i < 2 ? q.x : (i < 4 ? q.y : (i < 6 ? q.z : q.w));
    return __uint_as_float((i & 1) ? (w & 0xffff0000u) : (w << 16));
  }
};

// fp16 storage (IEEE half, the MFMA f16 operand type); math stays fp32.
typedef _Float16 f16;
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
template <> struct RawVec8<f16> {
  uint4 q;
  __device__ __forceinline__ void load(const f16* p) { q = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ float get(int i) const {
    const unsigned w = i < 2 ? q.x : (i < 4 ? q.y : (i < 6 ? q.z : q.w));
    return (float)__builtin_bit_cast(_Float16, (unsigned short)((i & 1) ? (w >> 16) : (w & 0xffffu)));
  }
};
template <> struct Vec8<f16> {
  static __device__ __forceinline__ void load(const f16* p, float* o) {
    const f16x8_t v = *reinterpret_cast<const f16x8_t*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void store(f16* p, const float* o) {
    f16x8_t v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (f16)o[i];
    *reinterpret_cast<f16x8_t*>(p) = v;
  }
};

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<bf16>(const bf16* p) { return bf2f(*reinterpret_cast<const u16*>(p)); }
template <typename T> __device__ __forceinline__ void st1(T* p, float v);
template <> __device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st1<bf16>(bf16* p, float v) { *reinterpret_cast<u16*>(p) = f2bf(v); }
template <> __device__ __forceinline__ float ld1<f16>(const f16* p) { return (float)*p; }
template <> __device__ __forceinline__ void st1<f16>(f16* p, float v) { *p = (f16)v; }
// element i of a buffer whose dtype is only known at run time (0 fp32, 1 bf16, 2 fp16); dt is wave-uniform
__device__ __forceinline__ float ld_any(const void* p, int dt, long long i) {
  if (dt == 1) return ld1<bf16>(reinterpret_cast<const bf16*>(p) + i);
  if (dt == 2) return ld1<f16>(reinterpret_cast<const f16*>(p) + i);
  return reinterpret_cast<const float*>(p)[i];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide reduction for blockDim.x <= 1024 (multiple of 64). `red` needs blockDim/64 floats.
template <bool MAX>
__device__ __forceinline__ float block_reduce(float v, float* red) {
  v = MAX ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = MAX ? -INFINITY : 0.f;
  for (int i = 0; i < nw; ++i) r = MAX ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

#define HIP_LAUNCH_CHECK() (hipGetLastError())

// Index decomposition for grid-stride elementwise loops: 64-bit division by a runtime divisor is a long emulated
// sequence on CDNA, so indices below 2^31 (every realistic activation) take the 32-bit path.
// t = ((a3 * D2 + a2) * D1 + a1) * D0 + a0
__device__ __forceinline__ void idx_decomp4(long long t, int D0, int D1, int D2, int& a0, int& a1, int& a2, int& a3) {
  if (t < 0x7fffffffLL) {
    unsigned u = (unsigned)t;
    const unsigned q0 = u / (unsigned)D0;
    a0 = (int)(u - q0 * (unsigned)D0);
    const unsigned q1 = q0 / (unsigned)D1;
    a1 = (int)(q0 - q1 * (unsigned)D1);
    const unsigned q2 = q1 / (unsigned)D2;
    a2 = (int)(q1 - q2 * (unsigned)D2);
    a3 = (int)q2;
  } else {
    a0 = (int)(t % D0);
    long long r = t / D0;
    a1 = (int)(r % D1);
    r /= D1;
    a2 = (int)(r % D2);
    a3 = (int)(r / D2);
  }
}

__device__ __forceinline__ int idx_mod(long long t, int D) {
  return t < 0x7fffffffLL ? (int)((unsigned)t % (unsigned)D) : (int)(t % D);
}
