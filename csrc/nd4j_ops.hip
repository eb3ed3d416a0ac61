// ND4J op surface on the GPU: the generic elementwise / broadcast / reduction / data-movement ops behind INDArray,
// Transforms, the standalone activation functions and the shape-only layers (reference: libnd4j's legacy
// transform / pairwise / broadcast / reduce / indexreduce op families and the custom ops reverse, space_to_depth,
// depth_to_space, space_to_batch, upsampling2d(_bp), mergemax).
//
//   transform     y = f(x)           unary op table (DL4J activations + ND4J Transforms), 8 elements / thread
//   transform_bp  dz = eps * f'(z)   activation derivatives with the reference's edge conventions
//   binary        out = op(a, b)     rank <= 8 strided N-D broadcast (stride 0 = broadcast dim); contiguous same-shape
//                                    operands take a vectorised fast path
//   reduce        out[o][i] = R_r x[o][r][i] over a contiguous [O][R][I] view; R split into segments whose partial
//                 states combine in a fixed order (bitwise deterministic), Welford states for var/std, (value, index)
//                 states for argmax/argmin (first index wins ties, like ND4J)
//   strided_copy  out (contiguous, rank <= 8) = x at arbitrary (incl. 0 / negative) strides, optional zero padding
//                 per dim: reverse, permute materialisation, space<->depth, space<->batch, nearest upsampling
//   mergemax      elementwise max over up to 8 inputs + argmax bytes; mergemax_bp routes eps to the argmax input
//   im2col_rows / col2im_rows   row-per-output-pixel im2col (padding in the same pass) and its gather-form adjoint
//                 onto a channels-last image: the exact-fp32 conv as three single GEMMs (ops/conv.py)
// dtype codes: 0 fp32, 1 bf16, 2 fp16 (fp32 math everywhere).
#include "common.h"

namespace {

template <typename T> __device__ __forceinline__ float ldf(const T* p, long long i);
template <> __device__ __forceinline__ float ldf<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ldf<bf16>(const bf16* p, long long i) {
  return bf2f(reinterpret_cast<const u16*>(p)[i]);
}
template <> __device__ __forceinline__ float ldf<f16>(const f16* p, long long i) { return (float)p[i]; }
template <typename T> __device__ __forceinline__ void stf(T* p, long long i, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, long long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stf<bf16>(bf16* p, long long i, float v) {
  reinterpret_cast<u16*>(p)[i] = f2bf(v);
}
template <> __device__ __forceinline__ void stf<f16>(f16* p, long long i, float v) { p[i] = (f16)v; }

inline int grid1(long long work, int per_block = 256) {
  long long g = (work + per_block - 1) / per_block;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

// ------------------------------------------------------------------------------------------------ unary transforms
enum : int {
  OP_IDENTITY = 0, OP_RELU, OP_RELU6, OP_LEAKYRELU, OP_ELU, OP_SELU, OP_SIGMOID, OP_HARDSIGMOID, OP_TANH, OP_HARDTANH,
  OP_RATIONALTANH, OP_RECTIFIEDTANH, OP_SOFTPLUS, OP_SOFTSIGN, OP_CUBE, OP_SWISH, OP_GELU_TANH, OP_GELU_ERF, OP_RRELU,
  OP_EXP = 30, OP_LOG, OP_ABS, OP_NEG, OP_SQRT, OP_SQUARE, OP_SIGN, OP_POW, OP_RECIPROCAL, OP_FLOOR, OP_CEIL, OP_ROUND,
  OP_SIN, OP_COS, OP_CLIP, OP_STEP, OP_ADD_S, OP_MUL_S, OP_RSUB_S, OP_RDIV_S, OP_MAX_S, OP_MIN_S, OP_LOG1P, OP_EXPM1,
  OP_RSQRT, OP_ATAN, OP_ASIN, OP_ACOS, OP_SINH, OP_COSH, OP_ERF, OP_SUB_S, OP_DIV_S
};

constexpr float kSeluA = 1.6732632423543772848f, kSeluS = 1.0507009873554804934f;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ float unary(int op, float x, float a0, float a1) {
  switch (op) {
    case OP_IDENTITY: return x;
    case OP_RELU: return fmaxf(x, 0.f);
    case OP_RELU6: return fminf(fmaxf(x, 0.f), 6.f);
    case OP_LEAKYRELU: case OP_RRELU: return x > 0.f ? x : x * a0;
    case OP_ELU: return x > 0.f ? x : a0 * expm1f(x);
    case OP_SELU: return kSeluS * (x > 0.f ? x : kSeluA * expm1f(x));
    case OP_SIGMOID: return sigm(x);
    case OP_HARDSIGMOID: return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f);
    case OP_TANH: return tanhf(x);
    case OP_HARDTANH: return fminf(fmaxf(x, -1.f), 1.f);
    case OP_RATIONALTANH: {
      const float y = 2.f * x / 3.f, a = fabsf(y);
      const float s = y > 0.f ? 1.f : (y < 0.f ? -1.f : 0.f);
      return 1.7159f * s * (1.f - 1.f / (1.f + a + y * y + 1.41645f * y * y * y * y));
    }
    case OP_RECTIFIEDTANH: return fmaxf(tanhf(x), 0.f);
    case OP_SOFTPLUS: return x > 20.f ? x : log1pf(__expf(x));
    case OP_SOFTSIGN: return x / (1.f + fabsf(x));
    case OP_CUBE: return x * x * x;
    case OP_SWISH: return x * sigm(x);
    case OP_GELU_TANH: {
      const float c = 0.7978845608028654f;
      return 0.5f * x * (1.f + tanhf(c * (x + 0.044715f * x * x * x)));
    }
    case OP_GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case OP_EXP: return expf(x);
    case OP_LOG: return logf(x);
    case OP_ABS: return fabsf(x);
    case OP_NEG: return -x;
    case OP_SQRT: return sqrtf(x);
    case OP_SQUARE: return x * x;
    case OP_SIGN: return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    case OP_POW: return powf(x, a0);
    case OP_RECIPROCAL: return 1.f / x;
    case OP_FLOOR: return floorf(x);
    case OP_CEIL: return ceilf(x);
    case OP_ROUND: return rintf(x);
    case OP_SIN: return sinf(x);
    case OP_COS: return cosf(x);
    case OP_CLIP: return fminf(fmaxf(x, a0), a1);
    case OP_STEP: return x > a0 ? 1.f : 0.f;
    case OP_ADD_S: return x + a0;
    case OP_SUB_S: return x - a0;
    case OP_MUL_S: return x * a0;
    case OP_DIV_S: return x / a0;
    case OP_RSUB_S: return a0 - x;
    case OP_RDIV_S: return a0 / x;
    case OP_MAX_S: return fmaxf(x, a0);
    case OP_MIN_S: return fminf(x, a0);
    case OP_LOG1P: return log1pf(x);
    case OP_EXPM1: return expm1f(x);
    case OP_RSQRT: return rsqrtf(x);
    case OP_ATAN: return atanf(x);
    case OP_ASIN: return asinf(x);
    case OP_ACOS: return acosf(x);
    case OP_SINH: return sinhf(x);
    case OP_COSH: return coshf(x);
    case OP_ERF: return erff(x);
    default: return x;
  }
}

// f'(z) for the activation ops, edge conventions of nn/conf/activations.py (= the reference IActivation.backprop)
__device__ float dunary(int op, float z, float a0) {
  switch (op) {
    case OP_IDENTITY: return 1.f;
    case OP_RELU: return z > 0.f ? 1.f : 0.f;
    case OP_RELU6: return (z > 0.f && z < 6.f) ? 1.f : 0.f;
    case OP_LEAKYRELU: return z > 0.f ? 1.f : a0;
    case OP_RRELU: return z >= 0.f ? 1.f : a0;
    case OP_ELU: return z > 0.f ? 1.f : a0 * __expf(z);
    case OP_SELU: return z > 0.f ? kSeluS : kSeluS * kSeluA * __expf(z);
    case OP_SIGMOID: { const float s = sigm(z); return s * (1.f - s); }
    case OP_HARDSIGMOID: return (z > -2.5f && z < 2.5f) ? 0.2f : 0.f;
    case OP_TANH: { const float t = tanhf(z); return 1.f - t * t; }
    case OP_HARDTANH: return (z > -1.f && z < 1.f) ? 1.f : 0.f;
    case OP_RATIONALTANH: {
      const float y = 2.f * z / 3.f, a = fabsf(y);
      const float d = 1.f + a + y * y + 1.41645f * y * y * y * y;
      return 1.7159f * (2.f / 3.f) * (1.f + 2.f * a + 4.f * 1.41645f * a * a * a) / (d * d);
    }
    case OP_RECTIFIEDTANH: { const float t = tanhf(z); return z > 0.f ? 1.f - t * t : 0.f; }
    case OP_SOFTPLUS: return sigm(z);
    case OP_SOFTSIGN: { const float d = 1.f + fabsf(z); return 1.f / (d * d); }
    case OP_CUBE: return 3.f * z * z;
    case OP_SWISH: { const float s = sigm(z); return s + z * s * (1.f - s); }
    case OP_GELU_TANH: {
      const float c = 0.7978845608028654f;
      const float t = tanhf(c * (z + 0.044715f * z * z * z));
      return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * c * (1.f + 3.f * 0.044715f * z * z);
    }
    case OP_GELU_ERF:
      return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.3989422804014327f * __expf(-0.5f * z * z);
    default: return 1.f;
  }
}

template <typename T, bool BP>
__global__ __launch_bounds__(256) void transform_kernel(const T* __restrict__ x, const T* __restrict__ eps,
                                                        T* __restrict__ y, long long n, int op, float a0, float a1) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long n8 = n / 8;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += stride) {
    float a[8], e[8];
    Vec8<T>::load(x + v * 8, a);
    if (BP) Vec8<T>::load(eps + v * 8, e);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = BP ? e[k] * dunary(op, a[k], a0) : unary(op, a[k], a0, a1);
    Vec8<T>::store(y + v * 8, a);
  }
  for (long long i = n8 * 8 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float z = ldf(x, i);
    stf(y, i, BP ? ldf(eps, i) * dunary(op, z, a0) : unary(op, z, a0, a1));
  }
}

// ------------------------------------------------------------------------------------------------ N-D broadcast
enum : int {
  B_ADD = 0, B_SUB, B_MUL, B_DIV, B_RSUB, B_RDIV, B_MAX, B_MIN, B_POW, B_SQDIFF, B_EQ, B_NEQ, B_GT, B_GTE, B_LT, B_LTE,
  B_FMOD, B_ATAN2, B_REMAINDER
};

__device__ __forceinline__ float binop(int op, float a, float b) {
  switch (op) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_RSUB: return b - a;
    case B_RDIV: return b / a;
    case B_MAX: return fmaxf(a, b);
    case B_MIN: return fminf(a, b);
    case B_POW: return powf(a, b);
    case B_SQDIFF: { const float d = a - b; return d * d; }
    case B_EQ: return a == b ? 1.f : 0.f;
    case B_NEQ: return a != b ? 1.f : 0.f;
    case B_GT: return a > b ? 1.f : 0.f;
    case B_GTE: return a >= b ? 1.f : 0.f;
    case B_LT: return a < b ? 1.f : 0.f;
    case B_LTE: return a <= b ? 1.f : 0.f;
    case B_FMOD: return fmodf(a, b);
    case B_ATAN2: return atan2f(a, b);
    case B_REMAINDER: return a - floorf(a / b) * b;
    default: return a;
  }
}

struct NdShape {
  int rank;
  long long shape[8];
  long long sa[8];
  long long sb[8];
};

template <typename T>
__global__ __launch_bounds__(256) void binary_nd(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out,
                                                 long long n, NdShape s, int op) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long long r = i, oa = 0, ob = 0;
    for (int d = s.rank - 1; d >= 0; --d) {
      const long long c = r % s.shape[d];
      r /= s.shape[d];
      oa += c * s.sa[d];
      ob += c * s.sb[d];
    }
    stf(out, i, binop(op, ldf(a, oa), ldf(b, ob)));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void binary_flat(const T* __restrict__ a, const T* __restrict__ b,
                                                   T* __restrict__ out, long long n, int op) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long n8 = n / 8;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += stride) {
    float x[8], y[8];
    Vec8<T>::load(a + v * 8, x);
    Vec8<T>::load(b + v * 8, y);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = binop(op, x[k], y[k]);
    Vec8<T>::store(out + v * 8, x);
  }
  for (long long i = n8 * 8 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    stf(out, i, binop(op, ldf(a, i), ldf(b, i)));
}

// ------------------------------------------------------------------------------------------------ reductions
enum : int {
  R_SUM = 0, R_MEAN, R_MAX, R_MIN, R_PROD, R_NORM1, R_NORM2, R_NORMMAX, R_SUMSQ, R_AMAX, R_AMIN, R_VAR, R_STD, R_ARGMAX,
  R_ARGMIN, R_LOGSUMEXP
};

// partial state: a (value / Welford mean / max for logsumexp), b (Welford M2 / sum exp), c (count), idx (arg ops)
struct RState {
  float a, b, c;
  long long idx;
};

__device__ __forceinline__ RState r_init(int op) {
  RState s;
  s.b = 0.f; s.c = 0.f; s.idx = -1;
  switch (op) {
    case R_MAX: case R_ARGMAX: case R_LOGSUMEXP: s.a = -INFINITY; break;
    case R_MIN: case R_ARGMIN: case R_AMIN: s.a = INFINITY; break;
    case R_PROD: s.a = 1.f; break;
    default: s.a = 0.f;
  }
  return s;
}

__device__ __forceinline__ void r_add(int op, RState& s, float x, long long i) {
  switch (op) {
    case R_SUM: case R_MEAN: s.a += x; break;
    case R_MAX: s.a = fmaxf(s.a, x); break;
    case R_MIN: s.a = fminf(s.a, x); break;
    case R_PROD: s.a *= x; break;
    case R_NORM1: s.a += fabsf(x); break;
    case R_NORM2: case R_SUMSQ: s.a += x * x; break;
    case R_NORMMAX: case R_AMAX: s.a = fmaxf(s.a, fabsf(x)); break;
    case R_AMIN: s.a = fminf(s.a, fabsf(x)); break;
    case R_VAR: case R_STD: {
      s.c += 1.f;
      const float d = x - s.a;
      s.a += d / s.c;
      s.b += d * (x - s.a);
      break;
    }
    case R_ARGMAX: if (x > s.a || s.idx < 0) { s.a = x; s.idx = i; } break;
    case R_ARGMIN: if (x < s.a || s.idx < 0) { s.a = x; s.idx = i; } break;
    case R_LOGSUMEXP:
      if (x > s.a) { s.b = s.b * __expf(s.a - x) + 1.f; s.a = x; }
      else s.b += __expf(x - s.a);
      break;
  }
}

// combine t (later indices) into s (earlier indices)
__device__ __forceinline__ void r_merge(int op, RState& s, const RState& t) {
  switch (op) {
    case R_SUM: case R_MEAN: case R_NORM1: case R_NORM2: case R_SUMSQ: s.a += t.a; break;
    case R_MAX: case R_NORMMAX: case R_AMAX: s.a = fmaxf(s.a, t.a); break;
    case R_MIN: case R_AMIN: s.a = fminf(s.a, t.a); break;
    case R_PROD: s.a *= t.a; break;
    case R_VAR: case R_STD: {
      if (t.c == 0.f) break;
      if (s.c == 0.f) { s = t; break; }
      const float n = s.c + t.c, d = t.a - s.a;
      s.a += d * t.c / n;
      s.b += t.b + d * d * s.c * t.c / n;
      s.c = n;
      break;
    }
    case R_ARGMAX: if (t.idx >= 0 && (s.idx < 0 || t.a > s.a)) { s.a = t.a; s.idx = t.idx; } break;
    case R_ARGMIN: if (t.idx >= 0 && (s.idx < 0 || t.a < s.a)) { s.a = t.a; s.idx = t.idx; } break;
    case R_LOGSUMEXP: {
      if (t.b == 0.f) break;
      if (s.b == 0.f) { s = t; break; }
      const float m = fmaxf(s.a, t.a);
      s.b = s.b * __expf(s.a - m) + t.b * __expf(t.a - m);
      s.a = m;
      break;
    }
  }
}

// block = 64 columns (i) x 4 row phases; partial state of rows [seg*rps, ...) of column i -> part[o][seg][i]
template <typename T>
__global__ __launch_bounds__(256) void reduce_cols(const T* __restrict__ x, RState* __restrict__ part, long long O,
                                                   long long R, long long I, long long rps, int op) {
  const long long i = (long long)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const long long o = blockIdx.y;
  const int seg = blockIdx.z, nseg = gridDim.z;
  const long long r0 = seg * rps, r1 = min(R, r0 + rps);
  RState s = r_init(op);
  if (i < I)
    for (long long r = r0 + ph; r < r1; r += 4) r_add(op, s, ldf(x, (o * R + r) * I + i), r);
  __shared__ RState sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  if (ph == 0 && i < I) {
    // phases hold interleaved rows: merge by re-walking would change the order for arg ops only on ties; the arg
    // ops keep the first index on ties explicitly, so a fixed phase order is deterministic and ND4J-compatible
    RState t = sh[threadIdx.x];
    for (int p = 1; p < 4; ++p) {
      const RState u = sh[p * 64 + threadIdx.x];
      if ((op == R_ARGMAX || op == R_ARGMIN) && u.idx >= 0 && t.idx >= 0 && u.a == t.a) {
        if (u.idx < t.idx) t = u;
        continue;
      }
      r_merge(op, t, u);
    }
    part[(o * nseg + seg) * I + i] = t;
  }
}

// I == 1: one block per (o, segment), 256 threads strided over the segment, fixed-order tree in LDS
template <typename T>
__global__ __launch_bounds__(256) void reduce_rows(const T* __restrict__ x, RState* __restrict__ part, long long R,
                                                   long long rps, int op) {
  const long long o = blockIdx.y;
  const int seg = blockIdx.x, nseg = gridDim.x;
  const long long r0 = seg * rps, r1 = min(R, r0 + rps);
  RState s = r_init(op);
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) r_add(op, s, ldf(x, o * R + r), r);
  __shared__ RState sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      RState t = sh[threadIdx.x];
      const RState u = sh[threadIdx.x + w];
      if ((op == R_ARGMAX || op == R_ARGMIN) && u.idx >= 0 && t.idx >= 0 && u.a == t.a) {
        if (u.idx < t.idx) t = u;
      } else {
        r_merge(op, t, u);
      }
      sh[threadIdx.x] = t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[o * nseg + seg] = sh[0];
}

// combine the segments of every (o, i) in order and write the final value (fp32) or index (int64)
__global__ __launch_bounds__(256) void reduce_finalize(const RState* __restrict__ part, float* __restrict__ out,
                                                       long long* __restrict__ iout, long long O, long long I,
                                                       int nseg, long long R, int op, int bias_corrected) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < O * I; t += stride) {
    const long long o = t / I, i = t - o * I;
    RState s = part[(o * nseg) * I + i];
    for (int g = 1; g < nseg; ++g) {
      const RState u = part[(o * nseg + g) * I + i];
      if ((op == R_ARGMAX || op == R_ARGMIN) && u.idx >= 0 && s.idx >= 0 && u.a == s.a) continue;   // first wins
      r_merge(op, s, u);
    }
    float v = s.a;
    switch (op) {
      case R_MEAN: v = s.a / (float)R; break;
      case R_NORM2: v = sqrtf(s.a); break;
      case R_VAR: v = s.b / fmaxf(s.c - (bias_corrected ? 1.f : 0.f), 1.f); break;
      case R_STD: v = sqrtf(s.b / fmaxf(s.c - (bias_corrected ? 1.f : 0.f), 1.f)); break;
      case R_LOGSUMEXP: v = s.a + logf(s.b); break;
      default: break;
    }
    if (op == R_ARGMAX || op == R_ARGMIN) iout[t] = s.idx;
    else out[t] = v;
  }
}

// many outputs: one thread per (o, i) walks its R elements in order (consecutive threads = consecutive i: coalesced
// when I > 1) and writes the final value directly
template <typename T>
__global__ __launch_bounds__(256) void reduce_direct(const T* __restrict__ x, float* __restrict__ out,
                                                     long long* __restrict__ iout, long long O, long long R,
                                                     long long I, int op, int bias_corrected) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < O * I; t += stride) {
    const long long o = t / I, i = t - o * I;
    RState s = r_init(op);
    for (long long r = 0; r < R; ++r) r_add(op, s, ldf(x, (o * R + r) * I + i), r);
    float v = s.a;
    switch (op) {
      case R_MEAN: v = s.a / (float)R; break;
      case R_NORM2: v = sqrtf(s.a); break;
      case R_VAR: v = s.b / fmaxf(s.c - (bias_corrected ? 1.f : 0.f), 1.f); break;
      case R_STD: v = sqrtf(s.b / fmaxf(s.c - (bias_corrected ? 1.f : 0.f), 1.f)); break;
      case R_LOGSUMEXP: v = s.a + logf(s.b); break;
      default: break;
    }
    if (op == R_ARGMAX || op == R_ARGMIN) iout[t] = s.idx;
    else out[t] = v;
  }
}

// ------------------------------------------------------------------------------------------------ strided copy
struct CopyShape {
  int rank;
  long long shape[8];    // output shape (contiguous)
  long long st[8];       // source strides per output dim (may be 0 or negative)
  long long off[8];      // source coordinate = output coordinate + off (zero padding when outside [0, lim))
  long long lim[8];      // source extent per dim (0 = unbounded: no padding check)
  long long base;        // source element offset of coordinate 0
};

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void strided_copy(const TI* __restrict__ x, TO* __restrict__ y, long long n,
                                                    CopyShape s) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long long r = i, src = s.base;
    bool ok = true;
    for (int d = s.rank - 1; d >= 0; --d) {
      const long long c = r % s.shape[d] + s.off[d];
      r /= s.shape[d];
      if (s.lim[d] > 0 && (c < 0 || c >= s.lim[d])) ok = false;
      src += c * s.st[d];
    }
    stf(y, i, ok ? ldf(x, src) : 0.f);
  }
}

// ------------------------------------------------------------------------------------------------ col2im
// x[n][c][h][w] = sum over the (r, s) taps whose window position lands on (h, w) of cols[n][(c*R + r)*S + s][oh*OW + ow]
// (the adjoint of im2col / F.unfold layout); x is the PADDED image [N][C][Hp][Wp], gather form: no atomics.
template <typename T>
__global__ __launch_bounds__(256) void col2im_kernel(const T* __restrict__ cols, T* __restrict__ x, int N, int C,
                                                     int Hp, int Wp, int R, int S, int sh, int sw, int dh, int dw,
                                                     int OH, int OW) {
  const long long total = (long long)N * C * Hp * Wp;
  const long long L = (long long)OH * OW;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int w = (int)(i % Wp);
    long long t = i / Wp;
    const int h = (int)(t % Hp);
    t /= Hp;
    const int c = (int)(t % C);
    const long long n = t / C;
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
      const int ohn = h - r * dh;
      if (ohn < 0 || ohn % sh) continue;
      const int oh = ohn / sh;
      if (oh >= OH) continue;
      for (int q = 0; q < S; ++q) {
        const int own = w - q * dw;
        if (own < 0 || own % sw) continue;
        const int ow = own / sw;
        if (ow >= OW) continue;
        acc += ldf(cols, (n * C * R * S + ((long long)c * R + r) * S + q) * L + (long long)oh * OW + ow);
      }
    }
    stf(x, i, acc);
  }
}

// ------------------------------------------------------------------------------------------------ im2col rows
// Row-per-output-pixel im2col for the exact-fp32 conv (one GEMM over all images instead of one per image):
//   cols[(n*OH + oh)*OW + ow][(c*R + r)*S + q] = x[n][c][oh*sh + r*dh - pt][ow*sw + q*dw - pl]   (0 outside)
// x at element strides (sN, sC, sH, sW): NCHW or channels-last; the column order (c, r, q) matches the weight
// [K][C][R][S] reshaped to [K][C*R*S], so no weight copy is needed.
template <typename T>
__global__ __launch_bounds__(256) void im2col_rows_kernel(const T* __restrict__ x, T* __restrict__ cols, int N, int C,
                                                          int H, int W, long long sN, long long sC, long long sH,
                                                          long long sW, int R, int S, int sh, int sw, int pt, int pl,
                                                          int dh, int dw, int OH, int OW) {
  const long long CRS = (long long)C * R * S;
  const long long total = (long long)N * OH * OW * CRS;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long row = i / CRS;
    const int col = (int)(i - row * CRS);
    const int q = col % S, r = (col / S) % R, c = col / (R * S);
    const int ow = (int)(row % OW);
    const long long t = row / OW;
    const int oh = (int)(t % OH);
    const long long n = t / OH;
    const int h = oh * sh + r * dh - pt, w = ow * sw + q * dw - pl;
    const bool in = h >= 0 && h < H && w >= 0 && w < W;
    stf(cols, i, in ? ldf(x, n * sN + c * sC + h * sH + w * sW) : 0.f);
  }
}

// Adjoint of im2col_rows onto the UNPADDED image, written channels-last: dx[n][h][w][c] = sum of the dcols entries
// whose window tap lands on (h, w). Gather form (no atomics, deterministic), channel index fastest.
template <typename T>
__global__ __launch_bounds__(256) void col2im_rows_kernel(const T* __restrict__ cols, T* __restrict__ dx, int N, int C,
                                                          int H, int W, int R, int S, int sh, int sw, int pt, int pl,
                                                          int dh, int dw, int OH, int OW) {
  const long long CRS = (long long)C * R * S;
  const long long total = (long long)N * H * W * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const long long n = t / H;
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
      const int ohn = h + pt - r * dh;
      if (ohn < 0 || ohn % sh) continue;
      const int oh = ohn / sh;
      if (oh >= OH) continue;
      for (int q = 0; q < S; ++q) {
        const int own = w + pl - q * dw;
        if (own < 0 || own % sw) continue;
        const int ow = own / sw;
        if (ow >= OW) continue;
        acc += ldf(cols, ((n * OH + oh) * OW + ow) * CRS + ((long long)c * R + r) * S + q);
      }
    }
    stf(dx, i, acc);
  }
}

// ------------------------------------------------------------------------------------------------ mergemax
struct PtrList {
  const void* p[8];
  int n;
};

template <typename T>
__global__ __launch_bounds__(256) void mergemax_kernel(PtrList in, T* __restrict__ y, unsigned char* __restrict__ am,
                                                       long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float best = ldf(reinterpret_cast<const T*>(in.p[0]), i);
    int bi = 0;
    for (int k = 1; k < in.n; ++k) {
      const float v = ldf(reinterpret_cast<const T*>(in.p[k]), i);
      if (v > best) { best = v; bi = k; }
    }
    stf(y, i, best);
    if (am) am[i] = (unsigned char)bi;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mergemax_bp_kernel(const T* __restrict__ eps, const unsigned char* __restrict__ am,
                                                          PtrList out, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float e = ldf(eps, i);
    const int k = am[i];
    for (int j = 0; j < out.n; ++j) stf(reinterpret_cast<T*>(const_cast<void*>(out.p[j])), i, j == k ? e : 0.f);
  }
}

#define DT_DISPATCH(dt, MACRO) \
  do {                         \
    if ((dt) == 0) { MACRO(float); }       \
    else if ((dt) == 1) { MACRO(bf16); }   \
    else if ((dt) == 2) { MACRO(f16); }    \
    else return -1;            \
  } while (0)

}  // namespace

DL4J_API int dl4j_transform(int dt, int op, const void* x, void* y, long long n, float a0, float a1, hipStream_t s) {
  if (n <= 0) return 0;
  const int g = grid1((n + 7) / 8);
#define L(T) hipLaunchKernelGGL((transform_kernel<T, false>), dim3(g), dim3(256), 0, s, (const T*)x, (const T*)nullptr, \
                                (T*)y, n, op, a0, a1)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

DL4J_API int dl4j_transform_bp(int dt, int op, const void* z, const void* eps, void* out, long long n, float a0,
                               hipStream_t s) {
  if (n <= 0) return 0;
  if (op > OP_RRELU) return -1;
  const int g = grid1((n + 7) / 8);
#define L(T) hipLaunchKernelGGL((transform_kernel<T, true>), dim3(g), dim3(256), 0, s, (const T*)z, (const T*)eps, \
                                (T*)out, n, op, a0, 0.f)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

// shape / strides: rank entries each (element strides of a and b for the OUTPUT's dims; 0 = broadcast).
// flat != 0: a and b are contiguous with the output's shape (vectorised path; shape/strides ignored).
DL4J_API int dl4j_binary(int dt, int op, const void* a, const void* b, void* out, int rank, const long long* shape,
                         const long long* sa, const long long* sb, int flat, hipStream_t s) {
  if (rank < 0 || rank > 8) return -1;
  long long n = 1;
  for (int d = 0; d < rank; ++d) n *= shape[d];
  if (n <= 0) return 0;
  if (flat) {
    const int g = grid1((n + 7) / 8);
#define L(T) hipLaunchKernelGGL((binary_flat<T>), dim3(g), dim3(256), 0, s, (const T*)a, (const T*)b, (T*)out, n, op)
    DT_DISPATCH(dt, L);
#undef L
    return (int)hipGetLastError();
  }
  NdShape sh = {};
  sh.rank = rank;
  for (int d = 0; d < rank; ++d) { sh.shape[d] = shape[d]; sh.sa[d] = sa[d]; sh.sb[d] = sb[d]; }
  const int g = grid1(n);
#define L(T) hipLaunchKernelGGL((binary_nd<T>), dim3(g), dim3(256), 0, s, (const T*)a, (const T*)b, (T*)out, n, sh, op)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

constexpr long long kDirectOutputs = 32768;     // at least this many outputs: one thread per output, no segments

// Segments the R axis is split into (host sizes the partial-state workspace from it); 0 = direct path.
DL4J_API int dl4j_reduce_segments(long long O, long long R, long long I) {
  if (O * I >= kDirectOutputs) return 0;
  const long long cols = I == 1 ? 1 : (I + 63) / 64;
  long long seg = (1024 + O * cols - 1) / (O * cols);
  const long long maxs = (R + 1023) / 1024;
  if (seg > maxs) seg = maxs;
  if (seg > 4096) seg = 4096;
  return (int)(seg < 1 ? 1 : seg);
}

DL4J_API long long dl4j_reduce_ws_bytes(long long O, long long R, long long I) {
  return (long long)dl4j_reduce_segments(O, R, I) * O * I * (long long)sizeof(RState);
}

// x contiguous [O][R][I] (dt 0/1/2); out fp32 [O][I] (value ops) or iout int64 [O][I] (argmax / argmin).
DL4J_API int dl4j_reduce(int dt, int op, const void* x, float* out, long long* iout, long long O, long long R,
                         long long I, int bias_corrected, void* ws, hipStream_t s) {
  if (O <= 0 || I <= 0 || R <= 0) return -1;
  if ((op == R_ARGMAX || op == R_ARGMIN) ? iout == nullptr : out == nullptr) return -1;
  if (O * I >= kDirectOutputs) {
#define L(T) hipLaunchKernelGGL((reduce_direct<T>), dim3(grid1(O * I)), dim3(256), 0, s, (const T*)x, out, iout, O, R, I, \
                                op, bias_corrected)
    DT_DISPATCH(dt, L);
#undef L
    return (int)hipGetLastError();
  }
  const int nseg = dl4j_reduce_segments(O, R, I);
  const long long rps = (R + nseg - 1) / nseg;
  RState* part = reinterpret_cast<RState*>(ws);
  if (I == 1) {
#define L(T) hipLaunchKernelGGL((reduce_rows<T>), dim3(nseg, (unsigned)O), dim3(256), 0, s, (const T*)x, part, R, rps, op)
    DT_DISPATCH(dt, L);
#undef L
  } else {
#define L(T) hipLaunchKernelGGL((reduce_cols<T>), dim3((unsigned)((I + 63) / 64), (unsigned)O, nseg), dim3(256), 0, s, \
                                (const T*)x, part, O, R, I, rps, op)
    DT_DISPATCH(dt, L);
#undef L
  }
  hipLaunchKernelGGL(reduce_finalize, dim3(grid1(O * I)), dim3(256), 0, s, part, out, iout, O, I, nseg, R, op,
                     bias_corrected);
  return (int)hipGetLastError();
}

// out = contiguous tensor of shape[rank]; element at coordinate c reads x[base + sum_d (c_d + off_d) * st_d], or 0
// when some lim_d > 0 and (c_d + off_d) is outside [0, lim_d).
// Same with a dtype conversion: x in sdt, y in ddt (0 fp32, 1 bf16, 2 fp16) — e.g. permute + cast + zero-pad of a
// GEMM operand in one pass.
DL4J_API int dl4j_strided_copy2(int sdt, int ddt, const void* x, void* y, int rank, const long long* shape,
                                const long long* st, const long long* off, const long long* lim, long long base,
                                hipStream_t s);

DL4J_API int dl4j_strided_copy(int dt, const void* x, void* y, int rank, const long long* shape, const long long* st,
                               const long long* off, const long long* lim, long long base, hipStream_t s) {
  return dl4j_strided_copy2(dt, dt, x, y, rank, shape, st, off, lim, base, s);
}

DL4J_API int dl4j_strided_copy2(int sdt, int ddt, const void* x, void* y, int rank, const long long* shape,
                                const long long* st, const long long* off, const long long* lim, long long base,
                                hipStream_t s) {
  if (rank < 1 || rank > 8) return -1;
  CopyShape cs = {};
  cs.rank = rank;
  cs.base = base;
  long long n = 1;
  for (int d = 0; d < rank; ++d) {
    cs.shape[d] = shape[d];
    cs.st[d] = st[d];
    cs.off[d] = off ? off[d] : 0;
    cs.lim[d] = lim ? lim[d] : 0;
    n *= shape[d];
  }
  if (n <= 0) return 0;
  const int g = grid1(n);
#define L2(TI, TO) hipLaunchKernelGGL((strided_copy<TI, TO>), dim3(g), dim3(256), 0, s, (const TI*)x, (TO*)y, n, cs)
#define LO(TI)                          \
  do {                                  \
    if (ddt == 0) { L2(TI, float); }    \
    else if (ddt == 1) { L2(TI, bf16); } \
    else if (ddt == 2) { L2(TI, f16); }  \
    else return -1;                     \
  } while (0)
  DT_DISPATCH(sdt, LO);
#undef LO
#undef L2
  return (int)hipGetLastError();
}

DL4J_API int dl4j_mergemax(int dt, const void* const* inputs, int nin, void* y, unsigned char* am, long long n,
                           hipStream_t s) {
  if (nin < 1 || nin > 8) return -1;
  PtrList pl = {};
  for (int k = 0; k < nin; ++k) pl.p[k] = inputs[k];
  pl.n = nin;
  const int g = grid1(n);
#define L(T) hipLaunchKernelGGL((mergemax_kernel<T>), dim3(g), dim3(256), 0, s, pl, (T*)y, am, n)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

DL4J_API int dl4j_mergemax_bp(int dt, const void* eps, const unsigned char* am, void* const* outs, int nout, long long n,
                              hipStream_t s) {
  if (nout < 1 || nout > 8) return -1;
  PtrList pl = {};
  for (int k = 0; k < nout; ++k) pl.p[k] = outs[k];
  pl.n = nout;
  const int g = grid1(n);
#define L(T) hipLaunchKernelGGL((mergemax_bp_kernel<T>), dim3(g), dim3(256), 0, s, (const T*)eps, am, pl, n)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

// cols [N][C*R*S][OH*OW] (F.unfold layout) -> padded image [N][C][Hp][Wp], summing overlapping windows.
DL4J_API int dl4j_col2im(int dt, const void* cols, void* x, int N, int C, int Hp, int Wp, int R, int S, int sh, int sw,
                         int dh, int dw, int OH, int OW, hipStream_t s) {
  if (sh < 1 || sw < 1 || dh < 1 || dw < 1) return -1;
  const int g = grid1((long long)N * C * Hp * Wp);
#define L(T) hipLaunchKernelGGL((col2im_kernel<T>), dim3(g), dim3(256), 0, s, (const T*)cols, (T*)x, N, C, Hp, Wp, R, S, \
                                sh, sw, dh, dw, OH, OW)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

// cols [N*OH*OW][C*R*S] <- x [N][C][H][W] at element strides st[4] = (sN, sC, sH, sW); geometry g[12] =
// {R, S, sh, sw, pt, pl, dh, dw, OH, OW, H, W}.
DL4J_API int dl4j_im2col_rows(int dt, const void* x, void* cols, int N, int C, const long long* st, const int* g,
                              hipStream_t s) {
  const int R = g[0], S = g[1], sh = g[2], sw = g[3], pt = g[4], pl = g[5], dh = g[6], dw = g[7], OH = g[8],
            OW = g[9], H = g[10], W = g[11];
  if (sh < 1 || sw < 1 || dh < 1 || dw < 1 || R < 1 || S < 1 || OH < 1 || OW < 1) return -1;
  const int gr = grid1((long long)N * OH * OW * C * R * S);
#define L(T) hipLaunchKernelGGL((im2col_rows_kernel<T>), dim3(gr), dim3(256), 0, s, (const T*)x, (T*)cols, N, C, H, W, \
                                st[0], st[1], st[2], st[3], R, S, sh, sw, pt, pl, dh, dw, OH, OW)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

// dx [N][H][W][C] (channels-last, unpadded) <- dcols [N*OH*OW][C*R*S]; same geometry array as dl4j_im2col_rows.
DL4J_API int dl4j_col2im_rows(int dt, const void* cols, void* dx, int N, int C, const int* g, hipStream_t s) {
  const int R = g[0], S = g[1], sh = g[2], sw = g[3], pt = g[4], pl = g[5], dh = g[6], dw = g[7], OH = g[8],
            OW = g[9], H = g[10], W = g[11];
  if (sh < 1 || sw < 1 || dh < 1 || dw < 1 || R < 1 || S < 1) return -1;
  const int gr = grid1((long long)N * H * W * C);
#define L(T) hipLaunchKernelGGL((col2im_rows_kernel<T>), dim3(gr), dim3(256), 0, s, (const T*)cols, (T*)dx, N, C, H, W, \
                                R, S, sh, sw, pt, pl, dh, dw, OH, OW)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------ fill
// out[0 .. nbytes) = a repeated 4-byte pattern (fp32 value, or two copies of a 16-bit value): the zero fills of the
// training step (flat gradient before backward, the gaps of strided backward-data outputs) without a library kernel.
// 16-byte stores, grid-stride; a ragged head / tail (unaligned base or size) in 4-byte (2-byte) pieces.
__global__ __launch_bounds__(256) void fill_pattern(char* __restrict__ out, long long nbytes, unsigned pat) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const uintptr_t base = reinterpret_cast<uintptr_t>(out);
  const long long head = (long long)((16 - (base & 15)) & 15) > nbytes ? nbytes : (long long)((16 - (base & 15)) & 15);
  const long long nvec = (nbytes - head) / 16;
  uint4* v = reinterpret_cast<uint4*>(out + head);
  const uint4 q = make_uint4(pat, pat, pat, pat);
  for (long long i = tid; i < nvec; i += stride) v[i] = q;
  if (tid == 0) {
    // head and tail bytes: the pattern is 4-byte periodic from the base (2-byte fills are 2-byte aligned)
    for (long long b = 0; b < head; b += 2)
      *reinterpret_cast<unsigned short*>(out + b) = (unsigned short)(pat >> (8 * ((base + b) & 3)));
    for (long long b = head + nvec * 16; b < nbytes; b += 2)
      *reinterpret_cast<unsigned short*>(out + b) = (unsigned short)(pat >> (8 * ((base + b) & 3)));
  }
}

// elem_bytes 4 (pattern = the fp32 bits) or 2 (pattern = the 16-bit value in both halves); nbytes a multiple of 2.
DL4J_API int dl4j_fill(void* out, long long nbytes, unsigned pattern, hipStream_t s) {
  if (nbytes <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(out) & 1) || (nbytes & 1)) return -1;
  hipLaunchKernelGGL(fill_pattern, dim3(grid1((nbytes + 15) / 16)), dim3(256), 0, s, reinterpret_cast<char*>(out),
                     nbytes, pattern);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------ axpy
// y[i] += alpha * x[i] for an fp32 y and an x of dtype dt: the running-mean correction of a BatchNormalization whose
// producing convolution deferred its bias (the bias cancels in the batch statistics; the running mean must still
// track E[conv + bias]). A handful of channels per call: one grid-stride pass.
template <typename T>
__global__ __launch_bounds__(256) void axpy_kernel(const T* __restrict__ x, float* __restrict__ y, long long n,
                                                   float alpha) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] += alpha * ldf(x, i);
}

DL4J_API int dl4j_axpy(int dt, const void* x, float* y, long long n, float alpha, hipStream_t s) {
  if (n <= 0) return 0;
  const int g = grid1(n);
#define L(T) hipLaunchKernelGGL((axpy_kernel<T>), dim3(g), dim3(256), 0, s, (const T*)x, y, n, alpha)
  DT_DISPATCH(dt, L);
#undef L
  return (int)hipGetLastError();
}
