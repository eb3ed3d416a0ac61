// Per-segment summary statistics and histograms of a flat parameter / gradient / update / activation array,
// for the stats listener (reference: UIM:stats/BaseStatsListener.java:774 — Histogram op per parameter plus
// mean / stdev / mean-magnitude reductions over every (layer, param) view of the flat arrays).
//
// One launch covers every segment: grid.y = segment, grid.x = chunks of a segment. Each 256-thread block reduces
// its chunk with wave reductions (64 lanes, xor shuffles) and one LDS exchange, then merges into the segment's
// accumulator with atomics (float add; order-preserving int atomics for min/max). Histograms bin into an LDS
// histogram per block, flushed with one atomic per bin. Listener-only (runs every N iterations), so loads are
// plain coalesced scalar reads of fp32 or bf16.
#include "common.h"

namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmin(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// order-preserving float <-> int mapping for atomicMin/atomicMax on floats
__device__ __forceinline__ int f2o(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

template <typename T>
__global__ __launch_bounds__(256) void seg_stats_kernel(const T* __restrict__ x, const long long* __restrict__ off,
                                                        float* __restrict__ acc, int* __restrict__ mm) {
  const int s = blockIdx.y;
  const long long a = off[s], b = off[s + 1];
  float sum = 0.f, sq = 0.f, ab = 0.f, mn = INFINITY, mx = -INFINITY;
  for (long long i = a + (long long)blockIdx.x * 256 + threadIdx.x; i < b; i += (long long)gridDim.x * 256) {
    const float v = ld1<T>(x + i);
    sum += v; sq += v * v; ab += fabsf(v);
    mn = fminf(mn, v); mx = fmaxf(mx, v);
  }
  sum = wsum(sum); sq = wsum(sq); ab = wsum(ab); mn = wmin(mn); mx = wmax(mx);
  __shared__ float red[4][5];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[w][0] = sum; red[w][1] = sq; red[w][2] = ab; red[w][3] = mn; red[w][4] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      red[0][0] += red[k][0]; red[0][1] += red[k][1]; red[0][2] += red[k][2];
      red[0][3] = fminf(red[0][3], red[k][3]); red[0][4] = fmaxf(red[0][4], red[k][4]);
    }
    atomicAdd(acc + 3 * s + 0, red[0][0]);
    atomicAdd(acc + 3 * s + 1, red[0][1]);
    atomicAdd(acc + 3 * s + 2, red[0][2]);
    atomicMin(mm + 2 * s + 0, f2o(red[0][3]));
    atomicMax(mm + 2 * s + 1, f2o(red[0][4]));
  }
}

__global__ void seg_init_kernel(float* acc, int* mm, int nseg) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nseg) {
    acc[3 * s] = 0.f; acc[3 * s + 1] = 0.f; acc[3 * s + 2] = 0.f;
    mm[2 * s] = f2o(INFINITY); mm[2 * s + 1] = f2o(-INFINITY);
  }
}

// out[s] = {mean, stdev (population), mean |x|, min, max}
__global__ void seg_final_kernel(const float* acc, const int* mm, const long long* off, int nseg, float* out) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const float n = float(off[s + 1] - off[s]);
  const float mean = n > 0 ? acc[3 * s] / n : 0.f;
  const float var = n > 0 ? fmaxf(acc[3 * s + 1] / n - mean * mean, 0.f) : 0.f;
  out[5 * s + 0] = mean;
  out[5 * s + 1] = sqrtf(var);
  out[5 * s + 2] = n > 0 ? acc[3 * s + 2] / n : 0.f;
  out[5 * s + 3] = o2f(mm[2 * s]);
  out[5 * s + 4] = o2f(mm[2 * s + 1]);
}

template <typename T>
__global__ __launch_bounds__(256) void seg_hist_kernel(const T* __restrict__ x, const long long* __restrict__ off,
                                                       const float* __restrict__ stats, int bins,
                                                       unsigned* __restrict__ hist) {
  extern __shared__ unsigned lh[];
  const int s = blockIdx.y;
  for (int k = threadIdx.x; k < bins; k += 256) lh[k] = 0;
  __syncthreads();
  const float lo = stats[5 * s + 3], hi = stats[5 * s + 4];
  const float scale = hi > lo ? float(bins) / (hi - lo) : 0.f;
  const long long a = off[s], b = off[s + 1];
  for (long long i = a + (long long)blockIdx.x * 256 + threadIdx.x; i < b; i += (long long)gridDim.x * 256) {
    const float v = ld1<T>(x + i);
    int bin = int((v - lo) * scale);
    bin = bin < 0 ? 0 : (bin >= bins ? bins - 1 : bin);
    atomicAdd(&lh[bin], 1u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < bins; k += 256)
    if (lh[k]) atomicAdd(hist + (long long)s * bins + k, lh[k]);
}

int chunks_for(long long maxlen) {
  long long c = (maxlen + 256 * 16 - 1) / (256 * 16);   // ~16 elements per thread
  return int(c < 1 ? 1 : (c > 1024 ? 1024 : c));
}

}  // namespace

// x: flat array (dtype 0 fp32, 1 bf16); off: [nseg+1] int64 element offsets (device); ws: 5*nseg floats (device)
// out: [nseg, 5] {mean, std, meanAbs, min, max}; hist (optional): [nseg, bins] uint32.
DL4J_API int dl4j_segment_stats(int dtype, const void* x, const long long* off, int nseg, long long maxlen,
                                float* ws, float* out, int bins, unsigned* hist, hipStream_t stream) {
  if (nseg <= 0) return 0;
  float* acc = ws;
  int* mm = reinterpret_cast<int*>(ws + 3 * nseg);
  hipLaunchKernelGGL(seg_init_kernel, dim3((nseg + 255) / 256), dim3(256), 0, stream, acc, mm, nseg);
  dim3 grid(chunks_for(maxlen), nseg);
  if (dtype == 1)
    hipLaunchKernelGGL(seg_stats_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)x, off, acc, mm);
  else
    hipLaunchKernelGGL(seg_stats_kernel<float>, grid, dim3(256), 0, stream, (const float*)x, off, acc, mm);
  hipLaunchKernelGGL(seg_final_kernel, dim3((nseg + 255) / 256), dim3(256), 0, stream, acc, mm, off, nseg, out);
  if (hist && bins > 0) {
    if (bins > 4096) return -2;
    if (hipMemsetAsync(hist, 0, sizeof(unsigned) * size_t(nseg) * bins, stream) != hipSuccess) return -3;
    const size_t lds = sizeof(unsigned) * bins;
    if (dtype == 1)
      hipLaunchKernelGGL(seg_hist_kernel<bf16>, grid, dim3(256), lds, stream, (const bf16*)x, off, out, bins, hist);
    else
      hipLaunchKernelGGL(seg_hist_kernel<float>, grid, dim3(256), lds, stream, (const float*)x, off, out, bins,
                         hist);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------------
// Column sums of a row-major [M, C] bf16/fp16/fp32 matrix into fp32 out[C] (conv / dense bias gradients: dy in
// channels-last is exactly such a matrix). Each thread owns 8 consecutive channels (one 16-byte load for bf16) of a
// row; a block sweeps rows in a grid-stride loop and reduces through LDS into its own partial row part[block][C]
// (plain stores); channel_sum_reduce then sums the partial rows in block order. No float atomics: bitwise
// reproducible (DL4J_AMD_DETERMINISTIC data-parallel equivalence). C % 8 == 0: channels beyond 2048 are split over
// blockIdx.y chunks of 2048 (transformer bias gradients: 768 / 2304 / 3072 columns); other widths take the
// one-column-per-thread kernel below.
// ------------------------------------------------------------------------------------------------------
namespace {
template <typename T>
__global__ __launch_bounds__(256) void channel_sum_kernel(const T* __restrict__ xfull, long long M, int ld,
                                                          float* __restrict__ part) {
  extern __shared__ float red[];                         // [rows_per_iter][C]
  const int c0 = blockIdx.y * 2048;
  const int C = min(2048, ld - c0);
  const T* x = xfull + c0;
  const int groups = C / 8;                              // threads per row
  const int rows_per_iter = 256 / groups;
  const int g = threadIdx.x % groups, r0 = threadIdx.x / groups;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rows_per_iter) {
    long long r = (long long)blockIdx.x * rows_per_iter + r0;
    const long long step = (long long)gridDim.x * rows_per_iter;
    constexpr int U = 8;                                  // eight independent 16-byte loads in flight, kept packed
    for (; r + (U - 1) * step < M; r += U * step) {
      RawVec8<T> v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u].load(x + (r + u * step) * ld + g * 8);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[u].get(j);
    }
    for (; r < M; r += step) {
      float v[8];
      Vec8<T>::load(x + r * ld + g * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    for (int j = 0; j < 8; ++j) red[r0 * C + g * 8 + j] = acc[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < rows_per_iter; ++k) s += red[k * C + c];
    part[(long long)blockIdx.x * ld + c0 + c] = s;
  }
}

// partial rows [nblk][C] -> out[C]: a block owns 64 channels, its 4 row groups sum every 4th partial row in a fixed
// order and combine through LDS (the same shape as bn_reduce_rows; one thread per channel serialised 512 rows).
// Eight independent loads per trip: two per trip left the 128-row BERT reduces latency-bound (6.5 us a launch).
__global__ __launch_bounds__(256) void channel_sum_reduce(const float* __restrict__ part, int nblk, int C,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    for (int b0 = grp; b0 < nblk; b0 += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + 4 * u;
        v[u] = b < nblk ? part[(long long)b * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 += v[u];
        s1 += v[u + 1];
      }
    }
  }
  __shared__ float red[256];
  red[threadIdx.x] = s0 + s1;
  __syncthreads();
  if (grp == 0 && c < C) out[c] = (red[threadIdx.x] + red[threadIdx.x + 64]) + (red[threadIdx.x + 128] + red[threadIdx.x + 192]);
}

// C % 8 != 0 (LeNet's 20 / 50 / 500-wide bias gradients): one thread per column of a 256-column chunk
// (blockIdx.y), 256 / min(C, 256) rows per block iteration, eight independent loads in flight; same partial rows.
template <typename T>
__global__ __launch_bounds__(256) void channel_sum_scalar_kernel(const T* __restrict__ x, long long M, int ld,
                                                                 float* __restrict__ part) {
  extern __shared__ float red[];
  const int c0 = blockIdx.y * 256;
  const int Cc = min(256, ld - c0);
  const int Cw = min(ld, 256);                           // LDS row pitch: rows_per_iter * Cw <= 256 floats
  const int rows_per_iter = 256 / Cw;
  const int c = threadIdx.x % Cw, r0 = threadIdx.x / Cw;
  float acc = 0.f;
  if (r0 < rows_per_iter && c < Cc) {
    long long r = (long long)blockIdx.x * rows_per_iter + r0;
    const long long step = (long long)gridDim.x * rows_per_iter;
    constexpr int U = 8;
    for (; r + (U - 1) * step < M; r += U * step) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld1<T>(x + (r + u * step) * ld + c0 + c);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
    }
    for (; r < M; r += step) acc += ld1<T>(x + r * ld + c0 + c);
  }
  if (r0 < rows_per_iter) red[r0 * Cw + c] = acc;
  __syncthreads();
  for (int cc = threadIdx.x; cc < Cc; cc += 256) {
    float sum = 0.f;
    for (int k = 0; k < rows_per_iter; ++k) sum += red[k * Cw + cc];
    part[(long long)blockIdx.x * ld + c0 + cc] = sum;
  }
}

int channel_sum_blocks(long long M, int C) {
  const int Cc = C < 2048 ? C : 2048;                    // widest chunk; the last chunk may be narrower
  const int rows_per_iter = C % 8 ? 256 / (C < 256 ? C : 256) : 256 / (Cc / 8);
  long long blocks = (M + rows_per_iter * 32 - 1) / (rows_per_iter * 32);
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}
}  // namespace

// Workspace floats dl4j_channel_sum needs for an [M, C] input.
DL4J_API long long dl4j_channel_sum_ws_floats(long long M, int C) { return (long long)channel_sum_blocks(M, C) * C; }

// ws: >= dl4j_channel_sum_ws_floats(M, C) fp32 scratch.
DL4J_API int dl4j_channel_sum(int dtype, const void* x, long long M, int C, float* out, float* ws, hipStream_t stream) {
  if (C <= 0 || M <= 0 || !ws) return -1;
  const int blocks = channel_sum_blocks(M, C);
  const size_t lds = sizeof(float) * 256 * 8;             // >= rows_per_iter * chunk width for every chunk
  if (C % 8) {
    const dim3 gs((unsigned)blocks, (C + 255) / 256);
    if (dtype == 1)
      hipLaunchKernelGGL(channel_sum_scalar_kernel<bf16>, gs, dim3(256), lds, stream, (const bf16*)x, M, C, ws);
    else if (dtype == 2)
      hipLaunchKernelGGL(channel_sum_scalar_kernel<f16>, gs, dim3(256), lds, stream, (const f16*)x, M, C, ws);
    else
      hipLaunchKernelGGL(channel_sum_scalar_kernel<float>, gs, dim3(256), lds, stream, (const float*)x, M, C, ws);
    hipLaunchKernelGGL(channel_sum_reduce, dim3((C + 63) / 64), dim3(256), 0, stream, ws, blocks, C, out);
    return (int)hipGetLastError();
  }
  const dim3 grid((unsigned)blocks, (C + 2047) / 2048);
  if (dtype == 1)
    hipLaunchKernelGGL(channel_sum_kernel<bf16>, grid, dim3(256), lds, stream, (const bf16*)x, M, C, ws);
  else if (dtype == 2)
    hipLaunchKernelGGL(channel_sum_kernel<f16>, grid, dim3(256), lds, stream, (const f16*)x, M, C, ws);
  else
    hipLaunchKernelGGL(channel_sum_kernel<float>, grid, dim3(256), lds, stream, (const float*)x, M, C, ws);
  hipLaunchKernelGGL(channel_sum_reduce, dim3((C + 63) / 64), dim3(256), 0, stream, ws, blocks, C, out);
  return (int)hipGetLastError();
}
