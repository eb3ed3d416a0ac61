// Threshold / bitmap gradient-update compression for the encoded update-sharing mode
// (reference NN:optimize/solvers/accumulation/EncodingHandler.java:114-191, EncodedGradientsAccumulator.java:244-521,
// libnd4j thresholdEncode/thresholdDecode/bitmapEncode/bitmapDecode).
//
// Message layout (int32): [0] count, [1] n (vector length), [2] threshold (float bits), [3] type (0 = sparse
// threshold, 1 = bitmap), payload from [4].
//   sparse:  count entries, +(i+1) for +threshold, -(i+1) for -threshold, in ascending index order
//   bitmap:  ceil(n/16) words, 2 bits per element: 01 = +threshold, 10 = -threshold
// Encoding subtracts what it emits from the residual in place (residual semantics of storeUpdate).
//
// The sparse encoder is a deterministic stream compaction: (1) per-block counts with wave ballots,
// (2) one-block exclusive scan of the block counts, (3) in-order write. Each block owns 2048 elements
// (8 per thread), each wave 512 contiguous elements as 8 ballot rounds of 64.
#include "common.h"

#define TC_BLOCK 256
#define TC_PER_THREAD 8
#define TC_CHUNK (TC_BLOCK * TC_PER_THREAD)

__device__ __forceinline__ int flag_of(float v, float thr) { return v >= thr ? 1 : (v <= -thr ? -1 : 0); }

// wave w of the block handles elements [base + w*512, base + (w+1)*512) in 8 rounds of 64 consecutive
__global__ __launch_bounds__(TC_BLOCK) void tc_count(const float* __restrict__ r, long long n, float thr,
                                                     int* __restrict__ blk_counts) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long base = (long long)blockIdx.x * TC_CHUNK + (long long)w * 512;
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < TC_PER_THREAD; ++k) {
    const long long i = base + k * 64 + lane;
    const bool f = i < n && flag_of(r[i], thr) != 0;
    cnt += __popcll(__ballot(f));
  }
  __shared__ int wc[TC_BLOCK / 64];
  if (lane == 0) wc[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < TC_BLOCK / 64; ++i) s += wc[i];
    blk_counts[blockIdx.x] = s;
  }
}

// exclusive scan of nb block counts (single block of 1024 threads, chunked), total -> out[0..3] header
__global__ __launch_bounds__(1024) void tc_scan(int* __restrict__ blk, int nb, int* __restrict__ out, long long n,
                                                float thr, int capacity) {
  __shared__ int part[1024];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nb; b0 += 1024) {
    const int i = b0 + threadIdx.x;
    const int v = i < nb ? blk[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {       // Hillis-Steele inclusive scan
      const int t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) blk[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = carry < capacity ? carry : capacity;
    out[1] = (int)n;
    out[2] = __float_as_int(thr);
    out[3] = 0;
  }
}

__global__ __launch_bounds__(TC_BLOCK) void tc_write(float* __restrict__ r, long long n, float thr,
                                                     const int* __restrict__ blk_off, int* __restrict__ out,
                                                     int capacity) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long base = (long long)blockIdx.x * TC_CHUNK + (long long)w * 512;
  // count of this wave's flags -> wave offset within the block
  int mine = 0;
  int flags[TC_PER_THREAD];
#pragma unroll
  for (int k = 0; k < TC_PER_THREAD; ++k) {
    const long long i = base + k * 64 + lane;
    flags[k] = i < n ? flag_of(r[i], thr) : 0;
    mine += __popcll(__ballot(flags[k] != 0));
  }
  __shared__ int wc[TC_BLOCK / 64];
  if (lane == 0) wc[w] = mine;
  __syncthreads();
  int pos = blk_off[blockIdx.x];
  for (int i = 0; i < w; ++i) pos += wc[i];
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int k = 0; k < TC_PER_THREAD; ++k) {
    const unsigned long long b = __ballot(flags[k] != 0);
    if (flags[k] != 0) {
      const int p = pos + __popcll(b & lt);
      if (p < capacity) {
        const long long i = base + k * 64 + lane;
        out[4 + p] = flags[k] > 0 ? (int)(i + 1) : -(int)(i + 1);
        r[i] -= flags[k] * thr;
      }
    }
    pos += __popcll(b);
  }
}

__global__ void tc_decode(const int* __restrict__ enc, float* __restrict__ target, float scale) {
  if (enc[3] != 0) return;                  // not a sparse message
  const int cnt = enc[0];
  const float thr = __int_as_float(enc[2]) * scale;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
    const int e = enc[4 + j];
    const int i = (e > 0 ? e : -e) - 1;
    target[i] += e > 0 ? thr : -thr;        // indices are unique within one message: no atomics needed
  }
}

// bitmap: one thread per 16 elements -> one 32-bit word
__global__ void bm_encode(float* __restrict__ r, long long n, float thr, int* __restrict__ out,
                          int* __restrict__ counter) {
  const long long nw = (n + 15) / 16;
  int local = 0;
  for (long long wi = (long long)blockIdx.x * blockDim.x + threadIdx.x; wi < nw;
       wi += (long long)gridDim.x * blockDim.x) {
    unsigned word = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const long long i = wi * 16 + k;
      if (i < n) {
        const int f = flag_of(r[i], thr);
        if (f != 0) {
          word |= (f > 0 ? 1u : 2u) << (2 * k);
          r[i] -= f * thr;
          ++local;
        }
      }
    }
    out[4 + wi] = (int)word;
  }
  local = (int)wave_sum((float)local);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(counter, local);
}

__global__ void bm_header(int* out, const int* counter, long long n, float thr) {
  out[0] = *counter;
  out[1] = (int)n;
  out[2] = __float_as_int(thr);
  out[3] = 1;
}

__global__ void bm_decode(const int* __restrict__ enc, float* __restrict__ target, float scale) {
  if (enc[3] != 1) return;                  // not a bitmap message
  const long long n = enc[1];
  const float thr = __int_as_float(enc[2]) * scale;
  const long long nw = (n + 15) / 16;
  for (long long wi = (long long)blockIdx.x * blockDim.x + threadIdx.x; wi < nw;
       wi += (long long)gridDim.x * blockDim.x) {
    const unsigned word = (unsigned)enc[4 + wi];
    if (!word) continue;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const unsigned b = (word >> (2 * k)) & 3u;
      if (b) target[wi * 16 + k] += b == 1u ? thr : -thr;
    }
  }
}

static inline int grid_for(long long work, int per_block) {
  long long g = (work + per_block - 1) / per_block;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

// workspace: >= dl4j_threshold_ws_ints(n) ints. Returns immediately (async); count is out[0] on device.
DL4J_API long long dl4j_threshold_ws_ints(long long n) { return (n + TC_CHUNK - 1) / TC_CHUNK + 1; }

DL4J_API int dl4j_threshold_encode(float* residual, long long n, float thr, int* out, int capacity, int* ws,
                                   hipStream_t s) {
  const int nb = (int)((n + TC_CHUNK - 1) / TC_CHUNK);
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(tc_count, dim3(nb), dim3(TC_BLOCK), 0, s, residual, n, thr, ws);
  hipLaunchKernelGGL(tc_scan, dim3(1), dim3(1024), 0, s, ws, nb, out, n, thr, capacity);
  hipLaunchKernelGGL(tc_write, dim3(nb), dim3(TC_BLOCK), 0, s, residual, n, thr, ws, out, capacity);
  return (int)hipGetLastError();
}

// count only (for the host's sparse-vs-bitmap decision): hdr4[0] = number of |r| >= thr entries
DL4J_API int dl4j_threshold_count(const float* residual, long long n, float thr, int* ws, int* hdr4,
                                  hipStream_t s) {
  const int nb = (int)((n + TC_CHUNK - 1) / TC_CHUNK);
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(tc_count, dim3(nb), dim3(TC_BLOCK), 0, s, residual, n, thr, ws);
  hipLaunchKernelGGL(tc_scan, dim3(1), dim3(1024), 0, s, ws, nb, hdr4, n, thr, 0x7fffffff);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_threshold_decode(const int* enc, float* target, int max_count, float scale, hipStream_t s) {
  hipLaunchKernelGGL(tc_decode, dim3(grid_for(max_count, 256)), dim3(256), 0, s, enc, target, scale);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bitmap_encode(float* residual, long long n, float thr, int* out, int* counter, hipStream_t s) {
  hipMemsetAsync(counter, 0, sizeof(int), s);
  hipLaunchKernelGGL(bm_encode, dim3(grid_for((n + 15) / 16, 256)), dim3(256), 0, s, residual, n, thr, out, counter);
  hipLaunchKernelGGL(bm_header, dim3(1), dim3(1), 0, s, out, counter, n, thr);
  return (int)hipGetLastError();
}

// decode a message of either type without a host round trip: both kernels launch, each exits unless the
// device-side header says it is its type. max_payload = message length - 4.
DL4J_API int dl4j_decode_any(const int* enc, long long n, int max_payload, float* target, float scale, hipStream_t s) {
  hipLaunchKernelGGL(tc_decode, dim3(grid_for(max_payload, 256)), dim3(256), 0, s, enc, target, scale);
  hipLaunchKernelGGL(bm_decode, dim3(grid_for((n + 15) / 16, 256)), dim3(256), 0, s, enc, target, scale);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bitmap_decode(const int* enc, long long n, float* target, float scale, hipStream_t s) {
  hipLaunchKernelGGL(bm_decode, dim3(grid_for((n + 15) / 16, 256)), dim3(256), 0, s, enc, target, scale);
  return (int)hipGetLastError();
}
