// Embedding learners on gfx950: skip-gram / CBOW (hierarchical softmax + negative sampling) and GloVe (AdaGrad).
//
// Reference: the AggregateSkipGram / AggregateCBOW batches the NLP learners hand to libnd4j
// (NLP:models/embeddings/learning/impl/elements/SkipGram.java:271-283, CBOW.java) and GloVe.java:182-225.
// MI355X mapping: one 64-lane wavefront per work item; a D-dimensional row lives in registers as VPL values per
// lane (D <= 64*VPL), dot products are wave reductions (xor shuffles within the wave), and every row update is a
// coalesced 64-lane read-modify-write. Updates are Hogwild (no atomics between items) exactly like the reference's
// concurrent worker threads; within an item the wave is the only writer. The caller caps the number of resident
// waves relative to the vocabulary size (max_blocks) so that small vocabularies do not turn Hogwild into a storm of
// lost updates on the same few rows. Work items come from the host batcher
// (csrc/runtime/embeddings.cpp) and use the same per-item LCG seeds as the CPU applier there.
#include "common.h"

namespace {

constexpr float MAX_EXP = 6.0f;
enum { F_UPD_OUT = 1, F_UPD_IN = 2, F_HS = 4, F_NS = 8 };

__device__ __forceinline__ uint64_t lcg(uint64_t r) { return r * 25214903917ULL + 11ULL; }
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct Out {
  float* syn1; float* syn1neg; int D;
  const uint8_t* codes; const int32_t* points; const int32_t* codelen; int maxc;
  const int32_t* table; long long tsize; int negative; int flags;
};

template <int VPL>
__device__ __forceinline__ void load_row(const float* row, int D, int lane, float* v) {
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    int k = lane + 64 * j;
    v[j] = k < D ? row[k] : 0.f;
  }
}

// HS + NS for input l1 (registers) against target word tgt; accumulates neu1e; returns the item's loss (uniform).
template <int VPL>
__device__ float learn_wave(const Out& O, const float* l1, float* e, int tgt, uint64_t rng, float alpha, int lane) {
  const int D = O.D;
  float loss = 0.f;
  float w[VPL];
  if (O.flags & F_HS) {
    const int L = O.codelen[tgt];
    for (int c = 0; c < L; ++c) {
      float* row = O.syn1 + (long long)O.points[(long long)tgt * O.maxc + c] * D;
      load_row<VPL>(row, D, lane, w);
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < VPL; ++j) p += l1[j] * w[j];
      const float f = wave_sum(p);
      if (f <= -MAX_EXP || f >= MAX_EXP) continue;
      const float sg = 1.f / (1.f + __expf(-f));
      const int code = O.codes[(long long)tgt * O.maxc + c];
      const float g = (1.f - code - sg) * alpha;
      loss -= __logf(fmaxf(1e-7f, code ? 1.f - sg : sg));
#pragma unroll
      for (int j = 0; j < VPL; ++j) e[j] += g * w[j];
      if (O.flags & F_UPD_OUT) {
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          int k = lane + 64 * j;
          if (k < D) row[k] = w[j] + g * l1[j];
        }
      }
    }
  }
  if ((O.flags & F_NS) && O.negative > 0) {
    for (int d = 0; d <= O.negative; ++d) {
      int target, label;
      if (d == 0) { target = tgt; label = 1; }
      else {
        rng = lcg(rng);
        target = O.table[(rng >> 16) % (uint64_t)O.tsize];
        if (target == tgt) continue;
        label = 0;
      }
      float* row = O.syn1neg + (long long)target * D;
      load_row<VPL>(row, D, lane, w);
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < VPL; ++j) p += l1[j] * w[j];
      const float f = wave_sum(p);
      const float sg = f > MAX_EXP ? 1.f : (f < -MAX_EXP ? 0.f : 1.f / (1.f + __expf(-f)));
      const float g = (float(label) - sg) * alpha;
      loss -= __logf(fmaxf(1e-7f, label ? sg : 1.f - sg));
#pragma unroll
      for (int j = 0; j < VPL; ++j) e[j] += g * w[j];
      if (O.flags & F_UPD_OUT) {
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          int k = lane + 64 * j;
          if (k < D) row[k] = w[j] + g * l1[j];
        }
      }
    }
  }
  return loss;
}

template <int VPL>
__global__ __launch_bounds__(256) void w2v_sg_kernel(const int32_t* __restrict__ item_in,
                                                     const int32_t* __restrict__ item_tgt,
                                                     const float* __restrict__ item_alpha, long long n, float* syn0,
                                                     Out O, uint64_t seed, long long item_base, float* loss_out) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  float loss = 0.f;
  for (long long i = wave; i < n; i += nw) {
    float* in = syn0 + (long long)item_in[i] * O.D;
    float l1[VPL], e[VPL];
    load_row<VPL>(in, O.D, lane, l1);
#pragma unroll
    for (int j = 0; j < VPL; ++j) e[j] = 0.f;
    loss += learn_wave<VPL>(O, l1, e, item_tgt[i], mix(seed ^ (uint64_t)(item_base + i)), item_alpha[i], lane);
    if (O.flags & F_UPD_IN) {
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        int k = lane + 64 * j;
        if (k < O.D) in[k] += e[j];
      }
    }
  }
  if (loss_out && lane == 0 && loss != 0.f) atomicAdd(loss_out, loss);
}

template <int VPL>
__global__ __launch_bounds__(256) void w2v_cbow_kernel(const int32_t* __restrict__ item_tgt,
                                                       const float* __restrict__ item_alpha,
                                                       const int32_t* __restrict__ ctx_off,
                                                       const int32_t* __restrict__ ctx, long long n, float* syn0,
                                                       Out O, uint64_t seed, long long item_base,
                                                       const float* extra_in, int n_extra, float* extra_grad,
                                                       float* loss_out) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  const int D = O.D;
  float loss = 0.f;
  for (long long i = wave; i < n; i += nw) {
    const int c0 = ctx_off[i], c1 = ctx_off[i + 1];
    const int cw = c1 - c0 + n_extra;
    if (cw <= 0) continue;
    float l1[VPL], e[VPL], v[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) { l1[j] = 0.f; e[j] = 0.f; }
    for (int c = c0; c < c1; ++c) {
      load_row<VPL>(syn0 + (long long)ctx[c] * D, D, lane, v);
#pragma unroll
      for (int j = 0; j < VPL; ++j) l1[j] += v[j];
    }
    for (int x = 0; x < n_extra; ++x) {
      load_row<VPL>(extra_in + (long long)x * D, D, lane, v);
#pragma unroll
      for (int j = 0; j < VPL; ++j) l1[j] += v[j];
    }
    const float inv = 1.f / float(cw);
#pragma unroll
    for (int j = 0; j < VPL; ++j) l1[j] *= inv;
    loss += learn_wave<VPL>(O, l1, e, item_tgt[i], mix(seed ^ (uint64_t)(item_base + i)), item_alpha[i], lane);
    if (O.flags & F_UPD_IN) {
      for (int c = c0; c < c1; ++c) {
        float* row = syn0 + (long long)ctx[c] * D;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          int k = lane + 64 * j;
          if (k < D) row[k] += e[j];
        }
      }
    }
    if (extra_grad) {
      for (int x = 0; x < n_extra; ++x)
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          int k = lane + 64 * j;
          if (k < D) atomicAdd(extra_grad + (long long)x * D + k, e[j]);
        }
    }
  }
  if (loss_out && lane == 0 && loss != 0.f) atomicAdd(loss_out, loss);
}

template <int VPL>
__global__ __launch_bounds__(256) void glove_kernel(const int32_t* __restrict__ ei, const int32_t* __restrict__ ej,
                                                    const float* __restrict__ ex, long long n, float* W, float* b,
                                                    float* hW, float* hb, int D, float lr, float xmax, float alpha,
                                                    float* cost_out) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  float cost = 0.f;
  for (long long k = wave; k < n; k += nw) {
    const int i = ei[k], j = ej[k];
    float* wi = W + (long long)i * D;
    float* wj = W + (long long)j * D;
    float a[VPL], c[VPL];
    load_row<VPL>(wi, D, lane, a);
    load_row<VPL>(wj, D, lane, c);
    float p = 0.f;
#pragma unroll
    for (int q = 0; q < VPL; ++q) p += a[q] * c[q];
    const float x = ex[k];
    const float pred = wave_sum(p) + b[i] + b[j] - __logf(x);
    const float fd = (x > xmax ? 1.f : __powf(x / xmax, alpha)) * pred;
    cost += 0.5f * fd * pred;
    float* hi = hW + (long long)i * D;
    float* hj = hW + (long long)j * D;
#pragma unroll
    for (int q = 0; q < VPL; ++q) {
      int d = lane + 64 * q;
      if (d < D) {
        const float gi = fd * c[q], gj = fd * a[q];
        const float ni = hi[d] + gi * gi;
        hi[d] = ni;
        wi[d] = a[q] - lr * gi * rsqrtf(ni + 1e-8f);
        const float nj = hj[d] + gj * gj;
        hj[d] = nj;
        wj[d] = c[q] - lr * gj * rsqrtf(nj + 1e-8f);
      }
    }
    if (lane == 0) {
      float t = hb[i] + fd * fd;
      hb[i] = t;
      b[i] -= lr * fd * rsqrtf(t + 1e-8f);
      t = hb[j] + fd * fd;
      hb[j] = t;
      b[j] -= lr * fd * rsqrtf(t + 1e-8f);
    }
  }
  if (cost_out && lane == 0 && cost != 0.f) atomicAdd(cost_out, cost);
}

inline int vpl_for(int D) { return D <= 64 ? 1 : D <= 128 ? 2 : D <= 256 ? 4 : D <= 512 ? 8 : D <= 1024 ? 16 : 0; }
inline int grid_for(long long n) {
  long long b = (n + 3) / 4;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

#define VPL_DISPATCH(D, CALL)                          \
  switch (vpl_for(D)) {                                \
    case 1: { constexpr int V = 1; CALL; break; }      \
    case 2: { constexpr int V = 2; CALL; break; }      \
    case 4: { constexpr int V = 4; CALL; break; }      \
    case 8: { constexpr int V = 8; CALL; break; }      \
    case 16: { constexpr int V = 16; CALL; break; }    \
    default: return -2;                                \
  }

DL4J_API int dl4j_w2v_sg(const int32_t* item_in, const int32_t* item_tgt, const float* alpha, long long n,
                         float* syn0, float* syn1, float* syn1neg, int D, const uint8_t* codes, const int32_t* points,
                         const int32_t* codelen, int maxc, const int32_t* table, long long tsize, int negative,
                         int flags, unsigned long long seed, long long item_base, float* loss_out, int max_blocks,
                         hipStream_t stream) {
  if (n <= 0) return 0;
  Out O{syn1, syn1neg, D, codes, points, codelen, maxc, table, tsize, negative, flags};
  const int grid = max_blocks > 0 && grid_for(n) > max_blocks ? max_blocks : grid_for(n);
  VPL_DISPATCH(D, hipLaunchKernelGGL(w2v_sg_kernel<V>, dim3(grid), dim3(256), 0, stream, item_in, item_tgt,
                                     alpha, n, syn0, O, (uint64_t)seed, item_base, loss_out));
  return (int)hipGetLastError();
}

DL4J_API int dl4j_w2v_cbow(const int32_t* item_tgt, const float* alpha, const int32_t* ctx_off, const int32_t* ctx,
                           long long n, float* syn0, float* syn1, float* syn1neg, int D, const uint8_t* codes,
                           const int32_t* points, const int32_t* codelen, int maxc, const int32_t* table,
                           long long tsize, int negative, int flags, unsigned long long seed, long long item_base,
                           const float* extra_in, int n_extra, float* extra_grad, float* loss_out, int max_blocks,
                           hipStream_t stream) {
  if (n <= 0) return 0;
  Out O{syn1, syn1neg, D, codes, points, codelen, maxc, table, tsize, negative, flags};
  const int grid = max_blocks > 0 && grid_for(n) > max_blocks ? max_blocks : grid_for(n);
  VPL_DISPATCH(D, hipLaunchKernelGGL(w2v_cbow_kernel<V>, dim3(grid), dim3(256), 0, stream, item_tgt, alpha,
                                     ctx_off, ctx, n, syn0, O, (uint64_t)seed, item_base, extra_in, n_extra,
                                     extra_grad, loss_out));
  return (int)hipGetLastError();
}

DL4J_API int dl4j_glove(const int32_t* ei, const int32_t* ej, const float* ex, long long n, float* W, float* b,
                        float* hW, float* hb, int D, float lr, float xmax, float alpha, float* cost_out,
                        int max_blocks, hipStream_t stream) {
  if (n <= 0) return 0;
  const int grid = max_blocks > 0 && grid_for(n) > max_blocks ? max_blocks : grid_for(n);
  VPL_DISPATCH(D, hipLaunchKernelGGL(glove_kernel<V>, dim3(grid), dim3(256), 0, stream, ei, ej, ex, n, W, b,
                                     hW, hb, D, lr, xmax, alpha, cost_out));
  return (int)hipGetLastError();
}
