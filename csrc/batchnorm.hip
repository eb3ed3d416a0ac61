// Batch normalization for channels-last activations viewed as a row-major [M, C] matrix
// (M = N*H*W, C % 8 == 0), bf16 or fp32 storage, fp32 math.
// Optional fused epilogues (chosen by the graph planner):
//   RELU:  y = relu(bn(x))                       (BN -> ActivationLayer(ReLU))
//   RES:   y = relu(bn(x) + r)                   (BN -> ElementWiseVertex(Add, shortcut) -> ReLU: ResNet blocks)
//
// Semantics = reference nn/layers/normalization/BatchNormalization.java (biased batch variance, eps added
// before sqrt, running stats: run = decay*run + (1-decay)*stat, running var tracks var+eps).
//
// Forward (training): stats_partial -> finalize -> apply.   Backward: bwd_partial -> bwd_finalize -> bwd_apply.
// Each thread owns 8 consecutive channels (one 16-byte vector); a block covers R = 256/(C/8) rows per sweep,
// so every wave issues fully coalesced dwordx4 loads. Per-block partial sums go to a [nblk, C] fp32
// workspace (no atomics -> bitwise reproducible); with many partial rows a level-1 kernel first folds every 32 rows
// in parallel (bn_reduce_rows), then finalize reduces the rest in double with 4 row-groups x 64 channels per
// block. The ReLU mask in backward is recomputed from x (and r), so no activation needs to be stored.
#include "common.h"
#include <cstdlib>

// --------------------------------------------------------------------------------------------- forward
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial(const T* __restrict__ x, long long M, int C,
                                                        long long rows_per_blk, float* __restrict__ part_s1,
                                                        float* __restrict__ part_s2) {
  const int T8 = C >> 3;
  const int R = 256 / T8;                       // rows per sweep
  const int cg = threadIdx.x % T8, r0 = threadIdx.x / T8;
  float s1[8], s2[8], sh[8];
  Vec8<T>::load(x + cg * 8, sh);                // row 0 is the shift: sums of (x - x0) avoid cancellation
#pragma unroll
  for (int i = 0; i < 8; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  const long long rbeg = (long long)blockIdx.x * rows_per_blk;
  long long rend = rbeg + rows_per_blk;
  if (rend > M) rend = M;
  if (r0 < R) {
    long long r = rbeg + r0;
    // 4 independent 16-byte loads in flight per thread before any use (memory-level parallelism)
    for (; r + 3 * R < rend; r += 4 * R) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) Vec8<T>::load(x + (r + u * R) * C + cg * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = v[u][i] - sh[i]; s1[i] += d; s2[i] += d * d; }
    }
    for (; r < rend; r += R) {
      float v[8];
      Vec8<T>::load(x + r * C + cg * 8, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = v[i] - sh[i]; s1[i] += d; s2[i] += d * d; }
    }
  }
  __shared__ float red1[256 * 9];   // row pitch 9 floats: conflict-free 8-float stores
  __shared__ float red2[256 * 9];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red1[threadIdx.x * 9 + i] = (r0 < R) ? s1[i] : 0.f;
    red2[threadIdx.x * 9 + i] = (r0 < R) ? s2[i] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < R; ++rr) { a += red1[(rr * T8 + g) * 9 + k]; b += red2[(rr * T8 + g) * 9 + k]; }
    part_s1[(long long)blockIdx.x * C + c] = a;
    part_s2[(long long)blockIdx.x * C + c] = b;
  }
}

// Level-1 partial reduction: [nblk, C] -> [ceil(nblk/32), C]. grid = (ceil(C/64), ceil(nblk/32)); each of the 4
// row groups of a block sums 8 rows with independent loads (one HBM round trip), so even C = 64 spreads over
// nblk/32 blocks instead of serialising nblk rows in one block.
__global__ __launch_bounds__(256) void bn_reduce_rows(const float* __restrict__ p1, const float* __restrict__ p2,
                                                      int nblk, int C, float* __restrict__ q1, float* __restrict__ q2) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const int r0 = blockIdx.y * 32 + grp * 8;
  float a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = r0 + u;
    const bool ok = c < C && r < nblk;
    a[u] = ok ? p1[(long long)r * C + c] : 0.f;
    b[u] = ok ? p2[(long long)r * C + c] : 0.f;
  }
  float sa = 0.f, sb = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) { sa += a[u]; sb += b[u]; }
  __shared__ float ra[256], rb[256];
  ra[threadIdx.x] = sa; rb[threadIdx.x] = sb;
  __syncthreads();
  if (grp == 0 && c < C) {
    q1[(long long)blockIdx.y * C + c] = ra[threadIdx.x] + ra[threadIdx.x + 64] + ra[threadIdx.x + 128] + ra[threadIdx.x + 192];
    q2[(long long)blockIdx.y * C + c] = rb[threadIdx.x] + rb[threadIdx.x + 64] + rb[threadIdx.x + 128] + rb[threadIdx.x + 192];
  }
}

// Per-tile statistics from the conv epilogue (csrc/conv_igemm.hip, planes [3][P][C]: S1, S2 about a per-partial
// shift y_p, partial p = rows [rpp*p, rpp*p + rpp), rpp = 64 for the igemm kernels, one output row for the stem) -> the [ceil(P/32), C] partial-sum format of bn_stats_partial
// (sums about the GLOBAL shift x0 = row 0). Re-centring uses d = y_p - x0 (both samples of the same channel, so
// O(std), no cancellation): S1' = S1 + n d, S2' = S2 + 2 d S1 + n d^2. grid = (ceil(C/64), ceil(P/32)).
template <typename T>
__global__ __launch_bounds__(256) void bn_tiles_reduce(const float* __restrict__ ts, long long P, int C, long long M,
                                                       const T* __restrict__ x, float* __restrict__ q1,
                                                       float* __restrict__ q2, int rpp) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const long long p0 = (long long)blockIdx.y * 32 + grp * 8;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    const float x0 = ld1<T>(x + c);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long p = p0 + u;
      if (p >= P) break;
      const long long nrow = M - (long long)rpp * p;
      const float n = (float)(nrow < rpp ? (nrow < 0 ? 0 : nrow) : rpp);
      const float s1 = ts[p * C + c], s2 = ts[(P + p) * C + c], d = ts[(2 * P + p) * C + c] - x0;
      sa += s1 + n * d;
      sb += s2 + 2.f * d * s1 + n * d * d;
    }
  }
  __shared__ float ra[256], rb[256];
  ra[threadIdx.x] = sa;
  rb[threadIdx.x] = sb;
  __syncthreads();
  if (grp == 0 && c < C) {
    q1[(long long)blockIdx.y * C + c] = ra[threadIdx.x] + ra[threadIdx.x + 64] + ra[threadIdx.x + 128] + ra[threadIdx.x + 192];
    q2[(long long)blockIdx.y * C + c] = rb[threadIdx.x] + rb[threadIdx.x + 64] + rb[threadIdx.x + 128] + rb[threadIdx.x + 192];
  }
}

// Reduce [nblk, C] partials: block = 64 channels x 4 row groups.
__device__ __forceinline__ void reduce_partials(const float* __restrict__ p1, const float* __restrict__ p2, int nblk,
                                                int C, int c, double& a, double& b) {
  const int grp = threadIdx.x >> 6;
  a = 0.0; b = 0.0;
  if (c < C)
    for (int i = grp; i < nblk; i += 4) { a += p1[(long long)i * C + c]; b += p2[(long long)i * C + c]; }
  __shared__ double ra[256], rb[256];
  ra[threadIdx.x] = a; rb[threadIdx.x] = b;
  __syncthreads();
  if (grp == 0) {
    a = ra[threadIdx.x] + ra[threadIdx.x + 64] + ra[threadIdx.x + 128] + ra[threadIdx.x + 192];
    b = rb[threadIdx.x] + rb[threadIdx.x + 64] + rb[threadIdx.x + 128] + rb[threadIdx.x + 192];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_finalize(const float* __restrict__ part_s1, const float* __restrict__ part_s2,
                                                   int nblk, int C, long long M, const T* __restrict__ x,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float gconst, float bconst, float* __restrict__ run_mean,
                                                   float* __restrict__ run_var, float decay, float eps, int training,
                                                   float* __restrict__ ctx) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double a = 0.0, b = 0.0;
  if (training) reduce_partials(part_s1, part_s2, nblk, C, c, a, b);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  float mean, var;
  if (training) {
    const double m1 = a / (double)M;
    mean = (float)((double)ld1<T>(x + c) + m1);
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
  ctx[c] = mean;
  ctx[C + c] = inv;
  ctx[2 * C + c] = g * inv;                 // scale
  ctx[3 * C + c] = bb - mean * g * inv;     // shift
}

// mask (optional, RES only): one byte per 8-channel vector, bit i = ReLU active for channel 8*(v % (C/8)) + i, so
// the backward pass reads 1/16 of the residual's bytes instead of re-reading the residual.
// RBN (residual BatchNorm folded in): the residual is the RAW output of the shortcut branch's conv and that branch's
// own training BN (context rctx, statistics already folded) is applied here: y = relu(bn(x) + bn_r(res)). The
// shortcut BN layer then never materialises its output (ResNet convBlock: conv -> BN -> add); see bn_bwd_* RBN.
template <typename T, bool RELU, bool RES, bool RBN = false>
__global__ __launch_bounds__(256) void bn_apply(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                                                long long M, int C, const float* __restrict__ ctx,
                                                unsigned char* __restrict__ mask, const float* __restrict__ rctx) {
  const long long nvec = M * (C >> 3);
  const int T8 = C >> 3;
  const float* scale = ctx + 2 * C;
  const float* shift = ctx + 3 * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long v0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (stride % T8 == 0) {
    // every grid-stride step keeps this thread on the same 8 channels: per-channel factors live in registers and
    // two independent vectors are in flight per iteration (instead of 16 L1 parameter loads per 16-byte vector)
    const int c0 = idx_mod(v0, T8) * 8;
    float sc[8], sf[8], rsc[8], rsf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale[c0 + i]; sf[i] = shift[c0 + i];
      rsc[i] = RBN ? rctx[2 * C + c0 + i] : 1.f;
      rsf[i] = RBN ? rctx[3 * C + c0 + i] : 0.f;
    }
    long long v = v0;
    for (; v + stride < nvec; v += 2 * stride) {
      float a[2][8], r[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        Vec8<T>::load(x + (v + u * stride) * 8, a[u]);
        if (RES) Vec8<T>::load(res + (v + u * stride) * 8, r[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        unsigned bits = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float t = a[u][i] * sc[i] + sf[i];
          if (RES) t += RBN ? fmaf(r[u][i], rsc[i], rsf[i]) : r[u][i];
          bits |= (t > 0.f ? 1u : 0u) << i;
          a[u][i] = RELU ? fmaxf(t, 0.f) : t;
        }
        Vec8<T>::store(y + (v + u * stride) * 8, a[u]);
        if (RES && mask) mask[v + u * stride] = (unsigned char)bits;
      }
    }
    if (v < nvec) {
      float a[8], r[8];
      Vec8<T>::load(x + v * 8, a);
      if (RES) Vec8<T>::load(res + v * 8, r);
      unsigned bits = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float t = a[i] * sc[i] + sf[i];
        if (RES) t += RBN ? fmaf(r[i], rsc[i], rsf[i]) : r[i];
        bits |= (t > 0.f ? 1u : 0u) << i;
        a[i] = RELU ? fmaxf(t, 0.f) : t;
      }
      Vec8<T>::store(y + v * 8, a);
      if (RES && mask) mask[v] = (unsigned char)bits;
    }
    return;
  }
  for (long long v = v0; v < nvec; v += stride) {
    const int c0 = idx_mod(v, T8) * 8;
    float a[8], r[8];
    Vec8<T>::load(x + v * 8, a);
    if (RES) Vec8<T>::load(res + v * 8, r);
    unsigned bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = a[i] * scale[c0 + i] + shift[c0 + i];
      if (RES) t += RBN ? fmaf(r[i], rctx[2 * C + c0 + i], rctx[3 * C + c0 + i]) : r[i];
      bits |= (t > 0.f ? 1u : 0u) << i;
      a[i] = RELU ? fmaxf(t, 0.f) : t;
    }
    Vec8<T>::store(y + v * 8, a);
    if (RES && mask) mask[v] = (unsigned char)bits;
  }
}

// -------------------------------------------------------------------------------------------- backward
// RBN: the residual is the raw shortcut-conv output and its BN (rctx) was applied inside bn_apply: the same masked
// d also feeds that BN's backward, so its sums sum(d) (= db) and sum(d * xhat_r) (part_dg2) come from this pass too.
template <typename T, bool RELU, bool RES, bool RBN = false>
__global__ __launch_bounds__(256) void bn_bwd_partial(const T* __restrict__ x, const T* __restrict__ res,
                                                      const T* __restrict__ dy, long long M, int C,
                                                      long long rows_per_blk, const float* __restrict__ ctx,
                                                      float* __restrict__ part_db, float* __restrict__ part_dg,
                                                      const unsigned char* __restrict__ mask,
                                                      const float* __restrict__ rctx, float* __restrict__ part_dg2) {
  const int T8 = C >> 3;
  const int R = 256 / T8;
  const int cg = threadIdx.x % T8, r0 = threadIdx.x / T8;
  float db[8], dg[8], mu[8], is[8], sc[8], sf[8], dg2[8], mu2[8], is2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    db[i] = 0.f; dg[i] = 0.f; dg2[i] = 0.f;
    mu[i] = ctx[cg * 8 + i]; is[i] = ctx[C + cg * 8 + i];
    sc[i] = ctx[2 * C + cg * 8 + i]; sf[i] = ctx[3 * C + cg * 8 + i];
    mu2[i] = RBN ? rctx[cg * 8 + i] : 0.f;
    is2[i] = RBN ? rctx[C + cg * 8 + i] : 0.f;
  }
  const long long rbeg = (long long)blockIdx.x * rows_per_blk;
  long long rend = rbeg + rows_per_blk;
  if (rend > M) rend = M;
  if (r0 < R) {
    // U independent rows per batch; the next batch's loads are issued before the current batch is consumed, so a
    // thread keeps 2U rows of x / dy in flight across the whole loop (the previous form waited for every batch:
    // 1.4-2.7 TB/s on the ResNet-50 shapes)
    constexpr int U = 4;
    // loads stay packed until consumed (RawVec8): two batches in flight at ~half the registers of unpacked floats
    struct Batch { RawVec8<T> xv[U], gv[U], rv[RES ? U : 1]; unsigned mb[U]; };
    auto load = [&](long long r, Batch& b) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long ru = r + u * R;
        const long long rr = ru < rend ? ru : rbeg + r0;       // clamped: always a valid row of this block
        const long long o = rr * C + cg * 8;
        b.xv[u].load(x + o);
        b.gv[u].load(dy + o);
        if (RES) {
          if (mask) b.mb[u] = mask[rr * T8 + cg];
          if (!mask || RBN) b.rv[RES ? u : 0].load(res + o);
        }
      }
    };
    auto consume = [&](long long r, const Batch& b) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * R >= rend) continue;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xf = b.xv[u].get(i);
          float d = b.gv[u].get(i);
          if (RES && mask) {
            d = (b.mb[u] >> i) & 1u ? d : 0.f;
          } else if (RELU) {
            float t = xf * sc[i] + sf[i];
            if (RES) t += RBN ? fmaf(b.rv[RES ? u : 0].get(i), rctx[2 * C + cg * 8 + i], rctx[3 * C + cg * 8 + i])
                              : b.rv[RES ? u : 0].get(i);
            d = t > 0.f ? d : 0.f;
          }
          db[i] += d;
          dg[i] += d * (xf - mu[i]) * is[i];
          if (RBN) dg2[i] += d * (b.rv[RES ? u : 0].get(i) - mu2[i]) * is2[i];
        }
      }
    };
    long long r = rbeg + r0;
    Batch b0, b1;
    if (r < rend) load(r, b0);
    while (r < rend) {                                  // two batches per trip: b0 / b1 alternate, no copies
      const long long r1 = r + U * R;
      if (r1 < rend) load(r1, b1);
      consume(r, b0);
      if (r1 >= rend) break;
      const long long r2 = r1 + U * R;
      if (r2 < rend) load(r2, b0);
      consume(r1, b1);
      r = r2;
    }
  }
  __shared__ float red1[256 * 9];   // row pitch 9 floats: conflict-free 8-float stores
  __shared__ float red2[256 * 9];
  __shared__ float red3[RBN ? 256 * 9 : 1];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red1[threadIdx.x * 9 + i] = (r0 < R) ? db[i] : 0.f;
    red2[threadIdx.x * 9 + i] = (r0 < R) ? dg[i] : 0.f;
    if (RBN) red3[threadIdx.x * 9 + i] = (r0 < R) ? dg2[i] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f, e = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      a += red1[(rr * T8 + g) * 9 + k];
      b += red2[(rr * T8 + g) * 9 + k];
      if (RBN) e += red3[(rr * T8 + g) * 9 + k];
    }
    part_db[(long long)blockIdx.x * C + c] = a;
    part_dg[(long long)blockIdx.x * C + c] = b;
    if (RBN) part_dg2[(long long)blockIdx.x * C + c] = e;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_finalize(const float* __restrict__ part_db,
                                                       const float* __restrict__ part_dg, int nblk, int C, long long M,
                                                       float* __restrict__ dbeta, float* __restrict__ dgamma,
                                                       float* __restrict__ cdb, float* __restrict__ cdg) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  double a, b;
  reduce_partials(part_db, part_dg, nblk, C, c, a, b);
  if ((threadIdx.x >> 6) != 0 || c >= C) return;
  if (dbeta) dbeta[c] = (float)a;
  if (dgamma) dgamma[c] = (float)b;
  cdb[c] = (float)(a / (double)M);
  cdg[c] = (float)(b / (double)M);
}

// ------------------------------------------------------------------------ fused partial fold + finalize
// One launch replaces bn_reduce_rows + bn_finalize / bn_bwd_finalize: grid (ceil(C/64), S), each block folds 32
// partial rows of 64 channels (4 row groups x 8 independent loads, same order as bn_reduce_rows) into q; with S > 1
// the last block of each channel column (agent-scope ticket; the folded rows are stored write-through with agent-scope
// atomic stores and drained before the relaxed fetch_add, and the reducer reads them with agent-scope atomic loads —
// the guide's sc1 hand-off form, so no block pays a release fence, i.e. an L2 write-back of everything the previous
// kernel left dirty) sums the S folded rows in double and finalizes. The ticket counters live in a zero-initialised device array, each launch draws a slot
// round-robin on the host and the reducer resets its counter, so no per-call memset is needed.
// SRC 0: p1/p2 are [nrows, C] partial sums about row 0 (bn_stats_partial / bn_bwd_partial).
// SRC 1: p1 is the conv epilogue's [3][P][C] tile-statistics planes (bn_tiles_reduce's re-centring).
struct BnFin {
  long long M;
  const void* x;                           // fwd: row 0 = the statistics shift
  const float* gamma; const float* beta;
  float gconst, bconst;
  float* run_mean; float* run_var;
  float decay, eps;
  float* ctx;                              // fwd out: mean, invstd, scale, shift
  float* dbeta; float* dgamma;             // bwd outs (optional)
  float* cdb; float* cdg;                  // bwd out: mean(d), mean(d*xhat)
  unsigned* ticket;                        // ceil(C/64) counters (S > 1 only)
  int rpp;                                 // SRC 1: rows per tile partial
  int rpb;                                 // SRC 0: partial rows folded per block (multiple of 32; set by the launcher)
};

template <typename T, int FIN>
__device__ __forceinline__ void bn_fin_store(int c, int C, double a, double b, const BnFin& f) {
  if (FIN == 0) {
    const double m1 = a / (double)f.M;
    const float mean = (float)((double)ld1<T>((const T*)f.x + c) + m1);
    double v = b / (double)f.M - m1 * m1;
    if (v < 0) v = 0;
    const float var = (float)v + f.eps;
    f.run_mean[c] = f.decay * f.run_mean[c] + (1.f - f.decay) * mean;
    f.run_var[c] = f.decay * f.run_var[c] + (1.f - f.decay) * var;
    const float inv = rsqrtf(var);
    const float g = f.gamma ? f.gamma[c] : f.gconst;
    const float bb = f.beta ? f.beta[c] : f.bconst;
    f.ctx[c] = mean;
    f.ctx[C + c] = inv;
    f.ctx[2 * C + c] = g * inv;
    f.ctx[3 * C + c] = bb - mean * g * inv;
  } else {
    if (f.dbeta) f.dbeta[c] = (float)a;
    if (f.dgamma) f.dgamma[c] = (float)b;
    f.cdb[c] = (float)(a / (double)f.M);
    f.cdg[c] = (float)(b / (double)f.M);
  }
}

// Work split (float4 over channels): a block covers 64 channels (blockIdx.x) and f.rpb partial rows (blockIdx.y);
// lane q = tid & 15 owns channels 4q..4q+3 of the column, row group g = tid >> 4 takes rows g, g+16, ... of the
// block's range, 8 rows (SRC 1: 3 planes x 8 float4) in flight per trip. The 16 row groups are summed in a fixed order
// through LDS, the block's folded row goes out write-through (sc1 stores), and the last block of a column (ticket)
// reads all S folded rows with the same 16-group split, sums in double and finalizes. Every sum has a fixed order, so
// the result is bitwise reproducible. (The scalar-per-channel version read 4 bytes per lane per load and left the
// many-partial folds latency-bound: 12 us per launch for 6272 tile partials.)
template <typename T, int SRC, int FIN>
__global__ __launch_bounds__(256) void bn_fold(const float* __restrict__ p1, const float* __restrict__ p2,
                                               long long nrows, int C, float* __restrict__ q1,
                                               float* __restrict__ q2, BnFin f) {
  const int lq = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + 4 * lq;
  const bool cok = c < C;                                  // C % 4 == 0 (host-checked)
  float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
  const long long rbeg = (long long)blockIdx.y * f.rpb;
  const long long rend = rbeg + f.rpb < nrows ? rbeg + f.rpb : nrows;
  if (cok) {
    if (SRC == 0) {
      for (long long r0 = rbeg + rg; r0 < rend; r0 += 16 * 8) {
        float4 va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long long r = r0 + 16 * u;
          const bool ok = r < rend;
          va[u] = ok ? *reinterpret_cast<const float4*>(p1 + r * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
          vb[u] = ok ? *reinterpret_cast<const float4*>(p2 + r * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sa[0] += va[u].x; sa[1] += va[u].y; sa[2] += va[u].z; sa[3] += va[u].w;
          sb[0] += vb[u].x; sb[1] += vb[u].y; sb[2] += vb[u].z; sb[3] += vb[u].w;
        }
      }
    } else {
      // tile partials: s1 = sum(y - y0), s2 = sum((y - y0)^2) about the tile's own shift y0 (plane 3), re-centred
      // on the global shift x0 (row 0 of x); a tile holds f.rpp rows except the last
      float x0[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x0[j] = ld1<T>((const T*)f.x + c + j);
      const long long P = nrows;
      for (long long r0 = rbeg + rg; r0 < rend; r0 += 16 * 8) {
        float4 v1[8], v2[8], vd[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long long pp = r0 + 16 * u;
          const bool ok = pp < rend;
          v1[u] = ok ? *reinterpret_cast<const float4*>(p1 + pp * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
          v2[u] = ok ? *reinterpret_cast<const float4*>(p1 + (P + pp) * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
          vd[u] = ok ? *reinterpret_cast<const float4*>(p1 + (2 * P + pp) * C + c)
                     : make_float4(x0[0], x0[1], x0[2], x0[3]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long long pp = r0 + 16 * u;
          const long long nrow = pp < rend ? f.M - (long long)f.rpp * pp : 0;
          const float n = (float)(nrow < f.rpp ? (nrow < 0 ? 0 : nrow) : f.rpp);
          const float e1[4] = {v1[u].x, v1[u].y, v1[u].z, v1[u].w};
          const float e2[4] = {v2[u].x, v2[u].y, v2[u].z, v2[u].w};
          const float ed[4] = {vd[u].x, vd[u].y, vd[u].z, vd[u].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = ed[j] - x0[j];
            sa[j] += e1[j] + n * d;
            sb[j] += e2[j] + 2.f * d * e1[j] + n * d * d;
          }
        }
      }
    }
  }
  // fixed-order sum of the 16 row groups: LDS [2][16][64] floats
  __shared__ double rd[2][16 * 64];
  float* rf = reinterpret_cast<float*>(&rd[0][0]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rf[rg * 64 + 4 * lq + j] = sa[j];
    rf[1024 + rg * 64 + 4 * lq + j] = sb[j];
  }
  __syncthreads();
  const int ch = threadIdx.x & 63;                         // threads 0..63: one channel each
  const int cc = blockIdx.x * 64 + ch;
  float ta = 0.f, tb = 0.f;
  if (threadIdx.x < 64) {
#pragma unroll
    for (int g = 0; g < 16; ++g) { ta += rf[g * 64 + ch]; tb += rf[1024 + g * 64 + ch]; }
  }
  if (gridDim.y == 1) {
    if (threadIdx.x < 64 && cc < C) bn_fin_store<T, FIN>(cc, C, (double)ta, (double)tb, f);
    return;
  }
  typedef __attribute__((address_space(1))) unsigned gq32;
  if (threadIdx.x < 64 && cc < C) {
    __hip_atomic_store((gq32*)(q1 + (long long)blockIdx.y * C + cc), __float_as_uint(ta), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gq32*)(q2 + (long long)blockIdx.y * C + cc), __float_as_uint(tb), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                   // every wave's q stores drained; rf reads done
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add((gq32*)&f.ticket[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == gridDim.y - 1;
    if (last) {
      __hip_atomic_store((gq32*)&f.ticket[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // one acquire for the block, then PLAIN loads that can all be in flight together
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    rf[0] = last ? 1.f : 0.f;                        // "I am last" through the existing LDS array
  }
  __syncthreads();
  if (rf[0] == 0.f) return;
  __syncthreads();                                   // rf[0] read by every wave before the array is reused
  const int S = gridDim.y;
  double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
  if (cok) {
    for (int i0 = rg; i0 < S; i0 += 16 * 8) {
      float4 va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 16 * u;
        va[u] = i < S ? *reinterpret_cast<const float4*>(q1 + (long long)i * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        vb[u] = i < S ? *reinterpret_cast<const float4*>(q2 + (long long)i * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[0] += va[u].x; a[1] += va[u].y; a[2] += va[u].z; a[3] += va[u].w;
        b[0] += vb[u].x; b[1] += vb[u].y; b[2] += vb[u].z; b[3] += vb[u].w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rd[0][rg * 64 + 4 * lq + j] = a[j];
    rd[1][rg * 64 + 4 * lq + j] = b[j];
  }
  __syncthreads();
  if (threadIdx.x < 64 && cc < C) {
    double ra = 0.0, rb = 0.0;
#pragma unroll
    for (int g = 0; g < 16; ++g) { ra += rd[0][g * 64 + ch]; rb += rd[1][g * 64 + ch]; }
    bn_fin_store<T, FIN>(cc, C, ra, rb, f);
  }
}

// Ticket slots for bn_fold: 256 launches in flight x 32 channel columns (C <= 2048), one array per device.
__device__ unsigned g_bn_ticket[256 * 32];

static unsigned* bn_ticket_slot() {
  static unsigned* base[64] = {nullptr};
  static unsigned next = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_bn_ticket)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  const unsigned k = __atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED) % 256u;
  return base[dev] + 32 * k;
}

// DL4J_AMD_BN_FOLD=0: the previous separate launches (bn_reduce_rows + bn_finalize / bn_bwd_finalize) for A/B runs.
static bool bn_fold_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DL4J_AMD_BN_FOLD");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

static inline void bn_reduce_stage(float*& p1, float*& p2, int& nblk, int C, float* q, hipStream_t s);

// Launches bn_fold over `nrows` partial rows; q: >= 2*ceil(nrows/32)*C floats of workspace.
template <typename T, int SRC, int FIN>
static int bn_fold_launch(const float* p1, const float* p2, long long nrows, int C, float* q, BnFin f,
                          hipStream_t s) {
  if (SRC == 0 && !bn_fold_enabled() && nrows <= 0x7fffffff) {
    float* a = const_cast<float*>(p1);
    float* b = const_cast<float*>(p2);
    int n = (int)nrows;
    bn_reduce_stage(a, b, n, C, q, s);
    if (FIN == 0)
      hipLaunchKernelGGL(bn_finalize<T>, dim3((C + 63) / 64), dim3(256), 0, s, a, b, n, C, f.M, (const T*)f.x, f.gamma,
                         f.beta, f.gconst, f.bconst, f.run_mean, f.run_var, f.decay, f.eps, 1, f.ctx);
    else
      hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + 63) / 64), dim3(256), 0, s, a, b, n, C, f.M, f.dbeta, f.dgamma,
                         f.cdb, f.cdg);
    return 0;
  }
  // many partial rows (the conv epilogues' 64-row tile partials): 128 rows per block keeps the reducer's serial pass
  // short (stage-1 ResNet-50 tiles: 6272 partials -> 49 folded rows instead of 196)
  // (bn_bwd_partial's <= 2048 block rows fold faster 32 to a block: measured 0.56 vs 0.66 ms/step)
  // 128 rows per block (one trip of 8 rows x 16 row groups); more per block once that would exceed 1024 blocks
  // per channel column, so the last block's serial pass stays short
  if (C % 4 != 0) return -1;
  f.rpb = 128;
  while ((nrows + f.rpb - 1) / f.rpb > 1024) f.rpb *= 2;
  const long long S = (nrows + f.rpb - 1) / f.rpb;
  if (S > 65535) return -1;
  f.ticket = nullptr;
  if (S > 1) {
    f.ticket = bn_ticket_slot();
    if (!f.ticket) return -2;
  }
  hipLaunchKernelGGL((bn_fold<T, SRC, FIN>), dim3((C + 63) / 64, (unsigned)S), dim3(256), 0, s, p1, p2, nrows, C, q,
                     q + S * C, f);
  return 0;
}

// one dx/dres element: d = relu'(.)*dy; dx = gamma*invstd*(d - mean(d) - xhat*mean(d*xhat)) written as
// dx = A*d - B*x - Cq with per-channel A = scale (= gamma*invstd), B = scale*invstd*cdg, Cq = scale*(cdb - mean*invstd*cdg)
template <bool RELU, bool RES>
__device__ __forceinline__ void bn_bwd_elem(float& xv, float& gv, float& rv, float A, float B, float Cq, float sf,
                                            int mbit) {
  float d = gv;
  if (mbit >= 0) {
    d = mbit ? d : 0.f;
  } else if (RELU) {
    float t = xv * A + sf;
    if (RES) t += rv;
    d = t > 0.f ? d : 0.f;
  }
  if (RES) rv = d;
  xv = A * d - B * xv - Cq;
}

// RBN: dres receives the gradient w.r.t. the shortcut BN's INPUT (that BN's backward of the masked d, with its
// context rctx and its mean(d * xhat_r) cdg2; mean(d) is cdb, shared), so that layer needs no pass of its own.
template <typename T, bool RELU, bool RES, bool RBN = false>
__global__ __launch_bounds__(256) void bn_bwd_apply(const T* __restrict__ x, const T* __restrict__ res,
                                                    const T* __restrict__ dy, T* __restrict__ dx, T* __restrict__ dres,
                                                    long long M, int C, const float* __restrict__ ctx,
                                                    const float* __restrict__ cdb, const float* __restrict__ cdg,
                                                    const unsigned char* __restrict__ mask,
                                                    const float* __restrict__ rctx, const float* __restrict__ cdg2) {
  const bool use_mask = RES && mask != nullptr;
  const long long nvec = M * (C >> 3);
  const int T8 = C >> 3;
  const float *mean = ctx, *invstd = ctx + C, *scale = ctx + 2 * C, *shift = ctx + 3 * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long v0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool fixed = stride % T8 == 0;   // the thread's channel group never changes: factors in registers
  float A[8], B[8], Cq[8], sf[8], A2[8], B2[8], Cq2[8];
  auto factors = [&](int c0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = c0 + i;
      A[i] = scale[c];
      B[i] = scale[c] * invstd[c] * cdg[c];
      Cq[i] = scale[c] * (cdb[c] - mean[c] * invstd[c] * cdg[c]);
      sf[i] = shift[c];
      if (RBN) {
        const float s2 = rctx[2 * C + c], i2 = rctx[C + c];
        A2[i] = s2;
        B2[i] = s2 * i2 * cdg2[c];
        Cq2[i] = s2 * (cdb[c] - rctx[c] * i2 * cdg2[c]);
      }
    }
  };
  if (fixed) factors(idx_mod(v0, T8) * 8);
  long long v = v0;
  if (fixed) {
    // four independent vectors in flight, kept packed until used (RawVec8: half the registers of unpacked floats)
    constexpr int U = 4;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
      RawVec8<T> xr[U], gr[U], rr[RES ? U : 1];
      unsigned mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xr[u].load(x + (v + u * stride) * 8);
        gr[u].load(dy + (v + u * stride) * 8);
        mb[u] = 0u;
        if (use_mask) mb[u] = mask[v + u * stride];
        if (RES && (!use_mask || RBN)) rr[RES ? u : 0].load(res + (v + u * stride) * 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float xv[8], gv[8], rv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xv[i] = xr[u].get(i);
          gv[i] = gr[u].get(i);
          rv[i] = (RES && (!use_mask || RBN)) ? rr[RES ? u : 0].get(i) : 0.f;
          const float r_in = rv[i];
          if (RBN && !use_mask) rv[i] = fmaf(r_in, A2[i], rctx[3 * C + idx_mod(v + u * stride, T8) * 8 + i]);
          bn_bwd_elem<RELU, RES>(xv[i], gv[i], rv[i], A[i], B[i], Cq[i], sf[i],
                                 use_mask ? (int)((mb[u] >> i) & 1u) : -1);
          if (RBN) rv[i] = A2[i] * rv[i] - B2[i] * r_in - Cq2[i];
        }
        Vec8<T>::store(dx + (v + u * stride) * 8, xv);
        if (RES) Vec8<T>::store(dres + (v + u * stride) * 8, rv);
      }
    }
  }
  for (; v < nvec; v += stride) {
    if (!fixed) factors(idx_mod(v, T8) * 8);
    float xv[8], gv[8], rv[8];
    unsigned mb = 0u;
    Vec8<T>::load(x + v * 8, xv);
    Vec8<T>::load(dy + v * 8, gv);
    if (use_mask) mb = mask[v];
    if (RES && (!use_mask || RBN)) Vec8<T>::load(res + v * 8, rv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float r_in = rv[i];
      if (RBN && !use_mask) rv[i] = fmaf(r_in, A2[i], rctx[3 * C + idx_mod(v, T8) * 8 + i]);
      bn_bwd_elem<RELU, RES>(xv[i], gv[i], rv[i], A[i], B[i], Cq[i], sf[i], use_mask ? (int)((mb >> i) & 1u) : -1);
      if (RBN) rv[i] = A2[i] * rv[i] - B2[i] * r_in - Cq2[i];
    }
    Vec8<T>::store(dx + v * 8, xv);
    if (RES) Vec8<T>::store(dres + v * 8, rv);
  }
}

static inline void bn_grid(long long M, int C, int* nblk, long long* rows_per_blk) {
  const int T8 = C / 8;
  const long long work = M * T8;                  // vector loads
  long long nb = work / (256LL * 24);             // ~24 vector loads per thread, up to 4 blocks per CU
  if (nb < 1) nb = 1;
  if (nb > 2048) nb = 2048;
  long long rpb = (M + nb - 1) / nb;
  nb = (M + rpb - 1) / rpb;
  *nblk = (int)nb;
  *rows_per_blk = rpb;
}

// Backward partial-sum grid: ~32 rows-vectors of x and dy per thread, and at least 256 blocks spread evenly (a
// multiple of the 256 CUs once there is enough work, so no CU runs one block more than the others).
static inline void bn_bwd_grid(long long M, int C, int* nblk, long long* rows_per_blk) {
  const int T8 = C / 8;
  const long long work = M * T8;
  long long nb = work / (256LL * 32);
  if (nb >= 256) nb = (nb + 255) / 256 * 256;
  if (nb < 1) nb = 1;
  if (nb > 2048) nb = 2048;
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
  int nblk, nb2; long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  bn_bwd_grid(M, C, &nb2, &rpb);
  if (nb2 > nblk) nblk = nb2;
  return 2 * nblk * C + 2 * ((nblk + 31) / 32) * C + 8 * C;
}

// Two-stage partial reduction when there are many partial rows; returns the buffers/rows finalize should read.
static inline void bn_reduce_stage(float*& p1, float*& p2, int& nblk, int C, float* q, hipStream_t s) {
  if (nblk <= 64) return;
  const int S = (nblk + 31) / 32;
  float* q1 = q;
  float* q2 = q + (long long)S * C;
  hipLaunchKernelGGL(bn_reduce_rows, dim3((C + 63) / 64, S), dim3(256), 0, s, p1, p2, nblk, C, q1, q2);
  p1 = q1; p2 = q2; nblk = S;
}

#define BN_DISPATCH3(KERNEL, T, relu, res, ...)                                         \
  do {                                                                                  \
    if (res) hipLaunchKernelGGL((KERNEL<T, true, true>), __VA_ARGS__);                 \
    else if (relu) hipLaunchKernelGGL((KERNEL<T, true, false>), __VA_ARGS__);          \
    else hipLaunchKernelGGL((KERNEL<T, false, false>), __VA_ARGS__);                   \
  } while (0)

// dtype: 0 fp32, 1 bf16, 2 fp16. ws: >= dl4j_bn_workspace_floats floats. ctx_out: 4*C floats (mean, invstd,
// scale, shift). res: optional residual (same layout as x) -> y = relu(bn(x) + res) (relu forced on).
template <typename T>
static int bn_fwd_impl(const T* x, const T* res, T* y, long long M, int C, const float* gamma, const float* beta,
                       float gconst, float bconst, float* run_mean, float* run_var, float decay, float eps,
                       int training, int relu, float* ws, float* ctx_out, unsigned char* mask, hipStream_t s,
                       const float* rctx = nullptr) {
  int nblk; long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* q = p2 + (long long)nblk * C;
  if (training) {
    hipLaunchKernelGGL(bn_stats_partial<T>, dim3(nblk), dim3(256), 0, s, x, M, C, rpb, p1, p2);
    BnFin f{M, x, gamma, beta, gconst, bconst, run_mean, run_var, decay, eps, ctx_out,
            nullptr, nullptr, nullptr, nullptr, nullptr, 0};
    const int rc = bn_fold_launch<T, 0, 0>(p1, p2, nblk, C, q, f, s);
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(bn_finalize<T>, dim3((C + 63) / 64), dim3(256), 0, s, p1, p2, nblk, C, M, x, gamma, beta,
                       gconst, bconst, run_mean, run_var, decay, eps, training, ctx_out);
  }
  if (!y) return (int)hipGetLastError();              // statistics only (a shortcut BN folded into its consumer)
  if (rctx && res)
    hipLaunchKernelGGL((bn_apply<T, true, true, true>), dim3(apply_grid(M, C)), dim3(256), 0, s, x, res, y, M, C,
                       ctx_out, mask, rctx);
  else
    BN_DISPATCH3(bn_apply, T, relu, res, dim3(apply_grid(M, C)), dim3(256), 0, s, x, res, y, M, C, ctx_out, mask,
                 (const float*)nullptr);
  return (int)hipGetLastError();
}

// mask: optional (res != nullptr only) M*C/8-byte ReLU bitmask for dl4j_bn_bwd (bn_apply).
DL4J_API int dl4j_bn_fwd(int dtype, const void* x, const void* res, void* y, long long M, int C, const float* gamma,
                         const float* beta, float gconst, float bconst, float* run_mean, float* run_var, float decay,
                         float eps, int training, int relu, float* ws, float* ctx_out, unsigned char* mask,
                         hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256) return -1;
  if (res) relu = 1;
  else mask = nullptr;
#define BNF(T) return bn_fwd_impl<T>((const T*)x, (const T*)res, (T*)y, M, C, gamma, beta, gconst, bconst, run_mean, \
                                     run_var, decay, eps, training, relu, ws, ctx_out, mask, s)
  if (dtype == 1) BNF(bf16);
  if (dtype == 2) BNF(f16);
  BNF(float);
#undef BNF
}

// Training forward with the statistics already reduced per tile by the producing conv kernel (tstats, P partials):
// skips bn_stats_partial's full read of x. ws: >= dl4j_bn_tiles_workspace_floats(P, C) floats.
DL4J_API long long dl4j_bn_tiles_workspace_floats(long long P, int C) {
  const long long S = (P + 31) / 32;
  return 2 * S * C + 2 * ((S + 31) / 32) * C + 8LL * C;
}

template <typename T>
static int bn_fwd_tiles_impl(const T* xb, const T* res, T* y, long long M, int C, const float* tstats, long long P,
                             int rpp, const float* gamma, const float* beta, float gconst, float bconst,
                             float* run_mean, float* run_var, float decay, float eps, int relu, float* ws,
                             float* ctx_out, unsigned char* mask, hipStream_t s, const float* rctx = nullptr) {
  const long long S = (P + 31) / 32;
  BnFin f{M, xb, gamma, beta, gconst, bconst, run_mean, run_var, decay, eps, ctx_out,
          nullptr, nullptr, nullptr, nullptr, nullptr, rpp};
  int rc;
  if (bn_fold_enabled()) {
    // one launch: tile re-centring + fold + finalize
    rc = bn_fold_launch<T, 1, 0>(tstats, nullptr, P, C, ws, f, s);
  } else {
    float* p1 = ws;
    float* p2 = ws + S * C;
    hipLaunchKernelGGL(bn_tiles_reduce<T>, dim3((C + 63) / 64, (unsigned)S), dim3(256), 0, s, tstats, P, C, M, xb, p1,
                       p2, rpp);
    rc = bn_fold_launch<T, 0, 0>(p1, p2, S, C, p2 + S * C, f, s);
  }
  if (rc) return rc;
  if (!y) return (int)hipGetLastError();              // statistics only (a shortcut BN folded into its consumer)
  if (rctx && res)
    hipLaunchKernelGGL((bn_apply<T, true, true, true>), dim3(apply_grid(M, C)), dim3(256), 0, s, xb, res, y, M, C,
                       ctx_out, mask, rctx);
  else
    BN_DISPATCH3(bn_apply, T, relu, res, dim3(apply_grid(M, C)), dim3(256), 0, s, xb, res, y, M, C, ctx_out,
                 mask, (const float*)nullptr);
  return (int)hipGetLastError();
}

// rpp: rows per partial (64 for the implicit-GEMM / GEMM epilogues, the chunk's pixel count for dl4j_conv_halo);
// partial p covers rows [rpp*p, rpp*p + rpp).
DL4J_API int dl4j_bn_fwd_tiles(int dtype, const void* x, const void* res, void* y, long long M, int C,
                               const float* tstats, long long P, int rpp, const float* gamma, const float* beta,
                               float gconst, float bconst, float* run_mean, float* run_var, float decay, float eps,
                               int relu, float* ws, float* ctx_out, unsigned char* mask, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || (dtype != 1 && dtype != 2) || P < 1 || rpp < 1 || P * (long long)rpp < M)
    return -1;
  if (res) relu = 1;
  else mask = nullptr;
  if (dtype == 2)
    return bn_fwd_tiles_impl<f16>((const f16*)x, (const f16*)res, (f16*)y, M, C, tstats, P, rpp, gamma, beta, gconst,
                                  bconst, run_mean, run_var, decay, eps, relu, ws, ctx_out, mask, s);
  return bn_fwd_tiles_impl<bf16>((const bf16*)x, (const bf16*)res, (bf16*)y, M, C, tstats, P, rpp, gamma, beta,
                                 gconst, bconst, run_mean, run_var, decay, eps, relu, ws, ctx_out, mask, s);
}

// dres: gradient w.r.t. the fused residual input (required when res != nullptr).
template <typename T>
static int bn_bwd_impl(const T* x, const T* res, const T* dy, T* dx, T* dres, long long M, int C, const float* ctx,
                       float* dgamma, float* dbeta, int relu, float* ws, const unsigned char* mask, hipStream_t s) {
  int nblk; long long rpb;
  bn_bwd_grid(M, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* q = p2 + (long long)nblk * C;
  float* cdb = q + 2LL * ((nblk + 31) / 32) * C;
  float* cdg = cdb + C;
  BN_DISPATCH3(bn_bwd_partial, T, relu, res, dim3(nblk), dim3(256), 0, s, x, res, dy, M, C, rpb, ctx, p1, p2, mask,
               (const float*)nullptr, (float*)nullptr);
  BnFin f{M, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, 0.f, 0.f, nullptr, dbeta, dgamma, cdb, cdg,
          nullptr, 0};
  const int rc = bn_fold_launch<T, 0, 1>(p1, p2, nblk, C, q, f, s);
  if (rc) return rc;
  BN_DISPATCH3(bn_bwd_apply, T, relu, res, dim3(apply_grid(M, C)), dim3(256), 0, s, x, res, dy, dx, dres, M, C, ctx,
               cdb, cdg, mask, (const float*)nullptr, (const float*)nullptr);
  return (int)hipGetLastError();
}

// Residual layer whose shortcut BN is folded in (RBN): one partial pass gives both layers' sums, two folds, one apply
// writing dx and the gradient w.r.t. the shortcut BN's input (dres). Workspace: dl4j_bn_bwd_rbn_workspace_floats.
DL4J_API long long dl4j_bn_bwd_rbn_workspace_floats(long long M, int C) {
  int nblk; long long rpb;
  bn_bwd_grid(M, C, &nblk, &rpb);
  return 3LL * nblk * C + 4LL * ((nblk + 31) / 32) * C + 4LL * C;
}

template <typename T>
static int bn_bwd_rbn_impl(const T* x, const T* res, const T* dy, T* dx, T* dres, long long M, int C, const float* ctx,
                           float* dgamma, float* dbeta, const float* rctx, float* dgamma2, float* dbeta2, float* ws,
                           const unsigned char* mask, hipStream_t s) {
  int nblk; long long rpb;
  bn_bwd_grid(M, C, &nblk, &rpb);
  const long long S = (nblk + 31) / 32;
  float* p1 = ws;
  float* p2 = p1 + (long long)nblk * C;
  float* p3 = p2 + (long long)nblk * C;
  float* q = p3 + (long long)nblk * C;
  float* q2 = q + 2 * S * C;
  float* cdb = q2 + 2 * S * C;
  float* cdg = cdb + C;
  float* cdb2 = cdg + C;
  float* cdg2 = cdb2 + C;
  hipLaunchKernelGGL((bn_bwd_partial<T, true, true, true>), dim3(nblk), dim3(256), 0, s, x, res, dy, M, C, rpb, ctx, p1,
                     p2, mask, rctx, p3);
  BnFin f{M, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, 0.f, 0.f, nullptr, dbeta, dgamma, cdb, cdg,
          nullptr, 0};
  int rc = bn_fold_launch<T, 0, 1>(p1, p2, nblk, C, q, f, s);
  if (rc) return rc;
  BnFin f2{M, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, 0.f, 0.f, nullptr, dbeta2, dgamma2, cdb2, cdg2,
           nullptr, 0};
  rc = bn_fold_launch<T, 0, 1>(p1, p3, nblk, C, q2, f2, s);
  if (rc) return rc;
  hipLaunchKernelGGL((bn_bwd_apply<T, true, true, true>), dim3(apply_grid(M, C)), dim3(256), 0, s, x, res, dy, dx, dres,
                     M, C, ctx, cdb, cdg, mask, rctx, cdg2);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bn_bwd_rbn(int dtype, const void* x, const void* res, const void* dy, void* dx, void* dres,
                             long long M, int C, const float* ctx, float* dgamma, float* dbeta, const float* rctx,
                             float* dgamma2, float* dbeta2, float* ws, const unsigned char* mask, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || !res || !dres || !rctx || (dtype != 1 && dtype != 2)) return -1;
  if (dtype == 2)
    return bn_bwd_rbn_impl<f16>((const f16*)x, (const f16*)res, (const f16*)dy, (f16*)dx, (f16*)dres, M, C, ctx, dgamma,
                                dbeta, rctx, dgamma2, dbeta2, ws, mask, s);
  return bn_bwd_rbn_impl<bf16>((const bf16*)x, (const bf16*)res, (const bf16*)dy, (bf16*)dx, (bf16*)dres, M, C, ctx,
                               dgamma, dbeta, rctx, dgamma2, dbeta2, ws, mask, s);
}

// Residual forward with the shortcut BN folded in: y = relu(bn(x) + bn_r(res)), rctx the shortcut BN's finalized
// context (its statistics-only forward). tstats / P: the producing conv's tile statistics (or null: full pass).
DL4J_API int dl4j_bn_fwd_rbn(int dtype, const void* x, const void* res, const float* rctx, void* y, long long M, int C,
                             const float* gamma, const float* beta, float gconst, float bconst, float* run_mean,
                             float* run_var, float decay, float eps, float* ws, float* ctx_out, unsigned char* mask,
                             const float* tstats, long long P, int rpp, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || !res || !rctx || !y || (dtype != 1 && dtype != 2)) return -1;
  if (tstats) {
    if (rpp < 1) return -1;
    if (dtype == 2)
      return bn_fwd_tiles_impl<f16>((const f16*)x, (const f16*)res, (f16*)y, M, C, tstats, P, rpp, gamma, beta,
                                    gconst, bconst, run_mean, run_var, decay, eps, 1, ws, ctx_out, mask, s, rctx);
    return bn_fwd_tiles_impl<bf16>((const bf16*)x, (const bf16*)res, (bf16*)y, M, C, tstats, P, rpp, gamma, beta,
                                   gconst, bconst, run_mean, run_var, decay, eps, 1, ws, ctx_out, mask, s, rctx);
  }
  if (dtype == 2)
    return bn_fwd_impl<f16>((const f16*)x, (const f16*)res, (f16*)y, M, C, gamma, beta, gconst, bconst, run_mean,
                            run_var, decay, eps, 1, 1, ws, ctx_out, mask, s, rctx);
  return bn_fwd_impl<bf16>((const bf16*)x, (const bf16*)res, (bf16*)y, M, C, gamma, beta, gconst, bconst, run_mean,
                           run_var, decay, eps, 1, 1, ws, ctx_out, mask, s, rctx);
}

DL4J_API int dl4j_bn_bwd(int dtype, const void* x, const void* res, const void* dy, void* dx, void* dres, long long M,
                         int C, const float* ctx, float* dgamma, float* dbeta, int relu, float* ws,
                         const unsigned char* mask, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256) return -1;
  if (res) relu = 1;
  else mask = nullptr;
#define BNB(T) return bn_bwd_impl<T>((const T*)x, (const T*)res, (const T*)dy, (T*)dx, (T*)dres, M, C, ctx, dgamma, \
                                     dbeta, relu, ws, mask, s)
  if (dtype == 1) BNB(bf16);
  if (dtype == 2) BNB(f16);
  BNB(float);
#undef BNB
}

// Backward with the partial sums already produced by the epilogue of the kernel that wrote dy (csrc/mfma_tile.h
// epi_bnbwd_wave, armed by dl4j_bnb_arm): planes [2][P][C] of sum(d), sum(d*xhat) per 64-row partial. One fold +
// finalize launch and the apply pass; bn_bwd_partial's full read of x and dy is gone. With a fused residual (res
// flag) the ReLU comes from the forward's bitmask and dres (the masked dy) is written as in dl4j_bn_bwd.
DL4J_API long long dl4j_bn_bwd_planes_workspace_floats(long long P, int C) {
  return 2 * ((P + 31) / 32) * (long long)C + 4LL * C;
}

template <typename T>
static int bn_bwd_planes_impl(const T* x, const T* dy, T* dx, T* dres, const unsigned char* mask, long long M, int C,
                              const float* ctx, float* dgamma, float* dbeta, int relu, const float* planes,
                              long long P, float* ws, hipStream_t s) {
  float* q = ws;
  float* cdb = q + 2 * ((P + 31) / 32) * (long long)C;
  float* cdg = cdb + C;
  BnFin f{M, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, 0.f, 0.f, nullptr, dbeta, dgamma, cdb, cdg,
          nullptr, 0};
  const int rc = bn_fold_launch<T, 0, 1>(planes, planes + P * C, P, C, q, f, s);
  if (rc) return rc;
  if (dres)
    hipLaunchKernelGGL((bn_bwd_apply<T, true, true>), dim3(apply_grid(M, C)), dim3(256), 0, s, x, nullptr, dy, dx,
                       dres, M, C, ctx, cdb, cdg, mask, nullptr, nullptr);
  else if (relu)
    hipLaunchKernelGGL((bn_bwd_apply<T, true, false>), dim3(apply_grid(M, C)), dim3(256), 0, s, x, nullptr, dy, dx,
                       nullptr, M, C, ctx, cdb, cdg, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_apply<T, false, false>), dim3(apply_grid(M, C)), dim3(256), 0, s, x, nullptr, dy, dx,
                       nullptr, M, C, ctx, cdb, cdg, nullptr, nullptr, nullptr);
  return (int)hipGetLastError();
}

// dres / mask: both or neither (residual BN layers: dres = the masked dy, ReLU from the forward's bitmask).
DL4J_API int dl4j_bn_bwd_planes(int dtype, const void* x, const void* dy, void* dx, void* dres,
                                const unsigned char* mask, long long M, int C, const float* ctx, float* dgamma,
                                float* dbeta, int relu, const float* planes, long long P, float* ws, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || P < 1 || P != (M + 63) / 64 || ((dres == nullptr) != (mask == nullptr))) return -1;
  if (dtype == 1)
    return bn_bwd_planes_impl<bf16>((const bf16*)x, (const bf16*)dy, (bf16*)dx, (bf16*)dres, mask, M, C, ctx, dgamma,
                                    dbeta, relu, planes, P, ws, s);
  if (dtype == 2)
    return bn_bwd_planes_impl<f16>((const f16*)x, (const f16*)dy, (f16*)dx, (f16*)dres, mask, M, C, ctx, dgamma,
                                   dbeta, relu, planes, P, ws, s);
  return -1;
}

// -------------------------------------------------------------------------------------------- BN + ReLU + max pool
// Fused stem tail (ResNet: conv7x7 -> BN -> ReLU -> maxpool 3x3/2). The BN output is never materialised:
//   forward  : pooled = max over the window of relu(x*scale + shift); per pooled element also stores the window
//              argmax byte (index | 0x80 when the max is > 0, i.e. the ReLU is active there) and x_hat at the
//              argmax (bf16/fp32 like x).
//   backward : (1) dbeta = sum(dy_p * active), dgamma = sum(dy_p * active * x_hat_p) over the POOLED tensor only:
//              every input position receives the pooled gradients routed to it, and the routing is linear, so the
//              BN reductions over the full-resolution gradient equal these sums over the pooled one;
//              (2) one gather pass over x: g = sum of the active pooled gradients whose argmax is this position,
//              dx = scale * (g - dbeta/M - x_hat * dgamma/M).
// Replaces bn_apply + pool_fwd (fwd) and pool_bwd + bn_bwd_partial + bn_bwd_apply (bwd): ~2.6 fewer full-size
// passes over the conv output.
template <typename T>
__global__ __launch_bounds__(256) void bnpool_fwd(const T* __restrict__ x, T* __restrict__ y,
                                                  unsigned char* __restrict__ am, T* __restrict__ xh,
                                                  const float* __restrict__ ctx, int N, int H, int W, int C, int OH,
                                                  int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * OH * OW * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int cg, ow, oh, n;
    idx_decomp4(t, CG, OW, OH, cg, ow, oh, n);
    float sc[8], sf[8], best[8], bx[8];
    unsigned char idx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = ctx[2 * C + cg * 8 + i];
      sf[i] = ctx[3 * C + cg * 8 + i];
      best[i] = -INFINITY;
      bx[i] = 0.f;
      idx[i] = 0;
    }
    for (int i = 0; i < kh; ++i) {
      const int ih = oh * sh - pt + i;
      if (ih < 0 || ih >= H) continue;
      for (int j = 0; j < kw; ++j) {
        const int iw = ow * sw - pl + j;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        Vec8<T>::load(x + (((long long)n * H + ih) * W + iw) * C + cg * 8, v);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float a = fmaxf(v[c] * sc[c] + sf[c], 0.f);
          if (a > best[c]) {                               // first maximum wins, as in pool_fwd
            best[c] = a;
            bx[c] = v[c];
            idx[c] = (unsigned char)(i * kw + j);
          }
        }
      }
    }
    Vec8<T>::store(y + t * 8, best);
    if (am) {
      unsigned long long pk = 0;
#pragma unroll
      for (int c = 0; c < 8; ++c)
        pk |= ((unsigned long long)(idx[c] | (best[c] > 0.f ? 0x80 : 0))) << (8 * c);
      *reinterpret_cast<unsigned long long*>(am + t * 8) = pk;
    }
    if (xh) {
#pragma unroll
      for (int c = 0; c < 8; ++c) bx[c] = (bx[c] - ctx[cg * 8 + c]) * ctx[C + cg * 8 + c];
      Vec8<T>::store(xh + t * 8, bx);
    }
  }
}

// Same as bnpool_fwd for a compile-time window: every window load is issued before any is consumed (clamped
// addresses + validity flags), so a wave keeps KH*KW 16-byte loads in flight instead of one.
template <typename T, int KH, int KW>
__global__ __launch_bounds__(256) void bnpool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                    unsigned char* __restrict__ am, T* __restrict__ xh,
                                                    const float* __restrict__ ctx, int N, int H, int W, int C, int OH,
                                                    int OW, int sh, int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * OH * OW * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int cg, ow, oh, n;
    idx_decomp4(t, CG, OW, OH, cg, ow, oh, n);
    float v[KH * KW][8];
    bool ok[KH * KW];
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
      for (int j = 0; j < KW; ++j) {
        const int ih = oh * sh - pt + i, iw = ow * sw - pl + j;
        ok[i * KW + j] = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
        Vec8<T>::load(x + (((long long)n * H + ihc) * W + iwc) * C + cg * 8, v[i * KW + j]);
      }
    float sc[8], sf[8], best[8], bx[8];
    unsigned char idx[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      sc[c] = ctx[2 * C + cg * 8 + c];
      sf[c] = ctx[3 * C + cg * 8 + c];
      best[c] = -INFINITY;
      bx[c] = 0.f;
      idx[c] = 0;
    }
#pragma unroll
    for (int q = 0; q < KH * KW; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float a = fmaxf(v[q][c] * sc[c] + sf[c], 0.f);
        if (a > best[c]) {
          best[c] = a;
          bx[c] = v[q][c];
          idx[c] = (unsigned char)q;
        }
      }
    }
    Vec8<T>::store(y + t * 8, best);
    if (am) {
      unsigned long long pk = 0;
#pragma unroll
      for (int c = 0; c < 8; ++c)
        pk |= ((unsigned long long)(idx[c] | (best[c] > 0.f ? 0x80 : 0))) << (8 * c);
      *reinterpret_cast<unsigned long long*>(am + t * 8) = pk;
    }
    if (xh) {
#pragma unroll
      for (int c = 0; c < 8; ++c) bx[c] = (bx[c] - ctx[cg * 8 + c]) * ctx[C + cg * 8 + c];
      Vec8<T>::store(xh + t * 8, bx);
    }
  }
}

// bnpool_bwd_dx when at most 2 windows per dimension contain an input position (kh <= 2*sh, kw <= 2*sw, e.g.
// 3x3/2): the 4 candidate windows' gradient and argmax loads are issued together with the x load.
template <typename T>
__global__ __launch_bounds__(256) void bnpool_bwd_dx2(const T* __restrict__ x, const T* __restrict__ dy,
                                                      const unsigned char* __restrict__ am, T* __restrict__ dx,
                                                      const float* __restrict__ ctx, const float* __restrict__ cdb,
                                                      const float* __restrict__ cdg, int N, int H, int W, int C,
                                                      int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * H * W * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int cg, iw, ih, n;
    idx_decomp4(t, CG, W, H, cg, iw, ih, n);
    const int hp = ih + pt, wp = iw + pl;
    int oh0 = hp - kh + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + sh - 1) / sh;
    int ow0 = wp - kw + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + sw - 1) / sw;
    const int oh1 = min(hp / sh, OH - 1), ow1 = min(wp / sw, OW - 1);
    float g[4][8], xv[8];
    unsigned long long pk[4];
    unsigned me[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = oh0 + a, ow = ow0 + b, q = a * 2 + b;
        const bool ok = oh <= oh1 && ow <= ow1;
        const long long o = (((long long)n * OH + min(oh, OH - 1)) * OW + min(ow, OW - 1)) * C + cg * 8;
        Vec8<T>::load(dy + o, g[q]);
        pk[q] = *reinterpret_cast<const unsigned long long*>(am + o);
        me[q] = ok ? (0x80u | (unsigned)((hp - oh * sh) * kw + (wp - ow * sw))) : 0x100u;   // 0x100: never matches
      }
    Vec8<T>::load(x + t * 8, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (((pk[q] >> (8 * i)) & 0xff) == me[q]) acc += g[q][i];
      const int c = cg * 8 + i;
      const float xhat = (xv[i] - ctx[c]) * ctx[C + c];
      xv[i] = ctx[2 * C + c] * (acc - cdb[c] - xhat * cdg[c]);
    }
    Vec8<T>::store(dx + t * 8, xv);
  }
}

// bnpool_bwd_dx2 with the pooled gradient and argmax rows STAGED IN LDS: a workgroup owns 2 input rows of one
// image, copies the (<= 3) pooled rows whose windows cover them once (coalesced 8/16-byte copies), then gathers
// the candidate windows from LDS. Cuts the L2->CU traffic of the 4-candidate gather (~4x the pooled tensor) to
// ~1.5x, leaving the kernel bound by its x read + dx write.
template <typename T>
__global__ __launch_bounds__(256) void bnpool_bwd_dx_lds(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const unsigned char* __restrict__ am, T* __restrict__ dx,
                                                         const float* __restrict__ ctx, const float* __restrict__ cdb,
                                                         const float* __restrict__ cdg, int N, int H, int W, int C,
                                                         int OH, int OW, int kh, int kw, int sh, int sw, int pt,
                                                         int pl, int maxrows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int CG = C >> 3, RB = 2;
  const int rows_per_img = (H + RB - 1) / RB;
  const int n = blockIdx.x / rows_per_img, ih0 = (blockIdx.x - n * rows_per_img) * RB;
  int oh_lo = ih0 + pt - kh + 1;
  oh_lo = oh_lo <= 0 ? 0 : (oh_lo + sh - 1) / sh;
  const int oh_hi = min((min(ih0 + RB, H) - 1 + pt) / sh, OH - 1);
  const int nrows = oh_hi - oh_lo + 1;                     // <= maxrows (host-checked)
  T* sdy = reinterpret_cast<T*>(smem);                                        // [maxrows][OW*C]
  unsigned char* sam = smem + (size_t)maxrows * OW * C * sizeof(T);           // [maxrows][OW*C]
  const int row_elems = OW * C;
  if (nrows > 0) {
    const long long g0 = ((long long)n * OH + oh_lo) * row_elems;
    const int nv = nrows * row_elems / 8;                  // 8-element vectors
    for (int i = threadIdx.x; i < nv; i += 256) {
      if (sizeof(T) == 2)
        reinterpret_cast<uint4*>(sdy)[i] = reinterpret_cast<const uint4*>(dy + g0)[i];
      else {
        reinterpret_cast<uint4*>(sdy)[2 * i] = reinterpret_cast<const uint4*>(dy + g0)[2 * i];
        reinterpret_cast<uint4*>(sdy)[2 * i + 1] = reinterpret_cast<const uint4*>(dy + g0)[2 * i + 1];
      }
      reinterpret_cast<uint2*>(sam)[i] = reinterpret_cast<const uint2*>(am + g0)[i];
    }
  }
  __syncthreads();
  const int items = min(RB, H - ih0) * W * CG;
  // a thread keeps one channel group across its items when CG divides the block size: BN factors in registers
  // (dx = A*acc - B*x - Cq, see bn_bwd_elem) instead of 40 L1 parameter loads per 8-channel item
  const bool fixed = (256 % CG) == 0;
  float A[8], B[8], Cq[8];
  if (fixed) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = (threadIdx.x % CG) * 8 + i;
      A[i] = ctx[2 * C + c];
      B[i] = ctx[2 * C + c] * ctx[C + c] * cdg[c];
      Cq[i] = ctx[2 * C + c] * (cdb[c] - ctx[c] * ctx[C + c] * cdg[c]);
    }
  }
  for (int it = threadIdx.x; it < items; it += 256) {
    const int cg = it % CG, q1 = it / CG, iw = q1 % W, ih = ih0 + q1 / W;
    const int hp = ih + pt, wp = iw + pl;
    int oh0 = hp - kh + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + sh - 1) / sh;
    int ow0 = wp - kw + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + sw - 1) / sw;
    const int oh1 = min(hp / sh, OH - 1), ow1 = min(wp / sw, OW - 1);
    const long long t = (((long long)n * H + ih) * W + iw) * CG + cg;
    float xv[8], acc[8];
    Vec8<T>::load(x + t * 8, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = oh0 + a, ow = ow0 + b;
        if (oh > oh1 || ow > ow1) continue;
        const int o = ((oh - oh_lo) * OW + ow) * C + cg * 8;
        float g[8];
        Vec8<T>::load(sdy + o, g);
        const unsigned long long pk = *reinterpret_cast<const unsigned long long*>(sam + o);
        const unsigned me = 0x80u | (unsigned)((hp - oh * sh) * kw + (wp - ow * sw));
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (((pk >> (8 * i)) & 0xff) == me) acc[i] += g[i];
      }
    if (fixed) {
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = A[i] * acc[i] - B[i] * xv[i] - Cq[i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = cg * 8 + i;
        const float xhat = (xv[i] - ctx[c]) * ctx[C + c];
        xv[i] = ctx[2 * C + c] * (acc[i] - cdb[c] - xhat * cdg[c]);
      }
    }
    Vec8<T>::store(dx + t * 8, xv);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bnpool_bwd_partial(const T* __restrict__ dy, const unsigned char* __restrict__ am,
                                                          const T* __restrict__ xh, long long M, int C,
                                                          long long rows_per_blk, float* __restrict__ part_db,
                                                          float* __restrict__ part_dg) {
  const int T8 = C >> 3;
  const int R = 256 / T8;
  const int cg = threadIdx.x % T8, r0 = threadIdx.x / T8;
  float db[8], dg[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    db[i] = 0.f;
    dg[i] = 0.f;
  }
  const long long rbeg = (long long)blockIdx.x * rows_per_blk;
  long long rend = rbeg + rows_per_blk;
  if (rend > M) rend = M;
  if (r0 < R) {
    for (long long r = rbeg + r0; r < rend; r += R) {
      const long long o = r * C + cg * 8;
      float gv[8], hv[8];
      Vec8<T>::load(dy + o, gv);
      Vec8<T>::load(xh + o, hv);
      const unsigned long long pk = *reinterpret_cast<const unsigned long long*>(am + o);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = ((pk >> (8 * i)) & 0x80) ? gv[i] : 0.f;
        db[i] += d;
        dg[i] += d * hv[i];
      }
    }
  }
  __shared__ float red1[256 * 9];   // row pitch 9 floats: conflict-free 8-float stores
  __shared__ float red2[256 * 9];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red1[threadIdx.x * 9 + i] = (r0 < R) ? db[i] : 0.f;
    red2[threadIdx.x * 9 + i] = (r0 < R) ? dg[i] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c >> 3, k = c & 7;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      a += red1[(rr * T8 + g) * 9 + k];
      b += red2[(rr * T8 + g) * 9 + k];
    }
    part_db[(long long)blockIdx.x * C + c] = a;
    part_dg[(long long)blockIdx.x * C + c] = b;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bnpool_bwd_dx(const T* __restrict__ x, const T* __restrict__ dy,
                                                     const unsigned char* __restrict__ am, T* __restrict__ dx,
                                                     const float* __restrict__ ctx, const float* __restrict__ cdb,
                                                     const float* __restrict__ cdg, int N, int H, int W, int C, int OH,
                                                     int OW, int kh, int kw, int sh, int sw, int pt, int pl) {
  const int CG = C >> 3;
  const long long total = (long long)N * H * W * CG;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int cg, iw, ih, n;
    idx_decomp4(t, CG, W, H, cg, iw, ih, n);
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    const int hp = ih + pt, wp = iw + pl;
    int oh0 = hp - kh + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + sh - 1) / sh;
    int ow0 = wp - kw + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + sw - 1) / sw;
    const int oh1 = min(hp / sh, OH - 1), ow1 = min(wp / sw, OW - 1);
    for (int oh = oh0; oh <= oh1; ++oh) {
      for (int ow = ow0; ow <= ow1; ++ow) {
        const long long o = (((long long)n * OH + oh) * OW + ow) * C + cg * 8;
        float g[8];
        Vec8<T>::load(dy + o, g);
        const unsigned long long pk = *reinterpret_cast<const unsigned long long*>(am + o);
        const unsigned me = 0x80u | (unsigned)((hp - oh * sh) * kw + (wp - ow * sw));
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (((pk >> (8 * c)) & 0xff) == me) acc[c] += g[c];
      }
    }
    float xv[8];
    Vec8<T>::load(x + t * 8, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cg * 8 + i;
      const float xhat = (xv[i] - ctx[c]) * ctx[C + c];
      xv[i] = ctx[2 * C + c] * (acc[i] - cdb[c] - xhat * cdg[c]);
    }
    Vec8<T>::store(dx + t * 8, xv);
  }
}

static inline int ew_grid(long long total) {
  long long g = (total + 255) / 256;
  if (g > 256 * 32) g = 256 * 32;
  return (int)(g < 1 ? 1 : g);
}

template <typename T>
static void bnpool_fwd_launch(const T* x, T* y, unsigned char* am, T* xh, const float* ctx, int N, int H, int W, int C,
                              int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl, int pg, hipStream_t s) {
  if (kh == 3 && kw == 3)
    hipLaunchKernelGGL((bnpool_fwd_k<T, 3, 3>), dim3(pg), dim3(256), 0, s, x, y, am, xh, ctx, N, H, W, C, OH, OW, sh,
                       sw, pt, pl);
  else if (kh == 2 && kw == 2)
    hipLaunchKernelGGL((bnpool_fwd_k<T, 2, 2>), dim3(pg), dim3(256), 0, s, x, y, am, xh, ctx, N, H, W, C, OH, OW, sh,
                       sw, pt, pl);
  else
    hipLaunchKernelGGL(bnpool_fwd<T>, dim3(pg), dim3(256), 0, s, x, y, am, xh, ctx, N, H, W, C, OH, OW, kh, kw, sh, sw,
                       pt, pl);
}

// x: conv output NHWC [N,H,W,C]; y: pooled [N,OH,OW,C]; am / xh: per pooled element (training only, may be null).
// ws: >= dl4j_bn_workspace_floats(N*H*W, C). ctx_out: 4*C floats.
template <typename T>
static int bn_pool_fwd_impl(const T* xb, T* y, unsigned char* am, T* xh, int N, int H, int W, int C, int OH, int OW,
                            int kh, int kw, int sh, int sw, int pt, int pl, const float* gamma, const float* beta,
                            float gconst, float bconst, float* run_mean, float* run_var, float decay, float eps,
                            int training, const float* tstats, long long P, int rpp, float* ws, float* ctx_out,
                            hipStream_t s) {
  const long long M = (long long)N * H * W;
  int nblk;
  long long rpb;
  bn_grid(M, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* q = p2 + (long long)nblk * C;
  const dim3 fg((C + 63) / 64);
  const int pg = ew_grid((long long)N * OH * OW * (C / 8));
  if (training && tstats && sizeof(T) == 2) {
    // statistics already reduced per tile by the producing conv's epilogue (ws sized for P tiles)
    nblk = (int)((P + 31) / 32);
    p2 = ws + (long long)nblk * C;
    q = p2 + (long long)nblk * C;
    hipLaunchKernelGGL(bn_tiles_reduce<T>, dim3((C + 63) / 64, nblk), dim3(256), 0, s, tstats, P, C, M, xb, p1, p2,
                       rpp);
    bn_reduce_stage(p1, p2, nblk, C, q, s);
    hipLaunchKernelGGL(bn_finalize<T>, fg, dim3(256), 0, s, p1, p2, nblk, C, M, xb, gamma, beta, gconst, bconst,
                       run_mean, run_var, decay, eps, 1, ctx_out);
  } else {
    if (training) hipLaunchKernelGGL(bn_stats_partial<T>, dim3(nblk), dim3(256), 0, s, xb, M, C, rpb, p1, p2);
    if (training) bn_reduce_stage(p1, p2, nblk, C, q, s);
    hipLaunchKernelGGL(bn_finalize<T>, fg, dim3(256), 0, s, p1, p2, nblk, C, M, xb, gamma, beta, gconst, bconst,
                       run_mean, run_var, decay, eps, training, ctx_out);
  }
  bnpool_fwd_launch<T>(xb, y, am, xh, ctx_out, N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl, pg, s);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bn_pool_fwd(int dtype, const void* x, void* y, unsigned char* am, void* xh, int N, int H, int W,
                              int C, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                              const float* gamma, const float* beta, float gconst, float bconst, float* run_mean,
                              float* run_var, float decay, float eps, int training, const float* tstats,
                              long long P, int rpp, float* ws, float* ctx_out, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || kh * kw > 127 || kh < 1 || kw < 1) return -1;
#define BPF(T) return bn_pool_fwd_impl<T>((const T*)x, (T*)y, am, (T*)xh, N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl, \
                                          gamma, beta, gconst, bconst, run_mean, run_var, decay, eps, training,    \
                                          tstats, P, rpp, ws, ctx_out, s)
  if (dtype == 1) BPF(bf16);
  if (dtype == 2) BPF(f16);
  BPF(float);
#undef BPF
}

// dy: gradient w.r.t. the pooled output; dx: w.r.t. x (the BN input). ws: >= dl4j_bn_workspace_floats(N*OH*OW, C).
template <typename T>
static int bn_pool_bwd_impl(const T* x, const T* dy, const unsigned char* am, const T* xh, T* dx, int N, int H, int W,
                            int C, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl, const float* ctx,
                            float* dgamma, float* dbeta, float* ws, hipStream_t s) {
  const long long Mp = (long long)N * OH * OW, M = (long long)N * H * W;
  int nblk;
  long long rpb;
  bn_grid(Mp, C, &nblk, &rpb);
  float* p1 = ws;
  float* p2 = ws + (long long)nblk * C;
  float* q = p2 + (long long)nblk * C;
  float* cdb = q + 2LL * ((nblk + 31) / 32) * C;
  float* cdg = cdb + C;
  const int g = ew_grid(M * (C / 8));
  hipLaunchKernelGGL(bnpool_bwd_partial<T>, dim3(nblk), dim3(256), 0, s, dy, am, xh, Mp, C, rpb, p1, p2);
  bn_reduce_stage(p1, p2, nblk, C, q, s);
  hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + 63) / 64), dim3(256), 0, s, p1, p2, nblk, C, M, dbeta, dgamma, cdb,
                     cdg);
  const bool two = kh <= 2 * sh && kw <= 2 * sw;
  // staged variant: pooled rows covering 2 input rows, all in LDS
  const int maxrows = (2 - 1 + kh - 1) / sh + 1;
  const size_t lds = (size_t)maxrows * OW * C * (sizeof(T) + 1);
  if (two && lds <= 64 * 1024) {
    const int nb = N * ((H + 1) / 2);
    hipLaunchKernelGGL(bnpool_bwd_dx_lds<T>, dim3(nb), dim3(256), lds, s, x, dy, am, dx, ctx, cdb, cdg, N, H, W, C, OH,
                       OW, kh, kw, sh, sw, pt, pl, maxrows);
    return (int)hipGetLastError();
  }
  if (two)
    hipLaunchKernelGGL(bnpool_bwd_dx2<T>, dim3(g), dim3(256), 0, s, x, dy, am, dx, ctx, cdb, cdg, N, H, W, C, OH, OW,
                       kh, kw, sh, sw, pt, pl);
  else
    hipLaunchKernelGGL(bnpool_bwd_dx<T>, dim3(g), dim3(256), 0, s, x, dy, am, dx, ctx, cdb, cdg, N, H, W, C, OH, OW,
                       kh, kw, sh, sw, pt, pl);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_bn_pool_bwd(int dtype, const void* x, const void* dy, const unsigned char* am, const void* xh,
                              void* dx, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw,
                              int pt, int pl, const float* ctx, float* dgamma, float* dbeta, float* ws, hipStream_t s) {
  if (C % 8 != 0 || C / 8 > 256 || kh * kw > 127) return -1;
#define BPB(T) return bn_pool_bwd_impl<T>((const T*)x, (const T*)dy, am, (const T*)xh, (T*)dx, N, H, W, C, OH, OW, kh, \
                                          kw, sh, sw, pt, pl, ctx, dgamma, dbeta, ws, s)
  if (dtype == 1) BPB(bf16);
  if (dtype == 2) BPB(f16);
  BPB(float);
#undef BPB
}
