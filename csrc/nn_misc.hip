// Less common NN layers on gfx950: cross-channel LRN, counter-based (Philox-4x32-10) dropout family, embedding
// gather / scatter-add, the BERT input-embedding sum and its position / type gradients, depthwise convolution (fwd,
// bwd-data, bwd-weight).
//
// Reference semantics:
//   LRN            deeplearning4j-cuda CudnnLocalResponseNormalizationHelper.java:160,199 and
//                  NN:nn/layers/normalization/LocalResponseNormalization.java:47,187 (window n centred on the channel,
//                  y = x (k + alpha * sum x^2)^-beta).
//   dropout        NN:nn/conf/dropout/Dropout.java:84 (inverted, p = RETAIN probability), AlphaDropout.java:113,
//                  GaussianDropout.java:66, GaussianNoise.java:53. The mask is never stored: forward and backward
//                  regenerate it from (seed, per-call counter, element index), so the backward costs one read of the
//                  gradient and the counter lives on the device (HIP-graph replays advance it).
//   embedding      NN:nn/layers/feedforward/embedding/EmbeddingLayer.java:71 (scatter-add of the row gradients),
//                  :111 (row gather).
//   depthwise conv NN:nn/layers/convolution/DepthwiseConvolution2DLayer.java / SeparableConvolution2DLayer.java:126-236
//                  (weights [depthMultiplier, C, kh, kw]; output channel c*dm + m).
//
// All kernels are memory-bound elementwise / stencil work: 64-wide waves, channel index fastest so that
// channels-last activations are read and written contiguously, fp32 accumulation, bf16 or fp32 storage.
#include "common.h"

// ------------------------------------------------------------------------------------------------ LRN
// Logical tensor [N, C, P] (P = H*W) with element strides sn, sc, sp. cfast: the thread index runs over c fastest
// (channels-last storage) instead of p.
__device__ __forceinline__ void lrn_coords(long long t, int C, int P, int cfast, int& n, int& c, int& p) {
  if (cfast) {
    c = idx_mod(t, C);
    const long long r = t / C;
    p = idx_mod(r, P);
    n = (int)(r / P);
  } else {
    p = idx_mod(t, P);
    const long long r = t / P;
    c = idx_mod(r, C);
    n = (int)(r / C);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void lrn_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                      float* __restrict__ unit, long long total, int C, int P,
                                                      long long sn, long long sc, long long sp, int half, float k,
                                                      float alpha, float beta, int cfast) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int n, c, p;
    lrn_coords(t, C, P, cfast, n, c, p);
    const long long base = (long long)n * sn + (long long)p * sp;
    const int lo = max(0, c - half), hi = min(C - 1, c + half);
    float s = 0.f;
    for (int j = lo; j <= hi; ++j) {
      const float v = ld1<T>(x + base + (long long)j * sc);
      s += v * v;
    }
    const long long o = base + (long long)c * sc;
    const float u = k + alpha * s;
    st1<T>(y + o, ld1<T>(x + o) * __powf(u, -beta));
    unit[o] = u;
  }
}

// dx_i = g_i u_i^-b - 2 a b x_i sum_{j in win(i)} g_j x_j u_j^(-b-1)   (the window is symmetric)
template <typename T>
__global__ __launch_bounds__(256) void lrn_bwd_kernel(const T* __restrict__ x, const T* __restrict__ g,
                                                      const float* __restrict__ unit, T* __restrict__ dx,
                                                      long long total, int C, int P, long long sn, long long sc,
                                                      long long sp, int half, float alpha, float beta, int cfast) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int n, c, p;
    lrn_coords(t, C, P, cfast, n, c, p);
    const long long base = (long long)n * sn + (long long)p * sp;
    const int lo = max(0, c - half), hi = min(C - 1, c + half);
    float s = 0.f;
    for (int j = lo; j <= hi; ++j) {
      const long long o = base + (long long)j * sc;
      const float u = unit[o];
      s += ld1<T>(g + o) * ld1<T>(x + o) * __powf(u, -beta - 1.f);
    }
    const long long o = base + (long long)c * sc;
    st1<T>(dx + o, ld1<T>(g + o) * __powf(unit[o], -beta) - 2.f * alpha * beta * ld1<T>(x + o) * s);
  }
}

// ------------------------------------------------------------------------------------------------ Philox dropout
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
  const unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const unsigned hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

__device__ __forceinline__ float u01(unsigned r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

// mode 0 Dropout, 1 AlphaDropout, 2 GaussianDropout, 3 GaussianNoise.  bwd: apply the multiplicative part only.
// Element i uses lane (i & 3) of philox(counter = {i >> 2, offset}, key = seed).
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long long n,
                                                      unsigned long long seed, const long long* __restrict__ offset,
                                                      int mode, int bwd, float p, float a, float b, float alpha_p,
                                                      float sd) {
  const unsigned long long off = (unsigned long long)offset[0];
  const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32));
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n;
       q += (long long)gridDim.x * blockDim.x) {
    const uint4 r = philox4x32_10(make_uint4((unsigned)q, (unsigned)(q >> 32), (unsigned)off,
                                             (unsigned)(off >> 32)), key);
    float u[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
    float z[4];
    if (mode >= 2) {                       // Box-Muller on the two pairs
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float rad = sqrtf(-2.f * __logf(fmaxf(u[2 * h], 1e-7f)));
        float sn, cs;
        __sincosf(6.283185307179586f * u[2 * h + 1], &sn, &cs);
        z[2 * h] = rad * cs;
        z[2 * h + 1] = rad * sn;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = q * 4 + e;
      if (i >= n) break;
      const float v = ld1<T>(x + i);
      float o;
      if (mode == 0) {
        o = u[e] < p ? v / p : 0.f;
      } else if (mode == 1) {
        const bool keep = u[e] < p;
        o = bwd ? (keep ? a * v : 0.f) : (keep ? a * v + b : a * alpha_p + b);
      } else if (mode == 2) {
        o = v * (1.f + sd * z[e]);
      } else {
        o = bwd ? v : v + sd * z[e];
      }
      st1<T>(y + i, o);
    }
  }
}

// ------------------------------------------------------------------------------------------------ embedding
// out[i, :] = W[idx[i], :] (zero row for an out-of-range index). One wave per row, 8-element vectors when possible.
template <typename T>
__global__ __launch_bounds__(256) void emb_gather_kernel(const T* __restrict__ W, const long long* __restrict__ idx,
                                                         T* __restrict__ out, int rows, int D, long long swr,
                                                         long long swc, int V, int vec) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4) {
    const long long k = idx[r];
    const bool ok = k >= 0 && k < V;
    const T* src = W + (ok ? k : 0) * swr;
    T* dst = out + (long long)r * D;
    if (vec) {
      for (int c = lane * 8; c < D; c += 512) {
        float v[8];
        Vec8<T>::load(src + c, v);
        if (!ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
        Vec8<T>::store(dst + c, v);
      }
    } else {
      for (int c = lane; c < D; c += 64) st1<T>(dst + c, ok ? ld1<T>(src + c * swc) : 0.f);
    }
  }
}

// dW[idx[i], :] += g[i, :]  (fp32 gradient, float atomics: repeated indices are summed)
template <typename T>
__global__ __launch_bounds__(256) void emb_scatter_kernel(const T* __restrict__ g, const long long* __restrict__ idx,
                                                          float* __restrict__ dW, int rows, int D, long long sdr,
                                                          long long sdc, int V) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4) {
    const long long k = idx[r];
    if (k < 0 || k >= V) continue;
    const T* src = g + (long long)r * D;
    float* dst = dW + k * sdr;
    for (int c = lane; c < D; c += 64) atomicAdd(dst + c * sdc, ld1<T>(src + c));
  }
}

// BERT input embedding: e[r, :] = Wword[idx[r], :] + Wpos[r % T, :] + Wtype[0, :] for r = b*T + t, summed in fp32
// and rounded once (three gathers and two adds of the imported graph in one pass). Rows are 16-byte vectors.
template <typename T>
__global__ __launch_bounds__(256) void bert_embed_fwd_kernel(const T* __restrict__ Ww, const T* __restrict__ Wp,
                                                             const T* __restrict__ Wt,
                                                             const long long* __restrict__ idx, T* __restrict__ out,
                                                             int rows, int Tn, int E, long long sw, long long sp,
                                                             int V) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4) {
    const long long k = idx[r];
    const bool ok = k >= 0 && k < V;
    const T* a = Ww + (ok ? k : 0) * sw;
    const T* p = Wp + (long long)(r % Tn) * sp;
    T* dst = out + (long long)r * E;
    for (int c = lane * 8; c < E; c += 512) {
      float va[8], vp[8], vt[8];
      Vec8<T>::load(a + c, va);
      Vec8<T>::load(p + c, vp);
      Vec8<T>::load(Wt + c, vt);
#pragma unroll
      for (int e = 0; e < 8; ++e) va[e] = (ok ? va[e] : 0.f) + vp[e] + vt[e];
      Vec8<T>::store(dst + c, va);
    }
  }
}

// Position / token-type gradients of that sum, deterministic (no atomics):
//   gpos[t, c] = sum_b de[b*T + t, c] for t < T, 0 for T <= t < Tmax      (one thread per (t, c), c fastest)
template <typename T>
__global__ __launch_bounds__(256) void bert_embed_bwd_pos_kernel(const T* __restrict__ de, float* __restrict__ gpos,
                                                                 int B, int Tn, int Tmax, int E, long long sgr,
                                                                 long long sgc) {
  const long long total = (long long)Tmax * E;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / E), c = (int)(i - (long long)t * E);
    float s = 0.f;
    if (t < Tn)
      for (int b = 0; b < B; ++b) s += ld1<T>(de + ((long long)b * Tn + t) * E + c);
    gpos[t * sgr + c * sgc] = s;
  }
}

//   gtype[0, c] = sum_{t < T} gpos[t, c], gtype[j > 0, c] = 0                (after the kernel above)
__global__ __launch_bounds__(256) void bert_embed_bwd_type_kernel(const float* __restrict__ gpos,
                                                                  float* __restrict__ gtype, int Tn, int ntype, int E,
                                                                  long long sgr, long long sgc, long long str,
                                                                  long long stc) {
  const long long total = (long long)ntype * E;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(i / E), c = (int)(i - (long long)j * E);
    float s = 0.f;
    if (j == 0)
      for (int t = 0; t < Tn; ++t) s += gpos[t * sgr + c * sgc];
    gtype[j * str + c * stc] = s;
  }
}

// ------------------------------------------------------------------------------------------------ depthwise conv
// Channels-last activations: x [N, H, W, C], y [N, OH, OW, OC], OC = C*dm, oc = c*dm + m.
// Weights re-laid out by the host as wr [KH*KW, OC] (fp32).
struct DwGeom {
  int N, H, W, C, dm, OH, OW, KH, KW, sh, sw, pt, pl, dh, dw;
};

template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wr,
                                                     const float* __restrict__ bias, T* __restrict__ y, DwGeom g) {
  const int OC = g.C * g.dm;
  const long long total = (long long)g.N * g.OH * g.OW * OC;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int oc, ow, oh, n;
    idx_decomp4(t, OC, g.OW, g.OH, oc, ow, oh, n);
    const int c = oc / g.dm;
    float acc = bias ? bias[oc] : 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.pt + kh * g.dh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pl + kw * g.dw;
        if (iw < 0 || iw >= g.W) continue;
        acc += ld1<T>(x + (((long long)n * g.H + ih) * g.W + iw) * g.C + c) * wr[(kh * g.KW + kw) * OC + oc];
      }
    }
    st1<T>(y + t, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_data_kernel(const T* __restrict__ dy, const float* __restrict__ wr,
                                                          T* __restrict__ dx, DwGeom g) {
  const int OC = g.C * g.dm;
  const long long total = (long long)g.N * g.H * g.W * g.C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    int c, iw, ih, n;
    idx_decomp4(t, g.C, g.W, g.H, c, iw, ih, n);
    float acc = 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int hh = ih + g.pt - kh * g.dh;
      if (hh < 0 || hh % g.sh) continue;
      const int oh = hh / g.sh;
      if (oh >= g.OH) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int ww = iw + g.pl - kw * g.dw;
        if (ww < 0 || ww % g.sw) continue;
        const int ow = ww / g.sw;
        if (ow >= g.OW) continue;
        const long long ob = (((long long)n * g.OH + oh) * g.OW + ow) * OC + (long long)c * g.dm;
        const float* wt = wr + (kh * g.KW + kw) * OC + c * g.dm;
        for (int m = 0; m < g.dm; ++m) acc += ld1<T>(dy + ob + m) * wt[m];
      }
    }
    st1<T>(dx + t, acc);
  }
}

// dwr[tap, oc] += sum over output pixels of x * dy. grid (row chunks, taps, oc tiles of 64); 4 waves split a chunk.
template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_weight_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            float* __restrict__ dwr, DwGeom g, int rows_per_block) {
  __shared__ float red[4][64];
  const int OC = g.C * g.dm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int oc = blockIdx.z * 64 + lane;
  const int tap = blockIdx.y, kh = tap / g.KW, kw = tap - kh * g.KW;
  const long long rows = (long long)g.N * g.OH * g.OW;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(rows, r0 + rows_per_block);
  float acc = 0.f;
  if (oc < OC) {
    const int c = oc / g.dm;
    for (long long r = r0 + wv; r < r1; r += 4) {
      int ow, oh, n, dummy;
      idx_decomp4(r, g.OW, g.OH, 0x7fffffff, ow, oh, n, dummy);
      const int ih = oh * g.sh - g.pt + kh * g.dh;
      const int iw = ow * g.sw - g.pl + kw * g.dw;
      if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
      acc += ld1<T>(x + (((long long)n * g.H + ih) * g.W + iw) * g.C + c) * ld1<T>(dy + r * OC + oc);
    }
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && oc < OC) {
    const float s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (s != 0.f) atomicAdd(dwr + (long long)tap * OC + oc, s);
  }
}

// ------------------------------------------------------------------------------------------------ C API
static inline int grid_for(long long total, int per_block = 256) {
  long long b = (total + per_block - 1) / per_block;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}

#define DISPATCH_T(dt, ...)                                          \
  do {                                                               \
    if ((dt) == 1) { typedef bf16 T; __VA_ARGS__; }                  \
    else if ((dt) == 0) { typedef float T; __VA_ARGS__; }            \
    else if ((dt) == 2) { typedef f16 T; __VA_ARGS__; }              \
    else return 1;                                                   \
  } while (0)

DL4J_API int dl4j_lrn_fwd(int dt, const void* x, void* y, float* unit, long long total, int C, int P, long long sn,
                          long long sc, long long sp, int half, float k, float alpha, float beta, int cfast,
                          hipStream_t s) {
  if (total <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(lrn_fwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, (const T*)x, (T*)y,
                                    unit, total, C, P, sn, sc, sp, half, k, alpha, beta, cfast));
  return (int)HIP_LAUNCH_CHECK();
}

DL4J_API int dl4j_lrn_bwd(int dt, const void* x, const void* g, const float* unit, void* dx, long long total, int C,
                          int P, long long sn, long long sc, long long sp, int half, float alpha, float beta,
                          int cfast, hipStream_t s) {
  if (total <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(lrn_bwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, (const T*)x,
                                    (const T*)g, unit, (T*)dx, total, C, P, sn, sc, sp, half, alpha, beta, cfast));
  return (int)HIP_LAUNCH_CHECK();
}

DL4J_API int dl4j_dropout(int dt, const void* x, void* y, long long n, unsigned long long seed, const long long* offset,
                          int mode, int bwd, float p, float a, float b, float alpha_p, float sd, hipStream_t s) {
  if (n <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(dropout_kernel<T>, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, (const T*)x,
                                    (T*)y, n, seed, offset, mode, bwd, p, a, b, alpha_p, sd));
  return (int)HIP_LAUNCH_CHECK();
}

// W / dW element strides (row, col): the DL4J parameter layout of EmbeddingLayer W is column-major ('f').
DL4J_API int dl4j_emb_gather(int dt, const void* W, const long long* idx, void* out, int rows, int D, long long swr,
                             long long swc, int V, hipStream_t s) {
  if (rows <= 0) return 0;
  const int vec = swc == 1 && (D % 8 == 0) && (swr % 8 == 0) && ((((uintptr_t)W) & 15) == 0) &&
                  ((((uintptr_t)out) & 15) == 0);
  DISPATCH_T(dt, hipLaunchKernelGGL(emb_gather_kernel<T>, dim3(grid_for(rows, 4)), dim3(256), 0, s, (const T*)W, idx,
                                    (T*)out, rows, D, swr, swc, V, vec));
  return (int)HIP_LAUNCH_CHECK();
}

DL4J_API int dl4j_emb_scatter_add(int dt, const void* g, const long long* idx, float* dW, int rows, int D,
                                  long long sdr, long long sdc, int V, hipStream_t s) {
  if (rows <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(emb_scatter_kernel<T>, dim3(grid_for(rows, 4)), dim3(256), 0, s, (const T*)g, idx,
                                    dW, rows, D, sdr, sdc, V));
  return (int)HIP_LAUNCH_CHECK();
}

// Wword / Wpos: row strides sw / sp with unit column stride; Wtype row 0 contiguous; E % 8 == 0, 16-byte aligned.
DL4J_API int dl4j_bert_embed_fwd(int dt, const void* Ww, const void* Wp, const void* Wt, const long long* idx,
                                 void* out, int rows, int Tn, int E, long long sw, long long sp, int V,
                                 hipStream_t s) {
  if (rows <= 0) return 0;
  if (Tn <= 0 || E % 8 || sw % 8 || sp % 8) return -1;
  for (const void* q : {Ww, Wp, Wt, (const void*)out})
    if (reinterpret_cast<uintptr_t>(q) & 15) return -1;
  DISPATCH_T(dt, hipLaunchKernelGGL(bert_embed_fwd_kernel<T>, dim3(grid_for(rows, 4)), dim3(256), 0, s, (const T*)Ww,
                                    (const T*)Wp, (const T*)Wt, idx, (T*)out, rows, Tn, E, sw, sp, V));
  return (int)HIP_LAUNCH_CHECK();
}

// de [B*T, E] contiguous; gpos [Tmax, E] and gtype [ntype, E] fp32 views with element strides (row, col).
DL4J_API int dl4j_bert_embed_bwd_pt(int dt, const void* de, float* gpos, float* gtype, int B, int Tn, int Tmax, int E,
                                    long long sgr, long long sgc, int ntype, long long str, long long stc,
                                    hipStream_t s) {
  if (B <= 0 || Tn <= 0 || Tn > Tmax || E <= 0) return -1;
  DISPATCH_T(dt, hipLaunchKernelGGL(bert_embed_bwd_pos_kernel<T>, dim3(grid_for((long long)Tmax * E)), dim3(256), 0,
                                    s, (const T*)de, gpos, B, Tn, Tmax, E, sgr, sgc));
  if (gtype && ntype > 0)
    hipLaunchKernelGGL(bert_embed_bwd_type_kernel, dim3(grid_for((long long)ntype * E)), dim3(256), 0, s, gpos, gtype,
                       Tn, ntype, E, sgr, sgc, str, stc);
  return (int)HIP_LAUNCH_CHECK();
}

static inline DwGeom dw_geom(const int* gi) {
  DwGeom g;
  g.N = gi[0]; g.H = gi[1]; g.W = gi[2]; g.C = gi[3]; g.dm = gi[4]; g.OH = gi[5]; g.OW = gi[6]; g.KH = gi[7];
  g.KW = gi[8]; g.sh = gi[9]; g.sw = gi[10]; g.pt = gi[11]; g.pl = gi[12]; g.dh = gi[13]; g.dw = gi[14];
  return g;
}

// gi = {N, H, W, C, dm, OH, OW, KH, KW, sh, sw, pt, pl, dh, dw}
DL4J_API int dl4j_dwconv_fwd(int dt, const void* x, const float* wr, const float* bias, void* y, const int* gi,
                             hipStream_t s) {
  const DwGeom g = dw_geom(gi);
  const long long total = (long long)g.N * g.OH * g.OW * g.C * g.dm;
  if (total <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(dw_fwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, (const T*)x, wr, bias,
                                    (T*)y, g));
  return (int)HIP_LAUNCH_CHECK();
}

DL4J_API int dl4j_dwconv_bwd_data(int dt, const void* dy, const float* wr, void* dx, const int* gi, hipStream_t s) {
  const DwGeom g = dw_geom(gi);
  const long long total = (long long)g.N * g.H * g.W * g.C;
  if (total <= 0) return 0;
  DISPATCH_T(dt, hipLaunchKernelGGL(dw_bwd_data_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, (const T*)dy, wr,
                                    (T*)dx, g));
  return (int)HIP_LAUNCH_CHECK();
}

DL4J_API int dl4j_dwconv_bwd_weight(int dt, const void* x, const void* dy, float* dwr, const int* gi, hipStream_t s) {
  const DwGeom g = dw_geom(gi);
  const long long rows = (long long)g.N * g.OH * g.OW;
  if (rows <= 0) return 0;
  const int OC = g.C * g.dm;
  const int taps = g.KH * g.KW;
  // aim for >= 2048 workgroups in total while keeping each chunk long enough to amortise the atomics
  long long tiles = (long long)taps * ((OC + 63) / 64);
  long long chunks = (2048 + tiles - 1) / tiles;
  int rpb = (int)((rows + chunks - 1) / chunks);
  if (rpb < 64) rpb = 64;
  const int nchunks = (int)((rows + rpb - 1) / rpb);
  DISPATCH_T(dt, hipLaunchKernelGGL(dw_bwd_weight_kernel<T>, dim3(nchunks, taps, (OC + 63) / 64), dim3(256), 0, s,
                                    (const T*)x, (const T*)dy, dwr, g, rpb));
  return (int)HIP_LAUNCH_CHECK();
}
