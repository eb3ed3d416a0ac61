// LayerNorm forward / backward for gfx950, with the transformer residual add fused in:
//   s = x (+ r);  y = (s - mean(s)) * rstd * gamma + beta,  rstd = 1/sqrt(var(s) + eps)   (biased var)
// One wave per row: 16-byte vector loads (8 elements per lane per chunk), the row held in registers, fp32 stats by
// wave shuffles (exact two-pass: mean, then centred variance), no LDS and no block barriers. Saves mean/rstd
// (fp32, per row) for the backward.
// Backward: dxhat = dy*gamma; ds = rstd*(dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)) (the same gradient flows to
// x and r); dgamma/dbeta column sums are accumulated per block in registers and written as per-block partials,
// reduced by a second small kernel (no atomics: deterministic).
#include "common.h"
#include <cstdlib>

template <typename T> struct V8;
template <> struct V8<bf16> {
  static __device__ __forceinline__ void ld(const bf16* p, float* o) { Vec8<bf16>::load(p, o); }
  static __device__ __forceinline__ void st(bf16* p, const float* o) { Vec8<bf16>::store(p, o); }
};
template <> struct V8<f16> {
  static __device__ __forceinline__ void ld(const f16* p, float* o) { Vec8<f16>::load(p, o); }
  static __device__ __forceinline__ void st(f16* p, const float* o) { Vec8<f16>::store(p, o); }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void ld(const float* p, float* o) { Vec8<float>::load(p, o); }
  static __device__ __forceinline__ void st(float* p, const float* o) { Vec8<float>::store(p, o); }
};

// CH = 8-element chunks per lane (N <= 512*CH)
template <typename T, int CH, bool RES>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     T* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, long long M, int N, float eps) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = N >> 3;
  float v[CH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      V8<T>::ld(x + row * N + ch * 8, v[c]);
      if (RES) {
        float rr[8];
        V8<T>::ld(r + row * N + ch * 8, rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[c][k] += rr[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[c][k];
    }
  }
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    if (lane + c * 64 < nch) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[c][k] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float g[8], b[8], o[8];
      Vec8<float>::load(gamma + ch * 8, g);
      Vec8<float>::load(beta + ch * 8, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (v[c][k] - mean) * rstd * g[k] + b[k];
      V8<T>::st(y + row * N + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Each block: 4 waves x RPW rows; per-lane column partials of dgamma/dbeta written to part[blockIdx.x][2][N].
template <typename T, int CH, bool RES, int RPW>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ r, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     T* __restrict__ dx, float* __restrict__ part, long long M, int N) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = N >> 3;
  float dg[CH][8], db[CH][8], g[CH][8];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[c][k] = db[c][k] = 0.f;
    if (ch < nch) Vec8<float>::load(gamma + ch * 8, g[c]);
  }
  for (int i = 0; i < RPW; ++i) {
    const long long row = ((long long)blockIdx.x * 4 + wave) * RPW + i;
    if (row >= M) break;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[CH][8], d[CH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float xv[8], dv[8];
        V8<T>::ld(x + row * N + ch * 8, xv);
        if (RES) {
          float rr[8];
          V8<T>::ld(r + row * N + ch * 8, rr);
#pragma unroll
          for (int k = 0; k < 8; ++k) xv[k] += rr[k];
        }
        V8<T>::ld(dy + row * N + ch * 8, dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[c][k] = (xv[k] - mean) * rstd;
          d[c][k] = dv[k] * g[c][k];
          s1 += d[c][k];
          s2 += d[c][k] * xh[c][k];
          dg[c][k] += dv[k] * xh[c][k];
          db[c][k] += dv[k];
        }
      }
    }
    const float m1 = wave_sum(s1) / N, m2 = wave_sum(s2) / N;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (d[c][k] - m1 - xh[c][k] * m2);
        V8<T>::st(dx + row * N + ch * 8, o);
      }
    }
  }
  // per-wave partials: part[(blockIdx.x*4 + wave)][0/1][N]
  float* pg = part + ((long long)blockIdx.x * 4 + wave) * 2 * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::store(pg + ch * 8, dg[c]);
      Vec8<float>::store(pg + N + ch * 8, db[c]);
    }
  }
}

// Block-partial variant: W waves per block, wave w takes rows r0 + w, r0 + w + W, ... of the block's row range; the
// W per-wave dgamma/dbeta partials are summed through LDS so each BLOCK writes one [2][N] partial row. With ~512
// blocks of W = 8 waves every CU holds 16 waves of rows in flight (the per-wave-partial kernel above needs 16 rows
// per wave to keep its partial buffer small, which left M = 4096 on 64 blocks: 476-700 GB/s).
// DS: also the column sums of dx (a third partial plane): dx is the gradient of the dense layer that produced x
// (transformer FFN-2 / attention output), so this is that layer's bias gradient without another pass over dx.
template <typename T, int CH, bool RES, int W, bool DS>
__global__ void __launch_bounds__(64 * W) ln_bwd_block(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ r, const float* __restrict__ gamma,
                                                       const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                       float* __restrict__ part, long long M, int N, long long rpb) {
  constexpr int NP = DS ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) float lsum[];     // [W][NP][N]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = N >> 3;
  float dg[CH][8], db[CH][8], g[CH][8], dsum[DS ? CH : 1][8];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[c][k] = db[c][k] = 0.f;
    if (DS) {
#pragma unroll
      for (int k = 0; k < 8; ++k) dsum[DS ? c : 0][k] = 0.f;
    }
    if (ch < nch) Vec8<float>::load(gamma + ch * 8, g[c]);
  }
  const long long r0 = (long long)blockIdx.x * rpb;
  long long r1 = r0 + rpb;
  if (r1 > M) r1 = M;
  for (long long row = r0 + wave; row < r1; row += W) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xv[CH][8], dv[CH][8], rv[CH][8];
#pragma unroll
    for (int c = 0; c < CH; ++c) {                      // all of the row's loads in flight before any use
      const int ch = lane + c * 64;
      if (ch < nch) {
        V8<T>::ld(x + row * N + ch * 8, xv[c]);
        if (RES) V8<T>::ld(r + row * N + ch * 8, rv[c]);
        V8<T>::ld(dy + row * N + ch * 8, dv[c]);
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (lane + c * 64 < nch) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xs = RES ? xv[c][k] + rv[c][k] : xv[c][k];
          const float xh = (xs - mean) * rstd;
          const float d = dv[c][k] * g[c][k];
          xv[c][k] = xh;
          s1 += d;
          s2 += d * xh;
          dg[c][k] += dv[c][k] * xh;
          db[c][k] += dv[c][k];
          dv[c][k] = d;
        }
      }
    }
    const float m1 = wave_sum(s1) / N, m2 = wave_sum(s2) / N;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (dv[c][k] - m1 - xv[c][k] * m2);
        V8<T>::st(dx + row * N + ch * 8, o);
        if (DS) {
          // sum what was stored (rounded to T), so the bias gradient matches a column sum of the stored dx
          V8<T>::ld(dx + row * N + ch * 8, o);
#pragma unroll
          for (int k = 0; k < 8; ++k) dsum[DS ? c : 0][k] += o[k];
        }
      }
    }
  }
  float* mine = lsum + (long long)wave * NP * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::store(mine + ch * 8, dg[c]);
      Vec8<float>::store(mine + N + ch * 8, db[c]);
      if (DS) Vec8<float>::store(mine + 2 * N + ch * 8, dsum[DS ? c : 0]);
    }
  }
  __syncthreads();
  float* out = part + (long long)blockIdx.x * NP * N;
  for (int j = threadIdx.x; j < NP * N; j += 64 * W) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) t += lsum[w * NP * N + j];
    out[j] = t;
  }
}

// out[0/1][N] = sum over P partial rows. Block = 32 columns x 8 row groups (coalesced 128-byte row reads), the 8
// group sums combined through LDS. Eight independent row loads per trip (one per trip was latency-bound: 16
// dependent round trips for BERT's 128 partials).
__global__ void __launch_bounds__(256) ln_bwd_reduce(const float* __restrict__ part, int P, int N,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                     float* __restrict__ dsum, int NP) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + cl;                          // over the concatenated [dgamma | dbeta (| dsum)]
  float s = 0.f;
  if (j < NP * N) {
    const int which = j / N, col = j - which * N;
    const float* src = part + which * N + col;
    for (int p0 = rg; p0 < P; p0 += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = p0 + 8 * u;
        v[u] = p < P ? src[(long long)p * NP * N] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < NP * N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][cl];
    const int which = j / N, col = j - which * N;
    (which == 0 ? dgamma : (which == 1 ? dbeta : dsum))[col] = t;
  }
}

// Partial-row fold for the block kernel's [P][NP*N] partials: grid (ceil(NP*N/64), S = ceil(P/32)); each block sums
// 32 rows of 64 columns (4 row groups x 8 independent loads) and hands its row to the last block of its column chunk
// (agent-scope ticket; write-through atomic stores drained before the relaxed ticket add, atomic loads in the reducer:
// no fence), which sums the S rows in fixed order and writes dgamma / dbeta / dsum. ~36 x 16 blocks for BERT-base
// (P = 512, N = 768) instead of ln_bwd_reduce's 72 latency-bound blocks.
typedef __attribute__((address_space(1))) unsigned lq32;
__device__ unsigned g_ln_ticket[64 * 128];

__global__ void __launch_bounds__(256) ln_bwd_fold(const float* __restrict__ part, int P, int NPN, int N,
                                                   float* __restrict__ q, unsigned* __restrict__ ticket,
                                                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                   float* __restrict__ dsum) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * 32 + grp * 8;
  float v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = (j < NPN && r0 + u < P) ? part[(long long)(r0 + u) * NPN + j] : 0.f;
  float sacc = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) sacc += v[u];
  red[grp][cl] = sacc;
  __syncthreads();
  const float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
  auto out = [&](float x) {
    const int which = j / N, col = j - which * N;
    (which == 0 ? dgamma : (which == 1 ? dbeta : dsum))[col] = x;
  };
  if (gridDim.y == 1) {
    if (grp == 0 && j < NPN) out(t);
    return;
  }
  if (grp == 0 && j < NPN)
    __hip_atomic_store((lq32*)(q + (long long)blockIdx.y * NPN + j), __float_as_uint(t), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add((lq32*)&ticket[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == gridDim.y - 1;
    if (last) {
      __hip_atomic_store((lq32*)&ticket[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");        // one acquire, then plain loads all in flight
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    red[0][0] = last ? 1.f : 0.f;
  }
  __syncthreads();
  if (red[0][0] == 0.f) return;
  __syncthreads();                                               // everyone has read the flag before red is reused
  const int S = gridDim.y;
  float x = 0.f;
  if (j < NPN) {
    constexpr int UL = 8;
    for (int i0 = grp; i0 < S; i0 += 4 * UL) {
      float v2[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) v2[u] = i0 + 4 * u < S ? q[(long long)(i0 + 4 * u) * NPN + j] : 0.f;
#pragma unroll
      for (int u = 0; u < UL; ++u) x += v2[u];
    }
  }
  red[grp][cl] = x;
  __syncthreads();
  if (grp == 0 && j < NPN) out(red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]);
}

static unsigned* ln_ticket_slot(int cols) {
  static unsigned* base[64] = {nullptr};
  static unsigned next = 0;
  int dev = 0;
  if (cols > 128 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_ln_ticket)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  const unsigned k = __atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED) % 64u;
  return base[dev] + 128 * k;
}

template <typename T, int CH>
static int fwd_l(const void* x, const void* r, const float* g, const float* b, void* y, float* mean, float* rstd,
                 long long M, int N, float eps, hipStream_t s) {
  const dim3 grid((unsigned)((M + 3) / 4));
  if (r)
    hipLaunchKernelGGL((ln_fwd_kernel<T, CH, true>), grid, dim3(256), 0, s, (const T*)x, (const T*)r, g, b, (T*)y,
                       mean, rstd, M, N, eps);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<T, CH, false>), grid, dim3(256), 0, s, (const T*)x, (const T*)nullptr, g, b,
                       (T*)y, mean, rstd, M, N, eps);
  return (int)hipGetLastError();
}

static constexpr int kRPW = 16;

// Block-partial kernel geometry: up to g_ln_cap (512) blocks of W waves, at least one row per wave.
static int g_ln_cap = 128, g_ln_fold = 0;   // measured: tools/ln_bench.py (profiles/r3_ln_bwd_bench.log)
DL4J_API void dl4j_ln_set_config(int block_cap, int fold) {
  g_ln_cap = block_cap < 1 ? 1 : (block_cap > 512 ? 512 : block_cap);
  g_ln_fold = fold;
}
static inline int ln_waves(int N) { return N <= 1024 ? 8 : (N <= 2048 ? 4 : 2); }
static inline long long ln_blocks(long long M, int N) {
  const int W = ln_waves(N);
  long long b = (M + W - 1) / W;
  return b > g_ln_cap ? g_ln_cap : (b < 1 ? 1 : b);
}

static long long ln_bwd_partials(long long M) {
  const long long old = ((M + 4 * kRPW - 1) / (4 * kRPW)) * 4;
  long long blk = M < 512 ? M : 512;                         // the block kernel never needs more rows than this,
  blk += (blk + 31) / 32;                                    // plus the fold's ceil(rows / 32) rows of q
  return old > blk ? old : blk;
}

template <typename T, int CH, bool RES, int W>
static void bwd_block_launch(const void* dy, const void* x, const void* r, const float* g, const float* mean,
                             const float* rstd, void* dx, float* part, long long M, int N, long long blocks,
                             long long rpb, bool ds, hipStream_t s) {
  const size_t lds = (size_t)W * (ds ? 3 : 2) * N * sizeof(float);
  if (lds > 64 * 1024) {                                       // > 64 KB of dynamic LDS must be opted into
    static bool done[2] = {false, false};
    if (!done[ds ? 1 : 0]) {
      const void* k = ds ? reinterpret_cast<const void*>(ln_bwd_block<T, CH, RES, W, true>)
                         : reinterpret_cast<const void*>(ln_bwd_block<T, CH, RES, W, false>);
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      done[ds ? 1 : 0] = true;
    }
  }
  if (ds)
    hipLaunchKernelGGL((ln_bwd_block<T, CH, RES, W, true>), dim3((unsigned)blocks), dim3(64 * W), lds, s,
                       (const T*)dy, (const T*)x, (const T*)r, g, mean, rstd, (T*)dx, part, M, N, rpb);
  else
    hipLaunchKernelGGL((ln_bwd_block<T, CH, RES, W, false>), dim3((unsigned)blocks), dim3(64 * W), lds, s,
                       (const T*)dy, (const T*)x, (const T*)r, g, mean, rstd, (T*)dx, part, M, N, rpb);
}

template <typename T, int CH>
static int bwd_l(const void* dy, const void* x, const void* r, const float* g, const float* mean, const float* rstd,
                 void* dx, float* part, float* dgamma, float* dbeta, float* dsum, long long M, int N, hipStream_t s) {
  static int mode = -1;                                       // DL4J_AMD_LN_BWD=wave: per-wave-partial kernel (A/B)
  if (mode < 0) {
    const char* e = getenv("DL4J_AMD_LN_BWD");
    mode = (e && e[0] == 'w') ? 0 : 1;
  }
  if (mode == 1 || dsum) {
    const int W = ln_waves(N);
    const bool ds = dsum != nullptr;
    const long long blocks = ln_blocks(M, N);
    const long long rpb = (M + blocks - 1) / blocks;
#define LNB(RS, WW) bwd_block_launch<T, CH, RS, WW>(dy, x, r, g, mean, rstd, dx, part, M, N, blocks, rpb, ds, s)
    if (r) {
      if (W == 8) LNB(true, 8); else if (W == 4) LNB(true, 4); else LNB(true, 2);
    } else {
      if (W == 8) LNB(false, 8); else if (W == 4) LNB(false, 4); else LNB(false, 2);
    }
#undef LNB
    const int NP = ds ? 3 : 2;
    const int cols = (NP * N + 63) / 64, S = (int)((blocks + 31) / 32);
    unsigned* tk = S > 1 && g_ln_fold ? ln_ticket_slot(cols) : nullptr;
    if (g_ln_fold && (S == 1 || tk)) {
      // q (the folded rows) lives right after the partial rows in the caller's workspace (see ln_bwd_partials)
      float* q = part + blocks * NP * N;
      hipLaunchKernelGGL(ln_bwd_fold, dim3(cols, S), dim3(256), 0, s, part, (int)blocks, NP * N, N, q, tk, dgamma,
                         dbeta, dsum);
    } else {
      hipLaunchKernelGGL(ln_bwd_reduce, dim3((NP * N + 31) / 32), dim3(256), 0, s, part, (int)blocks, N, dgamma,
                         dbeta, dsum, NP);
    }
    return (int)hipGetLastError();
  }
  const long long blocks = (M + 4 * kRPW - 1) / (4 * kRPW);
  if (r)
    hipLaunchKernelGGL((ln_bwd_kernel<T, CH, true, kRPW>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)x, (const T*)r, g, mean, rstd, (T*)dx, part, M, N);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<T, CH, false, kRPW>), dim3((unsigned)blocks), dim3(256), 0, s, (const T*)dy,
                       (const T*)x, (const T*)nullptr, g, mean, rstd, (T*)dx, part, M, N);
  const int P = (int)(blocks * 4);
  hipLaunchKernelGGL(ln_bwd_reduce, dim3((2 * N + 31) / 32), dim3(256), 0, s, part, P, N, dgamma, dbeta, nullptr, 2);
  return (int)hipGetLastError();
}

#define LN_CH_DISPATCH(FN, T, ...)                       \
  do {                                                   \
    if (N <= 512) return FN<T, 1>(__VA_ARGS__);          \
    if (N <= 1024) return FN<T, 2>(__VA_ARGS__);         \
    if (N <= 2048) return FN<T, 4>(__VA_ARGS__);         \
    if (N <= 4096) return FN<T, 8>(__VA_ARGS__);         \
    return -1;                                           \
  } while (0)

DL4J_API long long dl4j_ln_partial_rows(long long M) { return ln_bwd_partials(M); }

// dtype 0 fp32, 1 bf16, 2 fp16. r may be null (no residual). Returns -1 when N is unsupported (N % 8 or N > 4096).
DL4J_API int dl4j_ln_fwd(int dtype, const void* x, const void* r, const float* gamma, const float* beta, void* y,
                         float* mean, float* rstd, long long M, int N, float eps, hipStream_t s) {
  if (N % 8 != 0 || N > 4096 || M < 1) return -1;
  if (dtype == 1) LN_CH_DISPATCH(fwd_l, bf16, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
  if (dtype == 2) LN_CH_DISPATCH(fwd_l, f16, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
  LN_CH_DISPATCH(fwd_l, float, x, r, gamma, beta, y, mean, rstd, M, N, eps, s);
}

// part: fp32 workspace of dl4j_ln_partial_rows(M) * 3 * N floats. dsum (optional, [N] fp32): column sums of dx.
DL4J_API int dl4j_ln_bwd(int dtype, const void* dy, const void* x, const void* r, const float* gamma,
                         const float* mean, const float* rstd, void* dx, float* part, float* dgamma, float* dbeta,
                         float* dsum, long long M, int N, hipStream_t s) {
  if (N % 8 != 0 || N > 4096 || M < 1) return -1;
  if (dtype == 1) LN_CH_DISPATCH(bwd_l, bf16, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, dsum, M, N, s);
  if (dtype == 2) LN_CH_DISPATCH(bwd_l, f16, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, dsum, M, N, s);
  LN_CH_DISPATCH(bwd_l, float, dy, x, r, gamma, mean, rstd, dx, part, dgamma, dbeta, dsum, M, N, s);
}
