// Shared building blocks of the LDS-DMA MFMA tile kernels (csrc/gemm.hip GEMM, csrc/conv_gemm.hip implicit-GEMM
// convolution): operand fragment reads from the swizzled K-contiguous / M-contiguous LDS images, the counted-vmcnt
// helpers, and the LDS epilogue (alpha / bias / beta*C / pre-activation / activation, 16-byte row stores, BatchNorm
// tile statistics). Everything lives in an anonymous namespace: each including translation unit gets its own copy.
#pragma once
#include "common.h"
#include <hip/hip_fp16.h>

typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef __attribute__((address_space(3))) void lds_void_t;

namespace {

__device__ __attribute__((aligned(64))) char gemm_zero_page[64];

template <int V> struct IC { static constexpr int value = V; };
// compile-time loop: f(IC<I>{}) for I in [B, E) — keeps register arrays statically indexed
template <int B, int E, typename F> __device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    sfor<B + 1, E>(f);
  }
}

template <int DT> struct MfmaT;
template <> struct MfmaT<1> {
  typedef __attribute__((ext_vector_type(8))) __bf16 v8;
  static __device__ __forceinline__ f32x16_t mma(v8 a, v8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MfmaT<2> {
  typedef __attribute__((ext_vector_type(8))) _Float16 v8;
  static __device__ __forceinline__ f32x16_t mma(v8 a, v8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  void* Z;                 // optional pre-activation output (same dtype / ldc as C)
  const float* bias;       // fp32, per column (bias_mode 1) or per row (bias_mode 2)
  float* ws;               // split-K slabs [splits][M][N] fp32
  long long lda, ldb, ldc;
  long long sA, sB, sC;    // batch strides (elements)
  int M, N, K;
  int kps;                 // K per split (multiple of 64)
  int splits;
  float alpha, beta;
  int bias_mode, act, out_dt;
  int tiles_m, tiles_n;
  int coalesce;             // 1: epilogue through LDS with 16-byte row stores (host-checked alignment)
  float* tstats;           // optional BatchNorm partial statistics of the output (8-phase kernel, no split-K)
  int stats_P;              // number of 64-row partials (planes [3][stats_P][N])
  // BatchNorm-backward statistics instead (bnb 1: plain, 2: ReLU recomputed from x): the output is the gradient of a
  // BN layer's output, bnx that layer's input (same layout as C), bnctx its forward [mean|invstd|scale|shift];
  // planes [2][stats_P][N] (see epi_bnbwd_wave)
  const void* bnx;
  const float* bnctx;
  const unsigned char* bnmask;   // bnb 3: the forward's ReLU bitmask (1 byte per 8 channels, residual BN layers)
  int bnb;
  int store_nt;                  // lean read-out: 1 = non-temporal (streaming) output stores (DL4J_AMD_GEMM_STORE_NT)
  unsigned* sk_ticket;           // split-K fixup in the kernel (gemm_glds): per-tile arrival counters, else null
};

// Non-temporal (streaming) output stores in the lean read-out for outputs of >= 32 MB, which no L2 keeps for the
// next kernel anyway: the write-heavy expanding 1x1 convolutions (K = 64..128, N = 256..512) measured 299 -> 271 us
// and 153 -> 115 us, the ResNet-50 step +0.8 % (tools/gemm_conv1x1_bench.py, profiles/r5_conv1x1_gemm.txt).
// DL4J_AMD_GEMM_STORE_NT=0 / 1 forces them off / on for every size.
inline int store_nt_for(long long out_bytes) {
  static const int v = [] {
    const char* e = getenv("DL4J_AMD_GEMM_STORE_NT");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  return v >= 0 ? v : (out_bytes >= (32LL << 20) ? 1 : 0);
}

// The BN-backward epilogue request armed by dl4j_bnb_arm (csrc/gemm.hip) for the next GEMM / conv launches of this
// host thread (read into GemmArgs at launch time, so HIP-graph capture records it by value).
}  // namespace
struct BnbArm {
  const void* x;
  const float* ctx;
  const unsigned char* mask;
  int mode;
};
BnbArm& bnb_armed();                 // defined once, in csrc/gemm.hip
namespace {

__device__ __forceinline__ int xcd_remap_g(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N> __device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

// ----------------------------------------------------------------------------------------------- epilogue
// erf for the GELU epilogues: Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the 16-bit output's rounding),
// one hardware reciprocal, one exp2 and five FMAs, returning exp(-x^2) as well so gelu' reuses it. A 256x256 tile's
// GELU read-out runs 128 values per lane on two waves per SIMD after the main loop, i.e. it is VALU-bound: the
// library erff (two polynomial branches, both evaluated by the wave) cost ~19 us of a 52 us BERT FFN1 GEMM.
__device__ __forceinline__ float erf_as(float x, float& ex2) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  ex2 = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-p, ex2, 1.f), x);
}
__device__ __forceinline__ float gelu_f(float v) {
  float e;
  return 0.5f * v * (1.f + erf_as(v * 0.70710678118654752f, e));
}

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return tanhf(v);
    case 3: return 1.f / (1.f + __expf(-v));
    case 4: return gelu_f(v);
    default: return v;
  }
}

// act 5 (DGELU, backward of exact GELU): v *= gelu'(z) with z READ from the pre-activation buffer Z (same layout as C),
// so dz = (dy·Wᵀ) * gelu'(z) is one GEMM instead of a GEMM plus an elementwise pass.
// gelu'(z) = Phi(z) + z phi(z), phi(z) = exp(-z^2/2) / sqrt(2 pi) = the erf's exp(-(z/sqrt2)^2) term.
constexpr int kActDGelu = 5;
__device__ __forceinline__ float dgelu(float z) {
  float e;
  const float cdf = 0.5f * (1.f + erf_as(z * 0.70710678118654752f, e));
  return fmaf(z * 0.39894228040143268f, e, cdf);
}

__device__ __forceinline__ float ld_out(const void* C, int dt, long long i) {
  if (dt == 0) return reinterpret_cast<const float*>(C)[i];
  const u16 u = reinterpret_cast<const u16*>(C)[i];
  if (dt == 1) return bf2f(u);
  return __half2float(__ushort_as_half(u));
}

__device__ __forceinline__ u16 to16(float v, int dt) {
  return dt == 1 ? f2bf(v) : __half_as_ushort(__float2half(v));
}

// 4 consecutive outputs (m, n..n+3) of one row: vector store when aligned and fully in range.
__device__ __forceinline__ void store4(const GemmArgs& g, void* C, void* Z, int m, int n, float* v) {
  const long long base = (long long)m * g.ldc + n;
  const bool full = (n + 3 < g.N);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x = v[j] * g.alpha;
    if (g.bias_mode == 1 && n + j < g.N) x += g.bias[n + j];
    else if (g.bias_mode == 2) x += g.bias[m];
    if (g.beta != 0.f && n + j < g.N) x += g.beta * ld_out(C, g.out_dt, base + j);
    v[j] = x;
  }
  const bool vec = full && ((g.ldc & 3) == 0) && ((n & 3) == 0);
  if (g.act == kActDGelu) {
    if (Z)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < g.N) v[j] *= dgelu(ld_out(Z, g.out_dt, base + j));
  } else if (Z) {
    if (g.out_dt == 0) {
      float* z = reinterpret_cast<float*>(Z) + base;
      if (vec) *reinterpret_cast<float4*>(z) = make_float4(v[0], v[1], v[2], v[3]);
      else for (int j = 0; j < 4; ++j) if (n + j < g.N) z[j] = v[j];
    } else {
      u16* z = reinterpret_cast<u16*>(Z) + base;
      if (vec) {
        uint2 pk;
        pk.x = (unsigned)to16(v[0], g.out_dt) | ((unsigned)to16(v[1], g.out_dt) << 16);
        pk.y = (unsigned)to16(v[2], g.out_dt) | ((unsigned)to16(v[3], g.out_dt) << 16);
        *reinterpret_cast<uint2*>(z) = pk;
      } else {
        for (int j = 0; j < 4; ++j) if (n + j < g.N) z[j] = to16(v[j], g.out_dt);
      }
    }
  }
  if (g.act && g.act != kActDGelu)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = apply_act(v[j], g.act);
  if (g.out_dt == 0) {
    float* c = reinterpret_cast<float*>(C) + base;
    if (vec) *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
    else for (int j = 0; j < 4; ++j) if (n + j < g.N) c[j] = v[j];
  } else {
    u16* c = reinterpret_cast<u16*>(C) + base;
    if (vec) {
      uint2 pk;
      pk.x = (unsigned)to16(v[0], g.out_dt) | ((unsigned)to16(v[1], g.out_dt) << 16);
      pk.y = (unsigned)to16(v[2], g.out_dt) | ((unsigned)to16(v[3], g.out_dt) << 16);
      *reinterpret_cast<uint2*>(c) = pk;
    } else {
      for (int j = 0; j < 4; ++j) if (n + j < g.N) c[j] = to16(v[j], g.out_dt);
    }
  }
}

// ----------------------------------------------------------------------------------------------- lean epilogue
// The common output case — 16-bit C = act(alpha * acc + bias[col]), act none / relu, no beta, no pre-activation, no
// statistics, no split-K — leaves the block through ONE 16-bit LDS image of the whole tile ([BM][BN] x 2 bytes, row
// pitch BN*2, 16-byte chunks XOR-swizzled by row): every wave converts its accumulators in registers and writes
// 4-column (8-byte) pieces, one barrier, then every thread stores 16-byte row chunks. Half the LDS bytes of the fp32
// image, one pass instead of two, and little epilogue state: the generic path (epi_readout) kept so many kernel
// arguments live that the 8-phase kernel spilled 76 SGPRs / 4 VGPRs inside its main loop (measured 37.1k vs 26.9k
// loop cycles at K = 768 with a minimal epilogue, tools/native/gemm_stamps.hip).
// Host contract (lean_ok in csrc/gemm.hip): out_dt 1/2, N % 8 == 0, ldc % 8 == 0, 16-byte aligned C, bias 16-byte
// aligned (or absent), batch strides multiples of 8.
template <int BN>
__device__ __forceinline__ int lean_off(int r, int c) {          // byte offset of column c (multiple of 4) of row r
  return r * (BN * 2) + ((((c >> 3) ^ (r & 7))) << 4) + (c & 7) * 2;
}

template <int BN>
__device__ __forceinline__ void lean_put4(char* T, int r, int c, float v0, float v1, float v2, float v3, int dt) {
  uint2 pk;
  pk.x = (unsigned)to16(v0, dt) | ((unsigned)to16(v1, dt) << 16);
  pk.y = (unsigned)to16(v2, dt) | ((unsigned)to16(v3, dt) << 16);
  *reinterpret_cast<uint2*>(T + lean_off<BN>(r, c)) = pk;
}

// activation applied by the lean writer: relu, or GELU when no pre-activation is kept (with Z the read-out applies it)
__device__ __forceinline__ void lean_act4(const GemmArgs& g, float* v) {
  if (g.act == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
  } else if (g.act == 4 && g.Z == nullptr) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_f(v[j]);
  }
}

// alpha, per-column bias (4 columns from column n), activation (0 / 1 = relu) on 4 consecutive values
__device__ __forceinline__ void lean_math4(const GemmArgs& g, int n, float* v) {
  float b[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.bias_mode == 1 && n < g.N) {
    const float4 q = *reinterpret_cast<const float4*>(g.bias + n);
    b[0] = q.x; b[1] = q.y; b[2] = q.z; b[3] = q.w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = v[j] * g.alpha + b[j];
    if (g.act == 1) v[j] = fmaxf(v[j], 0.f);
  }
}

// Read-out of the lean image: 16-byte row chunks to C. With a pre-activation buffer Z: act GELU stores the image (the
// rounded pre-activation) to Z and gelu(Z) to C; act DGELU multiplies the image by gelu'(Z) read from Z (loads for 4
// rows issued before their stores). Both match the library-product + elementwise-kernel numerics (the elementwise
// pass reads the rounded product).
template <int BM, int BN, int NT>
__device__ __forceinline__ void lean_readout(const GemmArgs& g, char* dst, const char* T, int m0, int n0, int tid,
                                             char* zdst = nullptr) {
  constexpr int CPR = BN / 8;
  constexpr int RSTEP = NT / CPR;
  constexpr int ITER = BM / RSTEP;
  constexpr int GROUP = ITER < 4 ? ITER : 4;
  static_assert(NT % CPR == 0 && BM % RSTEP == 0 && ITER % GROUP == 0, "lean read-out geometry");
  const int c = tid % CPR, r0 = tid / CPR;
  const int n = n0 + c * 8;
  if (n >= g.N) return;
  const int dt = g.out_dt;
  const int zmode = zdst == nullptr ? 0 : (g.act == kActDGelu ? 2 : 1);
  auto unpack = [&](const uint4& q, float* v) {
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u16 u = (u16)(w[j >> 1] >> (16 * (j & 1)));
      v[j] = dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
    }
  };
  auto pack = [&](const float* v) {
    uint4 q;
    q.x = (unsigned)to16(v[0], dt) | ((unsigned)to16(v[1], dt) << 16);
    q.y = (unsigned)to16(v[2], dt) | ((unsigned)to16(v[3], dt) << 16);
    q.z = (unsigned)to16(v[4], dt) | ((unsigned)to16(v[5], dt) << 16);
    q.w = (unsigned)to16(v[6], dt) | ((unsigned)to16(v[7], dt) << 16);
    return q;
  };
  if (zmode == 0) {
#pragma unroll 4
    for (int r = r0; r < BM; r += RSTEP) {
      const int m = m0 + r;
      const uint4 q = *reinterpret_cast<const uint4*>(T + r * (BN * 2) + ((c ^ (r & 7)) << 4));
      if (m < g.M) {
        char* p = dst + ((long long)m * g.ldc + n) * 2;
        if (g.store_nt) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          const u32x4_t v = {q.x, q.y, q.z, q.w};
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
        } else {
          *reinterpret_cast<uint4*>(p) = q;
        }
      }
    }
    return;
  }
#pragma unroll 1
  for (int G = 0; G < ITER; G += GROUP) {
    uint4 zq[GROUP];
#pragma unroll
    for (int i = 0; i < GROUP; ++i) {
      const int m = m0 + r0 + (G + i) * RSTEP;
      zq[i] = make_uint4(0u, 0u, 0u, 0u);
      if (zmode == 2 && m < g.M) zq[i] = *reinterpret_cast<const uint4*>(zdst + ((long long)m * g.ldc + n) * 2);
    }
#pragma unroll
    for (int i = 0; i < GROUP; ++i) {
      const int r = r0 + (G + i) * RSTEP;
      const int m = m0 + r;
      const uint4 q = *reinterpret_cast<const uint4*>(T + r * (BN * 2) + ((c ^ (r & 7)) << 4));
      if (m >= g.M) continue;
      const long long off = ((long long)m * g.ldc + n) * 2;
      float v[8];
      unpack(q, v);
      if (zmode == 1) {
        *reinterpret_cast<uint4*>(zdst + off) = q;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j]);
      } else {
        float z[8];
        unpack(zq[i], z);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= dgelu(z[j]);
      }
      *reinterpret_cast<uint4*>(dst + off) = pack(v);
    }
  }
}

// BatchNorm tile statistics from the lean 16-bit image (the values exactly as stored): same work split, sums and
// output planes as epi_stats_wave (below) — one wave per (64-row partial, 64-column slab), lane 16q + c takes
// columns 4c..4c+3 of rows 16q..16q+15 (8-byte LDS reads), row quarters combined by two xor-shuffles.
template <int BM, int BN, int NT>
__device__ __forceinline__ void lean_stats(const GemmArgs& g, const char* T, int m0, int n0, int tid) {
  static_assert(BN % 64 == 0 && BM % 64 == 0, "lean statistics need 64-row / 64-column tiles");
  constexpr int PARTS = BM / 64, SLABS = BN / 64, NW = NT / 64;
  const int lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  const int dt = g.out_dt;
  auto val = [&](unsigned wv, int j) {
    const u16 u = (u16)(wv >> (16 * (j & 1)));
    return dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
  };
  for (int item = w; item < PARTS * SLABS; item += NW) {
    const int part = item / SLABS, slab = item - (item / SLABS) * SLABS;
    const int rbeg = m0 + part * 64;
    const long long pidx = rbeg / 64;
    if (pidx >= g.stats_P) continue;
    const int rows = min(64, g.M - rbeg);
    const int col = slab * 64 + 4 * c;
    const int n = n0 + col;
    float sh[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    if (rows > 0) {
      const uint2 y0 = *reinterpret_cast<const uint2*>(T + lean_off<BN>(part * 64, col));
#pragma unroll
      for (int j = 0; j < 4; ++j) sh[j] = val(j < 2 ? y0.x : y0.y, j);
      const int r0 = 16 * q;
      const int rn = rows - r0 < 16 ? (rows - r0 > 0 ? rows - r0 : 0) : 16;
      if (rn == 16) {
        // whole 16-row quarter: 16 independent LDS reads, statically indexed (the earlier loop with a data-dependent
        // break put this array in scratch memory, whose loads then drained every outstanding store with vmcnt(0))
        uint2 v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          v[r] = *reinterpret_cast<const uint2*>(T + lean_off<BN>(part * 64 + r0 + r, col));
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = val(j < 2 ? v[r].x : v[r].y, j) - sh[j];
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
      } else {
        for (int r = 0; r < rn; ++r) {
          const uint2 w = *reinterpret_cast<const uint2*>(T + lean_off<BN>(part * 64 + r0 + r, col));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = val(j < 2 ? w.x : w.y, j) - sh[j];
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], 16);
      s2[j] += __shfl_xor(s2[j], 16);
      s1[j] += __shfl_xor(s1[j], 32);
      s2[j] += __shfl_xor(s2[j], 32);
    }
    if (q == 0 && n < g.N) {
      float* p1 = g.tstats + pidx * g.N + n;
      float* p2 = g.tstats + ((long long)g.stats_P + pidx) * g.N + n;
      float* p3 = g.tstats + (2LL * g.stats_P + pidx) * g.N + n;
      *reinterpret_cast<float4*>(p1) = make_float4(s1[0], s1[1], s1[2], s1[3]);
      *reinterpret_cast<float4*>(p2) = make_float4(s2[0], s2[1], s2[2], s2[3]);
      *reinterpret_cast<float4*>(p3) = make_float4(sh[0], sh[1], sh[2], sh[3]);
    }
  }
}

// ----------------------------------------------------------------------------------------------- LDS epilogue
// Finished fp32 accumulators leave a block through LDS: pass P, the waves owning tile rows [P*RPP, (P+1)*RPP)
// store their raw accumulators into an fp32 [RPP][BN] image (row pitch BN*4 + 16 bytes), then every thread takes
// 8-column chunks of whole rows, applies alpha / bias / beta*C / pre-activation Z / activation once per element
// (bias as vector loads), converts, and writes 16-byte row segments. Direct 8-byte stores from the MFMA fragment
// layout (16-32 rows per instruction) ran at ~1 TB/s; register pressure stays at the accumulators themselves.
struct EpiOut {
  char* dst;          // C (or the split-K slab)
  long long ld;       // destination row stride (elements)
  int dt;             // destination dtype (0 f32, 1 bf16, 2 f16)
  bool raw;           // split-K slab: no epilogue math
  bool vec;           // 16-byte aligned rows (ld and base) for vector stores
  bool coh;           // slab stores coherent at agent scope (sc1 write-through): read by another block's fixup
};

// 16-byte / 4-byte stores visible to every XCD once the storing wave's vmcnt drains (sc1: written through the
// XCD-local L2), for split-K slabs that the tile's last-arriving block sums (gemm_glds fixup)
__device__ __forceinline__ void st_coh16(void* p, float a, float b, float c, float d) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const f32x4v v = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_coh4(float* p, float a) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void epi_chunk8(const GemmArgs& g, const EpiOut& o, void* Zp, int m, int n, float* v) {
  if (!o.raw) {
    float b[8];
    if (g.bias_mode == 1) {
      if (n + 8 <= g.N && ((n & 3) == 0)) {
        const float4 b0 = *reinterpret_cast<const float4*>(g.bias + n);
        const float4 b1 = *reinterpret_cast<const float4*>(g.bias + n + 4);
        b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
      } else {
        for (int j = 0; j < 8; ++j) b[j] = n + j < g.N ? g.bias[n + j] : 0.f;
      }
    } else {
      const float bm = g.bias_mode == 2 ? g.bias[m] : 0.f;
      for (int j = 0; j < 8; ++j) b[j] = bm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * g.alpha + b[j];
    if (g.beta != 0.f)
      for (int j = 0; j < 8; ++j) if (n + j < g.N) v[j] += g.beta * ld_out(o.dst, o.dt, (long long)m * o.ld + n + j);
    if (g.act == kActDGelu) {
      if (Zp) {
        const long long i0 = (long long)m * o.ld + n;
        if (o.vec && n + 8 <= g.N && o.dt != 0) {
          const uint4 zz = *reinterpret_cast<const uint4*>(reinterpret_cast<const u16*>(Zp) + i0);
          const unsigned w[4] = {zz.x, zz.y, zz.z, zz.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const u16 u = (u16)(w[j >> 1] >> (16 * (j & 1)));
            const float z = o.dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
            v[j] *= dgelu(z);
          }
        } else {
          for (int j = 0; j < 8; ++j)
            if (n + j < g.N) v[j] *= dgelu(ld_out(Zp, o.dt, i0 + j));
        }
      }
    } else {
      if (Zp)
        for (int j = 0; j < 8; ++j)
          if (n + j < g.N) {
            const long long i = (long long)m * o.ld + n + j;
            if (o.dt == 0) reinterpret_cast<float*>(Zp)[i] = v[j];
            else reinterpret_cast<u16*>(Zp)[i] = to16(v[j], o.dt);
          }
      if (g.act)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j], g.act);
    }
  }
  char* p = o.dst + ((long long)m * o.ld + n) * (o.dt == 0 ? 4 : 2);
  if (o.coh) {
    for (int j = 0; j < 8; ++j)
      if (n + j < g.N) st_coh4(reinterpret_cast<float*>(p) + j, v[j]);
    return;
  }
  if (o.vec && n + 8 <= g.N) {
    if (o.dt == 0) {
      reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      uint4 pk;
      pk.x = (unsigned)to16(v[0], o.dt) | ((unsigned)to16(v[1], o.dt) << 16);
      pk.y = (unsigned)to16(v[2], o.dt) | ((unsigned)to16(v[3], o.dt) << 16);
      pk.z = (unsigned)to16(v[4], o.dt) | ((unsigned)to16(v[5], o.dt) << 16);
      pk.w = (unsigned)to16(v[6], o.dt) | ((unsigned)to16(v[7], o.dt) << 16);
      *reinterpret_cast<uint4*>(p) = pk;
    }
  } else {
    for (int j = 0; j < 8; ++j)
      if (n + j < g.N) {
        if (o.dt == 0) reinterpret_cast<float*>(p)[j] = v[j];
        else reinterpret_cast<u16*>(p)[j] = to16(v[j], o.dt);
      }
  }
}

// Fast read-out sweep: the whole tile lies inside the output's columns and rows are 16-byte aligned. Every thread
// owns one 8-column chunk (fixed column -> the per-column bias is loaded once) of RSTEP-strided rows. Any loads
// (beta*C, the pre-activation Z of the GELU backward) are issued for a GROUP of rows at a time before the first
// store of that group, so a pass waits on the memory counter at most once per group — the generic per-chunk
// routine below branches around its loads, and hipcc then drains the counter (outstanding stores included) once
// per chunk: measured 22.5k cycles for a 256x256 bf16 tile (tools/native/gemm_stamps.hip) against ~3k here.
template <int RPP, int BN, int NT, bool F32>
__device__ __forceinline__ void epi_sweep(const GemmArgs& g, const EpiOut& o, void* Zp, const char* T, int mrow0,
                                          int n0, int tid) {
  constexpr int PITCH = BN * 4 + 16;
  constexpr int CPR = BN / 8;
  constexpr int RSTEP = NT / CPR;
  constexpr int ITER = RPP / RSTEP;
  constexpr int GROUP = ITER < 4 ? ITER : 4;
  static_assert(NT % CPR == 0 && RPP % RSTEP == 0 && ITER % GROUP == 0, "epilogue sweep geometry");
  constexpr int ESZ = F32 ? 4 : 2;
  const int c = tid % CPR, r0 = tid / CPR;
  const int n = n0 + c * 8;
  const bool raw = o.raw;
  const int dt = o.dt;                    // 16-bit destinations: 1 bf16, 2 fp16 (a VALU select, no branch on loads)
  const float alpha = raw ? 1.f : g.alpha;
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (!raw && g.bias_mode == 1) {
    const float4 b0 = *reinterpret_cast<const float4*>(g.bias + n);
    const float4 b1 = *reinterpret_cast<const float4*>(g.bias + n + 4);
    b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
  }
  const bool loadc = !raw && g.beta != 0.f;
  const bool dg = !raw && g.act == kActDGelu;
  const bool loadz = dg && Zp != nullptr;
  const bool storez = !raw && !dg && Zp != nullptr;
  const int act = raw || dg ? 0 : g.act;  // 0, 1 (relu) or 4 (gelu) here: epi_readout routes the others
  const float beta = g.beta;
  auto unpack = [&](const uint4& lo, const uint4& hi, float* out) {
    const unsigned w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (F32) out[j] = __uint_as_float(w[j]);
      else {
        const u16 u = (u16)(w[j >> 1] >> (16 * (j & 1)));
        out[j] = dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
      }
    }
  };
  const bool coh = o.coh;
  auto store8 = [&](char* p, const float* w) {
    if constexpr (F32) {
      if (coh) {
        st_coh16(p, w[0], w[1], w[2], w[3]);
        st_coh16(p + 16, w[4], w[5], w[6], w[7]);
      } else {
        reinterpret_cast<float4*>(p)[0] = make_float4(w[0], w[1], w[2], w[3]);
        reinterpret_cast<float4*>(p)[1] = make_float4(w[4], w[5], w[6], w[7]);
      }
    } else {
      uint4 pk;
      pk.x = (unsigned)to16(w[0], dt) | ((unsigned)to16(w[1], dt) << 16);
      pk.y = (unsigned)to16(w[2], dt) | ((unsigned)to16(w[3], dt) << 16);
      pk.z = (unsigned)to16(w[4], dt) | ((unsigned)to16(w[5], dt) << 16);
      pk.w = (unsigned)to16(w[6], dt) | ((unsigned)to16(w[7], dt) << 16);
      *reinterpret_cast<uint4*>(p) = pk;
    }
  };
#pragma unroll 1
  for (int G = 0; G < ITER; G += GROUP) {
    // 16-bit: one uint4 per row chunk; fp32: two (the second in the *h arrays)
    uint4 cc[GROUP], cz[GROUP], cch[GROUP], czh[GROUP];
#pragma unroll
    for (int i = 0; i < GROUP; ++i) cc[i] = cz[i] = cch[i] = czh[i] = make_uint4(0u, 0u, 0u, 0u);
    if (loadc || loadz) {
#pragma unroll
      for (int i = 0; i < GROUP; ++i) {
        const int m = mrow0 + r0 + (G + i) * RSTEP;
        if (m < g.M) {
          const long long off = ((long long)m * o.ld + n) * ESZ;
          if (loadc) {
            cc[i] = *reinterpret_cast<const uint4*>(o.dst + off);
            if constexpr (F32) cch[i] = *reinterpret_cast<const uint4*>(o.dst + off + 16);
          }
          if (loadz) {
            cz[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(Zp) + off);
            if constexpr (F32) czh[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(Zp) + off + 16);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GROUP; ++i) {
      const int r = r0 + (G + i) * RSTEP;
      const int m = mrow0 + r;
      const float4 a = *reinterpret_cast<const float4*>(T + r * PITCH + c * 32);
      const float4 q = *reinterpret_cast<const float4*>(T + r * PITCH + c * 32 + 16);
      float v[8] = {a.x, a.y, a.z, a.w, q.x, q.y, q.z, q.w};
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * alpha + b[j];
      if (loadc) {
        float x[8];
        unpack(cc[i], cch[i], x);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += beta * x[j];
      }
      const long long off = ((long long)m * o.ld + n) * ESZ;
      if (loadz) {
        float z[8];
        unpack(cz[i], czh[i], z);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= dgelu(z[j]);
      }
#ifdef DL4J_EPI_NOSTORE
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(v[j]));
      continue;
#endif
      if (storez) store8(reinterpret_cast<char*>(Zp) + off, v);
      if (act == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      } else if (act == 4) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j]);
      }
      store8(o.dst + off, v);
    }
  }
}

// Read-out of one pass: RPP rows x BN columns of the fp32 LDS image. Whole-tile-in-range, vector-aligned tiles take
// the fast sweep above (block-uniform choice); ragged right-edge / unaligned tiles the generic per-chunk routine.
template <int RPP, int BN, int NT>
__device__ __forceinline__ void epi_readout(const GemmArgs& g, const EpiOut& o, void* Zp, const char* T, int mrow0,
                                            int n0, int tid) {
  constexpr int PITCH = BN * 4 + 16;
  constexpr int CPR = BN / 8;
  const bool fast = o.vec && n0 + BN <= g.N &&
                    (o.raw || (g.bias_mode != 2 && (g.act == 0 || g.act == 1 || g.act == 4 || g.act == kActDGelu) &&
                               (g.bias_mode != 1 || (reinterpret_cast<uintptr_t>(g.bias) & 15) == 0)));
  if constexpr (NT % CPR == 0 && RPP % (NT / CPR) == 0) {
    if (fast) {
      if (o.raw || o.dt == 0) epi_sweep<RPP, BN, NT, true>(g, o, Zp, T, mrow0, n0, tid);
      else epi_sweep<RPP, BN, NT, false>(g, o, Zp, T, mrow0, n0, tid);
      return;
    }
  }
  for (int idx = tid; idx < RPP * CPR; idx += NT) {
    const int r = idx / CPR, c = idx - (idx / CPR) * CPR;
    const int m = mrow0 + r, n = n0 + c * 8;
    if (m >= g.M || n >= g.N) continue;
    const float4 a = *reinterpret_cast<const float4*>(T + r * PITCH + c * 32);
    const float4 b = *reinterpret_cast<const float4*>(T + r * PITCH + c * 32 + 16);
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    epi_chunk8(g, o, Zp, m, n, v);
  }
}

// BatchNorm partial statistics of the bf16 outputs held in an fp32 LDS image (conv epilogue -> consuming BN layer):
// per (64-row partial, column) shifted sums S1 = sum(y - y0), S2 = sum((y - y0)^2) and the shift y0 (first row),
// y = bf16(alpha*acc + bias) exactly as stored. Planes [3][stats_P][N]; reduced by bn_tiles_reduce.
//
// Work split: one wave per (64-row partial, 64-column slab) item; lane = 16*q + c takes columns slab*64 + 4c..4c+3 of
// rows 16q..16q+15 (float4 LDS reads: the 16 lanes of a quarter read one contiguous 256-byte row segment), and the
// four row quarters are combined with two cross-lane xor-shuffles (same shift y0 -> plain sums): 16 independent
// float4 reads per lane instead of 64 dependent scalar ones per column. The per-column loop below (kept for tiles
// with BN % 64 != 0) added 25-120 us to a 400k-row 1x1 conv (tools/skinny_probe.py).
template <int DTO>
__device__ __forceinline__ float stored_as(float v) {
  if constexpr (DTO == 2) return __half2float(__float2half(v));
  else if constexpr (DTO == 1) return bf2f(to16(v, 1));
  else return v;
}

template <int RPP, int BN, int NT, int DTO>
__device__ __forceinline__ void epi_stats_wave(const GemmArgs& g, const char* T, int mrow0, int n0, int tid) {
  constexpr int PITCH = BN * 4 + 16;
  constexpr int PARTS = RPP / 64, SLABS = BN / 64, NW = NT / 64;
  const int lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  for (int item = w; item < PARTS * SLABS; item += NW) {
    const int part = item / SLABS, slab = item - (item / SLABS) * SLABS;
    const int rbeg = mrow0 + part * 64;
    const long long pidx = rbeg / 64;
    if (pidx >= g.stats_P) continue;
    const int rows = min(64, g.M - rbeg);
    const int col = slab * 64 + 4 * c;
    const int n = n0 + col;
    float bb[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias_mode == 1)
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = n + j < g.N ? g.bias[n + j] : 0.f;
    float sh[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    const char* src = T + (part * 64) * PITCH + col * 4;
    if (rows > 0) {
      const float4 y0 = *reinterpret_cast<const float4*>(src);
      sh[0] = stored_as<DTO>(y0.x * g.alpha + bb[0]);
      sh[1] = stored_as<DTO>(y0.y * g.alpha + bb[1]);
      sh[2] = stored_as<DTO>(y0.z * g.alpha + bb[2]);
      sh[3] = stored_as<DTO>(y0.w * g.alpha + bb[3]);
      const int r0 = 16 * q;
      if (r0 + 16 <= rows) {
        float4 v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = *reinterpret_cast<const float4*>(src + (r0 + r) * PITCH);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = stored_as<DTO>(e[j] * g.alpha + bb[j]) - sh[j];
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
        }
      } else {
        for (int r = r0; r < rows; ++r) {
          const float4 x = *reinterpret_cast<const float4*>(src + r * PITCH);
          const float e[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = stored_as<DTO>(e[j] * g.alpha + bb[j]) - sh[j];
            s1[j] += d;
            s2[j] = fmaf(d, d, s2[j]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], 16);
      s2[j] += __shfl_xor(s2[j], 16);
      s1[j] += __shfl_xor(s1[j], 32);
      s2[j] += __shfl_xor(s2[j], 32);
    }
    if (q == 0) {
      float* p1 = g.tstats + pidx * g.N + n;
      float* p2 = g.tstats + ((long long)g.stats_P + pidx) * g.N + n;
      float* p3 = g.tstats + (2LL * g.stats_P + pidx) * g.N + n;
      if (n + 4 <= g.N && (g.N & 3) == 0) {
        *reinterpret_cast<float4*>(p1) = make_float4(s1[0], s1[1], s1[2], s1[3]);
        *reinterpret_cast<float4*>(p2) = make_float4(s2[0], s2[1], s2[2], s2[3]);
        *reinterpret_cast<float4*>(p3) = make_float4(sh[0], sh[1], sh[2], sh[3]);
      } else {
        for (int j = 0; j < 4; ++j)
          if (n + j < g.N) { p1[j] = s1[j]; p2[j] = s2[j]; p3[j] = sh[j]; }
      }
    }
  }
}

// BatchNorm BACKWARD partial sums from the epilogue of the GEMM / bwd-data conv that produces dy, the gradient of a
// training BN layer's output (reference NN:nn/layers/normalization/BatchNormalization.java:131-210): per (64-row
// partial, column) S1 = sum(d) and S2 = sum(d * (x - mean) * invstd), d = dy exactly as stored (bf16 / fp16 rounding),
// zeroed where relu(x*scale + shift) was inactive (bnb == 2) or where the forward's ReLU bitmask is clear (bnb == 3:
// a BN layer with a fused residual, whose ReLU input is not recomputable from x alone). x (g.bnx, the BN input, same
// layout as C) is read from global memory: 8 bytes per lane-row, the 16 lanes of a row quarter cover one 128-byte
// segment. With beta != 0 (dX summed into another consumer's gradient, the last contribution) the old C is read the
// same way and d is the stored sum; the caller then separates these reads from the readout's stores by a barrier.
// Planes [2][stats_P][N] are folded by bn_fold<SRC 0, FIN 1> (dl4j_bn_bwd_planes): bn_bwd_partial's full re-read of dy
// and x disappears. Same wave / lane split as epi_stats_wave. Requires N % 4 == 0, ldc % 4 == 0 (bnb 3: ldc == N),
// no bias / activation (host-checked).
template <int RPP, int BN, int NT, int DTO>
__device__ __forceinline__ void epi_bnbwd_wave(const GemmArgs& g, const char* T, int mrow0, int n0, int tid) {
  constexpr int PITCH = BN * 4 + 16;
  constexpr int PARTS = RPP / 64, SLABS = BN / 64, NW = NT / 64;
  const int lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  const u16* xb = reinterpret_cast<const u16*>(g.bnx);
  const float* ctx = g.bnctx;
  for (int item = w; item < PARTS * SLABS; item += NW) {
    const int part = item / SLABS, slab = item - (item / SLABS) * SLABS;
    const int rbeg = mrow0 + part * 64;
    const long long pidx = rbeg / 64;
    if (pidx >= g.stats_P) continue;
    const int rows = min(64, g.M - rbeg);
    const int col = slab * 64 + 4 * c;
    const int n = n0 + col;
    const bool cok = n < g.N;
    float mu[4], is[4], sc[4], sf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cc = cok ? n + j : 0;
      mu[j] = ctx[cc];
      is[j] = ctx[g.N + cc];
      sc[j] = ctx[2 * g.N + cc];
      sf[j] = ctx[3 * g.N + cc];
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    const int r0 = 16 * q;
    if (cok && rows > r0) {
      // 4 rows per trip (x, old C and mask loads of the 4 in flight together, then consumed): the accumulators of the
      // later epilogue passes are still live here, and 16 rows at once spilled to scratch
      const int nr = min(16, rows - r0);
      const bool acc = g.beta != 0.f;
      const long long row0 = (long long)(rbeg + r0);
      const char* src = T + (part * 64 + r0) * PITCH + col * 4;
      const u16* xp = xb + row0 * g.ldc + n;
      const u16* cp = reinterpret_cast<const u16*>(g.C) + row0 * g.ldc + n;
      const unsigned char* mp = g.bnb == 3 ? g.bnmask + row0 * (g.N >> 3) + (n >> 3) : nullptr;
#pragma unroll 1
      for (int rb = 0; rb < nr; rb += 4) {
        uint2 xv[4], cv[4];
        unsigned mb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rb + i;
          const bool ok = r < nr;
          xv[i] = ok ? *reinterpret_cast<const uint2*>(xp + (long long)r * g.ldc) : make_uint2(0u, 0u);
          cv[i] = (ok && acc) ? *reinterpret_cast<const uint2*>(cp + (long long)r * g.ldc) : make_uint2(0u, 0u);
          mb[i] = (ok && mp) ? ((unsigned)mp[(long long)r * (g.N >> 3)] >> (n & 7)) : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rb + i;
          if (r < nr) {
            const float4 v = *reinterpret_cast<const float4*>(src + r * PITCH);
            const float e[4] = {v.x, v.y, v.z, v.w};
            const unsigned xw[2] = {xv[i].x, xv[i].y};
            const unsigned cw[2] = {cv[i].x, cv[i].y};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const u16 u = (u16)(xw[j >> 1] >> (16 * (j & 1)));
              const float xf = DTO == 2 ? __half2float(__ushort_as_half(u)) : bf2f(u);
              float t = e[j] * g.alpha + 0.f;
              if (acc) {
                const u16 uc = (u16)(cw[j >> 1] >> (16 * (j & 1)));
                t += g.beta * (DTO == 2 ? __half2float(__ushort_as_half(uc)) : bf2f(uc));
              }
              float d = stored_as<DTO>(t);
              if (g.bnb == 2 && !(xf * sc[j] + sf[j] > 0.f)) d = 0.f;
              if (g.bnb == 3 && !((mb[i] >> j) & 1u)) d = 0.f;
              s1[j] += d;
              s2[j] = fmaf(d, (xf - mu[j]) * is[j], s2[j]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], 16);
      s2[j] += __shfl_xor(s2[j], 16);
      s1[j] += __shfl_xor(s1[j], 32);
      s2[j] += __shfl_xor(s2[j], 32);
    }
    if (q == 0 && cok) {
      *reinterpret_cast<float4*>(g.tstats + pidx * g.N + n) = make_float4(s1[0], s1[1], s1[2], s1[3]);
      *reinterpret_cast<float4*>(g.tstats + ((long long)g.stats_P + pidx) * g.N + n) =
          make_float4(s2[0], s2[1], s2[2], s2[3]);
    }
  }
}

// Only in the kernels' BNB instantiations (template flag): its loads in flight would otherwise raise the register
// count, and so cut the occupancy, of every launch of the plain kernels.
template <int RPP, int BN, int NT>
__device__ __forceinline__ void epi_bnbwd(const GemmArgs& g, const char* T, int mrow0, int n0, int tid) {
  static_assert(BN % 64 == 0, "BN-backward statistics need 64-column slabs");
  if (g.out_dt == 2) epi_bnbwd_wave<RPP, BN, NT, 2>(g, T, mrow0, n0, tid);
  else epi_bnbwd_wave<RPP, BN, NT, 1>(g, T, mrow0, n0, tid);
  if (g.beta != 0.f) raw_barrier();   // every wave's reads of the old C precede the readout's stores
}

template <int RPP, int BN, int NT>
__device__ __forceinline__ void epi_stats(const GemmArgs& g, const char* T, int mrow0, int n0, int tid) {
  if constexpr (BN % 64 == 0) {
    if (g.out_dt == 1) epi_stats_wave<RPP, BN, NT, 1>(g, T, mrow0, n0, tid);
    else if (g.out_dt == 2) epi_stats_wave<RPP, BN, NT, 2>(g, T, mrow0, n0, tid);
    else epi_stats_wave<RPP, BN, NT, 0>(g, T, mrow0, n0, tid);
    return;
  }
  constexpr int PITCH = BN * 4 + 16;
  constexpr int PARTS = RPP / 64;
  for (int task = tid; task < PARTS * BN; task += NT) {
    const int col = task % BN, part = task / BN;
    const int n = n0 + col;
    const int rbeg = mrow0 + part * 64;
    if (n >= g.N) continue;
    const long long pidx = rbeg / 64;
    if (pidx >= g.stats_P) continue;
    const int rows = min(64, g.M - rbeg);
    const float bb = g.bias_mode == 1 ? g.bias[n] : 0.f;
    float s1 = 0.f, s2 = 0.f, sh = 0.f;
    // statistics of the values exactly as stored (bf16 or fp16 rounding of the output dtype)
    auto stored = [&](float v) {
      return g.out_dt == 2 ? __half2float(__float2half(v)) : (g.out_dt == 0 ? v : bf2f(to16(v, 1)));
    };
    if (rows > 0) {
      const char* src = T + (part * 64) * PITCH + col * 4;
      sh = stored(*reinterpret_cast<const float*>(src) * g.alpha + bb);
      for (int r = 0; r < rows; ++r) {
        const float d = stored(*reinterpret_cast<const float*>(src + r * PITCH) * g.alpha + bb) - sh;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
    }
    g.tstats[pidx * g.N + n] = s1;
    g.tstats[((long long)g.stats_P + pidx) * g.N + n] = s2;
    g.tstats[(2LL * g.stats_P + pidx) * g.N + n] = sh;
  }
}

// ----------------------------------------------------------------------------------------------- fast kernel
// LDS byte offsets
__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int mc_off(int k, int col) {
  return (col >> 7) * (64 * 256) + k * 256 + (((((col & 127) >> 3) ^ ((k & 3) << 2))) << 4) + (col & 7) * 2;
}

template <int DT, bool KC>
__device__ __forceinline__ typename MfmaT<DT>::v8 read_frag(const char* T, int rbase, int s, int lane) {
  typedef typename MfmaT<DT>::v8 v8;
  if constexpr (KC) {
    const int r = rbase + (lane & 31);
    return *reinterpret_cast<const v8*>(T + kc_off(r, 2 * s + (lane >> 5)));
  } else {
    const int grp = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int col = rbase + (grp & 1) * 16 + 4 * p;
    const int k0 = 16 * s + (grp >> 1) * 8 + q;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + mc_off(k0, col)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + mc_off(k0 + 4, col)));
    s16x8_t f = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8, f);
  }
}

}  // namespace
