// Implicit-GEMM convolution on MFMA (gfx950 / CDNA4), NHWC bf16 activations, fp32 accumulation.
//
// Replaces the reference's im2col + GEMM path (ConvolutionLayer.java:385-417 forward, :215-257 backward) and
// the cuDNN helper (CudnnConvolutionHelper.java:297-306,424-470) with three kernels that never materialise
// im2col in HBM:
//
//   FWD   D[n][m]  = sum_k Wkrsc[n][k] * im2col(X)[m][k]      (+bias[n])  -> Y[m][n]        (NHWC)
//   BWD-D D[c][m'] = sum_k Wflip[c][k] * im2col(dY)[m'][k]               -> dX[m'][c]
//         (stride-1: transposed conv = conv of dY with the flipped CRSK weights and pad' = R-1-pad;
//          1x1 stride-s: plain GEMM over dY rows + strided scatter of the output rows)
//   WRW   dW[k][rsc] = sum_m dY[m][k] * im2col(X)[m][rsc]   (split over m, fp32 atomics straight into the
//         network's flat fp32 gradient in DL4J's [K][C][R][S] order; conv-bias gradient fused as column sums)
//
// GEMM core: 256 threads = 4 waves in a 2x2 arrangement, block tile 128(n) x 128(m) x 32(k), each wave a
// 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators. Operand tiles are register-staged into a
// double-buffered LDS ring (global loads for step k+1 are issued before the MFMAs of step k). K-contiguous
// tiles use an XOR chunk swizzle so every ds_read_b128 lane group hits 16 distinct bank slots; the WRW tiles
// (m-contiguous) are read with ds_read_b64_tr_b16 (hardware transpose) from rows padded to 320 B, which makes
// the 4 rows of each half-wave read land on disjoint banks. Block ids are remapped so that consecutive tiles
// (sharing the weight panel) run on the same XCD (T1).
#include "common.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

struct ConvGeom {
  int N, H, W, C;       // input image (NHWC)
  int OH, OW, K;        // output image / out channels
  int R, S, sh, sw, ph, pw, dh, dw;
};

#define TILE_N 128
#define TILE_M 128
#define TILE_K 32
#define NTHREADS 256

// bijective XCD-aware remap of a linear block id (guide §5, "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Division by a runtime-uniform divisor via multiply-high (CUTLASS-style FastDivmod); valid for n < 2^31.
struct FastDiv {
  unsigned d, mul, shr;
};
static inline FastDiv make_fastdiv(unsigned d) {
  FastDiv f;
  f.d = d;
  if (d == 1) { f.mul = 0; f.shr = 0; return f; }
  unsigned l = 0;
  while ((1u << l) < d) ++l;                       // ceil(log2 d)
  const unsigned p = 31 + l;
  f.mul = (unsigned)(((1ull << p) + d - 1) / d);
  f.shr = p - 32;
  return f;
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

// byte offset of (row, 16-byte chunk) in a swizzled [rows][4 chunks] K-contiguous tile
__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// ------------------------------------------------------------------------------------------------------
// FWD / BWD-DATA kernel.  A operand = weight rows [Nout][Kred] (K contiguous), B operand = im2col pixels.
//   geometry g describes the "input" image the im2col reads (X for fwd, dY for bwd-data) and the output grid.
//   scatter > 0: 1x1 bwd-data with stride `scatter`: output pixel m=(n,oh,ow) goes to row (n, oh*s, ow*s) of
//   an image with dims (g.OH*s', g.OW*s') given by out_H/out_W.
// ------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHREADS) void igemm_fwd_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                                                              const float* __restrict__ bias, bf16* __restrict__ Y,
                                                              ConvGeom g, int Kred, int scatter, int out_H, int out_W,
                                                              int accum, float* __restrict__ tstats) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_N * TILE_K * 2];   // 2 buffers x (A + B) = 32 KB
  const int M = g.N * g.OH * g.OW;
  const int Nout = g.K;
  const int tiles_m = (M + TILE_M - 1) / TILE_M;
  const int tiles_n = (Nout + TILE_N - 1) / TILE_N;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // n-major inside an XCD chunk: consecutive blocks share the pixel panel? -> pixel panels are bigger, so
  // iterate n fastest to reuse the im2col tile from L2 across the Nout tiles.
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  if (tm >= tiles_m) return;
  const int n0 = tn * TILE_N, m0 = tm * TILE_M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wm = wid & 1;

  // ---- per-thread load assignment: 2 rows (r0, r0+64) x chunk c of each 128x32 tile
  const int lrow = tid >> 2, lchunk = tid & 3;
  // weight rows
  const bf16* wrow[2];
  bool wok[2];
  for (int i = 0; i < 2; ++i) {
    const int n = n0 + lrow + 64 * i;
    wok[i] = n < Nout;
    wrow[i] = Wt + (long long)(wok[i] ? n : 0) * Kred;
  }
  // pixel rows: (image n, ih0, iw0)
  int pn[2], pih[2], piw[2];
  bool pok[2];
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + lrow + 64 * i;
    pok[i] = m < M;
    const int mm = pok[i] ? m : 0;
    const int ow = mm % g.OW, t = mm / g.OW;
    const int oh = t % g.OH;
    pn[i] = t / g.OH;
    pih[i] = oh * g.sh - g.ph;
    piw[i] = ow * g.sw - g.pw;
  }
  // k -> (r, s, c) decomposition of this thread's chunk, advanced by TILE_K every step
  int kc = lchunk * 8;
  int cc = kc % g.C, rs = kc / g.C;
  int rr = rs / g.S, ss = rs % g.S;

  f32x16_t acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  uint4 wreg[2], xreg[2];
  const int nk = (Kred + TILE_K - 1) / TILE_K;

  auto gload = [&](int kt) {
    const int k = kt * TILE_K + kc;
    const bool kin = k < Kred;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (wok[i] && kin) wreg[i] = *reinterpret_cast<const uint4*>(wrow[i] + k);
      else wreg[i] = make_uint4(0, 0, 0, 0);
      const int ih = pih[i] + rr * g.dh, iw = piw[i] + ss * g.dw;
      if (pok[i] && kin && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
        xreg[i] = *reinterpret_cast<const uint4*>(X + (((long long)pn[i] * g.H + ih) * g.W + iw) * g.C + cc);
      else xreg[i] = make_uint4(0, 0, 0, 0);
    }
    // advance (r, s, c) by TILE_K for the next step
    cc += TILE_K;
    while (cc >= g.C) { cc -= g.C; if (++ss == g.S) { ss = 0; ++rr; } }
  };
  auto sstore = [&](int buf) {
    char* A = smem + buf * (2 * TILE_N * TILE_K * 2);
    char* B = A + TILE_N * TILE_K * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = lrow + 64 * i;
      *reinterpret_cast<uint4*>(A + swz(row, lchunk)) = wreg[i];
      *reinterpret_cast<uint4*>(B + swz(row, lchunk)) = xreg[i];
    }
  };

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* A = smem + buf * (2 * TILE_N * TILE_K * 2);
    const char* B = A + TILE_N * TILE_K * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 2 + (lane >> 5);
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int row = wn * 64 + a * 32 + (lane & 31);
        af[a] = *reinterpret_cast<const bf16x8_t*>(A + swz(row, chunk));
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int row = wm * 64 + b * 32 + (lane & 31);
        bfr[b] = *reinterpret_cast<const bf16x8_t*>(B + swz(row, chunk));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: D[n][m] -> Y[row(m)][n], 4 consecutive channels per 8-byte store
  const int hh = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int m = m0 + wm * 64 + b * 32 + (lane & 31);
    if (m >= M) continue;
    long long orow;
    if (scatter > 0) {
      const int ow = m % g.OW, t = m / g.OW;
      const int oh = t % g.OH, n = t / g.OH;
      orow = ((long long)n * out_H + oh * scatter) * out_W + ow * scatter;
    } else {
      orow = m;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 64 + a * 32 + 8 * q + 4 * hh;
        if (n >= Nout) continue;
        u16 o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[a][b][4 * q + j];
          if (bias) v += bias[n + j];
          o[j] = f2bf(v);
        }
        if (accum) {                                    // dX += result (fan-out gradient summed in place)
          const uint2 old = *reinterpret_cast<const uint2*>(Y + orow * Nout + n);
          o[0] = f2bf(bf2f(o[0]) + bf2f((u16)(old.x & 0xffff)));
          o[1] = f2bf(bf2f(o[1]) + bf2f((u16)(old.x >> 16)));
          o[2] = f2bf(bf2f(o[2]) + bf2f((u16)(old.y & 0xffff)));
          o[3] = f2bf(bf2f(o[3]) + bf2f((u16)(old.y >> 16)));
        }
        uint2 pk;
        pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
        pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *reinterpret_cast<uint2*>(Y + orow * Nout + n) = pk;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// FWD / BWD-DATA, LDS-DMA pipeline (v2). Same math and output as igemm_fwd_kernel, but operand tiles go
// global -> LDS with global_load_lds_dwordx4 (no VGPR staging) through a G_STAGES-deep ring, so up to
// G_STAGES-1 K-steps of loads are in flight per block. The ResNet convs here have only 2-72 K-steps and
// 100-800 tiles: per-block load latency, not MFMA issue, sets their time, so the pipeline depth is the lever.
// LDS image is lane-linear per wave-instruction (16 rows x 64 B); the XOR chunk swizzle is applied on the
// SOURCE address (lane slot s of row r loads chunk s ^ f(r)) and undone by the same swz() on the read.
// Padding / out-of-range lanes load from a 16-byte zero page, which keeps every DMA unconditional.
// Waits: counted `s_waitcnt vmcnt` (4 DMAs per thread per stage) + raw s_barrier, never __syncthreads() (its
// fence would drain the DMAs still in flight for the next stages).
// ------------------------------------------------------------------------------------------------------
#define G_STAGES 4
#define G_STAGE_BYTES (2 * TILE_N * TILE_K * 2)

__device__ __attribute__((aligned(64))) char g_zero_page[64];

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_stage(int ahead) {
  // ahead = number of later stages whose 4 DMAs/thread may stay in flight
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// FAST (C % TILE_K == 0): every K-step stays inside one filter tap (r, s), so the step's source offset is a
// wave-uniform scalar (SALU) added to a per-lane pixel base, and tap validity is one bit of a per-lane mask —
// the DMA issue costs a handful of VALU ops instead of a division/while-loop/bounds-check chain per step.
template <bool FAST>
__global__ __launch_bounds__(NTHREADS) void igemm_fwd_glds(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                                                            const float* __restrict__ bias, bf16* __restrict__ Y,
                                                            ConvGeom g, int Kred, int scatter, int out_H, int out_W,
                                                            int accum, float* __restrict__ tstats) {
  __shared__ __attribute__((aligned(16))) char smem[G_STAGES * G_STAGE_BYTES];   // 64 KB -> 2 blocks / CU
  const int M = g.N * g.OH * g.OW;
  const int Nout = g.K;
  const int tiles_m = (M + TILE_M - 1) / TILE_M;
  const int tiles_n = (Nout + TILE_N - 1) / TILE_N;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % tiles_n, tm = bid / tiles_n;
  if (tm >= tiles_m) return;
  const int n0 = tn * TILE_N, m0 = tm * TILE_M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wm = wid & 1;

  // DMA assignment: round i covers rows (i*4 + wid)*16 + lane/4, lane slot lane&3 -> source chunk slot^f(row)
  const bf16* wrow[2];
  bool wok[2];
  int chunk[2], pn[2], pih[2], piw[2], cc[2], rr[2], ss[2];
  bool pok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (i * 4 + wid) * 16 + (lane >> 2);
    chunk[i] = (lane & 3) ^ ((row >> 2) & 3);
    const int n = n0 + row;
    wok[i] = n < Nout;
    wrow[i] = Wt + (long long)(wok[i] ? n : 0) * Kred + chunk[i] * 8;
    const int m = m0 + row;
    pok[i] = m < M;
    const int mm = pok[i] ? m : 0;
    const int ow = mm % g.OW, t = mm / g.OW;
    const int oh = t % g.OH;
    pn[i] = t / g.OH;
    pih[i] = oh * g.sh - g.ph;
    piw[i] = ow * g.sw - g.pw;
    const int kc = chunk[i] * 8;
    cc[i] = kc % g.C;
    const int rs = kc / g.C;
    rr[i] = rs / g.S;
    ss[i] = rs % g.S;
  }
  const int nk = (Kred + TILE_K - 1) / TILE_K;
  // FAST-path state: per-lane pixel base offsets + tap-validity masks, uniform tap counters
  long long pbase[2];
  unsigned long long vmask[2];
  if (FAST) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      pbase[i] = (((long long)pn[i] * g.H + pih[i]) * g.W + piw[i]) * g.C + chunk[i] * 8;
      unsigned long long mk = 0;
      for (int r = 0; r < g.R; ++r)
        for (int q = 0; q < g.S; ++q) {
          const int ih = pih[i] + r * g.dh, iw = piw[i] + q * g.dw;
          if (pok[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) mk |= 1ull << (r * g.S + q);
        }
      vmask[i] = mk;
    }
  }
  int u_c = 0, u_rs = 0, u_r = 0, u_s = 0;     // uniform: channel offset and tap of the next step to issue

  auto issue = [&](int kt, int buf) {
    char* A = smem + buf * G_STAGE_BYTES;
    char* B = A + TILE_N * TILE_K * 2;
    if (FAST) {
      const long long uoff = ((long long)(u_r * g.dh) * g.W + u_s * g.dw) * g.C + u_c;
      const int k0 = kt * TILE_K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const void* sa = wok[i] ? (const void*)(wrow[i] + k0) : (const void*)g_zero_page;
        const void* sb = ((vmask[i] >> u_rs) & 1ull) ? (const void*)(X + pbase[i] + uoff) : (const void*)g_zero_page;
        glds16(sa, A + (i * 4 + wid) * 1024);
        glds16(sb, B + (i * 4 + wid) * 1024);
      }
      u_c += TILE_K;
      if (u_c == g.C) { u_c = 0; ++u_rs; if (++u_s == g.S) { u_s = 0; ++u_r; } }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = kt * TILE_K + chunk[i] * 8;
      const bool kin = k < Kred;
      const void* sa = (wok[i] && kin) ? (const void*)(wrow[i] + kt * TILE_K) : (const void*)g_zero_page;
      const int ih = pih[i] + rr[i] * g.dh, iw = piw[i] + ss[i] * g.dw;
      const bool bok = pok[i] && kin && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const void* sb = bok ? (const void*)(X + (((long long)pn[i] * g.H + ih) * g.W + iw) * g.C + cc[i])
                           : (const void*)g_zero_page;
      glds16(sa, A + (i * 4 + wid) * 1024);
      glds16(sb, B + (i * 4 + wid) * 1024);
      cc[i] += TILE_K;
      while (cc[i] >= g.C) { cc[i] -= g.C; if (++ss[i] == g.S) { ss[i] = 0; ++rr[i]; } }
    }
  };

  f32x16_t acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

#pragma unroll
  for (int s = 0; s < G_STAGES - 1; ++s)
    if (s < nk) issue(s, s);

  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(G_STAGES - 2, nk - 1 - kt);
    wait_stage(ahead);
    raw_barrier();
    if (kt + G_STAGES - 1 < nk) issue(kt + G_STAGES - 1, (kt + G_STAGES - 1) % G_STAGES);
    const char* A = smem + (kt % G_STAGES) * G_STAGE_BYTES;
    const char* B = A + TILE_N * TILE_K * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 2 + (lane >> 5);
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = *reinterpret_cast<const bf16x8_t*>(A + swz(wn * 64 + a * 32 + (lane & 31), ch));
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = *reinterpret_cast<const bf16x8_t*>(B + swz(wm * 64 + b * 32 + (lane & 31), ch));
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
  }

  // ---- epilogue through LDS: acc (D[n][m]) -> bf16 tile [m][n] (row pitch 272 B) -> 16-byte coalesced row
  // stores (each output pixel row of the tile is 256 contiguous bytes in NHWC).
  const int hh = lane >> 5;
  if ((Nout & 7) == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();                                   // all waves are done reading the operand ring
    char* T = smem;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ml = wm * 64 + b * 32 + (lane & 31);
#pragma unroll
      for (int a = 0; a < 2; ++a) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int nl = wn * 64 + a * 32 + 8 * q + 4 * hh;
          const int n = n0 + nl;
          u16 o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = acc[a][b][4 * q + j];
            if (bias && n + j < Nout) v += bias[n + j];
            o[j] = f2bf(v);
          }
          uint2 pk;
          pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          *reinterpret_cast<uint2*>(T + ml * 272 + nl * 2) = pk;
        }
      }
    }
    raw_barrier();
    const int ch = tid & 15;
    const int n = n0 + ch * 8;
#pragma unroll 2
    for (int pass = 0; pass < 8; ++pass) {
      const int ml = pass * 16 + (tid >> 4);
      const int m = m0 + ml;
      if (m >= M || n >= Nout) continue;
      long long orow;
      if (scatter > 0) {
        const int ow = m % g.OW, t = m / g.OW;
        const int oh = t % g.OH, nn = t / g.OH;
        orow = ((long long)nn * out_H + oh * scatter) * out_W + ow * scatter;
      } else {
        orow = m;
      }
      uint4 v = *reinterpret_cast<const uint4*>(T + ml * 272 + ch * 16);
      if (accum) {                                      // dX += result: 8 bf16 read-modify-write, fp32 adds
        const uint4 old = *reinterpret_cast<const uint4*>(Y + orow * Nout + n);
        unsigned* pv = reinterpret_cast<unsigned*>(&v);
        const unsigned* po = reinterpret_cast<const unsigned*>(&old);
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
          const u16 lo = f2bf(bf2f((u16)(pv[w2] & 0xffff)) + bf2f((u16)(po[w2] & 0xffff)));
          const u16 hi = f2bf(bf2f((u16)(pv[w2] >> 16)) + bf2f((u16)(po[w2] >> 16)));
          pv[w2] = (unsigned)lo | ((unsigned)hi << 16);
        }
      }
      *reinterpret_cast<uint4*>(Y + orow * Nout + n) = v;
    }
    if (tstats) {
      // BatchNorm statistics of this tile, straight from the bf16 tile in LDS (the exact values BN will read):
      // per (64-row half, channel) shifted sums S1 = sum(y - y0), S2 = sum((y - y0)^2) and the shift y0 (first
      // row of the half). Planes [3][P][Nout], P = 2 * tiles_m; reduced by bn_tiles_reduce (csrc/batchnorm.hip).
      const int col = tid & 127, half = tid >> 7;
      const int nn = n0 + col;
      const int rbeg = half * 64;
      const int rows = min(64, M - (m0 + rbeg));
      const long long P = 2LL * tiles_m;
      const long long pidx = 2LL * tm + half;
      if (nn < Nout) {
        float s1 = 0.f, s2 = 0.f, sh = 0.f;
        if (rows > 0) {
          sh = bf2f(*reinterpret_cast<const u16*>(T + rbeg * 272 + col * 2));
          const char* src = T + rbeg * 272 + col * 2;
          if (rows == 64) {
            float a1 = 0.f, a2 = 0.f;
#pragma unroll 16
            for (int r = 0; r < 64; r += 2) {             // two independent chains, LDS reads batched by unrolling
              const float d0 = bf2f(*reinterpret_cast<const u16*>(src + r * 272)) - sh;
              const float d1 = bf2f(*reinterpret_cast<const u16*>(src + (r + 1) * 272)) - sh;
              s1 += d0;
              s2 = fmaf(d0, d0, s2);
              a1 += d1;
              a2 = fmaf(d1, d1, a2);
            }
            s1 += a1;
            s2 += a2;
          } else {
            for (int r = 0; r < rows; ++r) {
              const float d = bf2f(*reinterpret_cast<const u16*>(src + r * 272)) - sh;
              s1 += d;
              s2 = fmaf(d, d, s2);
            }
          }
        }
        tstats[pidx * Nout + nn] = s1;
        tstats[(P + pidx) * Nout + nn] = s2;
        tstats[(2 * P + pidx) * Nout + nn] = sh;
      }
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int m = m0 + wm * 64 + b * 32 + (lane & 31);
    if (m >= M) continue;
    long long orow;
    if (scatter > 0) {
      const int ow = m % g.OW, t = m / g.OW;
      const int oh = t % g.OH, n = t / g.OH;
      orow = ((long long)n * out_H + oh * scatter) * out_W + ow * scatter;
    } else {
      orow = m;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 64 + a * 32 + 8 * q + 4 * hh;
        if (n >= Nout) continue;
        u16 o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[a][b][4 * q + j];
          if (bias) v += bias[n + j];
          o[j] = f2bf(v);
        }
        if (accum) {                                    // dX += result (fan-out gradient summed in place)
          const uint2 old = *reinterpret_cast<const uint2*>(Y + orow * Nout + n);
          o[0] = f2bf(bf2f(o[0]) + bf2f((u16)(old.x & 0xffff)));
          o[1] = f2bf(bf2f(o[1]) + bf2f((u16)(old.x >> 16)));
          o[2] = f2bf(bf2f(o[2]) + bf2f((u16)(old.y & 0xffff)));
          o[3] = f2bf(bf2f(o[3]) + bf2f((u16)(old.y >> 16)));
        }
        uint2 pk;
        pk.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
        pk.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *reinterpret_cast<uint2*>(Y + orow * Nout + n) = pk;
      }
    }
  }
}

static int g_fwd_variant = 1;   // 1 = LDS-DMA pipeline (default), 0 = register-staged kernel
DL4J_API void dl4j_conv_set_variant(int v) { g_fwd_variant = v; }

#define LAUNCH_FWD(fast, grid, ...)                                                                        \
  do {                                                                                                      \
    if (g_fwd_variant == 1 && (fast))                                                                       \
      hipLaunchKernelGGL(igemm_fwd_glds<true>, grid, dim3(NTHREADS), 0, s, __VA_ARGS__);                    \
    else if (g_fwd_variant == 1) hipLaunchKernelGGL(igemm_fwd_glds<false>, grid, dim3(NTHREADS), 0, s, __VA_ARGS__); \
    else hipLaunchKernelGGL(igemm_fwd_kernel, grid, dim3(NTHREADS), 0, s, __VA_ARGS__);                    \
  } while (0)

// ------------------------------------------------------------------------------------------------------
// WRW: dW[k][rsc] += sum_m dY[m][k] * im2col(X)[m][rsc] over this block's m-range (split-K over pixels).
// Tiles are m-major ([32 m][128 cols], rows padded to 320 B) and read with ds_read_b64_tr_b16.
// ------------------------------------------------------------------------------------------------------
#define WRW_ROW 320

__global__ __launch_bounds__(NTHREADS) void igemm_wrw_kernel(const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                              float* __restrict__ dW, float* __restrict__ db,
                                                              ConvGeom g, int m_per_split, FastDiv fOW, FastDiv fOH,
                                                              int remap, float* __restrict__ part,
                                                              float* __restrict__ partb) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_K * WRW_ROW];   // 2 buffers x (A + B) = 40 KB
  const int M = g.N * g.OH * g.OW;
  const int Kout = g.K;
  const int RSC = g.R * g.S * g.C;
  const int tiles_k = (Kout + TILE_N - 1) / TILE_N;
  // XCD-aware order: logical ids are contiguous per XCD and tile-fastest, so every (k, j) tile of one pixel split
  // runs on the same XCD and the split's dY/X rows are fetched into one L2 instead of one per tile.
  const int hbid = blockIdx.x + blockIdx.y * gridDim.x;
  const int lbid = remap ? xcd_remap(hbid, gridDim.x * gridDim.y) : hbid;
  const int tile = lbid % gridDim.x, split = lbid / gridDim.x;
  const int tk = tile % tiles_k, tj = tile / tiles_k;
  const int k0 = tk * TILE_N, j0 = tj * TILE_M;
  const int mbeg = split * m_per_split;
  int mend = mbeg + m_per_split;
  if (mend > M) mend = M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid >> 1, wj = wid & 1;

  // loads: 32 rows x 16 chunks per tile; thread -> rows (tid>>4) and (tid>>4)+16, chunk tid&15
  const int lrow = tid >> 4, lchunk = tid & 15;
  const int kcol = k0 + lchunk * 8;
  const bool kok = kcol < Kout;
  // fixed im2col column chunk (r, s, c) of this thread
  const int jcol = j0 + lchunk * 8;
  const bool jok = jcol < RSC;
  const int jc = jok ? jcol : 0;
  const int cc = jc % g.C, rs = jc / g.C;
  const int rr = rs / g.S, ss = rs % g.S;
  // pixel rows of this thread (advanced by TILE_K per step; coordinates re-derived with multiply-high division)
  int pm[2];
  for (int i = 0; i < 2; ++i) pm[i] = mbeg + lrow + 16 * i;
  const int rdh = rr * g.dh - g.ph, sdw = ss * g.dw - g.pw;
  float bsum[8];
  const bool do_bias = (db != nullptr || partb != nullptr) && (tj == 0);
  for (int i = 0; i < 8; ++i) bsum[i] = 0.f;

  f32x16_t acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
  uint4 areg[2], breg[2];
  const int nsteps = (mend - mbeg + TILE_K - 1) / TILE_K;

  auto gload = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool mok = pm[i] < mend;
      if (mok && kok) areg[i] = *reinterpret_cast<const uint4*>(dY + (long long)pm[i] * Kout + kcol);
      else areg[i] = make_uint4(0, 0, 0, 0);
      const unsigned mm = mok ? (unsigned)pm[i] : 0u;
      const unsigned t = fdiv(mm, fOW);
      const int ow = (int)(mm - t * fOW.d);
      const unsigned pn = fdiv(t, fOH);
      const int oh = (int)(t - pn * fOH.d);
      const int ih = oh * g.sh + rdh, iw = ow * g.sw + sdw;
      if (mok && jok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
        breg[i] = *reinterpret_cast<const uint4*>(X + (((long long)pn * g.H + ih) * g.W + iw) * g.C + cc);
      else breg[i] = make_uint4(0, 0, 0, 0);
      if (do_bias && mok && kok) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned w = e == 0 ? areg[i].x : e == 1 ? areg[i].y : e == 2 ? areg[i].z : areg[i].w;
          bsum[2 * e] += bf2f((u16)(w & 0xffff));
          bsum[2 * e + 1] += bf2f((u16)(w >> 16));
        }
      }
      pm[i] += TILE_K;                                  // advance this row by 32 pixels
    }
  };
  auto sstore = [&](int buf) {
    char* A = smem + buf * (2 * TILE_K * WRW_ROW);
    char* B = A + TILE_K * WRW_ROW;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = lrow + 16 * i;
      *reinterpret_cast<uint4*>(A + row * WRW_ROW + lchunk * 16) = areg[i];
      *reinterpret_cast<uint4*>(B + row * WRW_ROW + lchunk * 16) = breg[i];
    }
  };
  // transposed fragment read: lanes of 16-group gi read rows kb+4t+q, cols colbase+4p (see T10)
  const int grp = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto frag = [&](const char* T, int colbase, int ks) -> bf16x8_t {
    const int col = colbase + (grp & 1) * 16 + 4 * p;
    const int r0 = ks * 16 + (grp >> 1) * 8 + q;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + r0 * WRW_ROW + col * 2));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + (r0 + 4) * WRW_ROW + col * 2));
    bf16x8_t f;
    const __bf16* l4 = reinterpret_cast<const __bf16*>(&lo);
    const __bf16* h4 = reinterpret_cast<const __bf16*>(&hi);
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] = l4[e]; f[e + 4] = h4[e]; }
    return f;
  };

  if (nsteps > 0) {
    gload();
    sstore(0);
    __syncthreads();
  }
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) gload();
    const char* A = smem + buf * (2 * TILE_K * WRW_ROW);
    const char* B = A + TILE_K * WRW_ROW;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = frag(A, wk * 64 + a * 32, ks);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = frag(B, wj * 64 + b * 32, ks);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (st + 1 < nsteps) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: atomically accumulate into the fp32 dW workspace laid out [K][R][S][C] (j contiguous), so
  // every atomic wave-instruction covers two full 128-byte row segments (the full-rate atomic shape).
  const int hh = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int j = j0 + wj * 64 + b * 32 + (lane & 31);
    if (j >= RSC) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + wk * 64 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (k >= Kout) continue;
        if (part) part[((long long)split * Kout + k) * RSC + j] = acc[a][b][e];   // deterministic: own slab
        else atomicAdd(dW + (long long)k * RSC + j, acc[a][b][e]);
      }
    }
  }
  if (do_bias) {
    // threads sharing a chunk column (same lchunk, 16 row-threads) reduce through LDS
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = bsum[e];
    __syncthreads();
    if (tid < 16) {
      for (int e = 0; e < 8; ++e) {
        float s = 0.f;
        for (int rrow = 0; rrow < 16; ++rrow) s += red[(rrow * 16 + tid) * 8 + e];
        const int k = k0 + tid * 8 + e;
        if (k < Kout) {
          if (partb) partb[(long long)split * Kout + k] = s;
          else atomicAdd(db + k, s);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// WRW, LDS-DMA pipeline (v2): same math/output as igemm_wrw_kernel. Per stage: A = dY[32 m][128 k] and
// B = im2col(X)[32 m][128 j], 256-byte rows, filled by global_load_lds (4 rows per wave-instruction, lane slot s
// of row r holds 16-byte chunk s ^ 2(r&3): the 4 rows a transposed 16-lane read touches then cover 8 distinct
// chunks = 32 distinct banks). Fragments are read with ds_read_b64_tr_b16 exactly as in the v1 kernel.
// Every lane owns one fixed column chunk (fixed filter tap), so the per-step work is one multiply-high pixel
// decode + bounds check per row.
// ------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wrw_addr(int row, int col) {
  return row * 256 + ((((col >> 3) ^ ((row & 3) << 1))) << 4) + (col & 7) * 2;
}

__global__ __launch_bounds__(NTHREADS) void igemm_wrw_glds(const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                            float* __restrict__ dW, float* __restrict__ db,
                                                            ConvGeom g, int m_per_split, FastDiv fOW, FastDiv fOH,
                                                            int remap) {
  __shared__ __attribute__((aligned(16))) char smem[G_STAGES * G_STAGE_BYTES];   // 4 x (8 KB + 8 KB)
  const int M = g.N * g.OH * g.OW;
  const int Kout = g.K;
  const int RSC = g.R * g.S * g.C;
  const int tiles_k = (Kout + TILE_N - 1) / TILE_N;
  // XCD-aware order: logical ids are contiguous per XCD and tile-fastest, so every (k, j) tile of one pixel split
  // runs on the same XCD and the split's dY/X rows are fetched into one L2 instead of one per tile.
  const int hbid = blockIdx.x + blockIdx.y * gridDim.x;
  const int lbid = remap ? xcd_remap(hbid, gridDim.x * gridDim.y) : hbid;
  const int tile = lbid % gridDim.x, split = lbid / gridDim.x;
  const int tk = tile % tiles_k, tj = tile / tiles_k;
  const int k0 = tk * TILE_N, j0 = tj * TILE_M;
  const int mbeg = split * m_per_split;
  int mend = mbeg + m_per_split;
  if (mend > M) mend = M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid >> 1, wj = wid & 1;

  int row[2], kcol[2], cc[2], rdh[2], sdw[2];
  bool kok[2], jok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    row[i] = (i * 4 + wid) * 4 + (lane >> 4);
    const int chunk = (lane & 15) ^ ((row[i] & 3) << 1);
    kcol[i] = k0 + chunk * 8;
    kok[i] = kcol[i] < Kout;
    const int jcol = j0 + chunk * 8;
    jok[i] = jcol < RSC;
    const int jc = jok[i] ? jcol : 0;
    cc[i] = jc % g.C;
    const int rs = jc / g.C;
    rdh[i] = (rs / g.S) * g.dh - g.ph;
    sdw[i] = (rs % g.S) * g.dw - g.pw;
  }
  const int nsteps = (mend - mbeg + TILE_K - 1) / TILE_K;
  const bool do_bias = (db != nullptr) && (tj == 0);
  float bsum = 0.f;

  auto issue = [&](int st, int buf) {
    char* A = smem + buf * G_STAGE_BYTES;
    char* B = A + TILE_K * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mbeg + st * TILE_K + row[i];
      const bool mok = m < mend;
      const void* sa = (mok && kok[i]) ? (const void*)(dY + (long long)m * Kout + kcol[i]) : (const void*)g_zero_page;
      const unsigned mm = mok ? (unsigned)m : 0u;
      const unsigned t = fdiv(mm, fOW);
      const int ow = (int)(mm - t * fOW.d);
      const unsigned pn = fdiv(t, fOH);
      const int oh = (int)(t - pn * fOH.d);
      const int ih = oh * g.sh + rdh[i], iw = ow * g.sw + sdw[i];
      const bool bok = mok && jok[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const void* sb = bok ? (const void*)(X + (((long long)pn * g.H + ih) * g.W + iw) * g.C + cc[i])
                           : (const void*)g_zero_page;
      glds16(sa, A + (i * 4 + wid) * 1024);
      glds16(sb, B + (i * 4 + wid) * 1024);
    }
  };
  const int grp = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto frag = [&](const char* T, int colbase, int ks) -> bf16x8_t {
    const int col = colbase + (grp & 1) * 16 + 4 * p;
    const int r0 = ks * 16 + (grp >> 1) * 8 + q;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + wrw_addr(r0, col)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(T + wrw_addr(r0 + 4, col)));
    bf16x8_t f;
    const __bf16* l4 = reinterpret_cast<const __bf16*>(&lo);
    const __bf16* h4 = reinterpret_cast<const __bf16*>(&hi);
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] = l4[e]; f[e + 4] = h4[e]; }
    return f;
  };

  f32x16_t acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

#pragma unroll
  for (int st = 0; st < G_STAGES - 1; ++st)
    if (st < nsteps) issue(st, st);

  for (int st = 0; st < nsteps; ++st) {
    const int ahead = min(G_STAGES - 2, nsteps - 1 - st);
    wait_stage(ahead);
    raw_barrier();
    if (st + G_STAGES - 1 < nsteps) issue(st + G_STAGES - 1, (st + G_STAGES - 1) % G_STAGES);
    const char* A = smem + (st % G_STAGES) * G_STAGE_BYTES;
    const char* B = A + TILE_K * 256;
    if (do_bias && tid < TILE_N) {                  // conv-bias gradient: column sums of the dY tile
#pragma unroll 8
      for (int r = 0; r < TILE_K; ++r) bsum += bf2f(*reinterpret_cast<const u16*>(A + wrw_addr(r, tid)));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = frag(A, wk * 64 + a * 32, ks);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = frag(B, wj * 64 + b * 32, ks);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
  }

  const int hh = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int j = j0 + wj * 64 + b * 32 + (lane & 31);
    if (j >= RSC) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + wk * 64 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (k < Kout) atomicAdd(dW + (long long)k * RSC + j, acc[a][b][e]);
      }
    }
  }
  if (do_bias && tid < TILE_N && k0 + tid < Kout) atomicAdd(db + k0 + tid, bsum);
}

static int g_wrw_variant = 0;   // v1 register-staged measured faster here (occupancy); v2 kept for A/B
DL4J_API void dl4j_conv_set_wrw_variant(int v) { g_wrw_variant = v; }
static int g_wrw_remap = 1;     // 1 = XCD-aware block order (all tiles of a pixel split on one XCD), 0 = launch order
DL4J_API void dl4j_conv_set_wrw_remap(int v) { g_wrw_remap = v; }

// ------------------------------------------------------------------------------------------------------
// Weight relayout (bf16): W[K][C][R][S] -> Wkrsc[K][R][S][C]  and  Wflip[C][R][S][K] = W[k][c][R-1-r][S-1-s]
// ------------------------------------------------------------------------------------------------------
__global__ void conv_w_relayout(const bf16* __restrict__ W, bf16* __restrict__ krsc, bf16* __restrict__ flip, int K,
                                int C, int R, int S) {
  const long long total = (long long)K * C * R * S;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    int s, r, c, k;
    idx_decomp4(i, S, R, C, s, r, c, k);
    const bf16 v = W[i];
    if (krsc) krsc[(((long long)k * R + r) * S + s) * C + c] = v;
    if (flip) flip[(((long long)c * R + (R - 1 - r)) * S + (S - 1 - s)) * K + k] = v;
  }
}

// Batched relayout of every conv weight of a network in ONE launch (replaces one scattered-write launch per weight
// per direction: ~100 launches/step on ResNet-50). Each job is one (weight, output layout) pair; a block owns 2048
// consecutive OUTPUT elements of one job, so writes are coalesced and the strided source reads hit L2 (a conv
// weight is at most a few MB). Jobs are located by binary search over their first block index.
struct RelayoutJob {
  const bf16* W;
  bf16* out;
  int K, C, R, S;
  int kind;                   // 0: krsc [K][R][S][C]   1: flip [C][R][S][K] (rotated 180 degrees)
  int pad_;
  long long first_block;
  long long n;
};

constexpr int RL_PER_BLOCK = 2048;

__global__ __launch_bounds__(256) void conv_w_relayout_batched(const RelayoutJob* __restrict__ jobs, int njobs) {
  int lo = 0, hi = njobs - 1;
  const long long b = blockIdx.x;
  while (lo < hi) {                       // last job with first_block <= b
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first_block <= b) lo = mid; else hi = mid - 1;
  }
  const RelayoutJob J = jobs[lo];
  const long long base = (b - J.first_block) * RL_PER_BLOCK;
  const int K = J.K, C = J.C, R = J.R, S = J.S;
  for (int t = threadIdx.x; t < RL_PER_BLOCK; t += 256) {
    const long long o = base + t;
    if (o >= J.n) break;
    long long src;
    if (J.kind == 0) {                    // o = ((k*R + r)*S + s)*C + c
      int c, sx, r, k;
      idx_decomp4(o, C, S, R, c, sx, r, k);
      src = (((long long)k * C + c) * R + r) * S + sx;
    } else {                              // o = ((c*R + r')*S + s')*K + k, source tap (R-1-r', S-1-s')
      int k, sx, r, c;
      idx_decomp4(o, K, S, R, k, sx, r, c);
      src = (((long long)k * C + c) * R + (R - 1 - r)) * S + (S - 1 - sx);
    }
    J.out[o] = J.W[src];
  }
}

DL4J_API int dl4j_conv_w_relayout_batched(const void* jobs, int njobs, long long total_blocks, hipStream_t s) {
  if (njobs <= 0) return 0;
  if (total_blocks <= 0 || total_blocks > 0x7FFFFFFF) return -2;
  hipLaunchKernelGGL(conv_w_relayout_batched, dim3((unsigned)total_blocks), dim3(256), 0, s,
                     (const RelayoutJob*)jobs, njobs);
  return (int)hipGetLastError();
}
DL4J_API int dl4j_conv_relayout_job_bytes() { return (int)sizeof(RelayoutJob); }
DL4J_API int dl4j_conv_relayout_per_block() { return RL_PER_BLOCK; }

// LDS-tiled relayout: one block = 64 output channels (k) x 32 input channels (c) x every tap of one weight. The source
// rows W[k][c0 .. c0+32)[taps] are contiguous, so the tile is read with 16-byte loads; both kernel layouts are
// written from LDS with 16-byte stores: krsc rows [k][tap][c0 .. c0+32) (64 B runs) and, when requested, the
// rotated CRSK copy [c][tap'][k0 .. k0+64) (128 B runs). Replaces the element-gather kernel above, whose flip reads
// touched one cache line per element (548 MB read per ResNet-50 step for 47 MB of weights).
struct RelayoutTileJob {
  const bf16* W;
  bf16* krsc;                 // may be null (1x1 weights: the weight itself is already [K][1][1][C])
  bf16* flip;                 // may be null
  int K, C, RS, tiles_c;
  long long first_block;
};
constexpr int RLT_K = 64, RLT_C = 32, RLT_MAX_RS = 16;

__global__ __launch_bounds__(256) void conv_w_relayout_tiled(const RelayoutTileJob* __restrict__ jobs, int njobs) {
  __shared__ __attribute__((aligned(16))) unsigned short T[RLT_K * RLT_C * RLT_MAX_RS];   // 64 KB max
  int lo = 0, hi = njobs - 1;
  const long long b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first_block <= b) lo = mid; else hi = mid - 1;
  }
  const RelayoutTileJob J = jobs[lo];
  const int t = (int)(b - J.first_block);
  const int k0 = (t / J.tiles_c) * RLT_K, c0 = (t % J.tiles_c) * RLT_C;
  const int kw = min(RLT_K, J.K - k0), cw = min(RLT_C, J.C - c0);     // cw % 8 == 0 (host-checked C % 8 == 0)
  const int RS = J.RS;
  const int rowlen = cw * RS;                                        // elements per k row of the tile, % 8 == 0
  const int pitch = RLT_C * RS;                                      // LDS row pitch (elements)
  const unsigned short* W = reinterpret_cast<const unsigned short*>(J.W);
  // load: chunks of 8 elements, row-major over (k, chunk)
  const int cpr = rowlen / 8;
  for (int i = threadIdx.x; i < kw * cpr; i += 256) {
    const int k = i / cpr, ch = i - k * cpr;
    const uint4 v = *reinterpret_cast<const uint4*>(W + ((long long)(k0 + k) * J.C + c0) * RS + ch * 8);
    *reinterpret_cast<uint4*>(T + k * pitch + ch * 8) = v;
  }
  __syncthreads();
  // krsc[k][tap][c]: 8 consecutive c per thread (LDS gather with stride RS)
  if (J.krsc) {
    unsigned short* O = reinterpret_cast<unsigned short*>(J.krsc);
    const int cg = cw / 8;
    for (int i = threadIdx.x; i < kw * RS * cg; i += 256) {
      const int g = i % cg, kt = i / cg;
      const int tap = kt % RS, k = kt / RS;
      unsigned short e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = T[k * pitch + (g * 8 + j) * RS + tap];
      uint4 v;
      v.x = e[0] | ((unsigned)e[1] << 16); v.y = e[2] | ((unsigned)e[3] << 16);
      v.z = e[4] | ((unsigned)e[5] << 16); v.w = e[6] | ((unsigned)e[7] << 16);
      *reinterpret_cast<uint4*>(O + ((long long)(k0 + k) * RS + tap) * J.C + c0 + g * 8) = v;
    }
  }
  // flip[c][tap'][k] = W[k][c][RS-1-tap']: 8 consecutive k per thread (K % 8 == 0 host-checked when flip is set)
  if (J.flip) {
    unsigned short* O = reinterpret_cast<unsigned short*>(J.flip);
    const int kg = kw / 8;
    for (int i = threadIdx.x; i < cw * RS * kg; i += 256) {
      const int g = i % kg, ct = i / kg;
      const int tp = ct % RS, c = ct / RS;
      const int src_tap = RS - 1 - tp;
      unsigned short e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = T[(g * 8 + j) * pitch + c * RS + src_tap];
      uint4 v;
      v.x = e[0] | ((unsigned)e[1] << 16); v.y = e[2] | ((unsigned)e[3] << 16);
      v.z = e[4] | ((unsigned)e[5] << 16); v.w = e[6] | ((unsigned)e[7] << 16);
      *reinterpret_cast<uint4*>(O + ((long long)(c0 + c) * RS + tp) * J.K + k0 + g * 8) = v;
    }
  }
}

DL4J_API int dl4j_conv_w_relayout_tiled(const void* jobs, int njobs, long long total_blocks, hipStream_t s) {
  if (njobs <= 0) return 0;
  if (total_blocks <= 0 || total_blocks > 0x7FFFFFFF) return -2;
  hipLaunchKernelGGL(conv_w_relayout_tiled, dim3((unsigned)total_blocks), dim3(256), 0, s,
                     (const RelayoutTileJob*)jobs, njobs);
  return (int)hipGetLastError();
}
DL4J_API int dl4j_conv_relayout_tile_job_bytes() { return (int)sizeof(RelayoutTileJob); }
DL4J_API int dl4j_conv_relayout_tile_max_rs() { return RLT_MAX_RS; }

// ------------------------------------------------------------------------------------------------------ API
static inline ConvGeom mk(int N, int H, int W, int C, int OH, int OW, int K, int R, int S, int sh, int sw, int ph, int pw,
                          int dh, int dw) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw;
  return g;
}

DL4J_API int dl4j_conv_w_relayout(const void* W, void* krsc, void* flip, int K, int C, int R, int S, hipStream_t s) {
  const long long total = (long long)K * C * R * S;
  long long gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(conv_w_relayout, dim3((unsigned)gsz), dim3(256), 0, s, (const bf16*)W, (bf16*)krsc, (bf16*)flip,
                     K, C, R, S);
  return (int)hipGetLastError();
}

// Forward: X NHWC [N,H,W,C] bf16, Wkrsc [K][R*S*C], bias fp32 [K] or null, Y NHWC [N,OH,OW,K].
// tstats (optional, fp32 [3][2*ceil(M/128)][K]): per-tile BatchNorm partial statistics of Y. Returns 1 when they
// were written, 0 when not (unsupported variant), a HIP error code otherwise.
DL4J_API int dl4j_conv_fwd(const void* X, const void* Wkrsc, const float* bias, void* Y, int N, int H, int W, int C,
                           int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW,
                           float* tstats, hipStream_t s) {
  if (C % 8 != 0 || K % 4 != 0) return -1;
  ConvGeom g = mk(N, H, W, C, OH, OW, K, R, S, sh, sw, ph, pw, dh, dw);
  const long long M = (long long)N * OH * OW;
  const int tiles = (int)(((M + TILE_M - 1) / TILE_M) * ((K + TILE_N - 1) / TILE_N));
  const int stats_ok = tstats != nullptr && g_fwd_variant == 1 && C % TILE_K == 0 && R * S <= 64 && K % 8 == 0;
  LAUNCH_FWD(C % TILE_K == 0 && R * S <= 64, dim3(tiles), (const bf16*)X, (const bf16*)Wkrsc, bias, (bf16*)Y, g, R * S * C, 0, 0, 0,
             0, stats_ok ? tstats : nullptr);
  const int e = (int)hipGetLastError();
  return e != 0 ? e : (stats_ok ? 1 : 0);
}

// Backward data, stride 1: dX[N,H,W,C] = conv(dY[N,OH,OW,K], Wflip[C][R][S][K], pad' = (R-1-ph, S-1-pw)).
// accum != 0: dX += result (dX already holds another consumer's gradient of the same tensor).
DL4J_API int dl4j_conv_bwd_data_s1(const void* dY, const void* Wflip, void* dX, int N, int H, int W, int C, int K,
                                   int R, int S, int ph, int pw, int OH, int OW, int accum, hipStream_t s) {
  if (K % 8 != 0 || C % 4 != 0) return -1;
  // "input" image = dY (OH x OW x K); output grid = H x W x C; kernel R x S stride 1, pad R-1-ph
  ConvGeom g = mk(N, OH, OW, K, H, W, C, R, S, 1, 1, R - 1 - ph, S - 1 - pw, 1, 1);
  const long long M = (long long)N * H * W;
  const int tiles = (int)(((M + TILE_M - 1) / TILE_M) * ((C + TILE_N - 1) / TILE_N));
  LAUNCH_FWD(K % TILE_K == 0 && R * S <= 64, dim3(tiles), (const bf16*)dY, (const bf16*)Wflip, (const float*)nullptr,
             (bf16*)dX, g, R * S * K, 0, 0, 0, accum, (float*)nullptr);
  return (int)hipGetLastError();
}

// Backward data, 1x1 kernel, stride s, no padding: dX (pre-zeroed) rows (n, oh*s, ow*s) = dY rows x Wflip[C][K].
DL4J_API int dl4j_conv_bwd_data_1x1(const void* dY, const void* Wflip, void* dX, int N, int H, int W, int C, int K,
                                    int stride, int OH, int OW, int accum, hipStream_t s) {
  if (K % 8 != 0 || C % 4 != 0) return -1;
  ConvGeom g = mk(N, OH, OW, K, OH, OW, C, 1, 1, 1, 1, 0, 0, 1, 1);
  const long long M = (long long)N * OH * OW;
  const int tiles = (int)(((M + TILE_M - 1) / TILE_M) * ((C + TILE_N - 1) / TILE_N));
  LAUNCH_FWD(K % TILE_K == 0, dim3(tiles), (const bf16*)dY, (const bf16*)Wflip, (const float*)nullptr, (bf16*)dX, g, K,
             stride, H, W, accum, (float*)nullptr);
  return (int)hipGetLastError();
}

// KRSC fp32 workspace -> DL4J [K][C][R][S] fp32 gradient view. With rezero the workspace is cleared as it is
// read, so a cached workspace is already zero for the next atomic accumulation (no separate memset launch).
__global__ void conv_wrw_permute(float* __restrict__ ws, float* __restrict__ dW, int K, int C, int R, int S,
                                 int rezero) {
  const long long total = (long long)K * C * R * S;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c, s, r, k;
    idx_decomp4(i, C, S, R, c, s, r, k);
    dW[(((long long)k * C + c) * R + r) * S + s] = ws[i];
    if (rezero) ws[i] = 0.f;
  }
}

DL4J_API int dl4j_conv_wrw_permute(float* ws, float* dW, int K, int C, int R, int S, int rezero, hipStream_t s) {
  const long long total = (long long)K * C * R * S;
  long long gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(conv_wrw_permute, dim3((unsigned)gsz), dim3(256), 0, s, ws, dW, K, C, R, S, rezero);
  return (int)hipGetLastError();
}

// Weight gradient: dW fp32 workspace [K][R][S][C] (pre-zeroed, accumulated atomically; equal to the DL4J layout
// when R == S == 1), db fp32 [K] (pre-zeroed) or null.
DL4J_API int dl4j_conv_wrw(const void* X, const void* dY, float* dW, float* db, int N, int H, int W, int C, int K,
                           int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW, int splits,
                           hipStream_t s) {
  if (C % 8 != 0 || K % 8 != 0) return -1;
  ConvGeom g = mk(N, H, W, C, OH, OW, K, R, S, sh, sw, ph, pw, dh, dw);
  const int M = N * OH * OW;
  const int RSC = R * S * C;
  const int tiles = ((K + TILE_N - 1) / TILE_N) * ((RSC + TILE_M - 1) / TILE_M);
  if (splits <= 0) {
    // ~1.5 workgroups per CU in total (measured sweet spot between fill and atomic traffic, tools/conv_bench.py
    // --sweep-wrw); every split keeps >= 8 k-steps so the atomic epilogue stays amortised
    splits = (384 + tiles - 1) / tiles;
    const int maxs = (M + 8 * TILE_K - 1) / (8 * TILE_K);
    if (splits > maxs) splits = maxs;
    if (splits < 1) splits = 1;
  }
  int mps = (M + splits - 1) / splits;
  mps = (mps + TILE_K - 1) / TILE_K * TILE_K;
  splits = (M + mps - 1) / mps;
  if (g_wrw_variant == 1)
    hipLaunchKernelGGL(igemm_wrw_glds, dim3(tiles, splits), dim3(NTHREADS), 0, s, (const bf16*)X, (const bf16*)dY, dW,
                       db, g, mps, make_fastdiv((unsigned)OW), make_fastdiv((unsigned)OH), g_wrw_remap);
  else
    hipLaunchKernelGGL(igemm_wrw_kernel, dim3(tiles, splits), dim3(NTHREADS), 0, s, (const bf16*)X, (const bf16*)dY, dW,
                       db, g, mps, make_fastdiv((unsigned)OW), make_fastdiv((unsigned)OH), g_wrw_remap,
                       (float*)nullptr, (float*)nullptr);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------------
// Deterministic weight gradient (DL4J_AMD_DETERMINISTIC=1; the reference's cuDNN helper offers deterministic
// backward-filter algorithms, CudnnConvolutionHelper.java:179-246). Every pixel split writes its own fp32 slab
// part[split][K][R*S*C] with plain stores (no atomics), then conv_wrw_reduce sums the slabs in split order and
// writes the DL4J [K][C][R][S] layout directly (no KRSC workspace / permute). Bitwise reproducible run to run.
// ------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_wrw_reduce(const float* __restrict__ part, const float* __restrict__ partb,
                                                       float* __restrict__ dW, float* __restrict__ db, int splits,
                                                       int K, int C, int RS) {
  const long long total = (long long)K * C * RS;
  const long long plane = total;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    // o indexes the DL4J layout [k][c][rs]; the slab layout is [k][rs][c]
    const int rs = (int)(o % RS);
    const long long t = o / RS;
    const int c = (int)(t % C);
    const long long k = t / C;
    const long long src = (k * RS + rs) * C + c;
    float a = 0.f;
    for (int sp = 0; sp < splits; ++sp) a += part[sp * plane + src];
    dW[o] = a;
  }
  if (db && blockIdx.x == 0) {
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      float a = 0.f;
      for (int sp = 0; sp < splits; ++sp) a += partb[(long long)sp * K + k];
      db[k] = a;
    }
  }
}

// Split count / slab sizes the deterministic path will use (host sizes the scratch from these).
DL4J_API long long dl4j_conv_wrw_det_floats(int N, int C, int K, int R, int S, int OH, int OW, int splits) {
  const int M = N * OH * OW;
  const int RSC = R * S * C;
  const int tiles = ((K + TILE_N - 1) / TILE_N) * ((RSC + TILE_M - 1) / TILE_M);
  if (splits <= 0) {
    splits = (384 + tiles - 1) / tiles;
    const int maxs = (M + 8 * TILE_K - 1) / (8 * TILE_K);
    if (splits > maxs) splits = maxs;
    if (splits < 1) splits = 1;
  }
  int mps = (M + splits - 1) / splits;
  mps = (mps + TILE_K - 1) / TILE_K * TILE_K;
  splits = (M + mps - 1) / mps;
  return (long long)splits * K * (RSC + 1);
}

// dW: DL4J-layout fp32 [K][C][R][S] (written, not accumulated); db fp32 [K] or null; part: >= dl4j_conv_wrw_det_floats.
DL4J_API int dl4j_conv_wrw_det(const void* X, const void* dY, float* dW, float* db, float* part, int N, int H, int W,
                               int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH,
                               int OW, int splits, hipStream_t s) {
  if (C % 8 != 0 || K % 8 != 0) return -1;
  ConvGeom g = mk(N, H, W, C, OH, OW, K, R, S, sh, sw, ph, pw, dh, dw);
  const int M = N * OH * OW;
  const int RSC = R * S * C;
  const int tiles = ((K + TILE_N - 1) / TILE_N) * ((RSC + TILE_M - 1) / TILE_M);
  if (splits <= 0) {
    splits = (384 + tiles - 1) / tiles;
    const int maxs = (M + 8 * TILE_K - 1) / (8 * TILE_K);
    if (splits > maxs) splits = maxs;
    if (splits < 1) splits = 1;
  }
  int mps = (M + splits - 1) / splits;
  mps = (mps + TILE_K - 1) / TILE_K * TILE_K;
  splits = (M + mps - 1) / mps;
  float* partb = part + (long long)splits * K * RSC;
  hipLaunchKernelGGL(igemm_wrw_kernel, dim3(tiles, splits), dim3(NTHREADS), 0, s, (const bf16*)X, (const bf16*)dY,
                     (float*)nullptr, (float*)nullptr, g, mps, make_fastdiv((unsigned)OW), make_fastdiv((unsigned)OH),
                     g_wrw_remap, part, db ? partb : (float*)nullptr);
  // a split whose pixel range is empty never stores: only possible when splits > ceil(M / mps), excluded above
  const long long total = (long long)K * RSC;
  long long gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(conv_wrw_reduce, dim3((unsigned)gsz), dim3(256), 0, s, part, partb, dW, db, splits, K, C, R * S);
  return (int)hipGetLastError();
}
