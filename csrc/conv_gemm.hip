// Implicit-GEMM convolution on the LDS-DMA MFMA tile engine (gfx950 / CDNA4), round-3 kernel.
//
// Same contract as the forward / stride-1 backward-data kernels of csrc/conv_igemm.hip (reference math:
// ConvolutionLayer.java:385-417 forward im2col + GEMM, :215-257 backward; cuDNN helper CudnnConvolutionHelper.java:
// 297-306,424-470), re-tiled for the hardware:
//
//   Y[m][n] = sum_k im2col(X)[m][k] * Wkrsc[n][k]  (+bias[n]) (+beta*Y)     m = pixel (NHWC row), n = out channel
//
// Why a second kernel: the round-2 kernel's 128x128x32 tile fetches 64-byte row pieces (half cache lines) and, on the
// many 64-channel ResNet layers, spends half its MFMAs on padding columns; its 3x3 convs ran at 4-5x their compute
// floor (profiles/r2_conv_bench_bs512_tuned_wrw.log). Here:
//   * K-steps are 64 deep (C % 64 == 0), so every im2col row piece is one whole 128-byte line of one pixel and one
//     filter tap: the tap / channel offset of a step is wave-uniform (SALU), the per-lane part is a fixed pixel base
//     plus one validity bit per tap (mask computed once per block);
//   * BM x BN tiles are template parameters (256x128, 128x128, 256x64, 128x64, 128x256), chosen per shape by the host
//     (first-call timing, ops/conv_native.py), so 64-channel layers run a 64-wide tile with no dead columns;
//   * operands go global -> LDS with global_load_lds_dwordx4 through a STAGES-deep ring with counted vmcnt waits and
//     raw s_barrier (guide §5 "Pipelining across barriers"); fragments, swizzles and the LDS epilogue (bias, beta
//     accumulation for fan-out gradients, 16-byte row stores, BatchNorm tile statistics) are the GEMM's (mfma_tile.h);
//   * bf16 or fp16 operands (v_mfma_f32_32x32x16_{bf16,f16}).
#include "mfma_tile.h"

namespace {

struct ConvA {
  const void* X;             // NHWC activations of the im2col operand
  int N, H, W, C;            // image
  int OH, OW;                // output grid (rows of the GEMM = N*OH*OW)
  int R, S, sh, sw, ph, pw, dh, dw;
};

template <int DT, int BM, int BN, int WGM, int WGN, int STAGES, bool BNB = false, bool LEAN = false>
__global__ __launch_bounds__(WGM* WGN * 64, 2) void conv_glds(GemmArgs g, ConvA ca) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, SBYTES = ABYTES + BBYTES;
  constexpr int NIA = BM / 8 / NW, NIB = BN / 8 / NW;     // 1-KB DMA instructions per wave per stage
  static_assert(NIA * NW * 8 == BM && NIB * NW * 8 == BN, "tile / wave count mismatch");
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile below one 32x32 fragment");
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SBYTES];

  // grouped, XCD-aware raster: consecutive ids of one XCD walk 8 pixel panels x all channel panels
  const int per_group = 8 * g.tiles_n;
  const int bid = xcd_remap_g(blockIdx.x, gridDim.x);
  const int grp_id = bid / per_group, first_m = grp_id * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int in_g = bid - grp_id * per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = g.K / 64;                                 // K = R*S*C, C % 64 == 0 (host-checked)

  typedef unsigned short E;
  const E* X = reinterpret_cast<const E*>(ca.X);
  const E* Wt = reinterpret_cast<const E*>(g.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // ---- A (im2col) per-lane state: pixel base offset of (n, oh*sh-ph, ow*sw-pw) + the lane's 16-byte chunk, and a
  // bit per filter tap telling whether that tap's input pixel is inside the image
  int pbase[NIA];
  unsigned long long vmask[NIA];
#pragma unroll
  for (int j = 0; j < NIA; ++j) {
    const int i = wid + NW * j;
    const int row = 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    const int m = m0 + row;
    const bool ok = m < g.M;
    const int mm = ok ? m : 0;
    const int ow = mm % ca.OW, t = mm / ca.OW;
    const int oh = t % ca.OH, n = t / ca.OH;
    const int ih0 = oh * ca.sh - ca.ph, iw0 = ow * ca.sw - ca.pw;
    pbase[j] = ((n * ca.H + ih0) * ca.W + iw0) * ca.C + ch * 8;
    unsigned long long mk = 0;
    if (ok) {
      for (int r = 0; r < ca.R; ++r) {
        const int ih = ih0 + r * ca.dh;
        if (ih < 0 || ih >= ca.H) continue;
        for (int q = 0; q < ca.S; ++q) {
          const int iw = iw0 + q * ca.dw;
          if (iw >= 0 && iw < ca.W) mk |= 1ull << (r * ca.S + q);
        }
      }
    }
    vmask[j] = mk;
  }
  // ---- B (weights [Nout][K], K-contiguous)
  const E* bp[NIB];
  bool bok[NIB];
#pragma unroll
  for (int j = 0; j < NIB; ++j) {
    const int i = wid + NW * j;
    const int row = 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    bok[j] = n0 + row < g.N;
    bp[j] = Wt + (long long)(bok[j] ? n0 + row : 0) * g.ldb + ch * 8;
  }

  // uniform im2col walk: channel offset and tap of the next K-step to issue
  int u_c = 0, u_rs = 0, u_r = 0, u_s = 0;
  auto issue = [&](int kt, int st) {
    char* sa = smem + st * SBYTES;
    char* sb = sa + ABYTES;
    const int uoff = (u_r * ca.dh * ca.W + u_s * ca.dw) * ca.C + u_c;
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const void* src = ((vmask[j] >> u_rs) & 1ull) ? (const void*)(X + pbase[j] + uoff) : (const void*)gemm_zero_page;
      glds16(src, sa + (wid + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const void* src = bok[j] ? (const void*)(bp[j] + kt * 64) : (const void*)gemm_zero_page;
      glds16(src, sb + (wid + NW * j) * 1024);
    }
    u_c += 64;
    if (u_c == ca.C) {
      u_c = 0;
      ++u_rs;
      if (++u_s == ca.S) { u_s = 0; ++u_r; }
    }
  };

  const int wm = wid / WGN, wn = wid % WGN;
  f32x16_t acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);

  constexpr int LPS = NIA + NIB;
  for (int kt = 0; kt < nk; ++kt) {
    if (STAGES > 2 && kt + 1 < nk) wait_vm<(STAGES > 2 ? (STAGES - 2) * LPS : 0)>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* sa = smem + (kt % STAGES) * SBYTES;
    const char* sb = sa + ABYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v8 fm[FM], fn[FN];
#pragma unroll
      for (int b = 0; b < FM; ++b) fm[b] = read_frag<DT, true>(sa, wm * WTM + 32 * b, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a) fn[a] = read_frag<DT, true>(sb, wn * WTN + 32 * a, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b) acc[a][b] = MfmaT<DT>::mma(fn[a], fm[b], acc[a][b]);
    }
  }

  if constexpr (LEAN) {
    // lean epilogue (mfma_tile.h): one 16-bit image of the tile, BN statistics from it, 16-byte row stores
    static_assert(BM * BN * 2 <= STAGES * SBYTES, "lean image exceeds the operand ring");
    const int h = lane >> 5;
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
#pragma unroll
    for (int a = 0; a < FN; ++a)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
        float4 bq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g.bias_mode == 1 && n0 + lc < g.N) bq = *reinterpret_cast<const float4*>(g.bias + n0 + lc);
#pragma unroll
        for (int b = 0; b < FM; ++b)
          lean_put4<BN>(smem, wm * WTM + 32 * b + (lane & 31), lc, acc[a][b][4 * q] + bq.x, acc[a][b][4 * q + 1] + bq.y,
                        acc[a][b][4 * q + 2] + bq.z, acc[a][b][4 * q + 3] + bq.w, g.out_dt);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (g.tstats) lean_stats<BM, BN, NW * 64>(g, smem, m0, n0, tid);
    lean_readout<BM, BN, NW * 64>(g, reinterpret_cast<char*>(g.C), smem, m0, n0, tid);
    return;
  }
  // ---- epilogue through LDS (mfma_tile.h epi_readout / epi_stats)
  constexpr int PITCH = BN * 4 + 16;
  constexpr int RPP0 = (STAGES * SBYTES) / PITCH;
  constexpr int RPP = RPP0 >= BM ? BM : (RPP0 >= BM / 2 ? BM / 2 : BM / 4);
  static_assert(RPP >= 64 && RPP % 64 == 0, "epilogue pass too small");
  const int h = lane >> 5;
  EpiOut o;
  o.coh = false;
  o.raw = false;
  o.dt = g.out_dt;
  o.dst = reinterpret_cast<char*>(g.C);
  o.ld = g.ldc;
  o.vec = g.coalesce != 0;
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int P = 0; P < BM / RPP; ++P) {
    sfor<0, FM>([&](auto B_) {
      constexpr int b = decltype(B_)::value;
      const int r0 = wm * WTM + 32 * b;
      if (r0 / RPP == P) {
        const int lr = r0 - P * RPP + (lane & 31);
        sfor<0, FN>([&](auto A_) {
          constexpr int a = decltype(A_)::value;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
            *reinterpret_cast<float4*>(smem + lr * PITCH + lc * 4) =
                make_float4(acc[a][b][4 * q], acc[a][b][4 * q + 1], acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]);
          }
        });
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if constexpr (BNB) epi_bnbwd<RPP, BN, NW * 64>(g, smem, m0 + P * RPP, n0, tid);
    else if (g.tstats) epi_stats<RPP, BN, NW * 64>(g, smem, m0 + P * RPP, n0, tid);
    epi_readout<RPP, BN, NW * 64>(g, o, nullptr, smem, m0 + P * RPP, n0, tid);
    if (P + 1 < BM / RPP) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
  }
}

struct TileCfg {
  int bm, bn;
};
// variant ids (kept stable: the host caches its per-shape choice by id)
//   0: 256x128, 8 waves 4x2, 3 stages     1: 128x128, 4 waves 2x2, 2 stages (2 blocks / CU)
//   2: 256x64,  4 waves 4x1, 3 stages     3: 128x64,  4 waves 2x2, 3 stages (2 blocks / CU)
//   4: 128x256, 8 waves 2x4, 3 stages
constexpr int kNumVariants = 5;
const TileCfg kTiles[kNumVariants] = {{256, 128}, {128, 128}, {256, 64}, {128, 64}, {128, 256}};

template <int DT, bool BNB, bool LEAN>
int launch_conv_t(int v, const GemmArgs& g, const ConvA& ca, hipStream_t s) {
  dim3 grid(g.tiles_m * g.tiles_n);
  switch (v) {
    case 0: hipLaunchKernelGGL((conv_glds<DT, 256, 128, 4, 2, 3, BNB, LEAN>), grid, dim3(512), 0, s, g, ca); break;
    case 1: hipLaunchKernelGGL((conv_glds<DT, 128, 128, 2, 2, 2, BNB, LEAN>), grid, dim3(256), 0, s, g, ca); break;
    case 2: hipLaunchKernelGGL((conv_glds<DT, 256, 64, 4, 1, 3, BNB, LEAN>), grid, dim3(256), 0, s, g, ca); break;
    case 3: hipLaunchKernelGGL((conv_glds<DT, 128, 64, 2, 2, 3, BNB, LEAN>), grid, dim3(256), 0, s, g, ca); break;
    default: hipLaunchKernelGGL((conv_glds<DT, 128, 256, 2, 4, 3, BNB, LEAN>), grid, dim3(512), 0, s, g, ca); break;
  }
  return (int)hipGetLastError();
}

// lean epilogue (mfma_tile.h): plain or biased 16-bit output, optional BN tile statistics; the fan-out beta
// accumulation and the BN-backward sums keep the generic LDS epilogue
bool conv_lean_ok(const GemmArgs& g) {
  static const int off = [] {
    const char* e = getenv("DL4J_AMD_GEMM_LEAN");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  if (off || g.bnb || g.beta != 0.f || g.act != 0) return false;
  if (g.bias_mode == 1 && (reinterpret_cast<uintptr_t>(g.bias) & 15)) return false;
  return (g.N & 7) == 0 && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0;
}

template <int DT>
int launch_conv(int v, const GemmArgs& g, const ConvA& ca, hipStream_t s) {
  if (g.bnb) return launch_conv_t<DT, true, false>(v, g, ca, s);
  return conv_lean_ok(g) ? launch_conv_t<DT, false, true>(v, g, ca, s) : launch_conv_t<DT, false, false>(v, g, ca, s);
}

// Default tile when the host has no timing for the shape: the largest tile whose width fits the channel count and
// that still gives >= one block per CU.
int default_variant(long long M, int Nout) {
  const int order64[] = {2, 3};
  const int order128[] = {0, 1};
  const int order256[] = {4, 0, 1};
  const int* ord;
  int n;
  if (Nout <= 64) { ord = order64; n = 2; }
  else if (Nout <= 128) { ord = order128; n = 2; }
  else { ord = order256; n = 3; }
  for (int i = 0; i < n; ++i) {
    const TileCfg t = kTiles[ord[i]];
    const long long tiles = ((M + t.bm - 1) / t.bm) * ((Nout + t.bn - 1) / t.bn);
    if (tiles >= 256) return ord[i];
  }
  return ord[n - 1];
}

}  // namespace

DL4J_API int dl4j_conv_v3_num_variants() { return kNumVariants; }
DL4J_API int dl4j_conv_v3_default_variant(long long M, int Nout) { return default_variant(M, Nout); }

// Y[N,OH,OW,K] (NHWC) = conv(X[N,H,W,C] NHWC, Wkrsc[K][R][S][C]) (+bias fp32[K]) (+beta * Y).
// dt: 1 bf16, 2 fp16 (X, W, Y all of it). tstats (optional): fp32 [3][ceil(M/64)][K] BatchNorm partials of Y
// (64-row partials, bn_tiles_reduce with rpp 64). variant < 0: default_variant. Also used for stride-1 backward-data
// (X = dY, W = flipped CRSK weights, pad' = R-1-pad). Returns 0, -1 when the shape is not supported (C % 64, K % 8,
// 32-bit offsets, R*S > 64), or a HIP error.
DL4J_API int dl4j_conv_fwd_v3(int dt, const void* X, const void* Wkrsc, const float* bias, void* Y, int N, int H, int W,
                              int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW,
                              float beta, float* tstats, int variant, hipStream_t s) {
  if ((dt != 1 && dt != 2) || C % 64 != 0 || K % 8 != 0 || R * S > 64 || R < 1 || S < 1) return -1;
  const long long M = (long long)N * OH * OW;
  if ((long long)N * H * W * C >= 0x7fffffffLL || M * K >= 0x7fffffffLL || M <= 0) return -1;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Wkrsc) & 15) ||
      (reinterpret_cast<uintptr_t>(Y) & 15))
    return -1;
  if (variant < 0 || variant >= kNumVariants) variant = default_variant(M, K);
  GemmArgs g = {};
  g.B = Wkrsc;
  g.C = Y;
  g.bias = bias;
  g.ldb = (long long)R * S * C;
  g.ldc = K;
  g.M = (int)M;
  g.N = K;
  g.K = R * S * C;
  g.kps = g.K;
  g.splits = 1;
  g.alpha = 1.f;
  g.beta = beta;
  g.bias_mode = bias ? 1 : 0;
  g.act = 0;
  g.out_dt = dt;
  g.tiles_m = (int)((M + kTiles[variant].bm - 1) / kTiles[variant].bm);
  g.tiles_n = (K + kTiles[variant].bn - 1) / kTiles[variant].bn;
  g.coalesce = 1;                                   // K % 8 == 0 and a 16-byte aligned Y: 16-byte row stores
  g.store_nt = store_nt_for(M * K * 2);
  g.tstats = tstats;
  g.stats_P = tstats ? (int)((M + 63) / 64) : 0;
  if (tstats && bnb_armed().mode) {                 // BN-backward sums of dX (stride-1 bwd-data as a transposed conv)
    if (bias || K % 4 != 0) return -1;             // beta != 0: sums of the stored dX + beta*Y (fan-out)
    g.bnx = bnb_armed().x;
    g.bnctx = bnb_armed().ctx;
    g.bnmask = bnb_armed().mask;
    g.bnb = bnb_armed().mode;
  }
  ConvA ca;
  ca.X = X;
  ca.N = N; ca.H = H; ca.W = W; ca.C = C; ca.OH = OH; ca.OW = OW;
  ca.R = R; ca.S = S; ca.sh = sh; ca.sw = sw; ca.ph = ph; ca.pw = pw; ca.dh = dh; ca.dw = dw;
  return dt == 1 ? launch_conv<1>(variant, g, ca, s) : launch_conv<2>(variant, g, ca, s);
}

// ==================================================================================================================
// Weight gradient on the same tile engine:  dW[k][j] = sum_m dY[m][k] * im2col(X)[m][j],  j = (r*S + s)*C + c.
// GEMM rows = output channels k (A = dY, M-contiguous: pixels are the reduction), columns = j (B = im2col(X),
// N-contiguous), reduction = pixels in 64-deep steps, split over grid.y into pixel ranges. Each split writes its fp32
// tile into its own slab part[split][K][RSC] (plain 16-byte stores via the LDS epilogue, no float atomics); the fixed-
// order reduce (conv_wrw_reduce, csrc/conv_igemm.hip) sums the slabs and writes the DL4J [K][C][R][S] layout straight
// into the flat gradient view: deterministic, and no separate permute / zeroing pass (the round-2 kernel's fp32
// atomics ran at ~1.3 TB/s and needed both).
// Fragments of both operands are transposed reads (ds_read_b64_tr_b16) of the M/N-contiguous LDS images. They are
// issued as inline asm: the builtin makes hipcc treat the read as aliasing the in-flight LDS-DMA stages and drain them
// (vmcnt(0)) before every read. Reads for sub-step s+1 are issued before the MFMAs of s (counted lgkmcnt + a
// sched_barrier after the wait, guide §5.4 rule 18).
// ==================================================================================================================
namespace {

// division by a runtime-uniform divisor via multiply-high (valid for n < 2^31)
struct FastDiv {
  unsigned d, mul, shr;
};
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

struct WrwGeom {
  const void* X;        // NHWC input
  const void* dY;       // NHWC output gradient
  int N, H, W, C, OH, OW, K;
  int R, S, sh, sw, ph, pw, dh, dw;
  int M;                // N*OH*OW
  int RSC;
  int mps;              // pixels per split (multiple of 64)
  FastDiv fOW, fOH;
  float* partb;         // conv-bias gradient partials [splits][K] (extra bias-only blocks), or null
};

template <int DT>
__device__ __forceinline__ typename MfmaT<DT>::v8 frag_tr_asm(const char* T, int rbase, int s, int ln) {
  typedef typename MfmaT<DT>::v8 v8;
  const int grp = ln >> 4, q = (ln & 15) >> 2, p = ln & 3;
  const int col = rbase + (grp & 1) * 16 + 4 * p;
  const int k0 = 16 * s + (grp >> 1) * 8 + q;
  typedef __attribute__((address_space(3))) const char* lds_cptr;
  const unsigned a0 = (unsigned)(uintptr_t)((lds_cptr)T + mc_off(k0, col));
  const unsigned a1 = (unsigned)(uintptr_t)((lds_cptr)T + mc_off(k0 + 4, col));
  s16x8_t f;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.hi) : "v"(a1));
  return __builtin_bit_cast(v8, f);
}

template <int N> __device__ __forceinline__ void wait_lgkm() {
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
  else static_assert(N < 0, "unsupported lgkmcnt");
}

template <int DT, int BM, int BN, int WGM, int WGN, int STAGES>
__global__ __launch_bounds__(WGM* WGN * 64, 2) void conv_wrw_glds(GemmArgs g, WrwGeom wg) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, SBYTES = ABYTES + BBYTES;
  constexpr int NIA = BM / 8 / NW, NIB = BN / 8 / NW;
  static_assert(NIA * NW * 8 == BM && NIB * NW * 8 == BN, "tile / wave count mismatch");
  static_assert(BM % 128 == 0 && BN % 128 == 0, "M/N-contiguous images are 128-column sub-images");
  constexpr int RPS = 2 * (FM + FN);                       // LDS reads per sub-step
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * SBYTES];

  const int per_group = 8 * g.tiles_n;
  const int ntile = gridDim.x;                             // tiles_m * tiles_n (+ tiles_m bias-only tasks)
  // all tiles of one pixel split on one XCD (they read the same dY / X rows): XCD-aware order over the whole grid
  const int hb = xcd_remap_g(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int split = hb / ntile, tile = hb - split * ntile;
  if (tile >= g.tiles_m * g.tiles_n) {
    // conv-bias gradient of output channels [k0, k0 + BM) over this split's pixels: column sums of dY rows
    constexpr int TPR = BM / 8;                            // threads per row (8 channels each)
    constexpr int RPI = NW * 64 / TPR;                     // rows per pass
    const int k0 = (tile - g.tiles_m * g.tiles_n) * BM;
    const int tid = threadIdx.x, cg = tid % TPR, r0 = tid / TPR;
    const int kc = k0 + cg * 8;
    const int pb = split * wg.mps, pe = min(wg.M, pb + wg.mps);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (kc < wg.K) {
      for (int p = pb + r0; p < pe; p += RPI) {
        float v[8];
        if constexpr (DT == 1) Vec8<bf16>::load(reinterpret_cast<const bf16*>(wg.dY) + (long long)p * wg.K + kc, v);
        else Vec8<f16>::load(reinterpret_cast<const f16*>(wg.dY) + (long long)p * wg.K + kc, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = acc[e];
    __syncthreads();
    if (tid < BM) {
      const int k = k0 + tid;
      float sacc = 0.f;
      for (int rr = 0; rr < RPI; ++rr) sacc += red[(rr * TPR + tid / 8) * 8 + (tid & 7)];
      if (k < wg.K) wg.partb[(long long)split * wg.K + k] = sacc;
    }
    return;
  }
  const int grp_id = tile / per_group, first_m = grp_id * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int in_g = tile - grp_id * per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;                    // m: output channel k, n: im2col column j
  const int pbeg = split * wg.mps;
  const int pend = min(wg.M, pbeg + wg.mps);
  const int nk = (pend - pbeg + 63) / 64;

  typedef unsigned short E;
  const E* X = reinterpret_cast<const E*>(wg.X);
  const E* dY = reinterpret_cast<const E*>(wg.dY);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // A = dY (rows k, reduction over pixels): lane -> (pixel row kr of the step, 8 channels at col)
  int a_col[NIA], a_kr[NIA];
  bool a_ok[NIA];
#pragma unroll
  for (int j = 0; j < NIA; ++j) {
    const int i = wid + NW * j;
    const int sub = i >> 4, kr = 4 * (i & 15) + (lane >> 4);
    const int ch = (lane & 15) ^ ((kr & 3) << 2);
    a_col[j] = m0 + sub * 128 + ch * 8;
    a_ok[j] = a_col[j] < wg.K;
    a_kr[j] = kr;
  }
  // B = im2col(X): lane -> fixed column chunk (filter tap (r, s), channels c..c+7), pixel row kr of the step
  int b_kr[NIB], b_c[NIB], b_rdh[NIB], b_sdw[NIB];
  bool b_ok[NIB];
#pragma unroll
  for (int j = 0; j < NIB; ++j) {
    const int i = wid + NW * j;
    const int sub = i >> 4, kr = 4 * (i & 15) + (lane >> 4);
    const int ch = (lane & 15) ^ ((kr & 3) << 2);
    const int col = n0 + sub * 128 + ch * 8;
    b_ok[j] = col < wg.RSC;
    const int cc = b_ok[j] ? col : 0;
    const int rs = cc / wg.C;
    b_c[j] = cc - rs * wg.C;
    b_rdh[j] = (rs / wg.S) * wg.dh - wg.ph;
    b_sdw[j] = (rs % wg.S) * wg.dw - wg.pw;
    b_kr[j] = kr;
  }

  auto issue = [&](int kt, int st) {
    char* sa = smem + st * SBYTES;
    char* sb = sa + ABYTES;
    const int p0 = pbeg + kt * 64;
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const int p = p0 + a_kr[j];
      const bool ok = a_ok[j] && p < pend;
      glds16(ok ? (const void*)(dY + (long long)p * wg.K + a_col[j]) : (const void*)gemm_zero_page,
             sa + (wid + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const int p = p0 + b_kr[j];
      const unsigned pp = p < pend ? (unsigned)p : 0u;
      const unsigned t = fdiv(pp, wg.fOW);
      const int ow = (int)(pp - t * wg.fOW.d);
      const unsigned n = fdiv(t, wg.fOH);
      const int oh = (int)(t - n * wg.fOH.d);
      const int ih = oh * wg.sh + b_rdh[j], iw = ow * wg.sw + b_sdw[j];
      const bool ok = b_ok[j] && p < pend && ih >= 0 && ih < wg.H && iw >= 0 && iw < wg.W;
      glds16(ok ? (const void*)(X + (((long long)n * wg.H + ih) * wg.W + iw) * wg.C + b_c[j])
                : (const void*)gemm_zero_page,
             sb + (wid + NW * j) * 1024);
    }
  };

  const int wm = wid / WGN, wn = wid % WGN;
  f32x16_t acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);

  int ln = lane;
  asm volatile("" : "+v"(ln));      // opaque lane id: the compiler recomputes the read addresses instead of hoisting
  constexpr int LPS = NIA + NIB;
  for (int kt = 0; kt < nk; ++kt) {
    if (STAGES > 2 && kt + 1 < nk) wait_vm<(STAGES > 2 ? (STAGES - 2) * LPS : 0)>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* sa = smem + (kt % STAGES) * SBYTES;
    const char* sb = sa + ABYTES;
    v8 fm[2][FM], fn[2][FN];
#pragma unroll
    for (int b = 0; b < FM; ++b) fm[0][b] = frag_tr_asm<DT>(sa, wm * WTM + 32 * b, 0, ln);
#pragma unroll
    for (int a = 0; a < FN; ++a) fn[0][a] = frag_tr_asm<DT>(sb, wn * WTN + 32 * a, 0, ln);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      if (s < 3) {
#pragma unroll
        for (int b = 0; b < FM; ++b) fm[nxt][b] = frag_tr_asm<DT>(sa, wm * WTM + 32 * b, s + 1, ln);
#pragma unroll
        for (int a = 0; a < FN; ++a) fn[nxt][a] = frag_tr_asm<DT>(sb, wn * WTN + 32 * a, s + 1, ln);
        wait_lgkm<RPS>();
      } else {
        wait_lgkm<0>();
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b) acc[a][b] = MfmaT<DT>::mma(fn[cur][a], fm[cur][b], acc[a][b]);
    }
  }

  // ---- epilogue: raw fp32 tile into this split's slab (mfma_tile.h epi_readout, raw mode)
  constexpr int PITCH = BN * 4 + 16;
  constexpr int RPP0 = (STAGES * SBYTES) / PITCH;
  constexpr int RPP = RPP0 >= BM ? BM : (RPP0 >= BM / 2 ? BM / 2 : BM / 4);
  static_assert(RPP >= 32, "epilogue pass too small");
  const int h = lane >> 5;
  EpiOut o;
  o.coh = false;
  o.raw = true;
  o.dt = 0;
  o.dst = reinterpret_cast<char*>(g.ws + (long long)split * g.M * g.N);
  o.ld = g.N;
  o.vec = (g.N & 3) == 0;
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
#pragma unroll
  for (int P = 0; P < BM / RPP; ++P) {
    sfor<0, FM>([&](auto B_) {
      constexpr int b = decltype(B_)::value;
      const int r0 = wm * WTM + 32 * b;
      if (r0 / RPP == P) {
        const int lr = r0 - P * RPP + (lane & 31);
        sfor<0, FN>([&](auto A_) {
          constexpr int a = decltype(A_)::value;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
            *reinterpret_cast<float4*>(smem + lr * PITCH + lc * 4) =
                make_float4(acc[a][b][4 * q], acc[a][b][4 * q + 1], acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]);
          }
        });
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    epi_readout<RPP, BN, NW * 64>(g, o, nullptr, smem, m0 + P * RPP, n0, tid);
    if (P + 1 < BM / RPP) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
  }
}

// slab reduce (fixed split order) + KRSC -> DL4J [K][C][R][S] relayout; see conv_wrw_reduce in conv_igemm.hip
__global__ __launch_bounds__(256) void conv_wrw_reduce_v3(const float* __restrict__ part, float* __restrict__ dW,
                                                          int splits, int K, int C, int RS,
                                                          const float* __restrict__ partb, float* __restrict__ db) {
  const long long total = (long long)K * C * RS;
  if (db && blockIdx.x == gridDim.x - 1) {
    // fixed-order bias reduce, 8 independent loads in flight per thread (a serial split loop here was the tail)
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      float a = 0.f;
      for (int sp0 = 0; sp0 < splits; sp0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = partb[(long long)min(sp0 + u, splits - 1) * K + k];
#pragma unroll
        for (int u = 0; u < 8; ++u) a += sp0 + u < splits ? v[u] : 0.f;
      }
      db[k] = a;
    }
  }
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int rs = (int)(o % RS);
    const long long t = o / RS;
    const int c = (int)(t % C);
    const long long k = t / C;
    const long long src = (k * RS + rs) * C + c;
    float a = 0.f;
    for (int sp = 0; sp < splits; ++sp) a += part[sp * total + src];
    dW[o] = a;
  }
}

struct WrwTile {
  int bm, bn;
};
// 0: 128x128 4 waves 2x2, 2 stages (2 blocks / CU)   1: 256x128 8 waves 4x2, 3 stages   2: 128x256 8 waves 2x4, 3 stages
// 3: 128x128 4 waves 2x2, 3 stages (96 KB)
constexpr int kWrwVariants = 4;
const WrwTile kWrw[kWrwVariants] = {{128, 128}, {256, 128}, {128, 256}, {128, 128}};

template <int DT>
int launch_wrw(int v, const GemmArgs& g, const WrwGeom& wg, int splits, hipStream_t s) {
  dim3 grid(g.tiles_m * g.tiles_n + (wg.partb ? g.tiles_m : 0), splits);
  switch (v) {
    case 0: hipLaunchKernelGGL((conv_wrw_glds<DT, 128, 128, 2, 2, 2>), grid, dim3(256), 0, s, g, wg); break;
    case 1: hipLaunchKernelGGL((conv_wrw_glds<DT, 256, 128, 4, 2, 3>), grid, dim3(512), 0, s, g, wg); break;
    case 2: hipLaunchKernelGGL((conv_wrw_glds<DT, 128, 256, 2, 4, 3>), grid, dim3(512), 0, s, g, wg); break;
    default: hipLaunchKernelGGL((conv_wrw_glds<DT, 128, 128, 2, 2, 3>), grid, dim3(256), 0, s, g, wg); break;
  }
  return (int)hipGetLastError();
}

static inline FastDiv make_fd(unsigned d) {
  FastDiv f;
  f.d = d;
  if (d == 1) { f.mul = 0; f.shr = 0; return f; }
  unsigned l = 0;
  while ((1u << l) < d) ++l;
  const unsigned p = 31 + l;
  f.mul = (unsigned)(((1ull << p) + d - 1) / d);
  f.shr = p - 32;
  return f;
}

// pixel splits: ~2 blocks per CU in total, every split >= 4 K-steps (256 pixels)
int wrw_splits(long long M, int tiles, int want) {
  int sp = want > 0 ? want : (int)((512 + tiles - 1) / tiles);
  const int maxs = (int)((M + 255) / 256);
  if (sp > maxs) sp = maxs;
  if (sp < 1) sp = 1;
  return sp;
}

}  // namespace

DL4J_API int dl4j_conv_wrw_v3_num_variants() { return kWrwVariants; }

// Slab floats needed by dl4j_conv_wrw_v3 for (variant, splits); splits <= 0 = heuristic. Writes the split count used.
DL4J_API long long dl4j_conv_wrw_v3_ws_floats(int N, int C, int K, int R, int S, int OH, int OW, int variant,
                                              int splits, int* splits_out) {
  if (variant < 0 || variant >= kWrwVariants) variant = 0;
  const long long M = (long long)N * OH * OW;
  const int RSC = R * S * C;
  const int tiles = ((K + kWrw[variant].bm - 1) / kWrw[variant].bm) * ((RSC + kWrw[variant].bn - 1) / kWrw[variant].bn);
  int sp = wrw_splits(M, tiles, splits);
  int mps = (int)((M + sp - 1) / sp);
  mps = (mps + 63) / 64 * 64;
  sp = (int)((M + mps - 1) / mps);
  if (splits_out) *splits_out = sp;
  return (long long)sp * K * (RSC + 1);                    // slabs + bias partials
}

// dW fp32 DL4J layout [K][C][R][S] and db fp32 [K] or null (both written, not accumulated). X NHWC [N,H,W,C], dY NHWC [N,OH,OW,K] (dt 1 bf16,
// 2 fp16). ws: >= dl4j_conv_wrw_v3_ws_floats. Requirements (else -1): C % 8, K % 8, 16-byte aligned operands,
// 32-bit element offsets.
DL4J_API int dl4j_conv_wrw_v3(int dt, const void* X, const void* dY, float* dW, float* db, float* ws, int N, int H,
                              int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH,
                              int OW, int variant, int splits, hipStream_t s) {
  if ((dt != 1 && dt != 2) || C % 8 != 0 || K % 8 != 0 || !ws || !dW) return -1;
  if ((long long)N * H * W * C >= 0x7fffffffLL || (long long)N * OH * OW * K >= 0x7fffffffLL) return -1;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(dY) & 15)) return -1;
  if (variant < 0 || variant >= kWrwVariants) variant = 0;
  const long long M = (long long)N * OH * OW;
  const int RSC = R * S * C;
  int sp = 0;
  dl4j_conv_wrw_v3_ws_floats(N, C, K, R, S, OH, OW, variant, splits, &sp);
  int mps = (int)((M + sp - 1) / sp);
  mps = (mps + 63) / 64 * 64;
  GemmArgs g = {};
  g.ws = ws;
  g.M = K;
  g.N = RSC;
  g.tiles_m = (K + kWrw[variant].bm - 1) / kWrw[variant].bm;
  g.tiles_n = (RSC + kWrw[variant].bn - 1) / kWrw[variant].bn;
  g.alpha = 1.f;
  WrwGeom wg;
  wg.X = X; wg.dY = dY;
  wg.N = N; wg.H = H; wg.W = W; wg.C = C; wg.OH = OH; wg.OW = OW; wg.K = K;
  wg.R = R; wg.S = S; wg.sh = sh; wg.sw = sw; wg.ph = ph; wg.pw = pw; wg.dh = dh; wg.dw = dw;
  wg.M = (int)M; wg.RSC = RSC; wg.mps = mps;
  wg.fOW = make_fd((unsigned)OW); wg.fOH = make_fd((unsigned)OH);
  wg.partb = db ? ws + (long long)sp * K * RSC : nullptr;
  int e = dt == 1 ? launch_wrw<1>(variant, g, wg, sp, s) : launch_wrw<2>(variant, g, wg, sp, s);
  if (e) return e;
  const long long total = (long long)K * RSC;
  long long gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(conv_wrw_reduce_v3, dim3((unsigned)gsz), dim3(256), 0, s, ws, dW, sp, K, C, R * S, wg.partb, db);
  return (int)hipGetLastError();
}
