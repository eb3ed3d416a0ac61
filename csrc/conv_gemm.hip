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

template <int DT, int BM, int BN, int WGM, int WGN, int STAGES>
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

  // ---- epilogue through LDS (mfma_tile.h epi_readout / epi_stats)
  constexpr int PITCH = BN * 4 + 16;
  constexpr int RPP0 = (STAGES * SBYTES) / PITCH;
  constexpr int RPP = RPP0 >= BM ? BM : (RPP0 >= BM / 2 ? BM / 2 : BM / 4);
  static_assert(RPP >= 64 && RPP % 64 == 0, "epilogue pass too small");
  const int h = lane >> 5;
  EpiOut o;
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
    if (g.tstats) epi_stats<RPP, BN, NW * 64>(g, smem, m0 + P * RPP, n0, tid);
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

template <int DT>
int launch_conv(int v, const GemmArgs& g, const ConvA& ca, hipStream_t s) {
  dim3 grid(g.tiles_m * g.tiles_n);
  switch (v) {
    case 0: hipLaunchKernelGGL((conv_glds<DT, 256, 128, 4, 2, 3>), grid, dim3(512), 0, s, g, ca); break;
    case 1: hipLaunchKernelGGL((conv_glds<DT, 128, 128, 2, 2, 2>), grid, dim3(256), 0, s, g, ca); break;
    case 2: hipLaunchKernelGGL((conv_glds<DT, 256, 64, 4, 1, 3>), grid, dim3(256), 0, s, g, ca); break;
    case 3: hipLaunchKernelGGL((conv_glds<DT, 128, 64, 2, 2, 3>), grid, dim3(256), 0, s, g, ca); break;
    default: hipLaunchKernelGGL((conv_glds<DT, 128, 256, 2, 4, 3>), grid, dim3(512), 0, s, g, ca); break;
  }
  return (int)hipGetLastError();
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
  g.tstats = tstats;
  g.stats_P = tstats ? (int)((M + 63) / 64) : 0;
  ConvA ca;
  ca.X = X;
  ca.N = N; ca.H = H; ca.W = W; ca.C = C; ca.OH = OH; ca.OW = OW;
  ca.R = R; ca.S = S; ca.sh = sh; ca.sw = sw; ca.ph = ph; ca.pw = pw; ca.dh = dh; ca.dw = dw;
  return dt == 1 ? launch_conv<1>(variant, g, ca, s) : launch_conv<2>(variant, g, ca, s);
}
