// Halo-staged 3x3 convolution (stride 1, pad 1) for 64 -> 64 channels, NHWC: Y[m][n] = sum_{r,s,c} X[pix(m)+(r,s)][c]
// W[n][r][s][c] (+ bias[n]), the ResNet stage-2 3x3 layers (forward, and their stride-1 backward-data, which is the
// same convolution of dY with the flipped, transposed weights). Reference math: ConvolutionLayer.java:385-417.
//
// Why: the implicit-GEMM kernels (conv_gemm.hip, gemm_stream.hip conv_stream) stream one 128-pixel x 64-channel
// im2col chunk per filter tap, i.e. every input element crosses L2 -> LDS nine times, and at C = 64 a tile's whole
// K loop is only 9 chunks long — too short for their pipelines to hide the L2 latency (151.8 us at batch 1024 x
// 28 x 28 against a 41 us HBM bound, profiles/r6_stream_kernels.txt). Here:
//   * all 9 x 64 x 64 weights stay resident in LDS for the whole kernel (72 KB);
//   * a pixel CHUNK = G images x TH output rows (<= 128 pixels) is computed from ONE LDS halo image of its input rows
//     ((TH+2) x (OW+2) padded pixels x 64 channels, zero page for the padding), read once from L2 / HBM; the 9 taps are
//     9 constant row offsets into that image, so input bytes cross L2 -> LDS ~1.3-1.9 times instead of 9;
//   * one block per CU walks a strided list of chunks (XCD-aware: an XCD owns a contiguous range, so the halo rows
//     two neighbouring chunks share come from that XCD's L2), a LOADER wave (the 5th) streams halo images through an
//     S-slot ring D = S-1 chunks ahead and issues nothing but loads (so its counted vmcnt waits are exact), and the 4
//     consumer waves run the 72 MFMAs per wave and chunk plus the epilogue (16-bit LDS image, optional BN statistics
//     of the chunk, 16-byte row stores) while the next chunks' loads are in flight.
// BatchNorm statistics: one partial per chunk (rows per partial = the chunk's pixel count), planes [3][chunks][64]
// (sum and sum of squares about the chunk's first row, and that row) — the format bn_fold reads with rpp = PC.
#include "common.h"
#include <hip/hip_fp16.h>

#include "mfma_tile.h"

namespace {

constexpr int kHaloLds = 160 * 1024;
constexpr int kWBytes = 9 * 64 * 128;           // resident weights: 9 taps x 64 n-rows x 128 B
constexpr int kImgBytes = 128 * 64 * 2;         // epilogue image [128][64] 16-bit

struct HaloFwd {
  const u16* X;
  const u16* Wt;                                 // [64 n][3][3][64 c]
  u16* Y;
  const float* bias;
  float* tstats;                                 // [3][nch][64] or null
  int N, H, W, OH, OW;
  int G, TH, PC;                                 // chunk = G images x TH output rows = PC pixels
  int HR, HW, HROWS;                             // halo rows / cols per image, halo image rows
  int bands, nch;                                // chunks per image group, chunks
  int out_dt, store_nt;
};

inline int halo_slot_bytes(int hrows) { return ((hrows + 7) / 8) * 1024; }

template <int N> __device__ __forceinline__ void lgkm_wait_h() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt is a 4-bit counter");
  __builtin_amdgcn_s_waitcnt((7 << 4) | (N << 8) | 15 | (3 << 14));   // lgkmcnt(N), vmcnt / expcnt: no wait
}

template <int N> __device__ __forceinline__ void wait_vm_h() {
  static_assert(N >= 0 && N <= 63, "vmcnt is a 6-bit counter");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// S ring slots, XI = DMA pieces (8 halo rows) per chunk
template <int DT, int S, int XI>
__global__ __launch_bounds__(320, 1) void conv_halo3x3(HaloFwd a) {
  constexpr int D = S - 1;
  constexpr int SLOT = XI * 1024;
  static_assert(D >= 1 && (D - 1) * XI <= 63, "vmcnt range");
  static_assert(kWBytes + S * SLOT + kImgBytes <= kHaloLds, "LDS budget");
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[kWBytes + S * SLOT + kImgBytes];
  char* const sW = smem;
  char* const sX = smem + kWBytes;
  char* const sC = sX + S * SLOT;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // chunks of this block: XCD x owns [x*nch/8, (x+1)*nch/8), its blocks take them round robin
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
  const int c_beg = (int)((long long)a.nch * xcd / 8), c_end = (int)((long long)a.nch * (xcd + 1) / 8);
  const int nloc = j < c_end - c_beg ? (c_end - c_beg - j + per_xcd - 1) / per_xcd : 0;
  auto chunk_of = [&](int i) { return c_beg + j + i * per_xcd; };

  if (wid == 4) {
    // ------------------------------------------------------------------ loader wave
    const int rl = lane >> 3;
    // weights: 72 pieces of 8 n-rows x 128 B, tap-major images [t][n][c] with the kc_off swizzle
#pragma unroll 1
    for (int i = 0; i < 72; ++i) {
      const int t = i >> 3, row = 8 * (i & 7) + rl;
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      glds16(a.Wt + ((long long)row * 9 + t) * 64 + ch * 8, sW + t * 8192 + (i & 7) * 1024);
    }
    // per-lane halo rows (chunk-invariant): image g, halo row rr, column cc -> relative element offset, or -1
    int xrel[XI], xrr[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int row = 8 * i + rl;
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      int rel = -1, rr = 0;
      if (row < a.HROWS) {
        const int g = row / (a.HR * a.HW), rem = row - g * (a.HR * a.HW);
        rr = rem / a.HW;
        const int iw = rem - rr * a.HW - 1;
        if (iw >= 0 && iw < a.W) rel = ((g * a.H + rr) * a.W + iw) * 64 + ch * 8;
      }
      xrel[i] = rel;
      xrr[i] = rr;
    }
    auto issue = [&](int i) {
      char* dst = sX + (i % S) * SLOT;
      if (i < nloc) {
        const int c = chunk_of(i);
        const int grp = c / a.bands, band = c - grp * a.bands;
        const int oh0 = band * a.TH;
        const long long xb = ((long long)grp * a.G * a.H + oh0 - 1) * a.W * 64;
#pragma unroll
        for (int q = 0; q < XI; ++q) {
          const int ih = oh0 - 1 + xrr[q];
          const bool ok = xrel[q] >= 0 && ih >= 0 && ih < a.H;
          glds16(ok ? (const void*)(a.X + xb + xrel[q]) : (const void*)gemm_zero_page, dst + q * 1024);
        }
      } else {
#pragma unroll
        for (int q = 0; q < XI; ++q) glds16(gemm_zero_page, dst + q * 1024);   // keeps the wait counts exact
      }
    };
#pragma unroll 1
    for (int i = 0; i < D; ++i) issue(i);
#pragma unroll 1
    for (int i = 0; i < nloc; ++i) {
      wait_vm_h<(D - 1) * XI>();                   // chunk i (and the weights) landed
      raw_barrier();                               // B1(i)
      issue(i + D);                                // into the slot chunk i-1 used (read before B1(i))
      raw_barrier();                               // B2(i): the consumers' epilogue image
    }
    wait_vm_h<0>();
    return;
  }

  // ------------------------------------------------------------------ consumer waves (4): rows 32*wid .. +31, 64 cols
  const int h = lane >> 5;
  float4 bq[2][4];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = 32 * f + 8 * q + 4 * h;
      bq[f][q] = a.bias ? *reinterpret_cast<const float4*>(a.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  __builtin_amdgcn_s_waitcnt(0x0F70);              // bias loads retired before the loop (see gemm_stream.hip)
  // this lane's pixel p = 32*wid + (lane & 31) of a chunk -> its halo-image row (tap (0, 0)); pixels past PC read row 0
  const int p = 32 * wid + (lane & 31);
  int xrow = 0;
  if (p < a.PC) {
    const int g = p / (a.TH * a.OW), rem = p - g * (a.TH * a.OW);
    const int t = rem / a.OW, ow = rem - t * a.OW;
    xrow = (g * a.HR + t) * a.HW + ow;
  }
  const int hw = a.HW;
  char* dst = reinterpret_cast<char*>(a.Y);

#pragma unroll 1
  for (int i = 0; i < nloc; ++i) {
    const int c = chunk_of(i);
    raw_barrier();                                 // B1(i)
    const char* xs = sX + (i % S) * SLOT;
    f32x16_t acc[2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[f][e] = 0.f;
    // 36 units (tap t = u / 4, 16-channel step s = u % 4), each 3 LDS fragment reads + 2 MFMAs; the reads run PD
    // units ahead in a register ring with counted lgkmcnt waits (the compiler's own schedule waited for the read
    // issued just before every MFMA: LDS latency exposed 72 times per chunk)
    constexpr int NU = 36, PD = 4, NB = PD + 1;
    v8 fa[NB], fb0[NB], fb1[NB];
    auto reads = [&](auto U_) {
      constexpr int u = decltype(U_)::value;
      constexpr int t = u / 4, s = u % 4;
      const int r = xrow + (t / 3) * hw + (t % 3);
      const char* ws = sW + t * 8192;
      fa[u % NB] = *reinterpret_cast<const v8*>(xs + kc_off(r, 2 * s + h));
      fb0[u % NB] = read_frag<DT, true>(ws, 0, s, lane);
      fb1[u % NB] = read_frag<DT, true>(ws, 32, s, lane);
    };
    sfor<0, PD>([&](auto U_) { reads(U_); });
    sfor<0, NU>([&](auto U_) {
      constexpr int u = decltype(U_)::value;
      if constexpr (u + PD < NU) reads(IC<u + PD>{});
      constexpr int ahead = (u + PD < NU ? PD : NU - 1 - u) * 3;   // reads issued after unit u's
      lgkm_wait_h<ahead>();
      __builtin_amdgcn_sched_barrier(0);
      acc[0] = MfmaT<DT>::mma(fb0[u % NB], fa[u % NB], acc[0]);
      acc[1] = MfmaT<DT>::mma(fb1[u % NB], fa[u % NB], acc[1]);
    });
    // acc[f] regs 4q..4q+3 <-> chunk row 32*wid + (lane & 31), columns 32f + 8q + 4h .. +3
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        lean_put4<64>(sC, p, 32 * f + 8 * q + 4 * h, acc[f][4 * q] + bq[f][q].x, acc[f][4 * q + 1] + bq[f][q].y,
                      acc[f][4 * q + 2] + bq[f][q].z, acc[f][4 * q + 3] + bq[f][q].w, a.out_dt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                                 // B2(i)
    const long long m0 = (long long)c * a.PC;
    if (a.tstats) {
      // one partial per chunk: wave w takes columns 16w..16w+15, lane = 4 column quads x 16 row groups of 8 rows
      const int cq = lane & 3, rg = lane >> 2;
      const int col = 16 * wid + 4 * cq;
      const int dt = a.out_dt;
      auto val = [&](unsigned wv, int jj) {
        const u16 u = (u16)(wv >> (16 * (jj & 1)));
        return dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
      };
      float sh[4], s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
      const uint2 y0 = *reinterpret_cast<const uint2*>(sC + lean_off<64>(0, col));
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) sh[jj] = val(jj < 2 ? y0.x : y0.y, jj);
      uint2 v[8];
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) v[rr] = *reinterpret_cast<const uint2*>(sC + lean_off<64>(8 * rg + rr, col));
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const bool live = 8 * rg + rr < a.PC;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float d = live ? val(jj < 2 ? v[rr].x : v[rr].y, jj) - sh[jj] : 0.f;
          s1[jj] += d;
          s2[jj] = fmaf(d, d, s2[jj]);
        }
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) {
          s1[jj] += __shfl_xor(s1[jj], o);
          s2[jj] += __shfl_xor(s2[jj], o);
        }
      if (rg == 0) {
        float* p1 = a.tstats + (long long)c * 64 + col;
        float* p2 = a.tstats + ((long long)a.nch + c) * 64 + col;
        float* p3 = a.tstats + (2LL * a.nch + c) * 64 + col;
        *reinterpret_cast<float4*>(p1) = make_float4(s1[0], s1[1], s1[2], s1[3]);
        *reinterpret_cast<float4*>(p2) = make_float4(s2[0], s2[1], s2[2], s2[3]);
        *reinterpret_cast<float4*>(p3) = make_float4(sh[0], sh[1], sh[2], sh[3]);
      }
    }
    // read-out: 8 x 16-byte chunks per row, 32 rows per pass, rows past PC belong to the next chunk
    {
      const int cc = tid & 7, r0 = tid >> 3;
#pragma unroll
      for (int rr = r0; rr < 128; rr += 32) {
        if (rr >= a.PC) break;
        const uint4 q = *reinterpret_cast<const uint4*>(sC + rr * 128 + ((cc ^ (rr & 7)) << 4));
        char* pp = dst + ((m0 + rr) * 64 + cc * 8) * 2;
        if (a.store_nt) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          const u32x4_t vv = {q.x, q.y, q.z, q.w};
          __builtin_nontemporal_store(vv, reinterpret_cast<u32x4_t*>(pp));
        } else {
          *reinterpret_cast<uint4*>(pp) = q;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

struct HaloPlan {
  int ok, G, TH, PC, HR, HW, HROWS, XI, S, bands, nch;
};

// chunk = G images x TH output rows with the most pixels <= 128 (ties: fewer halo rows), S = the deepest ring that
// fits next to the resident weights and the epilogue image
HaloPlan halo_plan(int N, int OH, int OW) {
  HaloPlan P = {};
  int best = 0, best_rows = 1 << 30;
  for (int mode = 0; mode < 2; ++mode) {
    const int lim = mode == 0 ? OH : N;
    for (int v = 1; v <= lim; ++v) {
      int G = 1, TH = OH;
      if (mode == 0) {
        if (OH % v) continue;
        TH = v;
      } else {
        if (N % v) continue;
        G = v;
      }
      const int pc = G * TH * OW;
      if (pc > 128) continue;
      const int hrows = G * (TH + 2) * (OW + 2);
      if (pc > best || (pc == best && hrows < best_rows)) {
        best = pc;
        best_rows = hrows;
        P.G = G;
        P.TH = TH;
      }
    }
  }
  if (best == 0) return P;
  P.PC = best;
  P.HR = P.TH + 2;
  P.HW = OW + 2;
  P.HROWS = best_rows;
  P.XI = (P.HROWS + 7) / 8;
  P.S = 0;
  for (int s = 4; s >= 2; --s)
    if (kWBytes + s * P.XI * 1024 + kImgBytes <= kHaloLds && (s - 2) * P.XI <= 63) {
      P.S = s;
      break;
    }
  if (!P.S) return P;
  P.bands = OH / P.TH;
  P.nch = (N / P.G) * P.bands;
  P.ok = 1;
  return P;
}

template <int DT, int S, int XI>
int launch_halo_sx(const HaloFwd& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((conv_halo3x3<DT, S, XI>), dim3(grid), dim3(320), 0, s, a);
  return (int)hipGetLastError();
}

// XI (halo DMA pieces) is a template parameter: the supported set covers OW <= 56 chunk plans
template <int DT>
int launch_halo(const HaloFwd& a, const HaloPlan& P, int grid, hipStream_t s) {
#define HX(SS, X) \
  if (P.S == SS && P.XI <= X) return launch_halo_sx<DT, SS, X>(a, grid, s)
  HX(4, 16);
  HX(4, 18);
  HX(3, 24);   // e.g. 28 x 28: 4 rows x 28 = 112 pixels, 6 x 30 = 180 halo rows
  HX(2, 30);   // e.g. 56 x 56: 2 rows x 56 = 112 pixels, 4 x 58 = 232 halo rows
  HX(2, 36);
#undef HX
  return -1;
}

}  // namespace

// Chunks (= BN-statistics partials) and pixels per chunk of dl4j_conv_halo for a shape; 0 when unsupported.
DL4J_API long long dl4j_conv_halo_plan(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                       int dh, int dw, int OH, int OW, int* pixels_per_chunk) {
  if (C != 64 || K != 64 || R != 3 || S != 3 || sh != 1 || sw != 1 || ph != 1 || pw != 1 || dh != 1 || dw != 1 ||
      OH != H || OW != W)
    return 0;
  const HaloPlan P = halo_plan(N, OH, OW);
  if (!P.ok) return 0;
  if (pixels_per_chunk) *pixels_per_chunk = P.PC;
  return P.nch;
}

// Y [N,OH,OW,64] = conv3x3(X [N,H,W,64] NHWC, Wkrsc [64][3][3][64]) (+ bias fp32 [64]), stride 1, pad 1; tstats:
// optional fp32 [3][chunks][64] (dl4j_conv_halo_plan). Returns -1 when the shape / arguments are not this kernel's.
DL4J_API int dl4j_conv_halo(int dt, const void* X, const void* Wkrsc, const float* bias, void* Y, int N, int H, int W,
                            int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW,
                            float beta, float* tstats, hipStream_t s) {
  if ((dt != 1 && dt != 2) || beta != 0.f) return -1;
  if (dl4j_conv_halo_plan(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW, nullptr) <= 0) return -1;
  if (tstats && bnb_armed().mode) return -1;         // BN-backward sums of dX: the round-3 kernels' epilogue only
  if ((long long)N * H * W * 64 >= 0x7fffffffLL) return -1;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Wkrsc) & 15) ||
      (reinterpret_cast<uintptr_t>(Y) & 15) || (bias && (reinterpret_cast<uintptr_t>(bias) & 15)))
    return -1;
  const HaloPlan P = halo_plan(N, OH, OW);
  HaloFwd a;
  a.X = reinterpret_cast<const u16*>(X);
  a.Wt = reinterpret_cast<const u16*>(Wkrsc);
  a.Y = reinterpret_cast<u16*>(Y);
  a.bias = bias;
  a.tstats = tstats;
  a.N = N; a.H = H; a.W = W; a.OH = OH; a.OW = OW;
  a.G = P.G; a.TH = P.TH; a.PC = P.PC; a.HR = P.HR; a.HW = P.HW; a.HROWS = P.HROWS;
  a.bands = P.bands; a.nch = P.nch;
  a.out_dt = dt;
  a.store_nt = store_nt_for((long long)N * OH * OW * 64 * 2);
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int grid = cus - cus % 8;
  if (grid <= 0) grid = 8;
  return dt == 1 ? launch_halo<1>(a, P, grid, s) : launch_halo<2>(a, P, grid, s);
}
