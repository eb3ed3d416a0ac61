// Persistent streaming GEMM (configuration 10 of dl4j_gemm, csrc/gemm.hip) for the tall, short-K products of the 1x1
// convolutions. Reference call site: NN:nn/layers/convolution/ConvolutionLayer.java:395-408 (im2col + gemm forward;
// a 1x1 convolution over NHWC activations is exactly C[M = N*H*W][Cout] = A[M][Cin] x W^T).
#include "common.h"
#include <hip/hip_fp16.h>

#include "mfma_tile.h"

namespace {
// ----------------------------------------------------------------------------------------------- streaming kernel
// gemm_stream: persistent GEMM for the tall, short-K products of the 1x1 convolutions (C[M][N] = A[M][K] B, both
// operands K-contiguous, K = 64..512, M % 128 == 0, N % BN == 0), e.g. the expanding ResNet-50 1x1 convs: 128-row
// tiles of 64..256 columns whose cost is the output write, not the MFMA work.
// The one-tile-per-block kernels serialise every block as [load A -> MFMA -> epilogue] and measured 2.0-2.5 TB/s on
// these shapes against a 6.2 TB/s write ceiling (profiles/r5_conv1x1_gemm.txt). Here:
//   * one block per CU walks a fixed n-tile and a strided list of m-tiles (XCD-aware: the n-tiles of one m-tile are
//     blocks of ONE XCD, so the A panel is read from HBM once and re-read from that XCD's L2);
//   * the block's B panel (BN x K) is DMA'd into LDS once and stays resident;
//   * a LOADER wave (the 9th) streams the A operand through an S-slot ring of 128 x 64 chunks with LDS-DMA, D = S-1
//     chunks ahead, and waits with a counted vmcnt on loads only (it issues no stores, so its counter never mixes
//     loads and stores); one s_barrier per chunk publishes a landed chunk to the 8 CONSUMER waves;
//   * the consumers run the MFMAs and the lean epilogue (16-bit LDS image, BN tile statistics, 16-byte row stores)
//     while the next tiles' chunks are already in flight, so the epilogue of tile t overlaps the loads of t+1..t+D/KC.
//   Barrier schedule (identical on every wave): B1 per chunk (chunk landed / previous slot free), B2 per tile (image
//   written). Output stores are never waited for inside the loop.
template <int BN, int KC, int S>
constexpr int stream_smem() {
  return BN * KC * 128 + S * 128 * 128 + 128 * BN * 2;
}

template <int N> __device__ __forceinline__ void wait_vm_s() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if constexpr (N == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

template <int DT, int BN, int KC, int S, int WGM, int WGN>
__global__ __launch_bounds__((WGM * WGN + 1) * 64) void gemm_stream(GemmArgs g) {
  constexpr int BM = 128;
  constexpr int NWC = WGM * WGN;                  // consumer waves; wave NWC is the loader
  constexpr int NT = NWC * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int BPANEL = BN * 128;                // one 64-deep K slice of the resident B panel
  constexpr int ASLOT = BM * 128;                 // one 128 x 64 A chunk
  constexpr int D = S - 1;                        // chunks in flight ahead of the one consumed
  constexpr int NIA = ASLOT / 1024;               // 16 DMA instructions per chunk
  static_assert(FM >= 1 && FN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "stream tile / wave layout");
  static_assert(D >= 1 && (D - 1) * NIA <= 48, "vmcnt range");
  static_assert(stream_smem<BN, KC, S>() <= 160 * 1024, "LDS budget");
  typedef typename MfmaT<DT>::v8 v8;
  typedef unsigned short E;
  __shared__ __attribute__((aligned(1024))) char smem[stream_smem<BN, KC, S>()];
  char* const sB = smem;
  char* const sA = smem + BPANEL * KC;
  char* const sC = sA + S * ASLOT;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = g.N / BN, tiles_m = g.M / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int nb = loc % tiles_n, mg = loc / tiles_n;
  const int Q = gridDim.x / tiles_n;              // m-tile stride of one block (host: gridDim.x % (8 * tiles_n) == 0)
  const int mb0 = mg * 8 + xcd;
  const int ntiles = mb0 < tiles_m ? (tiles_m - mb0 + Q - 1) / Q : 0;
  const int nchunks = ntiles * KC;
  const int n0 = nb * BN;

  if (wid == NWC) {
    // ------------------------------------------------------------------ loader wave
    const E* A = reinterpret_cast<const E*>(g.A);
    const E* B = reinterpret_cast<const E*>(g.B);
    const int rl = lane >> 3;                      // row within one 1-KB DMA piece (8 rows x 128 bytes)
#pragma unroll 1
    for (int i = 0; i < BN / 8 * KC; ++i) {        // B panel: KC slices of [BN rows][64 k]
      const int kc = i / (BN / 8), row = 8 * (i - kc * (BN / 8)) + rl;
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      glds16(B + (long long)(n0 + row) * g.ldb + kc * 64 + ch * 8, sB + kc * BPANEL + (i - kc * (BN / 8)) * 1024);
    }
    auto issue = [&](int c) {
      char* dst = sA + (c % S) * ASLOT;
      if (c < nchunks) {
        const int t = c / KC, kc = c - t * KC;
        const E* base = A + (long long)(mb0 + t * Q) * BM * g.lda + kc * 64;
#pragma unroll
        for (int i = 0; i < NIA; ++i) {
          const int row = 8 * i + rl;
          const int ch = (lane & 7) ^ ((row >> 1) & 7);
          glds16(base + (long long)row * g.lda + ch * 8, dst + i * 1024);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NIA; ++i) glds16(gemm_zero_page, dst + i * 1024);   // keeps the wait counts exact
      }
    };
#pragma unroll 1
    for (int c = 0; c < D; ++c) issue(c);
#pragma unroll 1
    for (int c = 0; c < nchunks; ++c) {
      wait_vm_s<(D - 1) * NIA>();                  // chunk c (and everything before it) has landed
      raw_barrier();                               // B1(c)
      issue(c + D);                                // into the slot chunk c-1 occupied (read before B1(c))
      if (c % KC == KC - 1) raw_barrier();         // B2: the consumers' epilogue image
    }
    wait_vm_s<0>();
    return;
  }

  // ------------------------------------------------------------------ consumer waves
  const int wm = wid / WGN, wn = wid % WGN;
  const int h = lane >> 5;
  float4 bq[FN][4];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
      bq[a][q] = g.bias_mode == 1 ? *reinterpret_cast<const float4*>(g.bias + n0 + lc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  // retire the bias loads HERE, with a wait the compiler's counter model sees (the builtin, not inline asm): else it
  // treats them as pending inside the loop, where the only vector-memory traffic is the epilogue's stores, and
  // emits vmcnt(0) before their first use in every epilogue — which drains the previous tile's output stores and
  // serialises the tiles (vmcnt(0), lgkmcnt / expcnt untouched)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  f32x16_t acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  char* dst = reinterpret_cast<char*>(g.C);

#pragma unroll 1
  for (int c = 0; c < nchunks; ++c) {
    raw_barrier();                                 // B1(c)
    const char* as = sA + (c % S) * ASLOT;
    const char* bs = sB + (c % KC) * BPANEL;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v8 fm[FM], fn[FN];
#pragma unroll
      for (int b = 0; b < FM; ++b) fm[b] = read_frag<DT, true>(as, wm * WTM + 32 * b, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a) fn[a] = read_frag<DT, true>(bs, wn * WTN + 32 * a, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b) acc[a][b] = MfmaT<DT>::mma(fn[a], fm[b], acc[a][b]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (c % KC == KC - 1) {
      const int m0 = (mb0 + (c / KC) * Q) * BM;
      // acc[a][b] regs 4q..4q+3 <-> tile row wm*WTM + 32b + (lane&31), columns wn*WTN + 32a + 8q + 4h .. +3
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
#pragma unroll
          for (int b = 0; b < FM; ++b) {
            float v[4] = {acc[a][b][4 * q] * g.alpha + bq[a][q].x, acc[a][b][4 * q + 1] * g.alpha + bq[a][q].y,
                          acc[a][b][4 * q + 2] * g.alpha + bq[a][q].z, acc[a][b][4 * q + 3] * g.alpha + bq[a][q].w};
            lean_act4(g, v);
            lean_put4<BN>(sC, wm * WTM + 32 * b + (lane & 31), lc, v[0], v[1], v[2], v[3], g.out_dt);
          }
        }
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();                               // B2
      if (g.tstats) lean_stats<BM, BN, NT>(g, sC, m0, n0, tid);
      lean_readout<BM, BN, NT>(g, dst, sC, m0, n0, tid, nullptr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

// Streaming-kernel variant for a shape: (BN, KC, S) with the largest BN that divides N, or -1.
int stream_variant(int N, int K) {
  const int kc = K / 64;
  if (K % 64 || (kc != 1 && kc != 2 && kc != 4 && kc != 8)) return -1;
  if (N % 256 == 0 && kc == 1) return 0;           // 256 x K64, 3 slots
  if (N % 128 == 0 && kc <= 4) return kc == 1 ? 1 : (kc == 2 ? 2 : 3);
  if (N % 64 == 0) return kc == 1 ? 4 : (kc == 2 ? 5 : (kc == 4 ? 6 : 7));
  return -1;
}
constexpr int kStreamBN[8] = {256, 128, 128, 128, 64, 64, 64, 64};

int stream_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
    return n;
  }();
  return cus;
}

template <int DT>
int launch_stream(const GemmArgs& g, hipStream_t s) {
  const int v = stream_variant(g.N, g.K);
  if (v < 0) return -4;
  const int tiles_n = g.N / kStreamBN[v];
  int G = stream_cus();
  G -= G % (8 * tiles_n);
  if (G <= 0) return -4;
  switch (v) {
    case 0: hipLaunchKernelGGL((gemm_stream<DT, 256, 1, 3, 2, 4>), dim3(G), dim3(576), 0, s, g); break;
    case 1: hipLaunchKernelGGL((gemm_stream<DT, 128, 1, 5, 2, 4>), dim3(G), dim3(576), 0, s, g); break;
    case 2: hipLaunchKernelGGL((gemm_stream<DT, 128, 2, 5, 2, 4>), dim3(G), dim3(576), 0, s, g); break;
    case 3: hipLaunchKernelGGL((gemm_stream<DT, 128, 4, 3, 2, 4>), dim3(G), dim3(576), 0, s, g); break;
    case 4: hipLaunchKernelGGL((gemm_stream<DT, 64, 1, 5, 4, 2>), dim3(G), dim3(576), 0, s, g); break;
    case 5: hipLaunchKernelGGL((gemm_stream<DT, 64, 2, 5, 4, 2>), dim3(G), dim3(576), 0, s, g); break;
    case 6: hipLaunchKernelGGL((gemm_stream<DT, 64, 4, 5, 4, 2>), dim3(G), dim3(576), 0, s, g); break;
    default: hipLaunchKernelGGL((gemm_stream<DT, 64, 8, 4, 4, 2>), dim3(G), dim3(576), 0, s, g); break;
  }
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------------------------- conv_stream
// The same persistent loader / consumer engine for implicit-GEMM convolution (NHWC): Y[m][n] = sum_k im2col(X)[m][k]
// W[n][k], m = output pixel, k = (r*S + s)*C + c, K-steps of 64 channels of one filter tap (C % 64 == 0). Here the
// B operand (the weights of the block's n-tile) is streamed with A through the ring (a slot = one 128 x 64 im2col
// chunk + one BN x 64 weight chunk): the 3x3 weight panels (K = 576 .. 4608) do not fit in LDS. The loader computes
// each tile's per-row pixel base and filter-tap validity mask when it starts issuing that tile's chunks (one
// tile's worth of rows per lane: 16 rows, one per DMA instruction), so the next tile's loads run while the consumers
// finish the current tile's MFMAs and epilogue. Reference math: ConvolutionLayer.java:385-417 (im2col + GEMM).
struct ConvS {
  const void* X;
  int N, H, W, C, OH, OW, R, S, sh, sw, ph, pw, dh, dw;
};

template <int BN, int S>
constexpr int conv_stream_smem() {
  return S * (128 * 128 + BN * 128) + 128 * BN * 2;
}

template <int DT, int BN, int S, int WGM, int WGN>
__global__ __launch_bounds__((WGM * WGN + 1) * 64) void conv_stream(GemmArgs g, ConvS cv) {
  constexpr int BM = 128;
  constexpr int NWC = WGM * WGN;
  constexpr int NT = NWC * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int ASLOT = BM * 128, BSLOT = BN * 128, SLOT = ASLOT + BSLOT;
  constexpr int D = S - 1;
  constexpr int NIA = ASLOT / 1024, NIB = BSLOT / 1024, NI = NIA + NIB;
  static_assert(FM >= 1 && FN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "conv stream tile / wave layout");
  static_assert(D >= 1 && (D - 1) * NI <= 48 && ((D - 1) * NI) % 16 == 0, "vmcnt range");
  static_assert(conv_stream_smem<BN, S>() <= 160 * 1024, "LDS budget");
  typedef typename MfmaT<DT>::v8 v8;
  typedef unsigned short E;
  __shared__ __attribute__((aligned(1024))) char smem[conv_stream_smem<BN, S>()];
  char* const sR = smem;                          // ring: S slots of [A chunk | B chunk]
  char* const sC = smem + S * SLOT;               // epilogue image

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = g.N / BN, tiles_m = g.M / BM;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int nb = loc % tiles_n, mg = loc / tiles_n;
  const int Q = gridDim.x / tiles_n;
  const int mb0 = mg * 8 + xcd;
  const int ntiles = mb0 < tiles_m ? (tiles_m - mb0 + Q - 1) / Q : 0;
  const int nk = g.K / 64;                        // K-steps per tile
  const int nchunks = ntiles * nk;
  const int n0 = nb * BN;

  if (wid == NWC) {
    // ------------------------------------------------------------------ loader wave
    const E* X = reinterpret_cast<const E*>(cv.X);
    const E* Wt = reinterpret_cast<const E*>(g.B);
    const int rl = lane >> 3;
    const int cpt = cv.C / 64;                    // K-steps per filter tap
    int pbase[NIA];
    unsigned long long vmask[NIA];
    int cur_tile = -1;
    auto rows_for = [&](int t) {                  // per-row pixel base + tap mask of tile t (this lane's 16 rows)
      const int m0 = (mb0 + t * Q) * BM;
#pragma unroll
      for (int i = 0; i < NIA; ++i) {
        const int row = 8 * i + rl;
        const int ch = (lane & 7) ^ ((row >> 1) & 7);
        const int m = m0 + row;
        const int ow = m % cv.OW, tq = m / cv.OW;
        const int oh = tq % cv.OH, n = tq / cv.OH;
        const int ih0 = oh * cv.sh - cv.ph, iw0 = ow * cv.sw - cv.pw;
        pbase[i] = ((n * cv.H + ih0) * cv.W + iw0) * cv.C + ch * 8;
        unsigned long long mk = 0;
        for (int r = 0; r < cv.R; ++r) {
          const int ih = ih0 + r * cv.dh;
          if (ih < 0 || ih >= cv.H) continue;
          for (int q = 0; q < cv.S; ++q) {
            const int iw = iw0 + q * cv.dw;
            if (iw >= 0 && iw < cv.W) mk |= 1ull << (r * cv.S + q);
          }
        }
        vmask[i] = mk;
      }
    };
    auto issue = [&](int c) {
      char* sa = sR + (c % S) * SLOT;
      char* sb = sa + ASLOT;
      if (c < nchunks) {
        const int t = c / nk, kt = c - t * nk;
        if (t != cur_tile) {
          rows_for(t);
          cur_tile = t;
        }
        const int rs = kt / cpt, c0 = (kt - rs * cpt) * 64;
        const int r = rs / cv.S, q = rs - r * cv.S;
        const int uoff = (r * cv.dh * cv.W + q * cv.dw) * cv.C + c0;
#pragma unroll
        for (int i = 0; i < NIA; ++i) {
          const void* src = ((vmask[i] >> rs) & 1ull) ? (const void*)(X + pbase[i] + uoff) : (const void*)gemm_zero_page;
          glds16(src, sa + i * 1024);
        }
#pragma unroll
        for (int i = 0; i < NIB; ++i) {
          const int row = 8 * i + rl;
          const int ch = (lane & 7) ^ ((row >> 1) & 7);
          glds16(Wt + (long long)(n0 + row) * g.ldb + kt * 64 + ch * 8, sb + i * 1024);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NIA; ++i) glds16(gemm_zero_page, sa + i * 1024);
#pragma unroll
        for (int i = 0; i < NIB; ++i) glds16(gemm_zero_page, sb + i * 1024);
      }
    };
#pragma unroll 1
    for (int c = 0; c < D; ++c) issue(c);
#pragma unroll 1
    for (int c = 0; c < nchunks; ++c) {
      wait_vm_s<(D - 1) * NI>();
      raw_barrier();                               // B1(c)
      issue(c + D);
      if (c % nk == nk - 1) raw_barrier();         // B2
    }
    wait_vm_s<0>();
    return;
  }

  // ------------------------------------------------------------------ consumer waves
  const int wm = wid / WGN, wn = wid % WGN;
  const int h = lane >> 5;
  float4 bq[FN][4];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
      bq[a][q] = g.bias_mode == 1 ? *reinterpret_cast<const float4*>(g.bias + n0 + lc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  __builtin_amdgcn_s_waitcnt(0x0F70);              // bias loads retired before the loop (see gemm_stream)
  f32x16_t acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  char* dst = reinterpret_cast<char*>(g.C);

#pragma unroll 1
  for (int c = 0; c < nchunks; ++c) {
    raw_barrier();                                 // B1(c)
    const char* as = sR + (c % S) * SLOT;
    const char* bs = as + ASLOT;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v8 fm[FM], fn[FN];
#pragma unroll
      for (int b = 0; b < FM; ++b) fm[b] = read_frag<DT, true>(as, wm * WTM + 32 * b, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a) fn[a] = read_frag<DT, true>(bs, wn * WTN + 32 * a, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b) acc[a][b] = MfmaT<DT>::mma(fn[a], fm[b], acc[a][b]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (c % nk == nk - 1) {
      const int m0 = (mb0 + (c / nk) * Q) * BM;
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int lc = wn * WTN + 32 * a + 8 * q + 4 * h;
#pragma unroll
          for (int b = 0; b < FM; ++b)
            lean_put4<BN>(sC, wm * WTM + 32 * b + (lane & 31), lc, acc[a][b][4 * q] + bq[a][q].x,
                          acc[a][b][4 * q + 1] + bq[a][q].y, acc[a][b][4 * q + 2] + bq[a][q].z,
                          acc[a][b][4 * q + 3] + bq[a][q].w, g.out_dt);
        }
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();                               // B2
      if (g.tstats) lean_stats<BM, BN, NT>(g, sC, m0, n0, tid);
      lean_readout<BM, BN, NT>(g, dst, sC, m0, n0, tid, nullptr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

template <int DT>
int launch_conv_stream(const GemmArgs& g, const ConvS& cv, hipStream_t s) {
  const int BN = g.N % 128 == 0 ? 128 : (g.N % 64 == 0 ? 64 : 0);
  if (!BN) return -1;
  const int tiles_n = g.N / BN;
  int G = stream_cus();
  G -= G % (8 * tiles_n);
  if (G <= 0) return -1;
  if (BN == 128) hipLaunchKernelGGL((conv_stream<DT, 128, 3, 2, 4>), dim3(G), dim3(576), 0, s, g, cv);
  else hipLaunchKernelGGL((conv_stream<DT, 64, 4, 4, 2>), dim3(G), dim3(576), 0, s, g, cv);
  return (int)hipGetLastError();
}

}  // namespace

// in_dt 1 bf16 / 2 f16; out_dt 1 / 2; bias_mode 0 / 1 (per column, 16-byte aligned); act 0 / 1 / 4 (relu / gelu);
// tstats: optional [3][stats_P][N] BN tile statistics (64-row partials). Returns -4 when the shape is not this kernel's
// (K % 64, K / 64 in {1, 2, 4, 8}, N % 64, M % 128, 16-byte aligned K-contiguous operands).
DL4J_API int dl4j_gemm_stream(int in_dt, const void* A, long long lda, const void* B, long long ldb, void* C,
                              long long ldc, int M, int N, int K, float alpha, const float* bias, int bias_mode,
                              int act, int out_dt, float* tstats, int stats_P, int store_nt, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if ((in_dt != 1 && in_dt != 2) || (out_dt != 1 && out_dt != 2) || (M % 128) || (lda & 7) || (ldb & 7) || (ldc & 7) ||
      (reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15) ||
      (reinterpret_cast<uintptr_t>(C) & 15) || (bias_mode == 1 && (reinterpret_cast<uintptr_t>(bias) & 15)) ||
      bias_mode == 2 || (act != 0 && act != 1 && act != 4) || (tstats && act != 0))
    return -4;
  GemmArgs g = {};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.bias_mode = bias ? bias_mode : 0; g.act = act; g.out_dt = out_dt;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.splits = 1; g.kps = K;
  g.tstats = tstats; g.stats_P = stats_P; g.store_nt = store_nt;
  return in_dt == 1 ? launch_stream<1>(g, s) : launch_stream<2>(g, s);
}


// Persistent implicit-GEMM convolution (conv_stream): Y[N,OH,OW,K] NHWC = conv(X NHWC, Wkrsc[K][R][S][C]) (+bias)
// with optional BN tile statistics (fp32 [3][M/64][K]); the contract of dl4j_conv_fwd_v3 (also used for stride-1
// backward-data) minus beta accumulation. Returns -1 when the shape is not this kernel's (C % 64, K % 64,
// M = N*OH*OW % 128, R*S <= 64, beta != 0, 32-bit offsets).
DL4J_API int dl4j_conv_stream(int dt, const void* X, const void* Wkrsc, const float* bias, void* Y, int N, int H, int W,
                              int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW,
                              float beta, float* tstats, hipStream_t s) {
  if ((dt != 1 && dt != 2) || C % 64 != 0 || K % 64 != 0 || R * S > 64 || R < 1 || S < 1 || beta != 0.f) return -1;
  if (tstats && bnb_armed().mode) return -1;        // BN-backward sums of dX: the round-3 kernels' epilogue only
  const long long M = (long long)N * OH * OW;
  if (M <= 0 || M % 128 || (long long)N * H * W * C >= 0x7fffffffLL || M * K >= 0x7fffffffLL) return -1;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Wkrsc) & 15) ||
      (reinterpret_cast<uintptr_t>(Y) & 15) || (bias && (reinterpret_cast<uintptr_t>(bias) & 15)))
    return -1;
  GemmArgs g = {};
  g.B = Wkrsc; g.C = Y; g.bias = bias; g.bias_mode = bias ? 1 : 0;
  g.ldb = (long long)R * S * C; g.ldc = K;
  g.M = (int)M; g.N = K; g.K = R * S * C; g.kps = g.K; g.splits = 1; g.alpha = 1.f; g.out_dt = dt;
  g.store_nt = store_nt_for(M * K * 2);
  g.tstats = tstats;
  g.stats_P = tstats ? (int)(M / 64) : 0;
  ConvS cv;
  cv.X = X; cv.N = N; cv.H = H; cv.W = W; cv.C = C; cv.OH = OH; cv.OW = OW;
  cv.R = R; cv.S = S; cv.sh = sh; cv.sw = sw; cv.ph = ph; cv.pw = pw; cv.dh = dh; cv.dw = dw;
  return dt == 1 ? launch_conv_stream<1>(g, cv, s) : launch_conv_stream<2>(g, cv, s);
}
