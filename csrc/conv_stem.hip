// ResNet stem convolution for gfx950: 7x7, stride 2, pad 3, C = 3 -> K = 64, NHWC bf16 (DL4J zoo ResNet50
// "stem-cnn1", reference zoo/model/ResNet50.java conv1 after ZeroPaddingLayer(3,3)).
//
// The generic implicit-GEMM kernels want C % 32 == 0; with C = 3 every im2col row is 147 values that straddle
// pixels, so the library path (MIOpen) ran at ~0.7 ms per direction for a batch of 512. Here:
//  * K layout k = r*24 + q, q = s*3 + c (< 21 valid, rows 21..23 and r = 7 are zero weights): for a fixed filter
//    row r the 21 inputs of an output pixel are CONTIGUOUS in NHWC memory, so every 8-value A fragment is one
//    contiguous 16-byte LDS read; K = 192 (6 MFMA k-steps of 32).
//  * A (persistent) workgroup walks blocks of 4 output rows (4*OW pixels) of one image: it stages the 13(+1) input
//    rows a block needs in LDS (8-byte copies, zero padded), keeps the whole 192x64 weight matrix as MFMA B fragments in registers (24 fragments per
//    lane), and emits 64-pixel rounds: 4 waves x 16 pixels x 64 channels with mfma_f32_16x16x32_bf16.
//  * Each round's 64x64 bf16 tile goes through LDS for 16-byte coalesced stores, and its per-channel BatchNorm
//    partial statistics (S1, S2 about the round's first pixel) are written in the tile-stats format of
//    csrc/conv_igemm.hip (planes [3][P][64], P = M / 64), so the following BN skips its statistics pass.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) float f4s_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8s_t;

namespace {
constexpr int KS = 6;           // k-steps of 32 (K = 192)
constexpr int ROWS_PER_WG = 4;  // output rows per workgroup
constexpr int IN_ROWS = 2 * ROWS_PER_WG + 6;   // 14 staged input rows (13 used + 1 zero row for r = 7 reads)
constexpr int OUT_LD = 64 + 8;  // bf16 elements per pixel row of the output staging tile
}  // namespace

__global__ void __launch_bounds__(256) stem_conv_fwd(const u16* __restrict__ x, const bf16x8s_t* __restrict__ wpk,
                                                     u16* __restrict__ y, float* __restrict__ tstats, int N, int H,
                                                     int W, int OH, int OW, int RS, long long P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u16* xin = reinterpret_cast<u16*>(smem);                                   // [IN_ROWS][RS]
  u16* ot = xin + IN_ROWS * RS;                                              // [64][OUT_LD]
  float* red = reinterpret_cast<float*>(ot + 64 * OUT_LD);                   // [2][4][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hg = lane >> 4;
  const int blocks_per_img = OH / ROWS_PER_WG, nblocks = N * blocks_per_img;
  // ---- weights: B fragments for 4 output-channel tiles x 6 k-steps, resident in registers for all blocks
  bf16x8s_t b[4][KS];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) b[nt][ks] = wpk[(nt * KS + ks) * 64 + lane];
  const int row_elems = 3 * W, row_u2 = row_elems / 4;                     // 8-byte chunks of one image row
  const int pix_per_wg = ROWS_PER_WG * OW;
  // persistent: each workgroup walks 4-output-row blocks (weights loaded once per workgroup)
  for (int blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const int n = blk / blocks_per_img, oh0 = (blk - n * blocks_per_img) * ROWS_PER_WG;
    // ---- stage input rows ih = 2*oh0 - 3 + rr; element (rr, iw, c) at rr*RS + (iw + 4)*3 + c: the image row
    // starts 24 bytes in (8-byte aligned copies), pads [0, 12) and [12 + 3W, RS) are zero
    __syncthreads();                                                         // previous block done with xin
    for (int i = threadIdx.x; i < (IN_ROWS - 1) * row_u2; i += 256) {
      const int rr = i / row_u2, j = i - rr * row_u2;
      const int ih = 2 * oh0 - 3 + rr;
      uint2 v = make_uint2(0u, 0u);
      if (ih >= 0 && ih < H) v = *reinterpret_cast<const uint2*>(x + ((long long)n * H + ih) * row_elems + 4 * j);
      *reinterpret_cast<uint2*>(xin + rr * RS + 12 + 4 * j) = v;
    }
    const int tail = RS - 12 - row_elems;                                    // zero columns per row (even)
    for (int i = threadIdx.x; i < IN_ROWS * (6 + tail / 2); i += 256) {
      const int rr = i / (6 + tail / 2), j = i - rr * (6 + tail / 2);
      const int e = j < 6 ? 2 * j : 12 + row_elems + 2 * (j - 6);
      *reinterpret_cast<unsigned*>(xin + rr * RS + e) = 0u;
    }
    for (int i = threadIdx.x; i < row_u2; i += 256)                          // last (r = 7 only) row: zero
      *reinterpret_cast<uint2*>(xin + (IN_ROWS - 1) * RS + 12 + 4 * i) = make_uint2(0u, 0u);
    __syncthreads();
    const long long m_base = ((long long)n * OH + oh0) * OW;
    for (int rnd = 0; rnd < pix_per_wg / 64; ++rnd) {
      // ---- MFMA: this wave's 16 pixels x 64 channels; window of output column ow starts at element 6*ow + 3 (odd):
      // read 5 aligned dwords and realign by 16 bits
      const int ml = rnd * 64 + wave * 16 + col;
      const int ohl = ml / OW, ow = ml - ohl * OW;
      const unsigned* abase = reinterpret_cast<const unsigned*>(xin + (2 * ohl) * RS + 6 * ow + 2);
      f4s_t acc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = f4s_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k0 = ks * 32 + hg * 8, r = k0 / 24, q0 = k0 - r * 24;
        const unsigned* ap = abase + (r * RS + q0) / 2;
        unsigned d[5];
#pragma unroll
        for (int jj = 0; jj < 5; ++jj) d[jj] = ap[jj];
        union {
          unsigned u[4];
          bf16x8s_t v;
        } a;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) a.u[jj] = __builtin_amdgcn_alignbit(d[jj + 1], d[jj], 16);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b[nt][ks], acc[nt], 0, 0, 0);
      }
      // ---- C tile -> LDS (bf16): lane holds rows 4*hg + j, column nt*16 + col
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) ot[(wave * 16 + hg * 4 + j) * OUT_LD + nt * 16 + col] = f2bf(acc[nt][j]);
      __syncthreads();
      // ---- BN tile statistics over the 64 rounded outputs of each channel (shift = the round's first pixel)
      if (tstats) {
        const int c = threadIdx.x & 63, qg = threadIdx.x >> 6;
        const float sh = bf2f(ot[c]);
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float dd = bf2f(ot[(qg * 16 + i) * OUT_LD + c]) - sh;
          s1 += dd;
          s2 += dd * dd;
        }
        red[qg * 64 + c] = s1;
        red[256 + qg * 64 + c] = s2;
      }
      // ---- 16-byte coalesced stores of the 64 x 64 tile
      const long long m0 = m_base + rnd * 64;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int id = threadIdx.x + 256 * j, row = id >> 3, c8 = id & 7;
        *reinterpret_cast<bf16x8*>(y + (m0 + row) * 64 + c8 * 8) =
            *reinterpret_cast<const bf16x8*>(ot + row * OUT_LD + c8 * 8);
      }
      __syncthreads();
      if (tstats && threadIdx.x < 64) {
        const int c = threadIdx.x;
        const long long p = m0 / 64;
        tstats[p * 64 + c] = red[c] + red[64 + c] + red[128 + c] + red[192 + c];
        tstats[(P + p) * 64 + c] = red[256 + c] + red[320 + c] + red[384 + c] + red[448 + c];
        tstats[(2 * P + p) * 64 + c] = bf2f(ot[c]);
      }
      __syncthreads();                                                       // ot / red reused next round
    }
  }
}

// x: [N,H,W,3] bf16; wpk: fragment-packed weights [4][6][64][8] bf16 (see deeplearning4j_amd/ops/conv_stem.py);
// y: [N,OH,OW,64] bf16; tstats: optional [3][N*OH*OW/64][64] fp32. Returns -1 when the shape is not the stem's.
DL4J_API int dl4j_stem_conv_fwd(const void* x, const void* wpk, void* y, float* tstats, int N, int H, int W,
                                      int OH, int OW, hipStream_t s) {
  if (N < 1 || OH % ROWS_PER_WG != 0 || (ROWS_PER_WG * OW) % 64 != 0 || OH != (H - 1) / 2 + 1 ||
      OW != (W - 1) / 2 + 1 || (3 * W) % 4 != 0)
    return -1;
  // row: 12 zero elements, the 3W image elements, zero tail covering window reads up to q = 23 (+1 realign dword)
  int RS = 12 + 3 * W;
  const int need = 6 * (OW - 1) + 3 + 24 + 2;
  if (RS < need) RS = need;
  RS = (RS + 15) & ~15;                           // 32-byte rows
  const size_t lds = (size_t)IN_ROWS * RS * 2 + 64 * OUT_LD * 2 + 512 * 4;
  if (lds > 64 * 1024) return -1;
  const long long P = (long long)N * OH * OW / 64;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int per = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, stem_conv_fwd, 256, lds) != hipSuccess || per < 1) per = 1;
  const int nblocks = N * (OH / ROWS_PER_WG);
  const int grid = nblocks < per * ncu ? nblocks : per * ncu;
  hipLaunchKernelGGL(stem_conv_fwd, dim3(grid), dim3(256), lds, s, (const u16*)x,
                     (const bf16x8s_t*)wpk, (u16*)y, tstats, N, H, W, OH, OW, RS, P);
  return (int)hipGetLastError();
}
