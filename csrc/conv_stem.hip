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
//  * Wave w of a block owns output row w: 16-pixel M-tiles go through a wave-private LDS tile for 16-byte coalesced
//    stores (no workgroup barrier outside the staging), and the row's per-channel BatchNorm partial statistics
//    (S1, S2 about the row's first pixel) are written in the tile-stats format of csrc/conv_igemm.hip with one
//    partial per output row (planes [3][N*OH][64]), so the following BN skips its statistics pass.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) float f4s_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8s_t;

namespace {
constexpr int KS = 6;           // k-steps of 32 (K = 192)
constexpr int ROWS_PER_WG = 4;  // output rows per workgroup
constexpr int IN_ROWS = 2 * ROWS_PER_WG + 6;   // 14 staged input rows (13 used + 1 zero row for r = 7 reads)
constexpr int OUT_LD = 64 + 8;  // bf16 elements per pixel row of the output staging tile
constexpr int STAGE_SLOTS = 12; // 8-byte staging chunks per thread (13 rows x 3W/4 <= 3072: W <= 315)
}  // namespace

__global__ void __launch_bounds__(256, 2) stem_conv_fwd(const u16* __restrict__ x, const bf16x8s_t* __restrict__ wpk,
                                                     u16* __restrict__ y, float* __restrict__ tstats, int N, int H,
                                                     int W, int OH, int OW, int RS, long long P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u16* xin = reinterpret_cast<u16*>(smem);                                   // [2][IN_ROWS][RS]
  u16* ot = xin + 2 * IN_ROWS * RS;                                          // [4 waves][16][OUT_LD]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hg = lane >> 4;
  const int blocks_per_img = OH / ROWS_PER_WG, nblocks = N * blocks_per_img;
  // ---- weights: B fragments for 4 output-channel tiles x 6 k-steps, resident in registers for all blocks
  bf16x8s_t b[4][KS];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) b[nt][ks] = wpk[(nt * KS + ks) * 64 + lane];
  const int row_elems = 3 * W, row_u2 = row_elems / 4;                     // 8-byte chunks of one image row
  const int nchunks = (IN_ROWS - 1) * row_u2;                              // <= STAGE_SLOTS * 256 (host-checked)
  // ---- zero pads once for both staging buffers: element (rr, iw, c) at rr*RS + (iw + 4)*3 + c; the image row
  // starts 24 bytes in, [0, 12) and [12 + 3W, RS) stay zero, as does the data part of the last (r = 7 only) row
  {
    const int tail = RS - 12 - row_elems, per_row = 6 + tail / 2;
    for (int i = threadIdx.x; i < 2 * IN_ROWS * per_row; i += 256) {
      const int rb = i / per_row, j = i - rb * per_row;
      const int e = j < 6 ? 2 * j : 12 + row_elems + 2 * (j - 6);
      *reinterpret_cast<unsigned*>(xin + rb * RS + e) = 0u;
    }
    for (int i = threadIdx.x; i < 2 * row_u2; i += 256) {
      const int b2 = i / row_u2, j = i - b2 * row_u2;
      *reinterpret_cast<uint2*>(xin + (b2 * IN_ROWS + IN_ROWS - 1) * RS + 12 + 4 * j) = make_uint2(0u, 0u);
    }
  }
  // ---- staging: all of a thread's 8-byte chunks are loaded before any is stored (one round trip per block); the
  // second resident workgroup of the CU computes while this one waits
  uint2 pre[STAGE_SLOTS];
  int buf = 0;
  for (int blk = blockIdx.x; blk < nblocks; blk += gridDim.x, buf ^= 1) {
    const int n = blk / blocks_per_img, oh0 = (blk - n * blocks_per_img) * ROWS_PER_WG;
    u16* xb = xin + buf * IN_ROWS * RS;
#pragma unroll
    for (int q = 0; q < STAGE_SLOTS; ++q) {
      const int i = threadIdx.x + q * 256;
      const int rr = i / row_u2, j = i - rr * row_u2;
      const int ih = 2 * oh0 - 3 + rr;
      pre[q] = make_uint2(0u, 0u);
      if (i < nchunks && ih >= 0 && ih < H)
        pre[q] = *reinterpret_cast<const uint2*>(x + ((long long)n * H + ih) * row_elems + 4 * j);
    }
#pragma unroll
    for (int q = 0; q < STAGE_SLOTS; ++q) {
      const int i = threadIdx.x + q * 256;
      const int rr = i / row_u2, j = i - rr * row_u2;
      if (i < nchunks) *reinterpret_cast<uint2*>(xb + rr * RS + 12 + 4 * j) = pre[q];
    }
    __syncthreads();
    // ---- wave w owns output row oh0 + w of the block: OW/16 M-tiles of 16 pixels x 64 channels, epilogue through
    // a wave-private LDS tile (no workgroup barriers), BN statistics of the row accumulated in registers
    const int oh = oh0 + wave;
    const long long mrow = ((long long)n * OH + oh) * OW;                    // first pixel of this wave's row
    u16* otw = ot + wave * 16 * OUT_LD;
    float s1[4], s2[4], shv[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) s1[nt] = s2[nt] = 0.f;
    for (int mt = 0; mt < OW / 16; ++mt) {
      const int ow = mt * 16 + col;                                          // A row (pixel) of this lane
      const unsigned* abase = reinterpret_cast<const unsigned*>(xb + (2 * wave) * RS + 6 * ow + 2);
      f4s_t acc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = f4s_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        // window of output column ow starts at element 6*ow + 3 (odd): read 5 aligned dwords, realign by 16 bits
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
      // ---- lane holds rows (pixels) 4*hg + j, channel nt*16 + col: round to bf16, stats, stage for the stores
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        u16 hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) hv[j] = f2bf(acc[nt][j]);
        if (mt == 0) shv[nt] = __shfl(bf2f(hv[0]), col, 64);                 // shift: the row's first pixel
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float dd = bf2f(hv[j]) - shv[nt];
          s1[nt] += dd;
          s2[nt] += dd * dd;
          otw[(hg * 4 + j) * OUT_LD + nt * 16 + col] = hv[j];
        }
      }
      // ---- 16-byte coalesced stores of the 16 x 64 tile (wave-local LDS round trip, in-order within the wave)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int id = lane + 64 * j, row = id >> 3, c8 = id & 7;
        *reinterpret_cast<bf16x8*>(y + (mrow + mt * 16 + row) * 64 + c8 * 8) =
            *reinterpret_cast<const bf16x8*>(otw + row * OUT_LD + c8 * 8);
      }
    }
    if (tstats) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        s1[nt] += __shfl_xor(s1[nt], 16, 64);
        s1[nt] += __shfl_xor(s1[nt], 32, 64);
        s2[nt] += __shfl_xor(s2[nt], 16, 64);
        s2[nt] += __shfl_xor(s2[nt], 32, 64);
      }
      if (hg == 0) {
        const long long p = (long long)n * OH + oh;                          // one partial per output row
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          tstats[p * 64 + nt * 16 + col] = s1[nt];
          tstats[(P + p) * 64 + nt * 16 + col] = s2[nt];
          tstats[(2 * P + p) * 64 + nt * 16 + col] = shv[nt];
        }
      }
    }
  }
}

// x: [N,H,W,3] bf16; wpk: fragment-packed weights [4][6][64][8] bf16 (see deeplearning4j_amd/ops/conv_stem.py);
// y: [N,OH,OW,64] bf16; tstats: optional [3][N*OH][64] fp32 (one partial per output row). Returns -1 when the shape is not the stem's.
DL4J_API int dl4j_stem_conv_fwd(const void* x, const void* wpk, void* y, float* tstats, int N, int H, int W,
                                      int OH, int OW, hipStream_t s) {
  if (N < 1 || OH % ROWS_PER_WG != 0 || OW % 16 != 0 || OH != (H - 1) / 2 + 1 ||
      OW != (W - 1) / 2 + 1 || (3 * W) % 4 != 0)
    return -1;
  // row: 12 zero elements, the 3W image elements, zero tail covering window reads up to q = 23 (+1 realign dword)
  int RS = 12 + 3 * W;
  const int need = 6 * (OW - 1) + 3 + 24 + 2;
  if (RS < need) RS = need;
  RS = (RS + 15) & ~15;                           // 32-byte rows
  const size_t lds = (size_t)2 * IN_ROWS * RS * 2 + 64 * OUT_LD * 2;
  if (lds > 64 * 1024 || (IN_ROWS - 1) * (3 * W / 4) > STAGE_SLOTS * 256) return -1;
  const long long P = (long long)N * OH;
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

// ------------------------------------------------------------------------------------------------ weight gradient
// dW[co][k] = sum over output pixels m of dy[m][co] * A[m][k] (A = the same contiguous-K im2col as the forward).
// MFMA view: C[co][k] (4 x 12 tiles of 16), reduction over pixels in chunks of 32:
//   A operand = dy^T (co rows): staged per 64-pixel round as dyT[64][64 + 8] in LDS (16-byte reads per fragment),
//   B operand = im2col (pixel rows, k columns): 8 pixels of one k per lane, gathered from the staged input rows
//   (8 x 2-byte LDS reads at a 12-byte stride).
// Wave w owns k-tiles 3w..3w+2 for all 4 co-tiles (12 accumulators). Each (persistent) workgroup writes its partial
// [64][192] sums (and the bias column sums) to a workspace; stem_wrw_reduce sums the partials in a fixed order
// (deterministic) straight into the DL4J [64][3][7][7] fp32 gradient.
constexpr int kWrwWgPerCu = 3;   // persistent weight-gradient workgroups per CU (LDS ~46 KB, 158 VGPRs: 3 fit)
__global__ void __launch_bounds__(256, kWrwWgPerCu) stem_conv_wrw(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                        float* __restrict__ part, float* __restrict__ part_db, int N,
                                                        int H, int W, int OH, int OW, int RS) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u16* xin = reinterpret_cast<u16*>(smem);                                   // [IN_ROWS][RS]
  u16* dyt = xin + IN_ROWS * RS;                                             // [2][64][OUT_LD]
  float* dbs = reinterpret_cast<float*>(dyt + 2 * 64 * OUT_LD);              // [256][8]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hg = lane >> 4;
  const int blocks_per_img = OH / ROWS_PER_WG, nblocks = N * blocks_per_img;
  const int row_elems = 3 * W, row_u2 = row_elems / 4;
  const int nchunks = (IN_ROWS - 1) * row_u2;
  const int rounds = ROWS_PER_WG * OW / 64;
  {  // zero pads and the r = 7 row once
    const int tail = RS - 12 - row_elems, per_row = 6 + tail / 2;
    for (int i = threadIdx.x; i < IN_ROWS * per_row; i += 256) {
      const int rb = i / per_row, j = i - rb * per_row;
      const int e = j < 6 ? 2 * j : 12 + row_elems + 2 * (j - 6);
      *reinterpret_cast<unsigned*>(xin + rb * RS + e) = 0u;
    }
    for (int i = threadIdx.x; i < row_u2; i += 256)
      *reinterpret_cast<uint2*>(xin + (IN_ROWS - 1) * RS + 12 + 4 * i) = make_uint2(0u, 0u);
  }
  // per lane: element offsets (within a window) of its 3 k columns; (r, q) of k = kt*16 + col
  int koff[3];
#pragma unroll
  for (int t3 = 0; t3 < 3; ++t3) {
    const int k = (wave * 3 + t3) * 16 + col, r = k / 24, q = k - r * 24;
    koff[t3] = r * RS + q;
  }
  f4s_t acc[4][3];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3) acc[ct][t3] = f4s_t{0.f, 0.f, 0.f, 0.f};
  float dbacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dbacc[i] = 0.f;
  uint2 pre[STAGE_SLOTS];
  for (int blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const int n = blk / blocks_per_img, oh0 = (blk - n * blocks_per_img) * ROWS_PER_WG;
    __syncthreads();                                                         // previous block done with xin / dyt
#pragma unroll
    for (int q = 0; q < STAGE_SLOTS; ++q) {
      const int i = threadIdx.x + q * 256;
      const int rr = i / row_u2, j = i - rr * row_u2;
      const int ih = 2 * oh0 - 3 + rr;
      pre[q] = make_uint2(0u, 0u);
      if (i < nchunks && ih >= 0 && ih < H)
        pre[q] = *reinterpret_cast<const uint2*>(x + ((long long)n * H + ih) * row_elems + 4 * j);
    }
#pragma unroll
    for (int q = 0; q < STAGE_SLOTS; ++q) {
      const int i = threadIdx.x + q * 256;
      const int rr = i / row_u2, j = i - rr * row_u2;
      if (i < nchunks) *reinterpret_cast<uint2*>(xin + rr * RS + 12 + 4 * j) = pre[q];
    }
    const long long m_base = ((long long)n * OH + oh0) * OW;
    // dy rounds two ahead (register sets gA / gB alternate): with three workgroups per CU this keeps enough dy in
    // flight to cover the HBM latency (one round of look-ahead with two workgroups per CU ran at ~2 TB/s)
    auto load_dy = [&](int rnd, uint4* dst) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dst[j] = *reinterpret_cast<const uint4*>(dy + (m_base + rnd * 64 + (threadIdx.x >> 3) + 32 * j) * 64 +
                                                 (threadIdx.x & 7) * 8);
    };
    auto round = [&](int rnd, uint4* gr) {
      u16* dt = dyt + (rnd & 1) * 64 * OUT_LD;
      // ---- transpose this round's dy tile into dyT[c][px]; bias column sums on the way
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int px = (threadIdx.x >> 3) + 32 * j, c8 = threadIdx.x & 7;
        const u16* hv = reinterpret_cast<const u16*>(&gr[j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          // 16-byte pixel chunks of channel row c8*8+i are XOR-swizzled by c8 (rows 8 apart are 1152 B apart, i.e.
          // the same bank: unswizzled, the 8 channel groups of a wave's store hit one bank 8 ways)
          dt[(c8 * 8 + i) * OUT_LD + (((px >> 3) ^ c8) << 3) + (px & 7)] = hv[i];
          dbacc[i] += bf2f(hv[i]);
        }
      }
      if (rnd + 2 < rounds) load_dy(rnd + 2, gr);
      __syncthreads();
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        // B fragments: pixels p = rnd*64 + ch*32 + 8*hg + j (same output row: OW % 8 == 0)
        const int p0 = rnd * 64 + ch * 32 + 8 * hg;
        const int ohl = p0 / OW, ow0 = p0 - ohl * OW;
        const u16* wb = xin + 2 * ohl * RS + (2 * ow0 + 1) * 3;
        bf16x8s_t bfr[3];
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3) {
          union {
            u16 h[8];
            bf16x8s_t v;
          } bb;
#pragma unroll
          for (int j = 0; j < 8; ++j) bb.h[j] = wb[koff[t3] + 6 * j];
          bfr[t3] = bb.v;
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int row = ct * 16 + col;
          const bf16x8s_t a =
              *reinterpret_cast<const bf16x8s_t*>(dt + row * OUT_LD + (((ch * 4 + hg) ^ (row >> 3)) << 3));
#pragma unroll
          for (int t3 = 0; t3 < 3; ++t3)
            acc[ct][t3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[t3], acc[ct][t3], 0, 0, 0);
        }
      }
    };
    uint4 gA[2], gB[2];
    load_dy(0, gA);
    if (rounds > 1) load_dy(1, gB);
    for (int rnd = 0; rnd < rounds; rnd += 2) {
      round(rnd, gA);
      if (rnd + 1 < rounds) round(rnd + 1, gB);
    }
  }
  // ---- partial dW: lane holds C[co = ct*16 + 4*hg + j][k = (3*wave + t3)*16 + col]
  float* pw = part + (long long)blockIdx.x * 64 * 192;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
      for (int j = 0; j < 4; ++j) pw[(ct * 16 + 4 * hg + j) * 192 + (3 * wave + t3) * 16 + col] = acc[ct][t3][j];
  // ---- partial bias sums: threads with the same channel group (threadIdx.x & 7) combine through LDS
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) dbs[threadIdx.x * 8 + i] = dbacc[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c8 = threadIdx.x >> 3, i = threadIdx.x & 7;
    float sum = 0.f;
    for (int t = c8; t < 256; t += 8) sum += dbs[t * 8 + i];
    part_db[(long long)blockIdx.x * 64 + c8 * 8 + i] = sum;
  }
}

// dW[co][c][r][s] = sum_g part[g][co][r*24 + s*3 + c]; db[co] = sum_g part_db[g][co]. A block covers 16 outputs x
// 16 partial slices (each thread sums every 16th partial, 4 loads in flight), then the 16 slice sums are added in a
// fixed order through LDS: deterministic, and ~600 blocks instead of 37 serial-latency-bound ones.
__global__ void __launch_bounds__(256) stem_wrw_reduce(const float* __restrict__ part, const float* __restrict__ part_db,
                                                       int G, float* __restrict__ dW, float* __restrict__ db) {
  __shared__ float red[16][17];
  const int ol = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + ol;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (o < 64 * 147) {
    const int co = o / 147, rem = o - co * 147, c = rem / 49, rs = rem - c * 49, r = rs / 7, s = rs - r * 7;
    const float* src = part + co * 192 + r * 24 + s * 3 + c;
    int g = sl;
    for (; g + 48 < G; g += 64) {
      a0 += src[(long long)g * 12288];
      a1 += src[(long long)(g + 16) * 12288];
      a2 += src[(long long)(g + 32) * 12288];
      a3 += src[(long long)(g + 48) * 12288];
    }
    for (; g < G; g += 16) a0 += src[(long long)g * 12288];
  } else if (db && o < 64 * 147 + 64) {
    const int co = o - 64 * 147;
    for (int g = sl; g < G; g += 16) a0 += part_db[(long long)g * 64 + co];
  }
  red[ol][sl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[ol][i];
    if (o < 64 * 147) dW[o] = t;
    else if (db && o < 64 * 147 + 64) db[o - 64 * 147] = t;
  }
}

DL4J_API long long dl4j_stem_wrw_workspace_floats(int N, int OH) {
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long long G = (long long)kWrwWgPerCu * ncu;
  return G * (64 * 192 + 64);
}

// x: [N,H,W,3] bf16 input; dy: [N,OH,OW,64] bf16; dW: [64][3][7][7] fp32 (overwritten); db: [64] fp32 or null.
// ws: >= dl4j_stem_wrw_workspace_floats floats. Returns -1 when the shape is not the stem's.
DL4J_API int dl4j_stem_conv_wrw(const void* x, const void* dy, float* dW, float* db, float* ws, int N, int H, int W,
                                int OH, int OW, hipStream_t s) {
  if (N < 1 || OH % ROWS_PER_WG != 0 || OW % 16 != 0 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1 ||
      (3 * W) % 4 != 0 || (ROWS_PER_WG * OW) % 64 != 0)
    return -1;
  int RS = 12 + 3 * W;
  const int need = 6 * (OW - 1) + 3 + 24 + 2;
  if (RS < need) RS = need;
  RS = (RS + 15) & ~15;
  const size_t lds = (size_t)IN_ROWS * RS * 2 + 2 * 64 * OUT_LD * 2 + 256 * 8 * 4;
  if (lds > 64 * 1024 || (IN_ROWS - 1) * (3 * W / 4) > STAGE_SLOTS * 256) return -1;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int nblocks = N * (OH / ROWS_PER_WG);
  const int G = nblocks < kWrwWgPerCu * ncu ? nblocks : kWrwWgPerCu * ncu;   // == the workspace's partial count
  float* part = ws;
  float* part_db = ws + (long long)G * 64 * 192;
  hipLaunchKernelGGL(stem_conv_wrw, dim3(G), dim3(256), lds, s, (const u16*)x, (const u16*)dy, part, part_db, N, H, W,
                     OH, OW, RS);
  hipLaunchKernelGGL(stem_wrw_reduce, dim3((64 * 147 + 64 + 15) / 16), dim3(256), 0, s, part, part_db, G, dW, db);
  return (int)hipGetLastError();
}

// Fragment-packed stem weights for stem_conv_fwd, rebuilt whenever the weights change (every training step): pk is
// bf16 [4][6][64][8]; element (i, j, m, n) holds tap row = j*32 + (m/16)*8 + n of a [192][64] image whose row
// r*24 + s*3 + c carries W[k][c][r][s] for k = i*16 + m%16 (rows with (row % 24) >= 21 are zero padding).
// W is read through element strides (k, c, r, s), so any view of the [64][3][7][7] weights works. One launch
// instead of the permute / index-copy / reshape sequence on the host side.
__global__ __launch_bounds__(256) void stem_pack_weights(const u16* __restrict__ w, u16* __restrict__ pk,
                                                         long long sk, long long sc, long long sr, long long ss) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 4 * 6 * 64 * 8) return;
  const int n = e & 7, m = (e >> 3) & 63, j = (e >> 9) % 6, i = e / (6 * 512);
  const int row = j * 32 + (m >> 4) * 8 + n, k = i * 16 + (m & 15);
  const int r = row / 24, rem = row - r * 24;
  u16 v = 0;
  if (r < 7 && rem < 21) {                     // rows 168..191 (r == 7) are padding too
    const int s_ = rem / 3, c = rem - s_ * 3;
    v = w[k * sk + c * sc + r * sr + s_ * ss];
  }
  pk[e] = v;
}

DL4J_API int dl4j_stem_pack_weights(const void* w, void* pk, long long sk, long long sc, long long sr, long long ss,
                                    hipStream_t s) {
  hipLaunchKernelGGL(stem_pack_weights, dim3((4 * 6 * 64 * 8 + 255) / 256), dim3(256), 0, s, (const u16*)w, (u16*)pk,
                     sk, sc, sr, ss);
  return (int)hipGetLastError();
}
