// Convolution weight gradient with the input halo staged once per pixel chunk (round-3 "tap reuse" kernel).
//
//   dW[k][c][r][s] = sum_p dY[p][k] * X[pix(p) + (r, s)][c]            (p = output pixel, NHWC operands)
//
// Why a separate kernel: the implicit-GEMM wrw kernels (conv_igemm.hip igemm_wrw, conv_gemm.hip conv_wrw_glds) treat
// the (r, s, c) columns as an im2col matrix, so every column tile re-reads dY and every tap re-reads X from L2/MALL:
// ~9x + 5x the operand bytes for a 3x3 conv with C = 64, which bounds them at 100-200 us per ResNet shape (the
// round-3 profile, profiles/r3_wrw_v3_vs_r2_bs512.log) while the FLOPs need ~12 us of MFMA time.
// Here one workgroup owns an output block of BK output channels x BC input channels x ALL taps and walks a range of
// pixel chunks (G images x TH output rows). Per chunk it DMAs (global_load_lds, 16 B per lane, zero page for the
// padding halo) the dY rows [PCP pixels][BK] and the X halo [G*(TH+R-1)*(OW+S-1)][BC] into LDS once; the 9 taps are
// 9 shifted address sets into the same X image. Fragments of both operands are hardware-transposed reads
// (ds_read_b64_tr_b16): the reduction runs over pixels, which are the LDS rows. The LDS rows are XOR-swizzled in
// 16-byte chunks so the 4 rows x 64 B a half-wave reads hit 16 distinct bank slots.
// Each (split, tile) writes its fp32 block into a slab part[split][K][RS*C] (no atomics); wrw_halo_reduce sums the
// slabs in a fixed order and writes the DL4J [K][C][R][S] layout (+ the conv-bias gradient from per-split column
// sums of the staged dY rows): bitwise deterministic. Opt-in alternative (DL4J_AMD_WRW_TREE): the slabs summed
// inside wrw_halo by a last-arrival reduction tree (tree_reduce below), measured slower (profiles/r6_wrw_tree.txt).
// 1x1 convolutions (any stride, no padding) use the same engine with a "gather" X image (row p = X pixel of p).
// Reference semantics: ConvolutionLayer.backpropGradient (deeplearning4j-nn/.../layers/convolution/
// ConvolutionLayer.java:131-265), cuDNN's backward-filter in CudnnConvolutionHelper.java:179-246.
#include "mfma_tile.h"

namespace {

struct FDv {
  unsigned d, mul, shr;
};
__device__ __forceinline__ unsigned fdv(unsigned n, const FDv& f) {
  return f.d == 1 ? n : (__umulhi(n, f.mul) >> f.shr);
}

struct HaloArgs {
  const u16* X;
  const u16* dY;
  float* part;           // [splits][K][RS*C]
  float* partb;          // [splits][K] conv-bias partials or null
  int N, H, W, C, K, OH, OW, sh, sw, ph, pw;
  int G, TH;             // halo chunk = G images x TH output rows (halo mode)
  int PC, PCP;           // real / padded (multiple of 16) pixels per chunk
  int HR, HW;            // halo rows / cols per image
  int bands;             // OH / TH
  int nch;               // number of chunks
  int cps;               // chunks per split
  int tiles_k, tiles_c;
  int M;                 // N*OH*OW (gather mode)
  FDv fHW, fHRHW, fOW, fTHOW, fOHOW;
  // in-kernel slab reduction (null ticket = separate wrw_halo_reduce launch): arrival counters of this launch,
  // tkpt per tile; fan-in of the reduction tree; the final outputs
  unsigned* ticket;
  int tkpt, fan, splits;
  float* dW;
  float* db;
};

template <int CPR>
__device__ __forceinline__ int swz(int row) {
  if constexpr (CPR >= 16) return (row & 3) << 2;
  else if constexpr (CPR == 8) return ((row >> 1) & 1) << 2;
  else return 0;
}
// byte offset of element (row, col) in an LDS image with CPR 16-byte chunks per row
template <int CPR>
__device__ __forceinline__ int loff(int row, int col) {
  return row * (CPR * 16) + ((((col >> 3) ^ swz<CPR>(row))) << 4) + ((col & 7) << 1);
}

typedef __attribute__((address_space(3))) const char* lds_cptr;

// transposed fragment: MFMA rows = image columns [cbase, cbase + 32), reduction = image rows r0 (k) / r1 (k + 4)
template <int DT, int CPR>
__device__ __forceinline__ typename MfmaT<DT>::v8 frag_rows(const char* T, int r0, int r1, int col) {
  typedef typename MfmaT<DT>::v8 v8;
  const unsigned a0 = (unsigned)(uintptr_t)((lds_cptr)T + loff<CPR>(r0, col));
  const unsigned a1 = (unsigned)(uintptr_t)((lds_cptr)T + loff<CPR>(r1, col));
  s16x8_t f;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.hi) : "v"(a1));
  return __builtin_bit_cast(v8, f);
}

template <int N> __device__ __forceinline__ void lgkm_wait() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt is a 4-bit counter");
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
  else if constexpr (N == 11) asm volatile("s_waitcnt lgkmcnt(11)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
  else if constexpr (N == 13) asm volatile("s_waitcnt lgkmcnt(13)" ::: "memory");
  else if constexpr (N == 14) asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
}

// transposed fragment from two precomputed LDS byte addresses (reduction rows k and k + 4 of this lane)
template <int DT>
__device__ __forceinline__ typename MfmaT<DT>::v8 frag_at(unsigned a0, unsigned a1) {
  typedef typename MfmaT<DT>::v8 v8;
  s16x8_t f;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.hi) : "v"(a1));
  return __builtin_bit_cast(v8, f);
}

// X halo image row pitch in 16-byte slots: 4 consecutive rows x 4 slots (one half-wave of a transposed read) land on
// 16 distinct slots when the pitch is 4 or 12 (mod 16); a LINEAR pitch makes every tap a constant byte offset.
template <int CPR> struct XPitch {
  static constexpr int slots = CPR == 4 ? 4 : CPR == 8 ? 12 : CPR == 16 ? 20 : 36;
};

template <int N> __device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt is a 6-bit counter");
  // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] (7 = no wait) | lgkmcnt[11:8] (15 = no wait) | vmcnt[5:4] at [15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// In-kernel fixed-order slab reduction (replaces the wrw_halo_reduce launch when HaloArgs::ticket is set).
// The splits of one tile form a tree with fan-in F: slab s is leaf s; the block that arrives last at a node (agent-
// scope arrival counter, reset by that block) sums the node's children in index order and stores the sum in place
// over its first child's slab, then climbs; at the root the sum goes to dW (DL4J [K][C][R][S] layout) and db. Every
// reader is the only block touching those slabs at that moment, slab stores are sc1 write-through and slab reads are
// agent-scope atomic loads, so no L2 invalidate is needed; the summation order depends only on the split count:
// bitwise deterministic. The serial tail per level is F slabs of one tile, against a whole-GPU reduce launch.
typedef __attribute__((address_space(1))) unsigned gq32_w;
typedef __attribute__((address_space(1))) unsigned long long gq64_w;
__device__ __forceinline__ float4 ld_coh16(const float* p) {
  const unsigned long long lo = __hip_atomic_load((gq64_w*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long hi = __hip_atomic_load((gq64_w*)(p + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float4(__uint_as_float((unsigned)lo), __uint_as_float((unsigned)(lo >> 32)),
                     __uint_as_float((unsigned)hi), __uint_as_float((unsigned)(hi >> 32)));
}
__device__ __forceinline__ float ld_coh4(const float* p) {
  return __uint_as_float(__hip_atomic_load((gq32_w*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int BK, int BC, int T>
__device__ __forceinline__ void tree_reduce(const HaloArgs& a, int split, int tile, int k0, int c0, bool do_bias, int tid,
                                         int* flag) {
  constexpr int C4 = BC / 4, ITEMS = BK * T * C4, PB = 8;
  const int RSC = T * a.C, F = a.fan;
  const long long slab_sz = (long long)a.K * RSC;
  unsigned* cnt = a.ticket + (long long)tile * a.tkpt;
  int node = split, n = a.splits, off = 0;
  long long stride = 1;                                  // leaves between consecutive nodes of this level
  for (;;) {
    const int parent = node / F, first = parent * F, nch = min(F, n - first), np = (n + F - 1) / F;
    if (n > 1) {
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add((gq32_w*)&cnt[off + parent], 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(nch - 1);
        if (last) __hip_atomic_store((gq32_w*)&cnt[off + parent], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      const int last = *flag;
      __syncthreads();
      if (!last) return;
    }
    const bool root = np == 1;
    float* dst = a.part + (long long)first * stride * slab_sz;
    // passes of PB float4 per thread (bounded registers; the block's main-loop accumulators are dead here)
#pragma unroll 1
    for (int p0 = 0; p0 < ITEMS; p0 += 256 * PB) {
      float4 v[PB];
      int o[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int it = p0 + tid + i * 256;
        const int k = k0 + it / (T * C4), rem = it % (T * C4), t = rem / C4, c = c0 + 4 * (rem % C4);
        o[i] = (it < ITEMS && k < a.K && c < a.C) ? k * RSC + t * a.C + c : -1;
      }
      for (int ch = 0; ch < nch; ++ch) {
        const float* src = a.part + (long long)(first + ch) * stride * slab_sz;
#pragma unroll
        for (int i = 0; i < PB; ++i)
          if (o[i] >= 0) {
            const float4 w = ld_coh16(src + o[i]);
            v[i].x += w.x; v[i].y += w.y; v[i].z += w.z; v[i].w += w.w;
          }
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        if (o[i] < 0) continue;
        if (root) {
          const int k = o[i] / RSC, rem = o[i] - k * RSC, t = rem / a.C, c = rem - t * a.C;
          float* q = a.dW + ((long long)k * a.C + c) * T + t;
          q[0] = v[i].x; q[T] = v[i].y; q[2 * T] = v[i].z; q[3 * T] = v[i].w;
        } else {
          st_coh16(dst + o[i], v[i].x, v[i].y, v[i].z, v[i].w);
        }
      }
    }
    if (do_bias && tid < BK && k0 + tid < a.K) {
      float sb = 0.f;
      for (int ch = 0; ch < nch; ++ch) sb += ld_coh4(a.partb + (long long)(first + ch) * stride * a.K + k0 + tid);
      if (root) a.db[k0 + tid] = sb;
      else st_coh4(a.partb + (long long)first * stride * a.K + k0 + tid, sb);
    }
    if (root) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    off += np;
    node = parent;
    n = np;
    stride *= F;
  }
}

// Compile-time stage geometry of one instantiation (shared with the host planner).
constexpr int kHaloStage = 52 * 1024;          // 3 stages = 156 KB of the 160 KB LDS (one block per CU)
constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
struct StageGeo {
  int DI, XI, DBYTES, XBYTES, STB;
};
constexpr StageGeo stage_geo(bool halo, int NB, int BK, int BC) {
  const int PCP = NB * 16;
  const int DI = cdiv(PCP * BK * 2, 4 * 1024);
  const int XI = halo ? (kHaloStage - DI * 4 * 1024) / (4 * 1024) : cdiv(PCP * BC * 2, 4 * 1024);
  return StageGeo{DI, XI, DI * 4096, XI * 4096, (DI + XI) * 4096};
}
constexpr int xpitch_slots(int BC) { return BC == 32 ? 4 : BC == 64 ? 12 : BC == 128 ? 20 : 36; }

// Waves: TG tap groups x WK x WC; each wave owns FK x FC fragments of 32x32 for the taps of its group.
// NB: 16-pixel reduction blocks per chunk (PCP = 16*NB). HALO: X image = padded halo of the chunk (RR x SS taps,
// stride 1, linear row pitch); else a 1x1 "gather" image (row p = input pixel of output pixel p, XOR rows).
// D: fragment-read units in flight ahead of the MFMAs (lgkmcnt <= 15).
// DMA: every wave issues exactly DI + XI global_load_lds per chunk (padding slots read the zero page) from per-lane
// descriptors computed once, so the NST-deep chunk ring waits with a counted vmcnt.
template <int DT, int WK, int WC, int TG, int FK, int FC, int RR, int SS, int NB, bool HALO, int D>
__global__ __launch_bounds__(WK* WC* TG * 64, 1) void wrw_halo(HaloArgs a) {
  constexpr int NW = WK * WC * TG;
  static_assert(NW == 4, "256-thread blocks");
  constexpr int BK = WK * FK * 32, BC = WC * FC * 32;
  constexpr int CPRK = BK / 8, CPRC = BC / 8;
  constexpr int XPS = HALO ? xpitch_slots(BC) : CPRC;             // X image slots per row
  constexpr int T = RR * SS;
  constexpr int TPG = (T + TG - 1) / TG;
  constexpr int PCP = NB * 16;
  constexpr int RA = 2 * FK, RB = 2 * FC;                           // LDS reads per A / B fragment set
  constexpr StageGeo SG = stage_geo(HALO, NB, BK, BC);
  constexpr int DI = SG.DI, XI = SG.XI, DBYTES = SG.DBYTES, STB = SG.STB;
  constexpr int NST = HALO ? 3 : 2;
  constexpr int PER = DI + XI;                                      // glds per wave per chunk
  static_assert(PER <= 63, "vmcnt range");
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[NST * STB];

  const int ntile = a.tiles_k * a.tiles_c;
  const int hb = xcd_remap_g(blockIdx.x, gridDim.x);         // the tiles of one split share an XCD (same chunks)
  const int split = hb / ntile, tile = hb - split * ntile;
  const int tk = tile % a.tiles_k, tc = tile / a.tiles_k;
  const int k0 = tk * BK, c0 = tc * BC;
  const int ch0 = split * a.cps, ch1 = min(a.nch, ch0 + a.cps);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u16* X = a.X;
  const u16* dY = a.dY;

  // ---- per-lane DMA descriptors (chunk-invariant): element offsets relative to the chunk base, -1 = zero page
  int drel[DI], drow[DI], xrel[XI], xrr[XI];
#pragma unroll
  for (int s = 0; s < DI; ++s) {
    const int q = (s * NW + wid) * 64 + lane;
    const int row = q / CPRK;
    const int kk = k0 + (((q % CPRK) ^ swz<CPRK>(row)) << 3);
    int rel = -1;
    if (kk < a.K && row < PCP) {
      if constexpr (HALO) {
        if (row < a.PC) {
          const int g = row / (a.TH * a.OW), rem = row - g * (a.TH * a.OW);
          const int t = rem / a.OW, ow = rem - t * a.OW;
          rel = ((g * a.OH + t) * a.OW + ow) * a.K + kk;
        }
      } else {
        rel = row * a.K + kk;
      }
    }
    drel[s] = rel;
    drow[s] = row;
  }
#pragma unroll
  for (int s = 0; s < XI; ++s) {
    const int q = (s * NW + wid) * 64 + lane;
    const int row = q / XPS;
    int rel = -1, rr = 0;
    if constexpr (HALO) {
      const int j = q - row * XPS;
      const int cc = c0 + (j << 3);
      if (j < CPRC && cc < a.C && row < a.G * a.HR * a.HW) {
        const int g = row / (a.HR * a.HW), rem = row - g * (a.HR * a.HW);
        rr = rem / a.HW;
        const int iw = rem - rr * a.HW - a.pw;
        if (iw >= 0 && iw < a.W) rel = ((g * a.H + rr) * a.W + iw) * a.C + cc;
      }
    } else {
      const int cc = c0 + (((q % CPRC) ^ swz<CPRC>(row)) << 3);
      if (cc < a.C && row < PCP) rel = cc;
      rr = row;
    }
    xrel[s] = rel;
    xrr[s] = rr;
  }

  // ---- DMA of one chunk into stage st
  auto issue = [&](int ch, int st) {
    char* sd = smem + st * STB;
    char* sx = sd + DBYTES;
    if constexpr (HALO) {
      const int img = ch / a.bands;
      const int n0 = img * a.G, oh0 = (ch - img * a.bands) * a.TH;
      const u16* db = dY + ((long long)n0 * a.OH + oh0) * a.OW * a.K;
      const long long xb = ((long long)n0 * a.H + oh0 - a.ph) * a.W * a.C;
#pragma unroll
      for (int s = 0; s < DI; ++s)
        glds16(drel[s] >= 0 ? (const void*)(db + drel[s]) : (const void*)gemm_zero_page, sd + (s * NW + wid) * 1024);
#pragma unroll
      for (int s = 0; s < XI; ++s) {
        const int ih = oh0 - a.ph + xrr[s];
        const bool ok = xrel[s] >= 0 && ih >= 0 && ih < a.H;
        glds16(ok ? (const void*)(X + xb + xrel[s]) : (const void*)gemm_zero_page, sx + (s * NW + wid) * 1024);
      }
    } else {
      const int pbase = ch * PCP;
      const int pc = min(PCP, a.M - pbase);
      const u16* db = dY + (long long)pbase * a.K;
#pragma unroll
      for (int s = 0; s < DI; ++s)
        glds16(drel[s] >= 0 && drow[s] < pc ? (const void*)(db + drel[s]) : (const void*)gemm_zero_page,
               sd + (s * NW + wid) * 1024);
#pragma unroll
      for (int s = 0; s < XI; ++s) {
        const void* src = gemm_zero_page;
        if (xrel[s] >= 0 && xrr[s] < pc) {
          const unsigned pix = (unsigned)(pbase + xrr[s]);
          long long xo;
          if (a.sh == 1 && a.sw == 1) {
            xo = pix;
          } else {
            const unsigned n = fdv(pix, a.fOHOW);
            const unsigned rem = pix - n * a.fOHOW.d;
            const unsigned oh = fdv(rem, a.fOW);
            const unsigned ow = rem - oh * a.fOW.d;
            xo = ((long long)n * a.H + oh * a.sh) * a.W + ow * a.sw;
          }
          src = X + xo * a.C + xrel[s];
        }
        glds16(src, sx + (s * NW + wid) * 1024);
      }
    }
  };

  // ---- per-lane fragment geometry. Reduction rows of block b: 16*b + kq (+4). Both XOR images have a swizzle of
  //      period 4 rows, so block b is block 0 + b*16 rows; the halo X image has a linear pitch, so tap t is + tdel[t].
  const int grp = lane >> 4;
  const int kq = (grp >> 1) * 8 + ((lane & 15) >> 2);
  const int colq = (grp & 1) * 16 + 4 * (lane & 3);
  const int tg = wid / (WK * WC), wrem = wid - tg * (WK * WC);
  const int wk = wrem / WC, wc = wrem - (wrem / WC) * WC;
  int aoff[2][FK];                                 // dY image byte offsets of block 0
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < FK; ++i) aoff[h][i] = loff<CPRK>(kq + 4 * h, (wk * FK + i) * 32 + colq);
  int boff[2][FC];                                 // X image byte offsets of block 0 (gather) / column part (halo)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < FC; ++j) {
      const int col = (wc * FC + j) * 32 + colq;
      boff[h][j] = HALO ? ((col >> 3) << 4) + ((col & 7) << 1) : loff<CPRC>(kq + 4 * h, col);
    }
  int xrow[NB][2];                                 // halo: X image byte offset of the row of reduction row (tap 0)
  if constexpr (HALO) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = 16 * b + kq + 4 * h;
        int v = 0;
        if (p < a.PC) {
          const int g = p / (a.TH * a.OW), rem = p - g * (a.TH * a.OW);
          const int t = rem / a.OW, ow = rem - t * a.OW;
          v = (g * a.HR + t) * a.HW + ow;
        }
        xrow[b][h] = v * (XPS * 16);
      }
  }
  const int hw_bytes = a.HW * XPS * 16;            // one halo row down (wave-uniform)

  // conv-bias partial: column sums of the staged dY rows (tiles with tc == 0 only), 16-byte reads
  const bool do_bias = a.partb != nullptr && tc == 0;
  constexpr int BRG = 256 / CPRK;                  // row groups
  const int blc = tid % CPRK, brg = tid / CPRK;
  float bs[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  // one chunk for the waves of tap group G_ (taps [G_*TPG, min(T, G_*TPG + TPG)))
  auto compute = [&](auto G_, unsigned sd, unsigned sx, auto& acc) {
    constexpr int G = decltype(G_)::value;
    constexpr int t0 = G * TPG;
    constexpr int NTG = (T - t0) < TPG ? (T - t0) : TPG;
    constexpr int NU = NB * NTG;                   // units = (block, tap)
    constexpr int NBUF = D + 1;
    // opaque per-chunk copies: keep the address arithmetic inside the chunk instead of hoisted + spilled
    unsigned ab[2][FK], bb[2][FC];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < FK; ++i) { ab[h][i] = sd + aoff[h][i]; asm volatile("" : "+v"(ab[h][i])); }
#pragma unroll
      for (int j = 0; j < FC; ++j) { bb[h][j] = sx + boff[h][j]; asm volatile("" : "+v"(bb[h][j])); }
    }
    v8 fa[2][FK], fb[NBUF][FC];
    auto reads = [&](auto U_) {
      constexpr int u = decltype(U_)::value;
      constexpr int b = u / NTG, ti = u % NTG, t = t0 + ti;
      if constexpr (ti == 0) {
#pragma unroll
        for (int i = 0; i < FK; ++i)
          fa[b & 1][i] = frag_at<DT>(ab[0][i] + b * 16 * CPRK * 16, ab[1][i] + b * 16 * CPRK * 16);
      }
#pragma unroll
      for (int j = 0; j < FC; ++j) {
        if constexpr (HALO) {
          const unsigned tap = (t / SS) * hw_bytes + (t % SS) * (XPS * 16);
          fb[u % NBUF][j] = frag_at<DT>(bb[0][j] + xrow[b][0] + tap, bb[1][j] + xrow[b][1] + tap);
        } else {
          fb[u % NBUF][j] = frag_at<DT>(bb[0][j] + b * 16 * CPRC * 16, bb[1][j] + b * 16 * CPRC * 16);
        }
      }
    };
    sfor<0, (D < NU ? D : NU)>([&](auto U_) { reads(U_); });
    sfor<0, NU>([&](auto U_) {
      constexpr int u = decltype(U_)::value;
      if constexpr (u + D < NU) reads(IC<u + D>{});
      // reads issued after unit u's: units u+1 .. min(u+D, NU-1)
      constexpr int after = [] {
        int n = 0;
        for (int v = u + 1; v <= u + D && v < NU; ++v) n += ((v % NTG) == 0 ? RA : 0) + RB;
        return n;
      }();
      lgkm_wait<after>();
      __builtin_amdgcn_sched_barrier(0);
      constexpr int b = u / NTG, ti = u % NTG;
#pragma unroll
      for (int i = 0; i < FK; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j)
          acc[ti][i][j] = MfmaT<DT>::mma(fb[u % NBUF][j], fa[b & 1][i], acc[ti][i][j]);
    });
  };

  // ---- slab stores: D[c][k] with k = lane & 31, c = 8*(e/4) + 4*(lane/32) + e%4 (4 consecutive channels per float4)
  const int RSC = T * a.C;
  float* slab = a.part + (long long)split * a.K * RSC;
  const int h = lane >> 5;
  // the whole chunk loop per tap group: the accumulators stay in place across chunks (a group branch inside the loop
  // made the compiler merge and re-copy them every chunk)
  auto body = [&](auto G_) {
    constexpr int G = decltype(G_)::value;
    constexpr int t0 = G * TPG;
    constexpr int NTG = (T - t0) < TPG ? (T - t0) : TPG;
    f32x16_t acc[NTG][FK][FC];
#pragma unroll
    for (int t = 0; t < NTG; ++t)
#pragma unroll
      for (int i = 0; i < FK; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[t][i][j][e] = 0.f;
    const int nloc = ch1 - ch0;
#pragma unroll
    for (int i = 0; i < NST - 1; ++i)
      if (i < nloc) issue(ch0 + i, i);
    for (int i = 0; i < nloc; ++i) {
      // chunk i landed (this wave's part): the ring still has chunk i+1 in flight when NST == 3
      if constexpr (NST == 3) {
        if (i + 1 < nloc) vm_wait<PER>();
        else vm_wait<0>();
      } else {
        vm_wait<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();                               // every wave's part landed; stage (i-1) % NST is free
      if (i + NST - 1 < nloc) issue(ch0 + i + NST - 1, (i + NST - 1) % NST);
      const char* sd = smem + (i % NST) * STB;
      const unsigned sdl = (unsigned)(uintptr_t)((lds_cptr)sd);
      if (do_bias) {
        constexpr int NR = (PCP + BRG - 1) / BRG;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          if (brg + r * BRG >= PCP) continue;
          const unsigned adr = sdl + loff<CPRK>(brg + r * BRG, blc * 8);
          s16x8_t v;
          // read + wait in one statement: the compiler must not see (and copy) the value before it has landed
          asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(adr) : "memory");
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const u16 u = (u16)v[e];
            bs[e] += DT == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
          }
        }
      }
      compute(G_, sdl, sdl + DBYTES, acc);
    }
#pragma unroll
    for (int i = 0; i < FK; ++i) {
      const int k = k0 + (wk * FK + i) * 32 + (lane & 31);
      if (k >= a.K) continue;
#pragma unroll
      for (int ti = 0; ti < NTG; ++ti)
#pragma unroll
        for (int j = 0; j < FC; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = c0 + (wc * FC + j) * 32 + 8 * q + 4 * h;
            if (c < a.C) {
              float* dst = slab + (long long)k * RSC + (t0 + ti) * a.C + c;
              if (a.ticket)     // read back by another block's tree step: written through the XCD-local L2
                st_coh16(dst, acc[ti][i][j][4 * q], acc[ti][i][j][4 * q + 1], acc[ti][i][j][4 * q + 2],
                         acc[ti][i][j][4 * q + 3]);
              else
                *reinterpret_cast<float4*>(dst) = make_float4(acc[ti][i][j][4 * q], acc[ti][i][j][4 * q + 1],
                                                              acc[ti][i][j][4 * q + 2], acc[ti][i][j][4 * q + 3]);
            }
          }
    }
  };
  if constexpr (TG == 1) {
    body(IC<0>{});
  } else {
    if (tg == 0) body(IC<0>{});
    else body(IC<1>{});
  }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);
    vm_wait<0>();
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[brg * BK + blc * 8 + e] = bs[e];
    __syncthreads();
    if (tid < BK && k0 + tid < a.K) {
      float sum = 0.f;
      for (int r = 0; r < BRG; ++r) sum += red[r * BK + tid];
      if (a.ticket) st_coh4(a.partb + (long long)split * a.K + k0 + tid, sum);
      else a.partb[(long long)split * a.K + k0 + tid] = sum;
    }
  }
  if (a.ticket) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // this wave's slab stores are in memory
    __syncthreads();                                               // ... and every wave's; LDS reads done
    tree_reduce<BK, BC, T>(a, split, tile, k0, c0, do_bias, tid, reinterpret_cast<int*>(smem));
  }
}

// Fixed-order slab reduction: part[split][K][RS][C] -> dW[K][C][R][S]. Block = 16 float4 columns (64 consecutive slab
// elements) x 16 split phases; phase ph sums splits ph, ph+16, ... with 8 unconditional (clamped) 16-byte loads in
// flight, the 16 phase sums are added in order: deterministic. Bias partials [splits][K] reduce in the extra block.
__global__ __launch_bounds__(256) void wrw_halo_reduce(const float* __restrict__ part, float* __restrict__ dW,
                                                       int splits, int K, int C, int RS, const float* __restrict__ partb,
                                                       float* __restrict__ db) {
  const long long total = (long long)K * C * RS;              // multiple of 8 (C % 8 == 0)
  const int nb = (int)((total + 63) / 64);
  if ((int)blockIdx.x >= nb) {
    // bias: 64 output channels x 4 split phases per block, 8 loads in flight per thread, fixed order
    __shared__ float rb[256];
    const int k = ((int)blockIdx.x - nb) * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
    float sb = 0.f;
    if (k < K)
      for (int sp0 = ph; sp0 < splits; sp0 += 4 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = partb[(long long)min(sp0 + 4 * u, splits - 1) * K + k];
#pragma unroll
        for (int u = 0; u < 8; ++u) sb += sp0 + 4 * u < splits ? v[u] : 0.f;
      }
    rb[threadIdx.x] = sb;
    __syncthreads();
    if (ph == 0 && k < K) db[k] = ((rb[threadIdx.x] + rb[threadIdx.x + 64]) + rb[threadIdx.x + 128]) + rb[threadIdx.x + 192];
    return;
  }
  const int col = threadIdx.x & 15, ph = threadIdx.x >> 4;
  long long src = (long long)blockIdx.x * 64 + col * 4;
  const bool live = src < total;
  if (!live) src = 0;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  for (int sp0 = ph; sp0 < splits; sp0 += 16 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int sp = min(sp0 + 16 * u, splits - 1);
      v[u] = *reinterpret_cast<const float4*>(part + sp * total + src);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float m = sp0 + 16 * u < splits ? 1.f : 0.f;
      float4& acc = (u & 1) ? s1 : s0;
      acc.x = fmaf(m, v[u].x, acc.x); acc.y = fmaf(m, v[u].y, acc.y);
      acc.z = fmaf(m, v[u].z, acc.z); acc.w = fmaf(m, v[u].w, acc.w);
    }
  }
  __shared__ float4 red[256];
  red[threadIdx.x] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
  __syncthreads();
  if (ph == 0 && live) {
    float4 v = red[col];
    for (int p = 1; p < 16; ++p) {
      const float4 w = red[p * 16 + col];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long o = src + e;
      const int c = (int)(o % C);
      const long long t = o / C;
      const int rs = (int)(t % RS);
      const long long k = t / RS;
      dW[(k * C + c) * RS + rs] = vv[e];
    }
  }
}

FDv make_fdv(unsigned d) {
  FDv f;
  f.d = d < 1 ? 1 : d;
  if (f.d == 1) { f.mul = 0; f.shr = 0; return f; }
  unsigned l = 0;
  while ((1u << l) < f.d) ++l;
  const unsigned p = 31 + l;
  f.mul = (unsigned)(((1ull << p) + f.d - 1) / f.d);
  f.shr = p - 32;
  return f;
}

// variants: 1 = 64x64 x 3x3 taps (stride 1, dilation 1, halo), 2 = 128x128 1x1, 3 = 256x64 1x1, 4 = 64x256 1x1
struct Plan {
  int ok, variant, NB, G, TH, BK, BC;
  HaloArgs a;
  int splits;
};


Plan make_plan(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int OH,
               int OW, int variant, int splits) {
  Plan P = {};
  P.ok = 0;
  if (C % 8 || K % 8) return P;
  const bool is1x1 = R == 1 && S == 1 && ph == 0 && pw == 0;
  const bool is3x3 = R == 3 && S == 3 && sh == 1 && sw == 1 && dh == 1 && dw == 1;
  if (variant == 0) {
    if (is3x3) variant = 1;
    else if (is1x1) variant = (C <= 64 && K >= 256) ? 3 : (K <= 64 && C >= 256) ? 4 : 2;
    else return P;
  }
  if (variant == 1 && !is3x3) return P;
  if (variant >= 2 && !is1x1) return P;
  if (variant < 1 || variant > 4) return P;
  static const int bk[5] = {0, 64, 128, 256, 64}, bc[5] = {0, 64, 128, 64, 256};
  P.variant = variant;
  P.BK = bk[variant];
  P.BC = bc[variant];
  HaloArgs& a = P.a;
  a.N = N; a.H = H; a.W = W; a.C = C; a.K = K; a.OH = OH; a.OW = OW; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.M = N * OH * OW;
  if (variant == 1) {
    // chunk = G images x TH rows with PCP = 16*NB, NB in {7, 4}; best padding efficiency within the LDS budget
    double best = 0.0;
    for (int nbv : {7, 4}) {
      for (int mode = 0; mode < 2; ++mode) {
        const int lim = mode == 0 ? OH : N;
        for (int v = 1; v <= lim; ++v) {
          int G = 1, TH = OH;
          if (mode == 0) { if (OH % v) continue; TH = v; }
          else { if (N % v) continue; G = v; }
          const int pc = G * TH * OW;
          if (pc > 16 * nbv || pc <= 16 * (nbv - 1)) continue;
          const int HR = TH + 2, HWd = OW + 2;
          const StageGeo sg = stage_geo(true, nbv, P.BK, P.BC);
          if ((long long)G * HR * HWd * xpitch_slots(P.BC) * 16 > sg.XBYTES) continue;
          const double eff = (double)pc / (16.0 * nbv) + (nbv == 7 ? 1e-3 : 0.0);
          if (eff > best) {
            best = eff;
            P.NB = nbv; P.G = G; P.TH = TH;
          }
        }
      }
    }
    if (best == 0.0) return P;
    a.G = P.G; a.TH = P.TH;
    a.PC = P.G * P.TH * OW;
    a.PCP = 16 * P.NB;
    a.HR = P.TH + 2; a.HW = OW + 2;
    a.bands = OH / P.TH;
    a.nch = (N / P.G) * a.bands;
  } else {
    P.NB = 4;
    a.G = 1; a.TH = 1;
    a.PC = 64; a.PCP = 64;
    a.HR = 1; a.HW = 1;
    a.bands = 1;
    a.nch = (a.M + 63) / 64;
  }
  a.tiles_k = (K + P.BK - 1) / P.BK;
  a.tiles_c = (C + P.BC - 1) / P.BC;
  const int ntile = a.tiles_k * a.tiles_c;
  int sp = splits > 0 ? splits : (512 + ntile - 1) / ntile;
  if (sp > a.nch) sp = a.nch;
  if (sp < 1) sp = 1;
  a.cps = (a.nch + sp - 1) / sp;
  P.splits = (a.nch + a.cps - 1) / a.cps;
  a.fHW = make_fdv(a.HW);
  a.fHRHW = make_fdv(a.HR * a.HW);
  a.fOW = make_fdv(OW);
  a.fTHOW = make_fdv(a.TH * OW);
  a.fOHOW = make_fdv(OH * OW);
  P.ok = 1;
  return P;
}

template <int DT>
int launch_halo(const Plan& P, hipStream_t s) {
  const dim3 grid(P.a.tiles_k * P.a.tiles_c * P.splits), blk(256);
  const size_t L = 0;
  switch (P.variant) {
    case 1:
      if (P.NB == 7) hipLaunchKernelGGL((wrw_halo<DT, 1, 2, 2, 2, 1, 3, 3, 7, true, 2>), grid, blk, L, s, P.a);
      else hipLaunchKernelGGL((wrw_halo<DT, 1, 2, 2, 2, 1, 3, 3, 4, true, 2>), grid, blk, L, s, P.a);
      break;
    case 2: hipLaunchKernelGGL((wrw_halo<DT, 2, 2, 1, 2, 2, 1, 1, 4, false, 1>), grid, blk, L, s, P.a); break;
    case 3: hipLaunchKernelGGL((wrw_halo<DT, 4, 1, 1, 2, 2, 1, 1, 4, false, 1>), grid, blk, L, s, P.a); break;
    default: hipLaunchKernelGGL((wrw_halo<DT, 1, 4, 1, 2, 2, 1, 1, 4, false, 1>), grid, blk, L, s, P.a); break;
  }
  return (int)hipGetLastError();
}

// Arrival counters of the in-kernel slab reduction: 256 launches in flight x kWrwTickets, zero-initialised; every
// counter is reset by the block that completes it, so a graph replay finds them at zero again.
constexpr int kWrwSlots = 256, kWrwTickets = 4096;
__device__ unsigned g_wrw_ticket[kWrwSlots * kWrwTickets];

unsigned* wrw_ticket_slot() {
  static unsigned* base[64] = {nullptr};
  static unsigned next = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_wrw_ticket)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  const unsigned k = __atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED) % (unsigned)kWrwSlots;
  return base[dev] + (long long)kWrwTickets * k;
}

// Fan-in of the in-kernel reduction tree; 0 or 1 = the separate wrw_halo_reduce launch (DL4J_AMD_WRW_TREE).
// Off by default: measured slower on the zoo ResNet-50 at batch 1024 (profiles/r6_wrw_tree.txt: fan 8 39.5k vs
// 41.5k images/s; limited to <= 16 splits still -1.2 %) — the write-through slab stores and the serial per-tile
// tail of the last levels cost more than the reduce launch they replace, which overlaps the data-gradient chain on
// the weight-gradient stream anyway.
int& wrw_tree_fan() {
  static int v = [] {
    const char* e = getenv("DL4J_AMD_WRW_TREE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// Largest split count that takes the in-kernel tree (DL4J_AMD_WRW_TREE_MAX): above it the serial tail of the
// tree's last levels (fan-in slabs of one tile per level) outlasts the separate reduce launch.
int wrw_tree_max_splits() {
  static const int v = [] {
    const char* e = getenv("DL4J_AMD_WRW_TREE_MAX");
    return e ? atoi(e) : 1 << 30;
  }();
  return v;
}

}  // namespace

// Sets the fan-in of the weight-gradient slab reduction tree (<= 1: separate reduce launch); returns the old value.
DL4J_API int dl4j_conv_wrw_set_tree(int fan) {
  const int old = wrw_tree_fan();
  wrw_tree_fan() = fan;
  return old;
}

// Workspace floats for dl4j_conv_wrw_halo (slabs + bias partials); 0 when the shape / variant is not supported.
// variant 0 = automatic. Writes the split count used to *splits_out.
DL4J_API long long dl4j_conv_wrw_halo_ws_floats(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph,
                                                int pw, int dh, int dw, int OH, int OW, int variant, int splits,
                                                int* splits_out) {
  const Plan P = make_plan(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW, variant, splits);
  if (!P.ok) return 0;
  if (splits_out) *splits_out = P.splits;
  return (long long)P.splits * K * ((long long)R * S * C + 1);
}

// dW fp32 [K][C][R][S] and db fp32 [K] (or null), both overwritten. X NHWC [N,H,W,C], dY NHWC [N,OH,OW,K], dt 1 bf16 /
// 2 fp16, 16-byte aligned. Returns -1 when the shape / variant is not supported (caller falls back).
DL4J_API int dl4j_conv_wrw_halo(int dt, const void* X, const void* dY, float* dW, float* db, float* ws, int N, int H,
                                int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                                int OH, int OW, int variant, int splits, hipStream_t s) {
  if ((dt != 1 && dt != 2) || !ws || !dW) return -1;
  if ((long long)N * H * W * C >= 0x7fffffffLL || (long long)N * OH * OW * K >= 0x7fffffffLL) return -1;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(dY) & 15)) return -1;
  Plan P = make_plan(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW, variant, splits);
  if (!P.ok) return -1;
  P.a.X = reinterpret_cast<const u16*>(X);
  P.a.dY = reinterpret_cast<const u16*>(dY);
  P.a.part = ws;
  const long long RSC = (long long)R * S * C;
  P.a.partb = db ? ws + (long long)P.splits * K * RSC : nullptr;
  P.a.splits = P.splits;
  P.a.dW = dW;
  P.a.db = db;
  P.a.fan = wrw_tree_fan();
  P.a.ticket = nullptr;
  if (P.a.fan > 1 && P.splits <= wrw_tree_max_splits()) {
    int tkpt = 0;
    for (int n = P.splits; n > 1;) {
      n = (n + P.a.fan - 1) / P.a.fan;
      tkpt += n;
    }
    P.a.tkpt = tkpt;
    if ((long long)P.a.tiles_k * P.a.tiles_c * tkpt <= kWrwTickets) P.a.ticket = wrw_ticket_slot();
  }
  int e = dt == 1 ? launch_halo<1>(P, s) : launch_halo<2>(P, s);
  if (e || P.a.ticket) return e;
  const long long total = (long long)K * RSC;
  const unsigned nb = (unsigned)((total + 63) / 64) + (db ? (unsigned)((K + 63) / 64) : 0u);
  hipLaunchKernelGGL(wrw_halo_reduce, dim3(nb), dim3(256), 0, s, ws, dW, P.splits, K, C, R * S, P.a.partb, db);
  return (int)hipGetLastError();
}
