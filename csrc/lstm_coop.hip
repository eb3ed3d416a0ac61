// Cooperative (multi-workgroup) LSTM recurrence for gfx950: the per-step RW·h GEMM is split over G workgroups per
// 16-row minibatch tile so that each workgroup's slice of the recurrent weights stays RESIDENT IN LDS for the
// whole sequence (128 KB per workgroup), instead of every step streaming all of RW from L2 (csrc/lstm.hip, which is
// bound by ~70 GB/s of L2->CU traffic per workgroup: 7.4 us per step at H = 256).
//
// Per step, workgroup g of a tile computes the four gates of its U hidden units (MFMA 16x16x32 bf16, A = h_{t-1}
// from LDS, B = its RW slice from LDS), keeps c in registers, and PUBLISHES its slice of h_t to the other G-1
// workgroups through 8-byte "granules" {tag = step+1, 2 x bf16} stored with agent-scope atomics: the data is its
// own flag (guide Guideline 16, R2), so there is no separate flag, fence or barrier between workgroups. Consumers
// sweep the granules of h_{t-1} with agent-scope atomic loads until every tag matches; every spin is bounded by the
// wall clock (a timeout sets *err and the kernel runs to completion instead of hanging). The exchange buffer is
// double-buffered by step parity. Tags are tag_base + step + 1 over one persistent buffer; the base lives on the
// device and the last workgroup of each launch advances it (coop_tag_end), so stale granules never match and no
// per-launch memset is needed, eager or inside a replayed HIP graph (the host zeroes the buffer on first use only).
//
// The grid (G x tiles workgroups, one per CU: LDS-bound, at most CUs - 8 of them) is launched stream-ordered (see
// coop_launch); shapes that do not fit fall back to csrc/lstm.hip.
// Math, gate order [a|f|o|g], peepholes, masks and outputs are identical to lstm_fwd_kernel.
#include "common.h"
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) float f4c_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8c_t;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ float sigm_c(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_c(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) / (1.f + e), x);
}

// Launch path. The grid is at most (CUs - 8) workgroups of one-per-CU occupancy and every cross-workgroup wait is
// bounded by the wall clock (a timeout sets *err, checked by the host), so a plain stream-ordered launch is safe:
// the stream's previous kernel has drained before any workgroup starts, and the few workgroups always find CUs.
// hipLaunchCooperativeKernel adds ~13 us of dispatch gap on each side of the kernel on this runtime (rocprofv3
// kernel trace, profiles/r3_lstm_window_kernels.txt), i.e. ~100 us per TBPTT window of the 2-layer text model;
// DL4J_AMD_LSTM_COOP_LAUNCH=coop restores the cooperative launch.
// That argument holds only while nothing on ANOTHER stream can hold CUs during the launch (a conv weight-gradient
// overlap stream, RCCL kernels of a data-parallel step): the host then asks for the cooperative launch
// (dl4j_lstm_coop_launch_mode, ops/rnn_native.py decides per launch). Either way a timed-out hand-off also raises the
// device-wide step guard below, and the fused updater skips its update while the guard is set, so the invalid
// outputs of such a launch never reach the parameters (the host raises at its next check).
static int g_coop_mode = -1;      // -1: environment default, 0: plain, 1: cooperative

static hipError_t coop_launch(const void* k, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s) {
  int mode = g_coop_mode;
  if (mode < 0) {
    const char* e = getenv("DL4J_AMD_LSTM_COOP_LAUNCH");
    mode = (e && e[0] == 'c') ? 1 : 0;
  }
  if (mode == 1) return hipLaunchCooperativeKernel(k, grid, block, args, lds, s);
  return hipLaunchKernel(k, grid, block, args, lds, s);
}

DL4J_API void dl4j_lstm_coop_launch_mode(int mode) { g_coop_mode = mode < -1 ? -1 : (mode > 1 ? 1 : mode); }

// Device-wide step guard: set (never cleared on the device) by any cooperative LSTM launch whose hand-off timed out;
// read by fused_update_kernel (csrc/updater.hip), which then leaves parameters and state untouched. The host clears
// it (dl4j_lstm_step_guard_reset) when it reports the failure.
__device__ unsigned g_lstm_step_guard;

unsigned* lstm_step_guard_ptr() {
  static unsigned* base[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_lstm_step_guard)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  return base[dev];
}

DL4J_API unsigned* dl4j_lstm_step_guard() { return lstm_step_guard_ptr(); }

DL4J_API int dl4j_lstm_step_guard_reset(hipStream_t s) {
  unsigned* g = lstm_step_guard_ptr();
  return g ? (int)hipMemsetAsync(g, 0, sizeof(unsigned), s) : -1;
}

// Device-side tag bookkeeping (tag argument == kDevTag): err[1] holds the tag base of the next launch and err[2]
// counts finished workgroups. Every workgroup reads the base at entry; the LAST workgroup to finish (all others have
// read it by then: no workgroup finishes before the launch's final exchange, and the counter spans every tile)
// advances it past this launch's tags. Stream-ordered launches therefore never reuse a tag and need no per-launch
// memset, eager or replayed inside a HIP graph. Before the 32-bit tags wrap, that last workgroup zeroes the exchange
// buffer and restarts at 0 (zeroed granules carry tag 0, which never matches: tags start at base + 1).
constexpr unsigned kDevTag = 0xFFFFFFFFu;

__device__ __forceinline__ unsigned coop_tag_begin(gu32* err, unsigned tag_arg) {
  return tag_arg == kDevTag ? __hip_atomic_load(err + 1, RLX_AGENT) : tag_arg;
}

// Called by every thread of the workgroup after its last exchange access; flag: any 4-byte LDS word.
__device__ __forceinline__ void coop_tag_end(gu32* err, gu64* exch, long long exch_words, unsigned tag_arg,
                                             unsigned base, unsigned used, unsigned* flag) {
  if (tag_arg != kDevTag) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nwg = gridDim.x * gridDim.y;
    const unsigned done = __hip_atomic_fetch_add(err + 2, 1u, RLX_AGENT);
    *flag = done == nwg - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (*flag == 0u) return;
  unsigned next = base + used;
  if (next >= 0xF0000000u) {
    for (long long i = threadIdx.x; i < exch_words; i += blockDim.x) __hip_atomic_store(exch + i, 0ull, RLX_AGENT);
    next = 0;
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(err + 2, 0u, RLX_AGENT);
    __hip_atomic_store(err + 1, next, RLX_AGENT);
  }
}

// U = hidden units per workgroup (16 per wave); KS = H / 32 k-steps
template <int U, bool PEEP>
__global__ void __launch_bounds__(4 * U) lstm_fwd_coop(
    const __bf16* __restrict__ zx, const __bf16* __restrict__ rwt, const float* __restrict__ peep,
    const float* __restrict__ h0, const float* __restrict__ c0, const float* __restrict__ mask,
    float* __restrict__ out, __bf16* __restrict__ out16, float* __restrict__ gates, float* __restrict__ call,
    float* __restrict__ hT, float* __restrict__ cT, unsigned long long* exch_raw, unsigned* err_raw, int Tn, int mb,
    int H, long long timeout_ticks, unsigned tag_arg, long long exch_words) {
  constexpr int NW = U / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int KS = H / 32, H16 = H / 16, H4 = 4 * H;
  bf16x8c_t* rws = reinterpret_cast<bf16x8c_t*>(smem);                       // [4][NW][KS][64] fragments
  __bf16* hbuf = reinterpret_cast<__bf16*>(smem + (size_t)4 * NW * KS * 64 * 16);   // [1 or 2][16][H + 8]
  const bool dbuf = H <= 256;        // double-buffered h tile when it fits next to the RW slice, else one more barrier
  const int ldh = H + 8;
  gu64* exch = (gu64*)exch_raw;
  gu32* err = (gu32*)err_raw;
  const unsigned tag_base = coop_tag_begin(err, tag_arg);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4, rg = hgrp * 4;
  const int grp = blockIdx.x, tile = blockIdx.y, G = gridDim.x;
  const int m0 = tile * 16;
  const int u0 = grp * U;                                  // first hidden unit of this workgroup
  const int j = u0 + wave * 16 + col;                      // this lane's hidden unit
  // ---- resident RW slice: fragments of (gate, this wave's 16-unit tile, k-step)
  for (int i = threadIdx.x; i < 4 * NW * KS * 64; i += blockDim.x) {
    const int ln = i & 63, t1 = i >> 6;
    const int ks = t1 % KS, t2 = t1 / KS;
    const int w = t2 % NW, g = t2 / NW;
    const long long gt = (long long)g * H16 + (u0 >> 4) + w;
    rws[i] = *reinterpret_cast<const bf16x8c_t*>(rwt + ((gt * KS + ks) * 64 + ln) * 8);
  }
  int mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float c[4], wff = 0.f, woo = 0.f, wgg = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = (c0 && m0 + rg + r < mb) ? c0[(long long)mrow[r] * H + j] : 0.f;
  if (PEEP) {
    wff = peep[j];
    woo = peep[H + j];
    wgg = peep[2 * H + j];
  }
  float zv[4][4], mv[4];
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long zrow = ((long long)t * mb + mrow[r]) * H4;
#pragma unroll
      for (int g = 0; g < 4; ++g) zv[g][r] = (float)zx[zrow + g * H + j];
      mv[r] = mask ? mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  load_step(0);
  const int npairs = 16 * (H / 2);                         // granules per step per tile
  for (int t = 0; t < Tn; ++t) {
    __bf16* hb = hbuf + (dbuf ? (t & 1) : 0) * 16 * ldh;
    // ---- gather h_{t-1} (16 rows x H) into LDS
    if (t == 0) {
      for (int i = threadIdx.x; i < 16 * H; i += blockDim.x) {
        const int r = i / H, k = i - r * H, m = m0 + r;
        hb[r * ldh + k] = (__bf16)((h0 && m < mb) ? h0[(long long)m * H + k] : 0.f);
      }
    } else {
      gu64* src = exch + ((long long)tile * 2 + ((t - 1) & 1)) * npairs;
      const long long deadline = wall_clock64() + timeout_ticks;   // per step: long sequences never time out
      // sweep: each thread issues its granule loads in batches of 8 (one round trip per batch), re-polling a batch
      // until every tag matches (guide Guideline 16, R2 sweep_granules)
      for (int base = 0; base < npairs; base += 8 * blockDim.x) {
        unsigned long long v[8];
        for (;;) {
          bool ok = true;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int i = base + q * blockDim.x + threadIdx.x;
            v[q] = i < npairs ? __hip_atomic_load(src + i, RLX_AGENT) : ((unsigned long long)(tag_base + t) << 32);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) ok &= (unsigned)(v[q] >> 32) == tag_base + (unsigned)t;
          if (ok) break;
          // once any hand-off has timed out the launch is already invalid: stop waiting at every later step
          if (wall_clock64() > deadline || __hip_atomic_load(err, RLX_AGENT) != 0u) {
            __hip_atomic_store(err, 1u, RLX_AGENT);
            __hip_atomic_store((gu32*)&g_lstm_step_guard, 1u, RLX_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int i = base + q * blockDim.x + threadIdx.x;
          if (i < npairs) {
            const int r = i / (H / 2), k = (i - r * (H / 2)) * 2;
            *reinterpret_cast<unsigned*>(hb + r * ldh + k) = (unsigned)v[q];
          }
        }
      }
    }
    __syncthreads();
    // ---- z = h_{t-1} . RW (this wave's 16 units x 4 gates), operands from LDS
    f4c_t acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f4c_t{0.f, 0.f, 0.f, 0.f};
    const __bf16* hA = hb + col * ldh + 8 * hgrp;
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8c_t a = *reinterpret_cast<const bf16x8c_t*>(hA + ks * 32);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, rws[((g * NW + wave) * KS + ks) * 64 + lane], acc[g], 0,
                                                         0, 0);
    }
    if (!dbuf) __syncthreads();                            // the next gather overwrites the only h tile
    // ---- gates, state, outputs, publish h_t
    gu64* dst = exch + ((long long)tile * 2 + (t & 1)) * npairs;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = rg + r;
      const bool valid = m0 + rr < mb;
      const float za = acc[0][r] + zv[0][r];
      float zf = acc[1][r] + zv[1][r];
      float zo = acc[2][r] + zv[2][r];
      float zg = acc[3][r] + zv[3][r];
      const float cp = c[r];
      if (PEEP) {
        zf += cp * wff;
        zg += cp * wgg;
      }
      const float a = tanh_c(za), f = sigm_c(zf), g = sigm_c(zg);
      float cc = f * cp + g * a;
      if (PEEP) zo += cc * woo;
      const float o = sigm_c(zo);
      float h = o * tanh_c(cc) * mv[r];
      cc *= mv[r];
      if (!valid) {
        h = 0.f;
        cc = 0.f;
      }
      c[r] = cc;
      if (valid) {
        const long long orow = ((long long)t * mb + m0 + rr) * H;
        out[orow + j] = h;
        if (out16) out16[orow + j] = (__bf16)h;
        if (call) call[orow + j] = cc;
        if (gates) {
          float* gp = gates + orow * 4 + j;
          gp[0] = a;
          gp[H] = f;
          gp[2 * H] = o;
          gp[3 * H] = g;
        }
      }
      // granule = {tag t+1, bf16(h[j]) | bf16(h[j+1]) << 16}, written by the even-unit lane of each pair
      const float hn = __shfl_xor(h, 1, 64);
      if ((col & 1) == 0) {
        const __bf16 lo = (__bf16)h, hi = (__bf16)hn;
        const unsigned pay = (unsigned)(*reinterpret_cast<const unsigned short*>(&lo)) |
                             ((unsigned)(*reinterpret_cast<const unsigned short*>(&hi)) << 16);
        __hip_atomic_store(dst + rr * (H / 2) + (j >> 1), ((unsigned long long)(tag_base + t + 1) << 32) | pay, RLX_AGENT);
      }
    }
    if (t + 1 < Tn) load_step(t + 1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + rg + r;
    if (m < mb) {
      if (cT) cT[(long long)m * H + j] = c[r];
      if (hT) hT[(long long)m * H + j] = out[((long long)(Tn - 1) * mb + m) * H + j];
    }
  }
  coop_tag_end(err, exch, exch_words, tag_arg, tag_base, (unsigned)Tn + 2u, reinterpret_cast<unsigned*>(smem));
  (void)G;
}

template <int U, bool PEEP>
static int coop_fwd_launch(const void* zx, const void* rwt, const float* peep, const float* h0, const float* c0,
                           const float* mask, float* out, void* out16, float* gates, float* call, float* hT,
                           float* cT, unsigned long long* exch, unsigned* err, int Tn, int mb, int H, unsigned tag_base,
                           int reset, hipStream_t s) {
  const int KS = H / 32, NW = U / 16;
  const size_t lds = (size_t)4 * NW * KS * 64 * 16 + (H <= 256 ? 2ull : 1ull) * 16 * (H + 8) * 2;
  auto k = lstm_fwd_coop<U, PEEP>;
  if (lds > 160 * 1024) return -1;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return -1;
  const dim3 grid(H / U, (mb + 15) / 16), block(64 * NW);
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, block.x, lds) != hipSuccess || per < 1) return -1;
  // one workgroup per CU (LDS-bound); keep a margin: the occupancy API can over-report by one block per CU at high
  // SGPR counts (MI355X_MICROARCH.md, correctness boundaries), so never rely on more than one block per CU
  if ((long long)grid.x * grid.y > (long long)ncu - 8) return -1;
  (void)per;
  const size_t exch_bytes = (size_t)((mb + 15) / 16) * 2 * 16 * (H / 2) * 8;
  if (reset && hipMemsetAsync(exch, 0, exch_bytes, s) != hipSuccess) return -1;
  if (reset && hipMemsetAsync(err, 0, 16, s) != hipSuccess) return -1;
  long long timeout = 200LL * 1000 * 1000;                  // wall_clock64 runs at 100 MHz: 2 s per wait
  long long exch_words = (long long)(exch_bytes / 8);
  void* args[] = {(void*)&zx, (void*)&rwt, (void*)&peep, (void*)&h0, (void*)&c0, (void*)&mask, (void*)&out,
                  (void*)&out16, (void*)&gates, (void*)&call, (void*)&hT, (void*)&cT, (void*)&exch, (void*)&err, (void*)&Tn,
                  (void*)&mb, (void*)&H, (void*)&timeout, (void*)&tag_base, (void*)&exch_words};
  const hipError_t e = coop_launch(reinterpret_cast<const void*>(k), grid, block, args, lds, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------ backward
// Cooperative backward time loop. The per-step product dh_{t-1} = dz_t . RW^T (K = 4H gate columns) is split over
// the G = H/U workgroups of a tile BY K: workgroup g owns the 4U gate columns of its U hidden units, so its slice
// of dz_t is produced locally (no exchange of dz), and its RW slice (RW[n][own gate columns] for all H outputs n,
// 128 KB at H = 256 / U = 64) stays resident in LDS. Each workgroup computes a PARTIAL dh (16 rows x H, fp32) and
// publishes it as {tag, fp32} granules addressed to the workgroup that owns each output unit; the owner sums the G
// partials of its units in a fixed producer order (deterministic) directly into the lanes that need them for the
// next step's gate deltas. Exchange per workgroup per step: 16 x H granules in, 16 x H out (vs 16 x 4H for
// gathering dz), fp32 partials (no bf16 rounding of dh). Same hand-off/timeout/cooperative-launch rules as the
// forward.
template <int U, int H, bool PEEP>
__global__ void __launch_bounds__(4 * U) lstm_bwd_coop(
    const void* __restrict__ eps, int eps_dt, const float* __restrict__ gates, const float* __restrict__ call,
    const float* __restrict__ c0, const __bf16* __restrict__ rw, const float* __restrict__ peep,
    const float* __restrict__ mask, const float* __restrict__ dh_last, const float* __restrict__ dc_last,
    float* __restrict__ dz, float* __restrict__ dh0, float* __restrict__ dc0, unsigned long long* exch_raw,
    unsigned* err_raw, int Tn, int mb, int t_end, long long timeout_ticks, unsigned tag_arg, long long exch_words) {
  constexpr int NW = U / 16, G = H / U, NTW = (H / 16) / NW, KL = 4 * U / 32, KSG = 4 * H / 32, LDZ = 4 * U + 8;
  constexpr int NE = 4 * G, BATCH = NE < 16 ? NE : 16;     // partial granules gathered per lane per step
  constexpr int H4 = 4 * H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16x8c_t* rws = reinterpret_cast<bf16x8c_t*>(smem);                       // [H/16][KL][64] fragments
  __bf16* zbuf = reinterpret_cast<__bf16*>(smem + (size_t)(H / 16) * KL * 64 * 16);   // [2][16][LDZ]
  gu64* exch = (gu64*)exch_raw;
  gu32* err = (gu32*)err_raw;
  const unsigned tag_base = coop_tag_begin(err, tag_arg);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4, rg = hgrp * 4;
  const int grp = blockIdx.x, tile = blockIdx.y;
  const int m0 = tile * 16, u0 = grp * U;
  const int ul = wave * 16 + col;                          // this lane's unit within the workgroup's U
  const int j = u0 + ul;
  // ---- resident RW slice: B[k][n] = RW[n][k] for k in this workgroup's gate columns, all n
  for (int i = threadIdx.x; i < (H / 16) * KL * 64; i += blockDim.x) {
    const int ln = i & 63, t1 = i >> 6;
    const int sl = t1 % KL, nt = t1 / KL;
    const int kg = ((32 * sl) / U) * (H / 32) + (u0 + (32 * sl) % U) / 32;   // global k-step of local k-step sl
    rws[i] = *reinterpret_cast<const bf16x8c_t*>(rw + (((long long)nt * KSG + kg) * 64 + ln) * 8);
  }
  int mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float dhn[4], dcn[4], wff = 0.f, woo = 0.f, wgg = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool v = m0 + rg + r < mb;
    dhn[r] = (dh_last && v) ? dh_last[(long long)mrow[r] * H + j] : 0.f;
    dcn[r] = (dc_last && v) ? dc_last[(long long)mrow[r] * H + j] : 0.f;
  }
  if (PEEP) {
    wff = peep[j];
    woo = peep[H + j];
    wgg = peep[2 * H + j];
  }
  float ev[4], av[4], fv[4], ov[4], gv[4], cv[4], pv[4], mv[4];
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long hrow = ((long long)t * mb + mrow[r]) * H, grow = hrow * 4;
      ev[r] = ld_any(eps, eps_dt, hrow + j);
      av[r] = gates[grow + j];
      fv[r] = gates[grow + H + j];
      ov[r] = gates[grow + 2 * H + j];
      gv[r] = gates[grow + 3 * H + j];
      cv[r] = call[hrow + j];
      pv[r] = t > 0 ? call[hrow - (long long)mb * H + j] : (c0 ? c0[(long long)mrow[r] * H + j] : 0.f);
      mv[r] = mask ? mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  const long long slot_sz = (long long)G * G * 16 * U;     // granules per (tile, slot)
  // sum of the G partials of (rows rg..rg+3, unit ul) published with tag `tag` into slot tag-1 & 1
  auto gather = [&](int tag, float* res) {
    const gu64* src = exch + ((long long)tile * 2 + ((tag - 1) & 1)) * slot_sz + (long long)grp * G * 16 * U;
    const long long deadline = wall_clock64() + timeout_ticks;
#pragma unroll
    for (int r = 0; r < 4; ++r) res[r] = 0.f;
#pragma unroll
    for (int b0 = 0; b0 < NE; b0 += BATCH) {
      unsigned long long v[BATCH];
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
          const int e = b0 + q, g = e >> 2, r = e & 3;     // producer-major: fixed summation order per unit
          v[q] = __hip_atomic_load(src + ((long long)g * 16 + rg + r) * U + ul, RLX_AGENT);
        }
#pragma unroll
        for (int q = 0; q < BATCH; ++q) ok &= (unsigned)(v[q] >> 32) == tag_base + (unsigned)tag;
        if (ok) break;
        if (wall_clock64() > deadline || __hip_atomic_load(err, RLX_AGENT) != 0u) {
          __hip_atomic_store(err, 1u, RLX_AGENT);
          __hip_atomic_store((gu32*)&g_lstm_step_guard, 1u, RLX_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int q = 0; q < BATCH; ++q) res[(b0 + q) & 3] += __uint_as_float((unsigned)v[q]);
    }
  };
  load_step(Tn - 1);
  int it = 0;
  for (int t = Tn - 1; t >= t_end; --t, ++it) {
    if (it > 0) gather(it, dhn);                           // dh_t from the previous iteration's partials
    __bf16* zb = zbuf + (it & 1) * 16 * LDZ;
    float dza[4], dzf[4], dzo[4], dzg[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool valid = m0 + rg + r < mb;
      const float dh = (ev[r] + dhn[r]) * mv[r];
      float dc = dcn[r] * mv[r];
      const float a = av[r], f = fv[r], o = ov[r], g = gv[r];
      const float ca = tanh_c(cv[r]);
      const float zo_ = dh * ca * o * (1.f - o);
      dc += dh * o * (1.f - ca * ca);
      if (PEEP) dc += zo_ * woo;
      const float zf_ = dc * pv[r] * f * (1.f - f);
      const float zg_ = dc * a * g * (1.f - g);
      const float za_ = dc * g * (1.f - a * a);
      float dcp = dc * f;
      if (PEEP) dcp += zf_ * wff + zg_ * wgg;
      dcn[r] = valid ? dcp : 0.f;
      dza[r] = valid ? za_ : 0.f;
      dzf[r] = valid ? zf_ : 0.f;
      dzo[r] = valid ? zo_ : 0.f;
      dzg[r] = valid ? zg_ : 0.f;
    }
    if (t - 1 >= t_end) load_step(t - 1);                  // next step's HBM operands in flight now
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = rg + r;
      zb[rr * LDZ + ul] = (__bf16)dza[r];
      zb[rr * LDZ + U + ul] = (__bf16)dzf[r];
      zb[rr * LDZ + 2 * U + ul] = (__bf16)dzo[r];
      zb[rr * LDZ + 3 * U + ul] = (__bf16)dzg[r];
      if (m0 + rr < mb) {
        float* dp = dz + ((long long)t * mb + m0 + rr) * H4 + j;
        dp[0] = dza[r];
        dp[H] = dzf[r];
        dp[2 * H] = dzo[r];
        dp[3 * H] = dzg[r];
      }
    }
    __syncthreads();
    if (t == t_end && !dh0) break;                         // nobody consumes the last partials
    // ---- partial dh (16 rows x this wave's NTW output tiles) over the local gate columns
    f4c_t acc[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc[nt] = f4c_t{0.f, 0.f, 0.f, 0.f};
    const __bf16* zA = zb + col * LDZ + 8 * hgrp;
#pragma unroll
    for (int sl = 0; sl < KL; ++sl) {
      const bf16x8c_t a = *reinterpret_cast<const bf16x8c_t*>(zA + sl * 32);
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, rws[((wave * NTW + nt) * KL + sl) * 64 + lane], acc[nt],
                                                          0, 0, 0);
    }
    // ---- publish: granule {tag it+1, fp32 partial} at [consumer][producer grp][row][unit in consumer]
    gu64* dst = exch + ((long long)tile * 2 + (it & 1)) * slot_sz;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n = (wave * NTW + nt) * 16 + col;
      const int cons = n / U, un = n - cons * U;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __hip_atomic_store(dst + (((long long)cons * G + grp) * 16 + rg + r) * U + un,
                           ((unsigned long long)(tag_base + it + 1) << 32) | __float_as_uint(acc[nt][r]), RLX_AGENT);
    }
  }
  const int iters = Tn - t_end;
  if (dh0) gather(iters, dhn);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + rg + r;
    if (m < mb) {
      if (dh0) dh0[(long long)m * H + j] = dhn[r];
      if (dc0) dc0[(long long)m * H + j] = dcn[r];
    }
  }
  coop_tag_end(err, exch, exch_words, tag_arg, tag_base, (unsigned)Tn + 2u, reinterpret_cast<unsigned*>(smem));
}

template <int U, int H, bool PEEP>
static int coop_bwd_launch(const void* eps, int eps_dt, const float* gates, const float* call, const float* c0, const void* rw,
                           const float* peep, const float* mask, const float* dhl, const float* dcl, float* dz,
                           float* dh0, float* dc0, unsigned long long* exch, unsigned* err, int Tn, int mb, int t_end,
                           unsigned tag_base, int reset, hipStream_t s) {
  const size_t lds = (size_t)(H / 16) * (4 * U / 32) * 64 * 16 + 2ull * 16 * (4 * U + 8) * 2;
  auto k = lstm_bwd_coop<U, H, PEEP>;
  if (lds > 160 * 1024) return -1;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return -1;
  const dim3 grid(H / U, (mb + 15) / 16), block(4 * U);
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, block.x, lds) != hipSuccess || per < 1) return -1;
  if ((long long)grid.x * grid.y > (long long)ncu - 8) return -1;    // one workgroup per CU, with margin
  const size_t exch_bytes = (size_t)((mb + 15) / 16) * 2 * (H / U) * 16 * H * 8;
  if (reset && hipMemsetAsync(exch, 0, exch_bytes, s) != hipSuccess) return -1;
  if (reset && hipMemsetAsync(err, 0, 16, s) != hipSuccess) return -1;
  long long exch_words = (long long)(exch_bytes / 8);
  long long timeout = 200LL * 1000 * 1000;                  // 2 s per wait at 100 MHz
  const __bf16* rwp = reinterpret_cast<const __bf16*>(rw);
  void* args[] = {(void*)&eps, (void*)&eps_dt, (void*)&gates, (void*)&call, (void*)&c0, (void*)&rwp, (void*)&peep, (void*)&mask,
                  (void*)&dhl, (void*)&dcl, (void*)&dz, (void*)&dh0, (void*)&dc0, (void*)&exch, (void*)&err,
                  (void*)&Tn, (void*)&mb, (void*)&t_end, (void*)&timeout, (void*)&tag_base, (void*)&exch_words};
  const hipError_t e = coop_launch(reinterpret_cast<const void*>(k), grid, block, args, lds, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

DL4J_API long long dl4j_lstm_coop_bwd_exch_bytes(int mb, int H) {
  const int U = H == 512 ? 32 : 64;
  return (long long)((mb + 15) / 16) * 2 * (H / U) * 16 * H * 8;
}

// bf16 RW only; H in {256 (U = 64), 512 (U = 32)}. Returns -1 when the cooperative path does not apply.
DL4J_API int dl4j_lstm_bwd_coop(const void* eps, int eps_dt, const float* gates, const float* call, const float* c0,
                                const void* rw, const float* peep, const float* mask, const float* dh_last,
                                const float* dc_last, float* dz, float* dh0, float* dc0, unsigned long long* exch,
                                unsigned* err, int Tn, int mb, int H, int t_end, unsigned tag_base, int reset,
                                hipStream_t s) {
  if (Tn < 1 || mb < 1 || t_end < 0 || t_end >= Tn) return -1;
  const bool pp = peep != nullptr;
#define BWD_ARGS eps, eps_dt, gates, call, c0, rw, peep, mask, dh_last, dc_last, dz, dh0, dc0, exch, err, Tn, mb, t_end, tag_base, \
                 reset, s
  if (H == 256) return pp ? coop_bwd_launch<64, 256, true>(BWD_ARGS) : coop_bwd_launch<64, 256, false>(BWD_ARGS);
  if (H == 512) return pp ? coop_bwd_launch<32, 512, true>(BWD_ARGS) : coop_bwd_launch<32, 512, false>(BWD_ARGS);
#undef BWD_ARGS
  return -1;
}

DL4J_API long long dl4j_lstm_coop_exch_bytes(int mb, int H) { return (long long)((mb + 15) / 16) * 2 * 16 * (H / 2) * 8; }

// bf16 only; H in {128, 256} (U = 64) or 512 (U = 32). Returns -1 when the cooperative path does not apply.
DL4J_API int dl4j_lstm_fwd_coop(const void* zx, const void* rwt, const float* peep, const float* h0, const float* c0,
                                const float* mask, float* out, void* out16, float* gates, float* call, float* hT,
                                float* cT, unsigned long long* exch, unsigned* err, int Tn, int mb, int H,
                                unsigned tag_base, int reset, hipStream_t s) {
  if (Tn < 1 || mb < 1) return -1;
  const bool pp = peep != nullptr;
#define FWD_ARGS zx, rwt, peep, h0, c0, mask, out, out16, gates, call, hT, cT, exch, err, Tn, mb, H, tag_base, reset, s
  if (H == 128 || H == 256) return pp ? coop_fwd_launch<64, true>(FWD_ARGS) : coop_fwd_launch<64, false>(FWD_ARGS);
  if (H == 512) return pp ? coop_fwd_launch<32, true>(FWD_ARGS) : coop_fwd_launch<32, false>(FWD_ARGS);
#undef FWD_ARGS
  return -1;
}

// ================================================================================================ two-layer stack
// Pipelined two-layer LSTM (the text models' GravesLSTM -> GravesLSTM stack, reference MultiLayerNetwork.java:
// 1521-1593 rnnTimeStep / TBPTT over stacked layers): ONE launch runs both layers' recurrences, layer 2 at step t
// concurrently with layer 1 at step t+1, so the serial chain of a window is T + 1 steps instead of 2T.
//   grid.x = 2G workgroups per 16-row tile (G = H / 32): blockIdx.x < G are layer 1, the rest layer 2; U = 32 units
//   per workgroup (2 waves), so layer 2's RW slice AND its input-weight slice fit in LDS together.
// Forward: layer 1 runs as lstm_fwd_coop and also publishes h1_t into a T-slot "cross ring" of tagged granules;
// layer 2 gathers h2_{t-1} (own exchange) and h1_t (cross ring) into one [16][2H] LDS row block and computes
// z = [h2_{t-1} | h1_t] . [RW2 ; W2] + b2 in one MFMA loop (its input projection moves into the recurrence).
// Backward: layer 2 runs as lstm_bwd_coop and additionally multiplies its dz2_t slice by its W2^T slice: those
// K-split partials of eps1_t = dz2_t . W2^T go through a T-slot cross ring to the layer-1 workgroup owning each unit,
// which sums them in a fixed producer order (deterministic) instead of reading eps from memory.
// Tags, timeouts, the step guard and the launch rules are those of the single-layer kernels; both rings are indexed
// by the time step (no slot reuse inside a launch), so the stack path is used for T <= kStackMaxT.
constexpr int kStackMaxT = 128;

struct Stack2Fwd {
  const __bf16* zx1; const __bf16* rw1; const __bf16* rw2; const __bf16* w2;
  const float* b2; const float* peep1; const float* peep2;
  const float* h0_1; const float* c0_1; const float* h0_2; const float* c0_2;
  const float* mask;
  float* out1; __bf16* o16_1; float* gates1; float* call1; float* hT1; float* cT1;
  float* out2; __bf16* o16_2; float* gates2; float* call2; float* hT2; float* cT2;
  unsigned long long* exch; unsigned* err;
  int Tn, mb;
  long long timeout;
  unsigned tag_arg;
  long long exch_words;
};

template <int H, bool PEEP>
__global__ void __launch_bounds__(128) lstm_fwd_stack2(Stack2Fwd a) {
  constexpr int U = 32, NW = 2, G = H / U, KS = H / 32, H16 = H / 16, H4 = 4 * H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int role = blockIdx.x / G, grp = blockIdx.x - role * G, tile = blockIdx.y, tiles = gridDim.y;
  const int KSR = role ? 2 * KS : KS;
  bf16x8c_t* rws = reinterpret_cast<bf16x8c_t*>(smem);                        // [4][NW][KSR][64]
  __bf16* hbuf = reinterpret_cast<__bf16*>(smem + (size_t)4 * NW * KSR * 64 * 16);
  const int ldh = role ? 2 * H + 8 : H + 8;                                   // role 1: [h2_{t-1} | h1_t]
  gu64* exch = (gu64*)a.exch;
  gu32* err = (gu32*)a.err;
  const unsigned tag_base = coop_tag_begin(err, a.tag_arg);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4, rg = hgrp * 4;
  const int m0 = tile * 16, u0 = grp * U, j = u0 + wave * 16 + col;
  const int Tn = a.Tn, mb = a.mb;
  const __bf16* RWp = role ? a.rw2 : a.rw1;
  for (int i = threadIdx.x; i < 4 * NW * KSR * 64; i += blockDim.x) {
    const int ln = i & 63, t1 = i >> 6;
    const int ks = t1 % KSR, t2 = t1 / KSR;
    const int w = t2 % NW, g = t2 / NW;
    const long long gt = (long long)g * H16 + (u0 >> 4) + w;
    const __bf16* src = ks < KS ? RWp : a.w2;
    rws[i] = *reinterpret_cast<const bf16x8c_t*>(src + ((gt * KS + (ks % KS)) * 64 + ln) * 8);
  }
  const float* peep = role ? a.peep2 : a.peep1;
  const float* h0 = role ? a.h0_2 : a.h0_1;
  const float* c0 = role ? a.c0_2 : a.c0_1;
  float* out = role ? a.out2 : a.out1;
  __bf16* out16 = role ? a.o16_2 : a.o16_1;
  float* gates = role ? a.gates2 : a.gates1;
  float* call = role ? a.call2 : a.call1;
  int mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float c[4], wff = 0.f, woo = 0.f, wgg = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = (c0 && m0 + rg + r < mb) ? c0[(long long)mrow[r] * H + j] : 0.f;
  if (PEEP) {
    wff = peep[j];
    woo = peep[H + j];
    wgg = peep[2 * H + j];
  }
  float zv[4][4], mv[4], bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (role) {
#pragma unroll
    for (int g = 0; g < 4; ++g) bv[g] = a.b2 ? a.b2[g * H + j] : 0.f;
  }
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (role == 0) {
        const long long zrow = ((long long)t * mb + mrow[r]) * H4;
#pragma unroll
        for (int g = 0; g < 4; ++g) zv[g][r] = (float)a.zx1[zrow + g * H + j];
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) zv[g][r] = bv[g];
      }
      mv[r] = a.mask ? a.mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  load_step(0);
  constexpr int npairs = 16 * (H / 2);
  gu64* own = exch + ((long long)role * tiles + tile) * 2 * npairs;
  gu64* ring = exch + 2LL * tiles * 2 * npairs + (long long)tile * Tn * npairs;
  // sweep the tagged granules of one [16][H] bf16 tile into columns [coff, coff + H) of hb; 16 loads per lane in
  // flight (128 lanes x 16 = one [16][256] tile per round trip)
  constexpr int SB = 16;
  auto sweep = [&](gu64* src, unsigned tag, __bf16* hb, int coff) {
    const long long deadline = wall_clock64() + a.timeout;
    for (int base = 0; base < npairs; base += SB * blockDim.x) {
      unsigned long long v[SB];
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int q = 0; q < SB; ++q) {
          const int i = base + q * blockDim.x + threadIdx.x;
          v[q] = i < npairs ? __hip_atomic_load(src + i, RLX_AGENT) : ((unsigned long long)tag << 32);
        }
#pragma unroll
        for (int q = 0; q < SB; ++q) ok &= (unsigned)(v[q] >> 32) == tag;
        if (ok) break;
        if (wall_clock64() > deadline || __hip_atomic_load(err, RLX_AGENT) != 0u) {
          __hip_atomic_store(err, 1u, RLX_AGENT);
          __hip_atomic_store((gu32*)&g_lstm_step_guard, 1u, RLX_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int q = 0; q < SB; ++q) {
        const int i = base + q * blockDim.x + threadIdx.x;
        if (i < npairs) {
          const int r = i / (H / 2), k = (i - r * (H / 2)) * 2;
          *reinterpret_cast<unsigned*>(hb + r * ldh + coff + k) = (unsigned)v[q];
        }
      }
    }
  };
  for (int t = 0; t < Tn; ++t) {
    __bf16* hb = hbuf + (role == 0 ? (t & 1) * 16 * ldh : 0);
    if (t == 0) {
      for (int i = threadIdx.x; i < 16 * H; i += blockDim.x) {
        const int r = i / H, k = i - r * H, m = m0 + r;
        hb[r * ldh + k] = (__bf16)((h0 && m < mb) ? h0[(long long)m * H + k] : 0.f);
      }
    } else {
      sweep(own + (long long)((t - 1) & 1) * npairs, tag_base + (unsigned)t, hb, 0);
    }
    if (role) sweep(ring + (long long)t * npairs, tag_base + (unsigned)t + 1u, hb, H);
    __syncthreads();
    f4c_t acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f4c_t{0.f, 0.f, 0.f, 0.f};
    const __bf16* hA = hb + col * ldh + 8 * hgrp;
    for (int ks = 0; ks < KSR; ++ks) {
      const bf16x8c_t av = *reinterpret_cast<const bf16x8c_t*>(hA + ks * 32);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, rws[((g * NW + wave) * KSR + ks) * 64 + lane], acc[g], 0,
                                                         0, 0);
    }
    if (role) __syncthreads();                             // single h tile: the next sweep overwrites it
    gu64* dst = own + (long long)(t & 1) * npairs;
    gu64* rdst = ring + (long long)t * npairs;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = rg + r;
      const bool valid = m0 + rr < mb;
      const float za = acc[0][r] + zv[0][r];
      float zf = acc[1][r] + zv[1][r];
      float zo = acc[2][r] + zv[2][r];
      float zg = acc[3][r] + zv[3][r];
      const float cp = c[r];
      if (PEEP) {
        zf += cp * wff;
        zg += cp * wgg;
      }
      const float av = tanh_c(za), f = sigm_c(zf), g = sigm_c(zg);
      float cc = f * cp + g * av;
      if (PEEP) zo += cc * woo;
      const float o = sigm_c(zo);
      float h = o * tanh_c(cc) * mv[r];
      cc *= mv[r];
      if (!valid) {
        h = 0.f;
        cc = 0.f;
      }
      c[r] = cc;
      if (valid) {
        const long long orow = ((long long)t * mb + m0 + rr) * H;
        out[orow + j] = h;
        if (out16) out16[orow + j] = (__bf16)h;
        if (call) call[orow + j] = cc;
        if (gates) {
          float* gp = gates + orow * 4 + j;
          gp[0] = av;
          gp[H] = f;
          gp[2 * H] = o;
          gp[3 * H] = g;
        }
      }
      const float hn = __shfl_xor(h, 1, 64);
      if ((col & 1) == 0) {
        const __bf16 lo = (__bf16)h, hi = (__bf16)hn;
        const unsigned pay = (unsigned)(*reinterpret_cast<const unsigned short*>(&lo)) |
                             ((unsigned)(*reinterpret_cast<const unsigned short*>(&hi)) << 16);
        const unsigned long long gv = ((unsigned long long)(tag_base + t + 1) << 32) | pay;
        __hip_atomic_store(dst + rr * (H / 2) + (j >> 1), gv, RLX_AGENT);
        if (role == 0) __hip_atomic_store(rdst + rr * (H / 2) + (j >> 1), gv, RLX_AGENT);
      }
    }
    if (t + 1 < Tn) load_step(t + 1);
  }
  float* hT = role ? a.hT2 : a.hT1;
  float* cT = role ? a.cT2 : a.cT1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + rg + r;
    if (m < mb) {
      if (cT) cT[(long long)m * H + j] = c[r];
      if (hT) hT[(long long)m * H + j] = out[((long long)(Tn - 1) * mb + m) * H + j];
    }
  }
  coop_tag_end(err, exch, a.exch_words, a.tag_arg, tag_base, (unsigned)Tn + 2u, reinterpret_cast<unsigned*>(smem));
}

struct Stack2Bwd {
  const void* eps2; int eps_dt; int pad_;
  const float* gates1; const float* call1; const float* c0_1;
  const float* gates2; const float* call2; const float* c0_2;
  const __bf16* rw1; const __bf16* rw2; const __bf16* w2;                     // backward (B = RW / W) images
  const float* peep1; const float* peep2; const float* mask;
  const float* dhl1; const float* dcl1; const float* dhl2; const float* dcl2;
  float* dz1; float* dz2; float* dh0_1; float* dc0_1; float* dh0_2; float* dc0_2;
  unsigned long long* exch; unsigned* err;
  int Tn, mb, t_end;
  long long timeout;
  unsigned tag_arg;
  long long exch_words;
};

template <int H, bool PEEP>
__global__ void __launch_bounds__(128) lstm_bwd_stack2(Stack2Bwd a) {
  constexpr int U = 32, NW = 2, G = H / U, NTW = (H / 16) / NW, KL = 4 * U / 32, KSG = 4 * H / 32, LDZ = 4 * U + 8;
  constexpr int NE = 4 * G, BATCH = NE < 32 ? NE : 32;     // all partials of a gather in one round trip
  constexpr int H4 = 4 * H;
  constexpr int RWS = (H / 16) * KL * 64;                 // fragments of one resident slice
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int role = blockIdx.x / G, grp = blockIdx.x - role * G, tile = blockIdx.y, tiles = gridDim.y;
  bf16x8c_t* rws = reinterpret_cast<bf16x8c_t*>(smem);                       // RW^T slice (+ W2^T slice, role 1)
  __bf16* zbuf = reinterpret_cast<__bf16*>(smem + (size_t)(role ? 2 : 1) * RWS * 16);   // [2][16][LDZ]
  gu64* exch = (gu64*)a.exch;
  gu32* err = (gu32*)a.err;
  const unsigned tag_base = coop_tag_begin(err, a.tag_arg);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4, rg = hgrp * 4;
  const int m0 = tile * 16, u0 = grp * U;
  const int ul = wave * 16 + col, j = u0 + ul;
  const int Tn = a.Tn, mb = a.mb, t_end = a.t_end;
  const __bf16* RWp = role ? a.rw2 : a.rw1;
  for (int i = threadIdx.x; i < (role ? 2 : 1) * RWS; i += blockDim.x) {
    const int ii = i % RWS;
    const int ln = ii & 63, t1 = ii >> 6;
    const int sl = t1 % KL, nt = t1 / KL;
    const int kg = ((32 * sl) / U) * (H / 32) + (u0 + (32 * sl) % U) / 32;
    const __bf16* src = i < RWS ? RWp : a.w2;
    rws[i] = *reinterpret_cast<const bf16x8c_t*>(src + (((long long)nt * KSG + kg) * 64 + ln) * 8);
  }
  const float* gates = role ? a.gates2 : a.gates1;
  const float* call = role ? a.call2 : a.call1;
  const float* c0 = role ? a.c0_2 : a.c0_1;
  const float* peep = role ? a.peep2 : a.peep1;
  const float* dh_last = role ? a.dhl2 : a.dhl1;
  const float* dc_last = role ? a.dcl2 : a.dcl1;
  float* dz = role ? a.dz2 : a.dz1;
  float* dh0 = role ? a.dh0_2 : a.dh0_1;
  float* dc0 = role ? a.dc0_2 : a.dc0_1;
  int mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float dhn[4], dcn[4], wff = 0.f, woo = 0.f, wgg = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool v = m0 + rg + r < mb;
    dhn[r] = (dh_last && v) ? dh_last[(long long)mrow[r] * H + j] : 0.f;
    dcn[r] = (dc_last && v) ? dc_last[(long long)mrow[r] * H + j] : 0.f;
  }
  if (PEEP) {
    wff = peep[j];
    woo = peep[H + j];
    wgg = peep[2 * H + j];
  }
  float ev[4], av[4], fv[4], ov[4], gv[4], cv[4], pv[4], mv[4];
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long hrow = ((long long)t * mb + mrow[r]) * H, grow = hrow * 4;
      if (role) ev[r] = ld_any(a.eps2, a.eps_dt, hrow + j);
      av[r] = gates[grow + j];
      fv[r] = gates[grow + H + j];
      ov[r] = gates[grow + 2 * H + j];
      gv[r] = gates[grow + 3 * H + j];
      cv[r] = call[hrow + j];
      pv[r] = t > 0 ? call[hrow - (long long)mb * H + j] : (c0 ? c0[(long long)mrow[r] * H + j] : 0.f);
      mv[r] = a.mask ? a.mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  const long long slot_sz = (long long)G * G * 16 * U;
  gu64* own = exch + ((long long)role * tiles + tile) * 2 * slot_sz;
  gu64* ring = exch + 2LL * tiles * 2 * slot_sz + (long long)tile * Tn * slot_sz;
  // sum of the G producers' partials of (rows rg..rg+3, unit ul) in slot `src` carrying tag `tag`
  auto gather = [&](const gu64* slot, unsigned tag, float* res) {
    const gu64* src = slot + (long long)grp * G * 16 * U;
    const long long deadline = wall_clock64() + a.timeout;
#pragma unroll
    for (int r = 0; r < 4; ++r) res[r] = 0.f;
#pragma unroll
    for (int b0 = 0; b0 < NE; b0 += BATCH) {
      unsigned long long v[BATCH];
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
          const int e = b0 + q, g = e >> 2, r = e & 3;
          v[q] = __hip_atomic_load(src + ((long long)g * 16 + rg + r) * U + ul, RLX_AGENT);
        }
#pragma unroll
        for (int q = 0; q < BATCH; ++q) ok &= (unsigned)(v[q] >> 32) == tag;
        if (ok) break;
        if (wall_clock64() > deadline || __hip_atomic_load(err, RLX_AGENT) != 0u) {
          __hip_atomic_store(err, 1u, RLX_AGENT);
          __hip_atomic_store((gu32*)&g_lstm_step_guard, 1u, RLX_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int q = 0; q < BATCH; ++q) res[(b0 + q) & 3] += __uint_as_float((unsigned)v[q]);
    }
  };
  // K-split partial of (16 rows x H) = zb . B over this workgroup's gate columns, published to the owners' slots
  auto partial = [&](const __bf16* zb, const bf16x8c_t* B, gu64* slot, unsigned tag) {
    f4c_t acc[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc[nt] = f4c_t{0.f, 0.f, 0.f, 0.f};
    const __bf16* zA = zb + col * LDZ + 8 * hgrp;
#pragma unroll
    for (int sl = 0; sl < KL; ++sl) {
      const bf16x8c_t av_ = *reinterpret_cast<const bf16x8c_t*>(zA + sl * 32);
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av_, B[((wave * NTW + nt) * KL + sl) * 64 + lane], acc[nt],
                                                          0, 0, 0);
    }
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n = (wave * NTW + nt) * 16 + col;
      const int cons = n / U, un = n - cons * U;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __hip_atomic_store(slot + (((long long)cons * G + grp) * 16 + rg + r) * U + un,
                           ((unsigned long long)tag << 32) | __float_as_uint(acc[nt][r]), RLX_AGENT);
    }
  };
  load_step(Tn - 1);
  int it = 0;
  for (int t = Tn - 1; t >= t_end; --t, ++it) {
    if (it > 0) gather(own + (long long)((it - 1) & 1) * slot_sz, tag_base + (unsigned)it, dhn);
    if (role == 0) gather(ring + (long long)t * slot_sz, tag_base + (unsigned)t + 1u, ev);   // eps1_t from layer 2
    __bf16* zb = zbuf + (it & 1) * 16 * LDZ;
    float dza[4], dzf[4], dzo[4], dzg[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool valid = m0 + rg + r < mb;
      const float dh = (ev[r] + dhn[r]) * mv[r];
      float dc = dcn[r] * mv[r];
      const float a_ = av[r], f = fv[r], o = ov[r], g = gv[r];
      const float ca = tanh_c(cv[r]);
      const float zo_ = dh * ca * o * (1.f - o);
      dc += dh * o * (1.f - ca * ca);
      if (PEEP) dc += zo_ * woo;
      const float zf_ = dc * pv[r] * f * (1.f - f);
      const float zg_ = dc * a_ * g * (1.f - g);
      const float za_ = dc * g * (1.f - a_ * a_);
      float dcp = dc * f;
      if (PEEP) dcp += zf_ * wff + zg_ * wgg;
      dcn[r] = valid ? dcp : 0.f;
      dza[r] = valid ? za_ : 0.f;
      dzf[r] = valid ? zf_ : 0.f;
      dzo[r] = valid ? zo_ : 0.f;
      dzg[r] = valid ? zg_ : 0.f;
    }
    if (t - 1 >= t_end) load_step(t - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = rg + r;
      zb[rr * LDZ + ul] = (__bf16)dza[r];
      zb[rr * LDZ + U + ul] = (__bf16)dzf[r];
      zb[rr * LDZ + 2 * U + ul] = (__bf16)dzo[r];
      zb[rr * LDZ + 3 * U + ul] = (__bf16)dzg[r];
      if (m0 + rr < mb) {
        float* dp = dz + ((long long)t * mb + m0 + rr) * H4 + j;
        dp[0] = dza[r];
        dp[H] = dzf[r];
        dp[2 * H] = dzo[r];
        dp[3 * H] = dzg[r];
      }
    }
    __syncthreads();
    if (role) partial(zb, rws + RWS, ring + (long long)t * slot_sz, tag_base + (unsigned)t + 1u);   // eps1_t
    if (t == t_end && !dh0) break;
    partial(zb, rws, own + (long long)(it & 1) * slot_sz, tag_base + (unsigned)it + 1u);           // dh_{t-1}
  }
  const int iters = Tn - t_end;
  if (dh0) gather(own + (long long)((iters - 1) & 1) * slot_sz, tag_base + (unsigned)iters, dhn);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + rg + r;
    if (m < mb) {
      if (dh0) dh0[(long long)m * H + j] = dhn[r];
      if (dc0) dc0[(long long)m * H + j] = dcn[r];
    }
  }
  coop_tag_end(err, exch, a.exch_words, a.tag_arg, tag_base, (unsigned)Tn + 2u, reinterpret_cast<unsigned*>(smem));
}

static long long stack2_fwd_exch_words(int mb, int H, int Tn) {
  const long long tiles = (mb + 15) / 16, npairs = 16LL * (H / 2);
  return 2 * tiles * 2 * npairs + tiles * Tn * npairs;
}

static long long stack2_bwd_exch_words(int mb, int H, int Tn) {
  const long long tiles = (mb + 15) / 16, G = H / 32, slot = G * G * 16 * 32;
  return 2 * tiles * 2 * slot + tiles * Tn * slot;
}

DL4J_API long long dl4j_lstm_stack2_exch_bytes(int mb, int H, int Tn, int bwd) {
  return 8 * (bwd ? stack2_bwd_exch_words(mb, H, Tn) : stack2_fwd_exch_words(mb, H, Tn));
}

DL4J_API int dl4j_lstm_stack2_max_t() { return kStackMaxT; }

template <typename K, typename A>
static int stack2_launch(K k, A& args, size_t lds, int H, int mb, int reset, long long words, hipStream_t s) {
  if (lds > 160 * 1024) return -1;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return -1;
  const dim3 grid(2 * (H / 32), (mb + 15) / 16), block(128);
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, block.x, lds) != hipSuccess || per < 1) return -1;
  if ((long long)grid.x * grid.y > (long long)ncu - 8) return -1;
  if (reset && hipMemsetAsync(args.exch, 0, (size_t)words * 8, s) != hipSuccess) return -1;
  if (reset && hipMemsetAsync(args.err, 0, 16, s) != hipSuccess) return -1;
  void* kargs[] = {(void*)&args};
  const hipError_t e = coop_launch(reinterpret_cast<const void*>(k), grid, block, kargs, lds, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

// bf16, H = 256 only, T <= kStackMaxT. Pointers of the per-layer outputs may be null where the single-layer kernel
// allows it (out16, gates, call, hT, cT). Returns -1 when the stack path does not apply.
DL4J_API int dl4j_lstm_fwd_stack2(const Stack2Fwd* p, int H, int reset, hipStream_t s) {
  Stack2Fwd a = *p;
  if (H != 256 || a.Tn < 1 || a.Tn > kStackMaxT || a.mb < 1) return -1;
  a.timeout = 200LL * 1000 * 1000;
  a.exch_words = stack2_fwd_exch_words(a.mb, H, a.Tn);
  constexpr int KS = 256 / 32;
  const size_t lds = (size_t)4 * 2 * (2 * KS) * 64 * 16 + 16ull * (2 * 256 + 8) * 2;   // role 1 (the larger)
  return a.peep1 ? stack2_launch(lstm_fwd_stack2<256, true>, a, lds, H, a.mb, reset, a.exch_words, s)
                 : stack2_launch(lstm_fwd_stack2<256, false>, a, lds, H, a.mb, reset, a.exch_words, s);
}

DL4J_API int dl4j_lstm_bwd_stack2(const Stack2Bwd* p, int H, int reset, hipStream_t s) {
  Stack2Bwd a = *p;
  if (H != 256 || a.Tn < 1 || a.Tn > kStackMaxT || a.mb < 1 || a.t_end < 0 || a.t_end >= a.Tn) return -1;
  a.timeout = 200LL * 1000 * 1000;
  a.exch_words = stack2_bwd_exch_words(a.mb, H, a.Tn);
  const size_t lds = (size_t)2 * (256 / 16) * 4 * 64 * 16 + 2ull * 16 * (4 * 32 + 8) * 2;
  return a.peep1 ? stack2_launch(lstm_bwd_stack2<256, true>, a, lds, H, a.mb, reset, a.exch_words, s)
                 : stack2_launch(lstm_bwd_stack2<256, false>, a, lds, H, a.mb, reset, a.exch_words, s);
}

DL4J_API int dl4j_lstm_stack2_struct_bytes(int bwd) { return bwd ? (int)sizeof(Stack2Bwd) : (int)sizeof(Stack2Fwd); }
