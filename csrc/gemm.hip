// General matrix multiply on MFMA (gfx950 / CDNA4): the `mmul` / gemm of the array engine.
//
// Replaces the library GEMM behind every dense-style product of the framework (reference call sites:
// nn/layers/BaseLayer.java:86,97,334-336 preOutput / backprop, BaseOutputLayer.java:151,178,
// recurrent/LSTMHelpers.java:206,212,522,616-676, SameDiff mmul) with in-tree kernels:
//
//   C[m][n] = act( alpha * sum_k A(m,k) B(k,n)  + bias  + beta * C[m][n] )      (optional pre-activation Z)
//
// Operand layouts are flags, not copies: A is either K-contiguous (A[m*lda + k]) or M-contiguous (A[k*lda + m]),
// B is K-contiguous (B[n*ldb + k]) or N-contiguous (B[k*ldb + n]); a transposed torch view is just the other flag.
// A column-major output is produced by the host wrapper as C^T = B^T A^T (swap operands and flags).
//
// gemm_glds  (bf16 / fp16 inputs, fp32 accumulation; fp32 / bf16 / fp16 output)
//   * block tile BM x BN x 64, 4 or 8 waves, each wave a (BM/WGM) x (BN/WGN) sub-tile of
//     v_mfma_f32_32x32x16 accumulators; the MFMA's A operand is the n-side fragment so every lane ends up holding
//     4 consecutive output columns of one row (8/16-byte stores).
//   * operands go global -> LDS with global_load_lds_dwordx4 (no VGPR staging) through a STAGES-deep ring; the
//     wait for a stage is a counted `s_waitcnt vmcnt(N)` + raw s_barrier (never __syncthreads(), whose fence would
//     drain the stages still in flight).
//   * K-contiguous images: [rows][64 k] with 128-byte rows, 16-byte chunk c of row r stored at slot c ^ ((r>>1)&7)
//     (each ds_read_b128 lane group then covers the 16 slots of a bank row). M/N-contiguous images: [rows/128]
//     sub-images of [64 k][128] with 256-byte rows, chunk c of k-row r at slot c ^ ((r&3)<<2), read with
//     ds_read_b64_tr_b16 (hardware transpose; the 16 (row, chunk) pairs of a half-wave read are distinct slots).
//     glds writes lane-linearly, so the swizzle is applied on the per-lane SOURCE address and undone on the read.
//   * XCD-aware, grouped block raster (consecutive block ids of one XCD share A row panels in its L2).
//   * split-K over grid.y: fp32 partial slabs + a deterministic fixed-order reduce kernel that applies the epilogue.
// gemm_simple (any dtype incl. fp32, any strides / shapes / alignment)
//   * 64 x 64 x 16 tile, operands converted to fp32 in LDS, exact-fp32 v_mfma_f32_32x32x2_f32; used for fp32
//     networks and for shapes the fast kernel's 16-byte DMA cannot address.
#include "common.h"
#include <hip/hip_fp16.h>

#include "mfma_tile.h"

// csrc/gemm_stream.hip: the persistent streaming kernel behind configuration 10 (-4 when the shape is not its own)
DL4J_API int dl4j_gemm_stream(int in_dt, const void* A, long long lda, const void* B, long long ldb, void* C,
                              long long ldc, int M, int N, int K, float alpha, const float* bias, int bias_mode,
                              int act, int out_dt, float* tstats, int stats_P, int store_nt, hipStream_t s);

// Diagnostic build only (tools/gemm_stamps.hip defines DL4J_GEMM_STAMPS): per-block phase timestamps of the 8-phase
// kernel, shader clock and 100 MHz real time, written by lane 0 of wave 0 with an ordinary vector store.
#ifdef DL4J_GEMM_STAMPS
__device__ unsigned long long* g_gemm_stamps;
#define GSTAMP(i)                                                                                   \
  do {                                                                                              \
    if (threadIdx.x == 0) {                                                                         \
      unsigned long long* p_ = g_gemm_stamps + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16; \
      p_[2 * (i)] = __builtin_amdgcn_s_memtime();                                                   \
      p_[2 * (i) + 1] = __builtin_amdgcn_s_memrealtime();                                           \
    }                                                                                               \
  } while (0)
#else
#define GSTAMP(i) do {} while (0)
#endif

namespace {

// In-kernel split-K fixup (gemm_glds with GemmArgs::sk_ticket): every split block writes its fp32 slab with sc1
// stores (written through the XCD-local L2), drains them, and bumps the tile's arrival counter; the block that arrives
// last sums the tile's slabs in split order — exactly the fixed order of gemm_splitk_reduce, so the result is
// bitwise the same — and applies the epilogue, instead of the separate reduce launch (BERT-base: 63 reduce launches,
// 0.51 ms of an 8.2 ms step). Slab reads are agent-scope atomic loads (sc1), so the last block never invalidates its
// L2. Opt-in: measured slower than the reduce launch (splitk_fixup_mode below).
typedef __attribute__((address_space(1))) unsigned gq32_t;
template <int BM, int BN, int NT>
__device__ __forceinline__ void splitk_fixup(const GemmArgs& g, int m0, int n0, int tid) {
  constexpr int C4 = BN / 4;
  constexpr int PER = BM * C4 / NT;
  static_assert((BM * C4) % NT == 0, "split-K fixup geometry");
  const long long MN = (long long)g.M * g.N;
  const bool vec = (g.N & 3) == 0;
  float v[PER][4];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
  for (int z = 0; z < g.splits; ++z) {
    const float* slab = g.ws + z * MN;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / C4, c = idx - (idx / C4) * C4;
      const int m = m0 + r, n = n0 + 4 * c;
      if (m >= g.M || n >= g.N) continue;
      const float* p = slab + (long long)m * g.N + n;
      typedef __attribute__((address_space(1))) unsigned long long gq64;
      if (vec) {
        const unsigned long long lo = __hip_atomic_load((gq64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long hi = __hip_atomic_load((gq64*)(p + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v[i][0] += __uint_as_float((unsigned)lo);
        v[i][1] += __uint_as_float((unsigned)(lo >> 32));
        v[i][2] += __uint_as_float((unsigned)hi);
        v[i][3] += __uint_as_float((unsigned)(hi >> 32));
      } else {
        for (int j = 0; j < 4; ++j)
          if (n + j < g.N)
            v[i][j] += __uint_as_float(__hip_atomic_load((gq32_t*)(p + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int idx = tid + i * NT;
    const int r = idx / C4, c = idx - (idx / C4) * C4;
    const int m = m0 + r, n = n0 + 4 * c;
    if (m < g.M && n < g.N) store4(g, g.C, g.Z, m, n, v[i]);
  }
}

constexpr int cmax(int a, int b) { return a > b ? a : b; }
// LDS bytes of a gemm_glds instantiation: the operand ring, grown where a single-stage wide tile's epilogue image
// (lean: [BM][BN] 16-bit; generic: >= 64 rows of fp32 at pitch BN*4+16) is larger than the ring
constexpr int glds_smem(int BM, int BN, int STAGES) {
  return cmax(STAGES * (BM + BN) * 128, cmax(BM * BN * 2, 64 * (BN * 4 + 16)));
}

template <int DT, int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int STAGES, bool BNB = false, bool LEAN = false>
__global__ __launch_bounds__(WGM* WGN * 64, (STAGES == 1 && WGM * WGN == 4 ? 4 : 2)) void gemm_glds(GemmArgs g) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, SBYTES = ABYTES + BBYTES;
  constexpr int SMEM = glds_smem(BM, BN, STAGES);
  constexpr int NIA = BM / 8 / NW, NIB = BN / 8 / NW;     // 1-KB DMA instructions per wave per stage
  static_assert(NIA * NW * 8 == BM && NIB * NW * 8 == BN, "tile / wave count mismatch");
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int per_group = 8 * g.tiles_n;
  const int bid = xcd_remap_g(blockIdx.x, gridDim.x);
  const int grp_id = bid / per_group, first_m = grp_id * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int in_g = bid - grp_id * per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.y, bz = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = (kend - kbeg + 63) / 64;

  typedef unsigned short E;
  const E* A = reinterpret_cast<const E*>(g.A) + (long long)bz * g.sA;
  const E* B = reinterpret_cast<const E*>(g.B) + (long long)bz * g.sB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // ---- per-lane DMA sources (fixed for the whole K loop; advanced by 64 along K per stage)
  const E* ap[NIA];
  int akey[NIA];       // K-contig: k offset of this lane's chunk; M-contig: k row of this lane
  bool aok[NIA];
#pragma unroll
  for (int j = 0; j < NIA; ++j) {
    const int i = wid + NW * j;
    if constexpr (AKC) {
      const int row = 8 * i + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      aok[j] = m0 + row < g.M;
      ap[j] = A + (long long)(aok[j] ? m0 + row : 0) * g.lda + kbeg + ch * 8;
      akey[j] = kbeg + ch * 8;
    } else {
      const int sub = i >> 4, kr = 4 * (i & 15) + (lane >> 4);
      const int ch = (lane & 15) ^ ((kr & 3) << 2);
      const int col = m0 + sub * 128 + ch * 8;
      aok[j] = col < g.M;
      ap[j] = A + (long long)(kbeg + kr) * g.lda + (aok[j] ? col : 0);
      akey[j] = kbeg + kr;
    }
  }
  const E* bp[NIB];
  int bkey[NIB];
  bool bok[NIB];
#pragma unroll
  for (int j = 0; j < NIB; ++j) {
    const int i = wid + NW * j;
    if constexpr (BKC) {
      const int row = 8 * i + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      bok[j] = n0 + row < g.N;
      bp[j] = B + (long long)(bok[j] ? n0 + row : 0) * g.ldb + kbeg + ch * 8;
      bkey[j] = kbeg + ch * 8;
    } else {
      const int sub = i >> 4, kr = 4 * (i & 15) + (lane >> 4);
      const int ch = (lane & 15) ^ ((kr & 3) << 2);
      const int col = n0 + sub * 128 + ch * 8;
      bok[j] = col < g.N;
      bp[j] = B + (long long)(kbeg + kr) * g.ldb + (bok[j] ? col : 0);
      bkey[j] = kbeg + kr;
    }
  }
  const long long astep = AKC ? 64 : 64 * g.lda;
  const long long bstep = BKC ? 64 : 64 * g.ldb;

  auto issue = [&](int kt, int st) {
    char* sa = smem + st * SBYTES;
    char* sb = sa + ABYTES;
    const int kof = kt * 64;
#pragma unroll
    for (int j = 0; j < NIA; ++j) {
      const void* src = (aok[j] && akey[j] + kof < kend) ? (const void*)(ap[j] + kt * astep) : (const void*)gemm_zero_page;
      glds16(src, sa + (wid + NW * j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < NIB; ++j) {
      const void* src = (bok[j] && bkey[j] + kof < kend) ? (const void*)(bp[j] + kt * bstep) : (const void*)gemm_zero_page;
      glds16(src, sb + (wid + NW * j) * 1024);
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
    if constexpr (STAGES == 1) {
      // single buffer (small-K streaming shapes, 4+ blocks per CU hide the latency instead of a ring):
      // every wave's fragment reads of the previous K-tile are done before the DMA overwrites the buffer
      if (kt > 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
      }
      issue(kt, 0);
      wait_vm<0>();
    } else {
      if (STAGES > 2 && kt + 1 < nk) wait_vm<(STAGES > 2 ? (STAGES - 2) * LPS : 0)>();
      else wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if constexpr (STAGES > 1)
      if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* sa = smem + (kt % STAGES) * SBYTES;
    const char* sb = sa + ABYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v8 fm[FM], fn[FN];
#pragma unroll
      for (int b = 0; b < FM; ++b) fm[b] = read_frag<DT, AKC>(sa, wm * WTM + 32 * b, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a) fn[a] = read_frag<DT, BKC>(sb, wn * WTN + 32 * a, s, lane);
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b) acc[a][b] = MfmaT<DT>::mma(fn[a], fm[b], acc[a][b]);
    }
  }

  if constexpr (LEAN) {
    // lean epilogue (mfma_tile.h): acc[a][b] regs 4q..4q+3 <-> tile row wm*WTM + 32b + (lane&31), columns
    // wn*WTN + 32a + 8q + 4h .. +3
    static_assert(BM * BN * 2 <= SMEM, "lean image exceeds the block's LDS");
    const int h = lane >> 5;
    char* dst = reinterpret_cast<char*>(g.C) + (long long)bz * g.sC * 2;
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
        for (int b = 0; b < FM; ++b) {
          float v[4] = {acc[a][b][4 * q] * g.alpha + bq.x, acc[a][b][4 * q + 1] * g.alpha + bq.y,
                        acc[a][b][4 * q + 2] * g.alpha + bq.z, acc[a][b][4 * q + 3] * g.alpha + bq.w};
          lean_act4(g, v);
          lean_put4<BN>(smem, wm * WTM + 32 * b + (lane & 31), lc, v[0], v[1], v[2], v[3], g.out_dt);
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (g.tstats) lean_stats<BM, BN, WGM * WGN * 64>(g, smem, m0, n0, tid);
    lean_readout<BM, BN, WGM * WGN * 64>(g, dst, smem, m0, n0, tid,
                                         g.Z ? reinterpret_cast<char*>(g.Z) + (long long)bz * g.sC * 2 : nullptr);
    return;
  }
  // ---- epilogue through LDS (see epi_readout): acc[a][b] reg e <-> tile column wn*WTN + 32a + (e&3) + 8(e>>2) +
  // 4h, tile row wm*WTM + 32b + (lane&31); passes of RPP rows sized to the operand ring's LDS
  constexpr int PITCH = BN * 4 + 16;
  constexpr int RPP0 = SMEM / PITCH;
  constexpr int RPP = RPP0 >= BM ? BM : (RPP0 >= BM / 2 ? BM / 2 : (RPP0 >= BM / 4 ? BM / 4 : 64));
  static_assert(RPP >= 64 && RPP % 64 == 0, "epilogue pass too small");
  const int h = lane >> 5;
  const bool split = g.splits > 1;
  EpiOut o;
  o.coh = false;
  o.raw = split;
  o.coh = split && g.sk_ticket != nullptr;
  o.dt = split ? 0 : g.out_dt;
  o.dst = split ? reinterpret_cast<char*>(g.ws + (long long)z * g.M * g.N)
                : reinterpret_cast<char*>(g.C) + (long long)bz * g.sC * (g.out_dt == 0 ? 4 : 2);
  o.ld = split ? g.N : g.ldc;
  o.vec = split ? ((g.N & 3) == 0) : (g.coalesce != 0);
  void* Zp = (!split && g.Z) ? reinterpret_cast<char*>(g.Z) + (long long)bz * g.sC * (g.out_dt == 0 ? 4 : 2) : nullptr;
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
    if constexpr (BNB) epi_bnbwd<RPP, BN, WGM * WGN * 64>(g, smem, m0 + P * RPP, n0, tid);
    else if (g.tstats) epi_stats<RPP, BN, WGM * WGN * 64>(g, smem, m0 + P * RPP, n0, tid);
    epi_readout<RPP, BN, WGM * WGN * 64>(g, o, Zp, smem, m0 + P * RPP, n0, tid);
    if (P + 1 < BM / RPP) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
  }
  if constexpr (!BNB) {
    if (o.coh) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // this wave's slab stores are in memory
      __syncthreads();                                               // ... and every other wave's; image reads done
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add((gq32_t*)&g.sk_ticket[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(g.splits - 1);
        if (last) __hip_atomic_store((gq32_t*)&g.sk_ticket[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      if (*flag == 0) return;
      splitk_fixup<BM, BN, WGM * WGN * 64>(g, m0, n0, tid);
    }
  }
}

// split-K reduce: out = epilogue(sum_z ws[z]) in fixed z order (deterministic)
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmArgs g) {
  const long long MN = (long long)g.M * g.N;
  const int nq = (g.N + 3) / 4;
  const long long total = (long long)g.M * nq;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(t / nq);
    const int n = (int)(t - (long long)m * nq) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < g.splits; ++z) {
      const float* p = g.ws + z * MN + (long long)m * g.N + n;
      if (n + 3 < g.N && (g.N & 3) == 0) {
        const float4 x = *reinterpret_cast<const float4*>(p);
        v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
      } else {
        for (int j = 0; j < 4; ++j) if (n + j < g.N) v[j] += p[j];
      }
    }
    store4(g, g.C, g.Z, m, n, v);
  }
}

// Deep split-K reduce: few outputs, many slabs (long-K weight gradients of small layers, e.g. 20 x 25 over 50k
// pixels in 242 slabs, where one thread per output quad serialised 242 loads: 92 us). A block owns 16 output quads;
// its 16 slab groups sum slabs grp, grp+16, ... with eight loads in flight, then combine through LDS in group order
// (fixed order: bitwise reproducible).
__global__ __launch_bounds__(256) void gemm_splitk_reduce_deep(GemmArgs g) {
  const long long MN = (long long)g.M * g.N;
  const int nq = (g.N + 3) / 4;
  const long long total = (long long)g.M * nq;
  const int ql = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long long q = (long long)blockIdx.x * 16 + ql;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  int m = 0, n = 0;
  if (q < total) {
    m = (int)(q / nq);
    n = (int)(q - (long long)m * nq) * 4;
    const float* base = g.ws + (long long)m * g.N + n;
    for (int z0 = grp; z0 < g.splits; z0 += 16 * 8) {
      float t[8][4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int z = z0 + 16 * u;
#pragma unroll
        for (int j = 0; j < 4; ++j) t[u][j] = (z < g.splits && n + j < g.N) ? base[(long long)z * MN + j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += t[u][j];
    }
  }
  __shared__ float red[16][16][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[grp][ql][j] = v[j];
  __syncthreads();
  if (grp == 0 && q < total) {
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += red[k][ql][j];
    store4(g, g.C, g.Z, m, n, o);
  }
}

// ----------------------------------------------------------------------------------------------- 8-phase kernel
// 256 x 256 x 64 tile, 8 waves (2 along M x 4 along N, 128 x 64 outputs each), v_mfma_f32_16x16x32, LDS-DMA staging
// in half-tiles with loads kept in flight across barriers (guide §5 "The 256² 8-phase template", T2-T5).
//   * LDS (128 KB, one array): [2 K-tile buffers][A h0, A h1, B h0, B h1] x 16 KB. Half-tile h of A holds the rows
//     {wr*128 + h*64 + 0..63} of both wave rows, half h of B the columns {wc*64 + h*32 + 0..31} of all four wave
//     columns, so the quadrant (h, h') a wave computes in one phase reads exactly A half h and B half h'.
//   * one iteration = 2 K-tiles = 8 phases. Phase p: ds_read this phase's register sub-tile -> stage ONE half-tile
//     (2 DMAs per thread) -> [counted vmcnt(6) in phases 4 and 8] -> s_barrier -> lgkmcnt(0) -> 16 MFMAs -> s_barrier.
//     Reads: P1 A-h0 + B-h0, P2 B-h1, P3 A-h1 (into the A-h0 registers), P4 none; P5-P8 the same on the odd buffer.
//     Staging: P1 odd A-h1 (tile 2i+1), P2-P5 even A-h0, B-h0, B-h1, A-h1 (tile 2i+2), P6-P8 odd A-h0, B-h0, B-h1
//     (tile 2i+3). Every restage is >= 1 phase after the last read of that half (retired by that phase's
//     lgkmcnt(0) before its second barrier); the vmcnt(6) of P4 retires the odd tile (3 younger half-tiles may stay
//     in flight), that of P8 the next even tile, each one barrier before its first reader.
//   * past the last K-tile every DMA reads the zero page, so the wait counts never change (K-tile count padded to
//     even with zeros).
// Requirements: K % 64 == 0 (per split), operand element offsets < 2^31.
__device__ __forceinline__ int mc16_off(int k, int col) {
  return k * 256 + (((col >> 3) ^ (((k & 3) << 2) | (((k >> 3) & 1) << 1))) << 4) + (col & 7) * 2;
}

template <int DT, bool KC>
__device__ __forceinline__ typename MfmaT<DT>::v8 frag16(const char* T, int rbase, int ks, int lane) {
  typedef typename MfmaT<DT>::v8 v8;
  if constexpr (KC) {
    return *reinterpret_cast<const v8*>(T + kc_off(rbase + (lane & 15), 4 * ks + (lane >> 4)));
  } else {
    // the swizzled transposed-read address is not base + immediate: recompute it per read from an opaque copy of
    // the lane id instead of letting the compiler hoist 24 live address registers out of the K loop.
    // Inline asm, not the builtin: hipcc treats the builtin's LDS read as aliasing the in-flight LDS-DMA stages and
    // drains them (vmcnt(0)) before every such read. The caller's lgkmcnt(0) + sched_barrier(0) orders the result.
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int g = ln >> 4, q = (ln & 15) >> 2, p = ln & 3;
    const int col = rbase + 4 * p;
    const int k = 32 * ks + 8 * g + q;
    typedef __attribute__((address_space(3))) const char* lds_cptr;
    const unsigned a0 = (unsigned)(uintptr_t)((lds_cptr)T + mc16_off(k, col));
    const unsigned a1 = (unsigned)(uintptr_t)((lds_cptr)T + mc16_off(k + 4, col));
    s16x8_t f;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.lo) : "v"(a0));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=&v"(f.hi) : "v"(a1));
    return __builtin_bit_cast(v8, f);
  }
}

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

template <int DT> struct Mfma16;
template <> struct Mfma16<1> {
  static __device__ __forceinline__ f32x4_t mma(MfmaT<1>::v8 a, MfmaT<1>::v8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma16<2> {
  static __device__ __forceinline__ f32x4_t mma(MfmaT<2>::v8 a, MfmaT<2>::v8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <int DT, bool AKC, bool BKC, bool BNB = false, bool LEAN = false>
__global__ __launch_bounds__(512) void gemm_8ph(GemmArgs g) {
  typedef typename MfmaT<DT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) char smem[2 * 4 * 16384 + 8192];   // + pad rows of the epilogue tile

  const int per_group = 8 * g.tiles_n;
  const int bid = xcd_remap_g(blockIdx.x, gridDim.x);
  const int grp_id = bid / per_group, first_m = grp_id * 8;
  const int gsz = min(g.tiles_m - first_m, 8);
  const int in_g = bid - grp_id * per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * 256, n0 = tn * 256;
  const int z = blockIdx.y, bz = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = (kend - kbeg) / 64;
  const int niter = (nk + 1) / 2;

  typedef unsigned short E;
  const E* A = reinterpret_cast<const E*>(g.A) + (long long)bz * g.sA;
  const E* B = reinterpret_cast<const E*>(g.B) + (long long)bz * g.sB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  GSTAMP(0);

  // Per-lane DMA source: one base element offset per operand (k = kbeg) plus the lane's row/column within the
  // half-tile pattern; half h and instruction j only add wave-uniform offsets (keeps the loop free of spills).
  // K-contig A: rows m0 + j*128 + h*64 + rl, rl = 8*wid + lane/8; K-contig B: n0 + j*128 + h*32 + rl', with
  // rl' = (rl/32)*64 + rl%32. M/N-contig: k-row 32j + 4*wid + lane/16, column (lc/64)*128 + h*64 + lc%64 (A) or
  // (lc/32)*64 + h*32 + lc%32 (B), lc = 8 * (swizzled chunk).
  int a_base, a_lim, b_base, b_lim;
  long long a_js, b_js;            // element offset between the j = 0 and j = 1 instruction
  int a_hs, b_hs;                  // element offset between half 0 and half 1
  {
    const int rl = 8 * wid + (lane >> 3);
    const int ch8 = (lane & 7) ^ ((rl >> 1) & 7);
    const int kl = 4 * wid + (lane >> 4);
    const int ch16 = (lane & 15) ^ (((kl & 3) << 2) | (((kl >> 3) & 1) << 1));
    if constexpr (AKC) {
      a_lim = g.M - m0 - rl;                                   // valid iff j*128 + h*64 < a_lim
      a_base = (int)((long long)(m0 + rl) * g.lda + kbeg + ch8 * 8);
      a_js = 128LL * g.lda;
      a_hs = 64 * (int)g.lda;
    } else {
      const int lc = ch16 * 8;
      const int cl = (lc >> 6) * 128 + (lc & 63);
      a_lim = g.M - m0 - cl;                                   // valid iff h*64 < a_lim
      a_base = (int)((long long)(kbeg + kl) * g.lda + m0 + cl);
      a_js = 32LL * g.lda;
      a_hs = 64;
    }
    if constexpr (BKC) {
      const int rr = (rl >> 5) * 64 + (rl & 31);
      b_lim = g.N - n0 - rr;
      b_base = (int)((long long)(n0 + rr) * g.ldb + kbeg + ch8 * 8);
      b_js = 128LL * g.ldb;
      b_hs = 32 * (int)g.ldb;
    } else {
      const int lc = ch16 * 8;
      const int cl = (lc >> 5) * 64 + (lc & 31);
      b_lim = g.N - n0 - cl;
      b_base = (int)((long long)(kbeg + kl) * g.ldb + n0 + cl);
      b_js = 32LL * g.ldb;
      b_hs = 32;
    }
  }
  const long long astep = AKC ? 64 : 64 * g.lda;
  const long long bstep = BKC ? 64 : 64 * g.ldb;

  // stage half-tile (op 0 = A, 1 = B; half h) of K-tile kt into buffer kt & 1
  auto stage = [&](int kt, int op, int h) {
    char* dst = smem + (kt & 1) * 65536 + (op * 2 + h) * 16384 + wid * 1024;
    const bool live = kt < nk;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bool ok;
      const void* src;
      if (op == 0) {
        ok = live && (AKC ? (j * 128 + h * 64 < a_lim) : (h * 64 < a_lim));
        src = A + (long long)a_base + j * a_js + h * a_hs + kt * astep;
      } else {
        ok = live && (BKC ? (j * 128 + h * 32 < b_lim) : (h * 32 < b_lim));
        src = B + (long long)b_base + j * b_js + h * b_hs + kt * bstep;
      }
      glds16(ok ? src : (const void*)gemm_zero_page, dst + j * 8192);
    }
  };

  f32x4_t acc[4][8];      // [n-block: h'*2 + cb][m-block: h*4 + rb]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  v8 af[4][2], bf0[2][2], bf1[2][2];

  auto readA = [&](const char* T) {
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[rb][ks] = frag16<DT, AKC>(T, wr * 64 + rb * 16, ks, lane);
  };
  auto readB = [&](const char* T, v8 (&bf)[2][2]) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf[cb][ks] = frag16<DT, BKC>(T, wc * 32 + cb * 16, ks, lane);
  };
  auto quad = [&](int h, int hp, v8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc[hp * 2 + cb][h * 4 + rb] = Mfma16<DT>::mma(bf[cb][ks], af[rb][ks], acc[hp * 2 + cb][h * 4 + rb]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar_lgkm = [&]() {
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // retire this phase's A reads before its first barrier (the A half is restaged one phase later; with the
  // staggered wave groups the other group may pass that barrier before our lgkmcnt(0) after it)
  auto wait_b_only = [&]() {
    if constexpr (BKC) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  };

  // prologue: even tile 0 (4 halves) + odd tile 1 (A-h0, B-h0, B-h1); retire the even tile
  stage(0, 0, 0); stage(0, 1, 0); stage(0, 1, 1); stage(0, 0, 1);
  stage(1, 0, 0); stage(1, 1, 0); stage(1, 1, 1);
  wait_vm<6>();
  raw_barrier();
  GSTAMP(1);
  // stagger the two wave rows by one barrier: while one group runs its MFMA cluster the other issues its reads
  const bool late = __builtin_amdgcn_readfirstlane(wr) == 1;
  if (late) raw_barrier();

  for (int it = 0; it < niter; ++it) {
    const int ke = 2 * it, ko = 2 * it + 1;
    const char* E0 = smem;
    const char* O0 = smem + 65536;
    // P1
    readA(E0 + 0 * 16384); readB(E0 + 2 * 16384, bf0);
    stage(ko, 0, 1);
    wait_b_only();
    bar_lgkm(); quad(0, 0, bf0); raw_barrier();
    // P2
    readB(E0 + 3 * 16384, bf1);
    stage(ke + 2, 0, 0);
    bar_lgkm(); quad(0, 1, bf1); raw_barrier();
    // P3
    readA(E0 + 1 * 16384);
    stage(ke + 2, 1, 0);
    bar_lgkm(); quad(1, 1, bf1); raw_barrier();
    // P4
    stage(ke + 2, 1, 1);
    wait_vm<6>();
    raw_barrier(); quad(1, 0, bf0); raw_barrier();
    // P5
    readA(O0 + 0 * 16384); readB(O0 + 2 * 16384, bf0);
    stage(ke + 2, 0, 1);
    wait_b_only();
    bar_lgkm(); quad(0, 0, bf0); raw_barrier();
    // P6
    readB(O0 + 3 * 16384, bf1);
    stage(ko + 2, 0, 0);
    bar_lgkm(); quad(0, 1, bf1); raw_barrier();
    // P7
    readA(O0 + 1 * 16384);
    stage(ko + 2, 1, 0);
    bar_lgkm(); quad(1, 1, bf1); raw_barrier();
    // P8
    stage(ko + 2, 1, 1);
    wait_vm<6>();
    raw_barrier(); quad(1, 0, bf0); raw_barrier();
  }
  if (!late) raw_barrier();
  wait_vm<0>();
  GSTAMP(2);

  // epilogue (see epi_readout): pass P = wave row wr. acc[nb][mb] reg e <-> tile row wr*128 + (mb>>2)*64 +
  // (mb&3)*16 + (lane&15), tile column wc*64 + (nb>>1)*32 + (nb&1)*16 + (lane>>4)*4 + e.
  if constexpr (LEAN) {
    char* dst = reinterpret_cast<char*>(g.C) + (long long)bz * g.sC * 2;
    float4 bq[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int lc = wc * 64 + (nb >> 1) * 32 + (nb & 1) * 16 + (lane >> 4) * 4;
      bq[nb] = (g.bias_mode == 1 && n0 + lc < g.N) ? *reinterpret_cast<const float4*>(g.bias + n0 + lc)
                                                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                                   // every wave is done reading the operand stages
    sfor<0, 8>([&](auto MB) {
      constexpr int mb = decltype(MB)::value;
      const int lr = wr * 128 + (mb >> 2) * 64 + (mb & 3) * 16 + (lane & 15);
      sfor<0, 4>([&](auto NB) {
        constexpr int nb = decltype(NB)::value;
        const int lc = wc * 64 + (nb >> 1) * 32 + (nb & 1) * 16 + (lane >> 4) * 4;
        float v[4] = {acc[nb][mb][0] * g.alpha + bq[nb].x, acc[nb][mb][1] * g.alpha + bq[nb].y,
                      acc[nb][mb][2] * g.alpha + bq[nb].z, acc[nb][mb][3] * g.alpha + bq[nb].w};
        lean_act4(g, v);
        lean_put4<256>(smem, lr, lc, v[0], v[1], v[2], v[3], g.out_dt);
      });
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    GSTAMP(4);
    if (g.tstats) lean_stats<256, 256, 512>(g, smem, m0, n0, tid);
    lean_readout<256, 256, 512>(g, dst, smem, m0, n0, tid,
                                g.Z ? reinterpret_cast<char*>(g.Z) + (long long)bz * g.sC * 2 : nullptr);
    GSTAMP(5);
  } else {
    const bool split = g.splits > 1;
    EpiOut o;
    o.coh = false;
    o.raw = split;
    o.dt = split ? 0 : g.out_dt;
    o.dst = split ? reinterpret_cast<char*>(g.ws + (long long)z * g.M * g.N)
                  : reinterpret_cast<char*>(g.C) + (long long)bz * g.sC * (g.out_dt == 0 ? 4 : 2);
    o.ld = split ? g.N : g.ldc;
    o.vec = split ? ((g.N & 3) == 0) : (g.coalesce != 0);
    void* Zp = (!split && g.Z) ? reinterpret_cast<char*>(g.Z) + (long long)bz * g.sC * (g.out_dt == 0 ? 4 : 2) : nullptr;
    constexpr int PITCH = 256 * 4 + 16;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                                   // every wave is done reading the operand stages
#ifdef DL4J_EPI_STOREONLY
    // diagnostic: the read-out's global stores alone (same addresses and widths, values from the accumulators)
    {
      const int c = tid % 32, r0 = tid / 32;
#pragma unroll
      for (int P = 0; P < 2; ++P) {
        GSTAMP(4 + 2 * P);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = m0 + P * 128 + r0 + 16 * i;
          uint4 pk;
          pk.x = __float_as_uint(acc[i & 3][i][0]);
          pk.y = __float_as_uint(acc[(i + 1) & 3][i][1]);
          pk.z = pk.x ^ pk.y; pk.w = pk.x + pk.y;
          if (m < g.M) *reinterpret_cast<uint4*>(o.dst + ((long long)m * o.ld + n0 + c * 8) * 2) = pk;
        }
        GSTAMP(5 + 2 * P);
      }
    }
    if (0)
#endif
#pragma unroll
    for (int P = 0; P < 2; ++P) {
      if (wr == P) {
        sfor<0, 8>([&](auto MB) {
          constexpr int mb = decltype(MB)::value;
          const int lr = (mb >> 2) * 64 + (mb & 3) * 16 + (lane & 15);
          sfor<0, 4>([&](auto NB) {
            constexpr int nb = decltype(NB)::value;
            const int lc = wc * 64 + (nb >> 1) * 32 + (nb & 1) * 16 + (lane >> 4) * 4;
            *reinterpret_cast<f32x4_t*>(smem + lr * PITCH + lc * 4) = acc[nb][mb];
          });
        });
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
      GSTAMP(4 + 2 * P);
      if constexpr (BNB) epi_bnbwd<128, 256, 512>(g, smem, m0 + P * 128, n0, tid);
      else if (g.tstats) epi_stats<128, 256, 512>(g, smem, m0 + P * 128, n0, tid);
      epi_readout<128, 256, 512>(g, o, Zp, smem, m0 + P * 128, n0, tid);
      GSTAMP(5 + 2 * P);
      if (P == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
      }
    }
  }
#ifdef DL4J_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  GSTAMP(3);
}

// ----------------------------------------------------------------------------------------------- simple kernel
struct SimpleArgs {
  const void* A;
  const void* B;
  long long sam, sak, sbk, sbn;     // element strides
  long long bA, bB, bC;             // batch strides
  int in_dt;                        // 0 f32, 1 bf16, 2 f16
};

__device__ __forceinline__ float ld_in(const void* p, int dt, long long i) {
  if (dt == 0) return reinterpret_cast<const float*>(p)[i];
  const u16 u = reinterpret_cast<const u16*>(p)[i];
  return dt == 1 ? bf2f(u) : __half2float(__ushort_as_half(u));
}

// 64x64 output tile, BK = 16, 4 waves (2x2) each 32x32 via v_mfma_f32_32x32x2_f32 (exact fp32 products).
__global__ __launch_bounds__(256) void gemm_simple(GemmArgs g, SimpleArgs s) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int tiles_n = (g.N + 63) / 64;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * 64, n0 = tn * 64;
  const int bz = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const long long aoff = (long long)bz * s.bA, boff = (long long)bz * s.bB;
  f32x16_t acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  // loader: 1024 elements per operand tile = 4 per thread; element (kk, r) with r fastest when the operand is
  // contiguous along m/n, kk fastest otherwise (coalesced either way)
  const bool a_mfast = s.sam == 1, b_nfast = s.sbn == 1;
  for (int k0 = 0; k0 < g.K; k0 += 16) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      int kk, r;
      if (a_mfast) { kk = e >> 6; r = e & 63; } else { r = e >> 4; kk = e & 15; }
      const int m = m0 + r, k = k0 + kk;
      As[kk][r] = (m < g.M && k < g.K) ? ld_in(s.A, s.in_dt, aoff + m * s.sam + k * s.sak) : 0.f;
      if (b_nfast) { kk = e >> 6; r = e & 63; } else { r = e >> 4; kk = e & 15; }
      const int n = n0 + r, k2 = k0 + kk;
      Bs[kk][r] = (n < g.N && k2 < g.K) ? ld_in(s.B, s.in_dt, boff + k2 * s.sbk + n * s.sbn) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map: row (m) = (e&3) + 8(e>>2) + 4h, col (n) = lane&31
  const int h = lane >> 5;
  void* C = reinterpret_cast<char*>(g.C) + (long long)bz * s.bC * (g.out_dt == 0 ? 4 : 2);
  void* Zp = g.Z ? reinterpret_cast<char*>(g.Z) + (long long)bz * s.bC * (g.out_dt == 0 ? 4 : 2) : nullptr;
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= g.N) return;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (m >= g.M) continue;
    float x = acc[e] * g.alpha;
    if (g.bias_mode == 1) x += g.bias[n];
    else if (g.bias_mode == 2) x += g.bias[m];
    const long long o = (long long)m * g.ldc + n;
    if (g.beta != 0.f) x += g.beta * ld_out(C, g.out_dt, o);
    if (g.act == kActDGelu) {
      if (Zp) x *= dgelu(ld_out(Zp, g.out_dt, o));
    } else {
      if (Zp) {
        if (g.out_dt == 0) reinterpret_cast<float*>(Zp)[o] = x;
        else reinterpret_cast<u16*>(Zp)[o] = to16(x, g.out_dt);
      }
      x = apply_act(x, g.act);
    }
    if (g.out_dt == 0) reinterpret_cast<float*>(C)[o] = x;
    else reinterpret_cast<u16*>(C)[o] = to16(x, g.out_dt);
  }
}

// ----------------------------------------------------------------------------------------------- exact fp32, tiled
// BM x BN x 16 tiles (4 waves as 2 x 2, each (BM/2) x (BN/2) of v_mfma_f32_32x32x2_f32 accumulators: exact fp32
// products), operands of any dtype / strides converted to fp32 while staging to LDS (two buffers: the next K-step's
// global loads are issued before the current step's MFMAs), and split-K over grid.y: each split writes its raw fp32
// tile to a slab and gemm_splitk_reduce applies the epilogue in a fixed order. The one-tile gemm_simple above is the
// fallback for the smallest problems.
template <int BM, int BN>
__global__ __launch_bounds__(256) void gemm_f32t(GemmArgs g, SimpleArgs s) {
  constexpr int FM = BM / 64, FN = BN / 64;          // 32x32 accumulators per wave along M / N
  constexpr int LA = BM * 16 / 256, LB = BN * 16 / 256;   // elements staged per thread per operand
  __shared__ float As[2][16][BM + 4];
  __shared__ float Bs[2][16][BN + 4];
  const int tiles_n = (g.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.y, bz = blockIdx.z;
  const int kbeg = z * g.kps, kend = min(g.K, kbeg + g.kps);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const long long aoff = (long long)bz * s.bA, boff = (long long)bz * s.bB;
  const bool a_mfast = s.sam == 1, b_nfast = s.sbn == 1;
  f32x16_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  float ra[LA], rb[LB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = tid + 256 * u;
      int kk, r;
      if (a_mfast) { kk = e / BM; r = e % BM; } else { r = e >> 4; kk = e & 15; }
      const int m = m0 + r, k = k0 + kk;
      ra[u] = (m < g.M && k < kend) ? ld_in(s.A, s.in_dt, aoff + m * s.sam + k * s.sak) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = tid + 256 * u;
      int kk, r;
      if (b_nfast) { kk = e / BN; r = e % BN; } else { r = e >> 4; kk = e & 15; }
      const int n = n0 + r, k = k0 + kk;
      rb[u] = (n < g.N && k < kend) ? ld_in(s.B, s.in_dt, boff + k * s.sbk + n * s.sbn) : 0.f;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = tid + 256 * u;
      int kk, r;
      if (a_mfast) { kk = e / BM; r = e % BM; } else { r = e >> 4; kk = e & 15; }
      As[buf][kk][r] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = tid + 256 * u;
      int kk, r;
      if (b_nfast) { kk = e / BN; r = e % BN; } else { r = e >> 4; kk = e & 15; }
      Bs[buf][kk][r] = rb[u];
    }
  };
  int buf = 0;
  if (kbeg < kend) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
    const bool more = k0 + 16 < kend;
    if (more) gload(k0 + 16);                        // in flight during this step's MFMAs
#pragma unroll
    for (int kk = 0; kk < 16; kk += 2) {
      float a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = As[buf][kk + (lane >> 5)][wm * (BM / 2) + 32 * i + (lane & 31)];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = Bs[buf][kk + (lane >> 5)][wn * (BN / 2) + 32 * j + (lane & 31)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // C/D map of each accumulator: row (m) = (e&3) + 8(e>>2) + 4h, col (n) = lane&31
  const int h = lane >> 5;
  const bool split = g.splits > 1;
  void* C = reinterpret_cast<char*>(g.C) + (long long)bz * s.bC * (g.out_dt == 0 ? 4 : 2);
  void* Zp = g.Z ? reinterpret_cast<char*>(g.Z) + (long long)bz * s.bC * (g.out_dt == 0 ? 4 : 2) : nullptr;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * (BN / 2) + 32 * j + (lane & 31);
    if (n >= g.N) continue;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * (BM / 2) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m >= g.M) continue;
        float x = acc[i][j][e];
        if (split) {
          g.ws[(long long)z * g.M * g.N + (long long)m * g.N + n] = x;
          continue;
        }
        x *= g.alpha;
        if (g.bias_mode == 1) x += g.bias[n];
        else if (g.bias_mode == 2) x += g.bias[m];
        const long long o = (long long)m * g.ldc + n;
        if (g.beta != 0.f) x += g.beta * ld_out(C, g.out_dt, o);
        if (g.act == kActDGelu) {
          if (Zp) x *= dgelu(ld_out(Zp, g.out_dt, o));
        } else {
          if (Zp) {
            if (g.out_dt == 0) reinterpret_cast<float*>(Zp)[o] = x;
            else reinterpret_cast<u16*>(Zp)[o] = to16(x, g.out_dt);
          }
          x = apply_act(x, g.act);
        }
        if (g.out_dt == 0) reinterpret_cast<float*>(C)[o] = x;
        else reinterpret_cast<u16*>(C)[o] = to16(x, g.out_dt);
      }
  }
}

// tile (64 or 128) and split count for the tiled exact-fp32 kernel: fill the 256 CUs with >= 256-deep K slices
// Tile and split-K count of the exact-fp32 kernel. Each K-step of a block waits on its own global loads, so the
// kernel needs several blocks per CU to hide load latency: split K until ~768 blocks are in flight, keeping >= 48
// K-elements per slab (tools/f32_gemm_probe.py on the LeNet shapes: conv2 forward 77 -> 39 us with 4 splits, its
// weight gradient 77 -> 39-51 us with 96-128, dense forward / data gradient 2-3x faster). 128-wide tiles only for
// large problems (they lost on every LeNet shape).
void plan_f32(int M, int N, int K, int batch, int* tile, int* splits) {
  const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  const long long t64 = (long long)((M + 63) / 64) * ((N + 63) / 64) * batch;
  *tile = (t128 >= 512) ? 128 : 64;
  const long long t = *tile == 128 ? t128 : t64;
  int sp = 1;
  if (batch == 1 && t < 768) {
    sp = (int)((768 + t - 1) / t);
    const int maxs = K / 48;
    if (sp > maxs) sp = maxs;
    if (sp > 256) sp = 256;
    if (sp < 1) sp = 1;
  }
  *splits = sp;
}


// ----------------------------------------------------------------------------------------------- dispatch
// DL4J_AMD_GEMM_LEAN=0 forces the generic LDS epilogue everywhere (A/B experiments)

// Arrival counters of the in-kernel split-K fixup: 512 launches in flight x 2048 tiles, zero-initialised, each
// counter reset by its tile's last block (so no per-launch memset; a graph replay finds them at zero again).
constexpr int kSkSlots = 512, kSkTiles = 2048;
__device__ unsigned g_sk_ticket[kSkSlots * kSkTiles];

// Off by default (DL4J_AMD_GEMM_SPLITK_FIXUP=1 turns it on): measured slower on BERT-base, 447k vs 529k tok/s
// (profiles/r5_splitk_fixup.txt) — the write-through slab stores and the tile's serial last-block pass cost more than
// the reduce launch they replace, and the autotuner then moves shapes to other configurations.
int& splitk_fixup_mode() {
  static int v = [] {
    const char* e = getenv("DL4J_AMD_GEMM_SPLITK_FIXUP");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v;
}

unsigned* sk_ticket_slot() {
  static unsigned* base[64] = {nullptr};
  static unsigned next = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_sk_ticket)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  const unsigned k = __atomic_fetch_add(&next, 1u, __ATOMIC_RELAXED) % (unsigned)kSkSlots;
  return base[dev] + (long long)kSkTiles * k;
}

bool lean_disabled() {
  static const int v = [] {
    const char* e = getenv("DL4J_AMD_GEMM_LEAN");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  return v != 0;
}

struct Cfg {
  int bm, bn;
};
// cfg ids: 0 = 256x256 (8 waves 2x4, 2 stages), 1 = 256x128 (8 waves 4x2, 3 stages),
//          2 = 128x128 (4 waves 2x2, 2 stages, 2 blocks/CU), 3 = 128x64 (4 waves 2x2 of 64x32, 3 stages)
//          4 = 256x256 8-phase (8 waves, 16x16x32 MFMA, K % 64 == 0)
//          5 = 128x64 single-buffered (24 KB LDS, up to 4 blocks/CU: memory-bound skinny / small-K shapes)
//          6 = 128x128 3 stages (96 KB, 1 block/CU: two K-tiles in flight across each barrier instead of one)
//          7 = 128x128 4 stages (128 KB: three K-tiles in flight) — latency-bound small-grid / split-K shapes
//          8 = 128x128 single-buffered (32 KB, 4 blocks/CU), 9 = 128x256 single-buffered (8 waves, 64 KB, 2 blocks/CU):
//              short-K, output-heavy products (the expanding 1x1 convolutions: K = 64..256, N = 256..1024), where
//              a wide tile loads each A row panel once for more output columns and halves the blocks per output
//          10 = gemm_stream (persistent, loader wave + resident B panel; tall short-K products, M % 128 == 0)
constexpr int kNumCfg = 11;
const Cfg kCfg[kNumCfg] = {{256, 256}, {256, 128}, {128, 128}, {128, 64}, {256, 256},
                           {128, 64},  {128, 128}, {128, 128}, {128, 128}, {128, 256}, {128, 128}};

template <int DT, bool AKC, bool BKC, bool LEAN>
int launch_fast(int cfg, const GemmArgs& g, int batch, hipStream_t s) {
  const int tiles = g.tiles_m * g.tiles_n;
  dim3 grid(tiles, g.splits, batch);
  switch (cfg) {
    case 0: hipLaunchKernelGGL((gemm_glds<DT, 256, 256, 2, 4, AKC, BKC, 2, false, LEAN>), grid, dim3(512), 0, s, g); break;
    case 1: hipLaunchKernelGGL((gemm_glds<DT, 256, 128, 4, 2, AKC, BKC, 3, false, LEAN>), grid, dim3(512), 0, s, g); break;
    case 2: hipLaunchKernelGGL((gemm_glds<DT, 128, 128, 2, 2, AKC, BKC, 2, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 3: hipLaunchKernelGGL((gemm_glds<DT, 128, 64, 2, 2, AKC, BKC, 3, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 5: hipLaunchKernelGGL((gemm_glds<DT, 128, 64, 2, 2, AKC, BKC, 1, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 6: hipLaunchKernelGGL((gemm_glds<DT, 128, 128, 2, 2, AKC, BKC, 3, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 7: hipLaunchKernelGGL((gemm_glds<DT, 128, 128, 2, 2, AKC, BKC, 4, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 8: hipLaunchKernelGGL((gemm_glds<DT, 128, 128, 2, 2, AKC, BKC, 1, false, LEAN>), grid, dim3(256), 0, s, g); break;
    case 9: hipLaunchKernelGGL((gemm_glds<DT, 128, 256, 2, 4, AKC, BKC, 1, false, LEAN>), grid, dim3(512), 0, s, g); break;
    default: hipLaunchKernelGGL((gemm_8ph<DT, AKC, BKC, false, LEAN>), grid, dim3(512), 0, s, g); break;
  }
  return (int)hipGetLastError();
}

// BN-backward epilogue instantiations: only the 1x1 bwd-data layout (dY rows K-contiguous, W [K][C] N-contiguous)
template <int DT>
int launch_fast_bnb(int cfg, const GemmArgs& g, hipStream_t s) {
  if (cfg >= 6) return -1;                      // the deep-ring 128x128 tiles have no BN-backward instantiation
  dim3 grid(g.tiles_m * g.tiles_n, 1, 1);
  switch (cfg) {
    case 0: hipLaunchKernelGGL((gemm_glds<DT, 256, 256, 2, 4, true, false, 2, true>), grid, dim3(512), 0, s, g); break;
    case 1: hipLaunchKernelGGL((gemm_glds<DT, 256, 128, 4, 2, true, false, 3, true>), grid, dim3(512), 0, s, g); break;
    case 2: hipLaunchKernelGGL((gemm_glds<DT, 128, 128, 2, 2, true, false, 2, true>), grid, dim3(256), 0, s, g); break;
    case 3: hipLaunchKernelGGL((gemm_glds<DT, 128, 64, 2, 2, true, false, 3, true>), grid, dim3(256), 0, s, g); break;
    case 5: hipLaunchKernelGGL((gemm_glds<DT, 128, 64, 2, 2, true, false, 1, true>), grid, dim3(256), 0, s, g); break;
    default: hipLaunchKernelGGL((gemm_8ph<DT, true, false, true>), grid, dim3(512), 0, s, g); break;
  }
  return (int)hipGetLastError();
}

template <int DT, bool LEAN>
int launch_fast_lay(int cfg, int akc, int bkc, const GemmArgs& g, int batch, hipStream_t s) {
  if (akc && bkc) return launch_fast<DT, true, true, LEAN>(cfg, g, batch, s);
  if (akc) return launch_fast<DT, true, false, LEAN>(cfg, g, batch, s);
  if (bkc) return launch_fast<DT, false, true, LEAN>(cfg, g, batch, s);
  return launch_fast<DT, false, false, LEAN>(cfg, g, batch, s);
}

template <int DT>
int launch_fast_l(int cfg, int akc, int bkc, const GemmArgs& g, int batch, bool lean, hipStream_t s) {
  if (g.bnb) return (akc && !bkc && batch == 1) ? launch_fast_bnb<DT>(cfg, g, s) : -3;
  return lean ? launch_fast_lay<DT, true>(cfg, akc, bkc, g, batch, s) : launch_fast_lay<DT, false>(cfg, akc, bkc, g, batch, s);
}

// The lean epilogue's contract (mfma_tile.h): 16-bit output, alpha + optional per-column bias + none / relu / gelu
// (pre-activation kept in Z or not) / gelu-backward from Z, no beta, no split-K slabs, 16-byte addressable rows; BN
// tile statistics from the 16-bit image.
bool lean_ok(const GemmArgs& g, int batch) {
  if (g.splits > 1 || g.bnb || g.out_dt == 0 || g.beta != 0.f) return false;
  if (g.tstats && g.act != 0) return false;        // statistics are of the stored pre-activation output
  if (g.act != 0 && g.act != 1 && g.act != 4 && g.act != kActDGelu) return false;
  if (g.act == kActDGelu && !g.Z) return false;
  if (g.Z && ((g.act != 4 && g.act != kActDGelu) || (reinterpret_cast<uintptr_t>(g.Z) & 15))) return false;
  if (g.bias_mode == 2 || (g.bias_mode == 1 && (reinterpret_cast<uintptr_t>(g.bias) & 15))) return false;
  if ((g.N & 7) || (g.ldc & 7) || (reinterpret_cast<uintptr_t>(g.C) & 15)) return false;
  if (batch > 1 && (g.sC & 7)) return false;
  return !lean_disabled();
}

// Choose tile config + split-K. The 8-phase 256x256 kernel when it can fill >= half the chip (split-K over >= 8
// K-tiles per split if needed), else the biggest 2/3-stage tile that reaches one block per CU.
void plan(int M, int N, int K, int batch, int* cfg, int* splits) {
  const int CUS = 256;
  const long long t256 = (long long)((M + 255) / 256) * ((N + 255) / 256) * batch;
  if (K % 64 == 0) {
    int sp = 1;
    if (batch == 1 && t256 < 224) {
      sp = (int)((CUS + t256 - 1) / t256);
      const int maxs = K / 512;
      if (sp > maxs) sp = maxs;
      if (sp > 256) sp = 256;
      if (sp < 1) sp = 1;
    }
    if (t256 * sp >= 128) { *cfg = 4; *splits = sp; return; }
  }
  int best = 3;
  for (int c = 0; c < 4; ++c) {
    const long long t = (long long)((M + kCfg[c].bm - 1) / kCfg[c].bm) * ((N + kCfg[c].bn - 1) / kCfg[c].bn) * batch;
    if (t >= CUS) { best = c; break; }
  }
  *cfg = best;
  const long long t = (long long)((M + kCfg[best].bm - 1) / kCfg[best].bm) * ((N + kCfg[best].bn - 1) / kCfg[best].bn) * batch;
  int sp = 1;
  if (batch == 1 && t < CUS) {
    sp = (int)((CUS + t - 1) / t);
    const int maxs = K / 512;                  // keep >= 8 K-tiles per split
    if (sp > maxs) sp = maxs;
    if (sp < 1) sp = 1;
    if (sp > 256) sp = 256;
  }
  *splits = sp;
}

}  // namespace

// 1: split-K products of the gemm_glds tiles sum their slabs in the kernel; 0 (default): separate reduce launch.
// Returns the previous mode.
DL4J_API int dl4j_gemm_set_splitk_fixup(int on) {
  const int old = splitk_fixup_mode();
  splitk_fixup_mode() = on ? 1 : 0;
  return old;
}

// Returns the workspace bytes the fast path needs for (M, N, K, batch) with config (cfg, splits) chosen by plan().
DL4J_API long long dl4j_gemm_plan(int M, int N, int K, int batch, int* cfg, int* splits) {
  plan(M, N, K, batch, cfg, splits);
  if (*splits <= 1) return 0;
  int kps = (K + *splits - 1) / *splits;
  kps = (kps + 63) / 64 * 64;
  *splits = (K + kps - 1) / kps;
  return *splits > 1 ? (long long)(*splits) * M * N * 4 : 0;
}

BnbArm& bnb_armed() {
  static thread_local BnbArm a{nullptr, nullptr, nullptr, 0};
  return a;
}

// Arms (mode 1: plain, 2: ReLU recomputed from x, 3: ReLU from the forward's bitmask) or disarms (mode 0)
// BatchNorm-backward statistics for the next dl4j_gemm / dl4j_conv_fwd_v3 launches of this thread that pass a
// statistics buffer: planes [2][P][N] of sum(d), sum(d*xhat) of the stored output instead of the forward [3][P][N]
// tile statistics. x: the BN layer's input, laid out like the output; ctx: its forward [mean | invstd | scale | shift]
// (csrc/batchnorm.hip); mask: bn_apply's ReLU bitmask (mode 3).
DL4J_API void dl4j_bnb_arm(const void* x, const float* ctx, const unsigned char* mask, int mode) {
  BnbArm& a = bnb_armed();
  const bool ok = mode && x && ctx && (mode != 3 || mask);
  a.x = ok ? x : nullptr;
  a.ctx = ok ? ctx : nullptr;
  a.mask = ok ? mask : nullptr;
  a.mode = ok ? mode : 0;
}

// Fast path. in_dt: 1 bf16, 2 f16. out_dt: 0 f32, 1 bf16, 2 f16. akc/bkc: operand layout flags (see top).
// Requirements (else -1): lda/ldb multiples of 8 elements and 16-byte aligned bases; K % 8 == 0 for K-contiguous
// operands, M % 8 == 0 (N % 8 == 0) for an M- (N-) contiguous A (B); batch > 1 only without split-K.
DL4J_API int dl4j_gemm(int in_dt, int out_dt, int M, int N, int K, int batch, const void* A, long long lda, int akc,
                       long long sA, const void* B, long long ldb, int bkc, long long sB, void* C, long long ldc,
                       long long sC, float alpha, float beta, const float* bias, int bias_mode, int act, void* Z,
                       int cfg, int splits, float* ws, float* tstats, int stats_P, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (in_dt != 1 && in_dt != 2) return -1;
  if ((lda & 7) || (ldb & 7) || (reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15)) return -1;
  if (batch > 1 && ((sA & 7) || (sB & 7))) return -1;
  // K-contiguous operands need K % 8 (a 16-byte chunk must not straddle K) unless flagged (bit 1 of akc/bkc) as
  // zero-padded to the next multiple of 8 inside their leading dimension: the straddling chunk then only brings zeros,
  // and an M/N-contiguous partner reads its rows >= K from the zero page. An M/N-contiguous operand only needs its
  // leading dimension % 8: the chunk past M (N) stays inside the row stride and only feeds discarded outputs.
  {
    const bool akz = (akc & 2) != 0, bkz = (bkc & 2) != 0;
    akc &= 1;
    bkc &= 1;
    if ((akc && (K & 7) && !(akz && lda >= ((K + 7) & ~7))) || (bkc && (K & 7) && !(bkz && ldb >= ((K + 7) & ~7))))
      return -1;
  }
  if (K <= 0) return -1;
  if (cfg < 0 || cfg >= kNumCfg || splits < 1) plan(M, N, K, batch, &cfg, &splits);
  if ((cfg == 3 || cfg == 5) && !bkc) cfg = 2;   // the 64-wide tile has no N-contiguous image
  if (cfg == 4) {                                // 8-phase: K % 64 and 32-bit element offsets
    const long long ea = akc ? (long long)(M - 1) * lda + K : (long long)(K - 1) * lda + M;
    const long long eb = bkc ? (long long)(N - 1) * ldb + K : (long long)(K - 1) * ldb + N;
    if (K % 64 != 0 || ea >= 0x7fffffffLL || eb >= 0x7fffffffLL) { cfg = 0; }
  }
  if (batch > 1) splits = 1;
  GemmArgs g;
  g.sk_ticket = nullptr;
  g.A = A; g.B = B; g.C = C; g.Z = Z; g.bias = bias; g.ws = ws;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.sA = sA; g.sB = sB; g.sC = sC;
  g.M = M; g.N = N; g.K = K;
  int kps = (K + splits - 1) / splits;
  kps = (kps + 63) / 64 * 64;
  splits = (K + kps - 1) / kps;
  if (splits > 1 && ws == nullptr) return -2;
  g.kps = kps; g.splits = splits;
  g.alpha = alpha; g.beta = beta; g.bias_mode = bias ? bias_mode : 0; g.act = act; g.out_dt = out_dt;
  g.tstats = nullptr;
  g.stats_P = 0;
  g.bnx = nullptr; g.bnctx = nullptr; g.bnmask = nullptr; g.bnb = 0;
  g.store_nt = store_nt_for((long long)M * N * batch * (out_dt == 0 ? 4 : 2));
  if (tstats) {                                   // statistics only from the 8-phase epilogue without split-K
    if (splits > 1 || batch > 1) return -3;
    g.tstats = tstats;
    g.stats_P = stats_P;
    const BnbArm& ba = bnb_armed();
    if (ba.mode) {                                // BN-backward sums of the stored output (mfma_tile.h epi_bnbwd_wave)
      if (bias || act || (N & 3) || (ldc & 3) || (out_dt != 1 && out_dt != 2) || (ba.mode == 3 && ldc != N) ||
          (reinterpret_cast<uintptr_t>(C) & 7))
        return -3;
      g.bnx = ba.x; g.bnctx = ba.ctx; g.bnmask = ba.mask; g.bnb = ba.mode;
    }
  }
  {
    const int esz = out_dt == 0 ? 4 : 2;
    g.coalesce = ((ldc * esz) % 16 == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0 &&
                  (batch == 1 || (sC * esz) % 16 == 0)) ? 1 : 0;
  }
  g.tiles_m = (M + kCfg[cfg].bm - 1) / kCfg[cfg].bm;
  g.tiles_n = (N + kCfg[cfg].bn - 1) / kCfg[cfg].bn;
  const bool lean = lean_ok(g, batch);
  if (cfg == 10) {                                // streaming kernel: its contract, else refused (-4)
    if (!akc || !bkc || batch != 1 || splits != 1 || !lean || g.bnb || g.Z || (M % 128)) return -4;
    return dl4j_gemm_stream(in_dt, A, lda, B, ldb, C, ldc, M, N, K, alpha, g.bias, g.bias_mode, act, out_dt, tstats,
                            stats_P, g.store_nt, s);
  }
  if (splits > 1 && cfg != 4 && batch == 1 && !g.bnb && splitk_fixup_mode() &&
      (long long)g.tiles_m * g.tiles_n <= kSkTiles)
    g.sk_ticket = sk_ticket_slot();            // gemm_glds sums the slabs itself: no reduce launch
  const int e = in_dt == 1 ? launch_fast_l<1>(cfg, akc, bkc, g, batch, lean, s)
                           : launch_fast_l<2>(cfg, akc, bkc, g, batch, lean, s);
  if (e || splits <= 1 || g.sk_ticket) return e;
  const long long total = (long long)M * ((N + 3) / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

// Tiled exact-fp32 path (gemm_f32t): workspace bytes for the split-K slabs of (M, N, K, batch); *tile, *splits out.
DL4J_API long long dl4j_gemm_f32_plan(int M, int N, int K, int batch, int* tile, int* splits) {
  plan_f32(M, N, K, batch, tile, splits);
  if (*splits <= 1) return 0;
  int kps = (K + *splits - 1) / *splits;
  kps = (kps + 15) / 16 * 16;
  *splits = (K + kps - 1) / kps;
  return *splits > 1 ? (long long)(*splits) * M * N * 4 : 0;
}

// Any dtype (0 f32 / 1 bf16 / 2 f16 input), any element strides, exact fp32 MFMA products, BM x BN tiles + split-K.
// tile: 64 or 128 (<= 0: planned); splits > 1 needs ws (dl4j_gemm_f32_plan bytes).
DL4J_API int dl4j_gemm_f32(int in_dt, int out_dt, int M, int N, int K, int batch, const void* A, long long sam,
                           long long sak, long long sA, const void* B, long long sbk, long long sbn, long long sB,
                           void* C, long long ldc, long long sC, float alpha, float beta, const float* bias,
                           int bias_mode, int act, void* Z, int tile, int splits, float* ws, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (tile <= 0) plan_f32(M, N, K, batch, &tile, &splits);
  if (batch > 1 || splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = (kps + 15) / 16 * 16;
  if (kps < 16) kps = 16;
  splits = (K + kps - 1) / kps;
  if (splits < 1) splits = 1;
  if (splits > 1 && !ws) return -2;
  GemmArgs g = {};
  g.C = C; g.Z = Z; g.bias = bias; g.ldc = ldc; g.M = M; g.N = N; g.K = K; g.ws = ws;
  g.kps = splits > 1 ? kps : (K > 0 ? K : 16);
  g.splits = splits;
  g.alpha = alpha; g.beta = beta; g.bias_mode = bias ? bias_mode : 0; g.act = act; g.out_dt = out_dt;
  SimpleArgs sa;
  sa.A = A; sa.B = B; sa.sam = sam; sa.sak = sak; sa.sbk = sbk; sa.sbn = sbn;
  sa.bA = sA; sa.bB = sB; sa.bC = sC; sa.in_dt = in_dt;
  const int tiles = tile == 128 ? ((M + 127) / 128) * ((N + 127) / 128) : ((M + 63) / 64) * ((N + 63) / 64);
  dim3 grid(tiles, splits, batch);
  if (tile == 128) hipLaunchKernelGGL((gemm_f32t<128, 128>), grid, dim3(256), 0, s, g, sa);
  else hipLaunchKernelGGL((gemm_f32t<64, 64>), grid, dim3(256), 0, s, g, sa);
  int e = (int)hipGetLastError();
  if (e || splits <= 1) return e;
  const long long total = (long long)M * ((N + 3) / 4);
  if (splits >= 16) {
    hipLaunchKernelGGL(gemm_splitk_reduce_deep, dim3((unsigned)((total + 15) / 16)), dim3(256), 0, s, g);
    return (int)hipGetLastError();
  }
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, g);
  return (int)hipGetLastError();
}

// Generic path: any dtype (0 f32 / 1 bf16 / 2 f16 input), any element strides, exact fp32 MFMA.
DL4J_API int dl4j_gemm_simple(int in_dt, int out_dt, int M, int N, int K, int batch, const void* A, long long sam,
                              long long sak, long long sA, const void* B, long long sbk, long long sbn, long long sB,
                              void* C, long long ldc, long long sC, float alpha, float beta, const float* bias,
                              int bias_mode, int act, void* Z, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  GemmArgs g = {};
  g.C = C; g.Z = Z; g.bias = bias; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
  g.alpha = alpha; g.beta = beta; g.bias_mode = bias ? bias_mode : 0; g.act = act; g.out_dt = out_dt;
  SimpleArgs sa;
  sa.A = A; sa.B = B; sa.sam = sam; sa.sak = sak; sa.sbk = sbk; sa.sbn = sbn;
  sa.bA = sA; sa.bB = sB; sa.bC = sC; sa.in_dt = in_dt;
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  hipLaunchKernelGGL(gemm_simple, dim3(tiles, 1, batch), dim3(256), 0, s, g, sa);
  return (int)hipGetLastError();
}
