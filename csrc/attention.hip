// Fused multi-head attention (flash-style) for gfx950, bf16 or fp16 in (template element type hb) / fp32 accumulate,
// head dim D in {64, 128}.
// Used by the transformer layers (BERT-base config of BASELINE.json; attention is new relative to the reference,
// SURVEY §2.6 / §5.7).
//
// Layout: Q, K, V are read in place from the fused projection output qkv[B, T, 3*E] (E = H*D; Q at column h*D,
// K at E + h*D, V at 2E + h*D), O is written to [B, T, E] and the backward writes dQ/dK/dV straight into a
// dqkv[B, T, 3*E] buffer — no permute copies around the kernels. Optional key-padding mask [B, T] (1 = keep) and
// causal masking.
//
// CDNA4 mapping (per 64-wide wave, v_mfma_f32_16x16x32_bf16):
//  * forward / dQ: a wave owns 16 queries. Scores are computed TRANSPOSED, Sᵀ = K·Qᵀ, so the query is the lane's
//    accumulator column: the online-softmax state (running max m, sum l) is one scalar per lane and the 64 keys of
//    a block reduce with two cross-group shuffles. Pᵀ stays in registers and feeds Oᵀ += Vᵀ·Pᵀ directly as the B
//    operand (the k-slot order of the accumulator layout is matched on the A side by reading Vᵀ from LDS in the same
//    permuted key order), so P never touches LDS.
//  * dK/dV: a wave owns 16 keys; S = Q·Kᵀ has the key on the lane; dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS take P / dS as B
//    operands the same way. dQ is a separate pass over query blocks (no atomics).
//  * K/V (or Q/dO) tiles are staged in LDS per 64-row block, both row-major and transposed as the operands need;
//    rows padded by 16 B.
// Softmax runs in the exp2 domain: s2 = q·k · scale·log2(e); lse2 = m2 + log2(l) is saved for the backward.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) float f4_t;
template <typename T> using V8 = T __attribute__((ext_vector_type(8)));
template <typename T> using V4 = T __attribute__((ext_vector_type(4)));

static constexpr int BLK = 64;             // rows (queries or keys) per block
static constexpr float kLog2e = 1.4426950408889634f;
static constexpr float kNegInf = -INFINITY;

// v_mfma_f32_16x16x32_{bf16,f16}: same fragment layout for both element types
__device__ __forceinline__ f4_t mma(V8<__bf16> a, V8<__bf16> b, f4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4_t mma(V8<_Float16> a, V8<_Float16> b, f4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <typename hb> __device__ __forceinline__ hb tobf(float v) { return (hb)v; }

// fragment of 8 hb from a row-major LDS/global row (16-byte aligned)
template <typename hb> __device__ __forceinline__ V8<hb> ld8(const hb* p) { return *reinterpret_cast<const V8<hb>*>(p); }
// two 4-element pieces (keys 4h..4h+3 and 16+4h..16+4h+3 of a 32-key step) of a transposed row
template <typename hb> __device__ __forceinline__ V8<hb> ld4x2(const hb* row, int h) {
  const V4<hb> a = *reinterpret_cast<const V4<hb>*>(row + 4 * h);
  const V4<hb> b = *reinterpret_cast<const V4<hb>*>(row + 16 + 4 * h);
  return V8<hb>{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// B fragment from two accumulator tiles (16 rows each) in the permuted k order matching ld4x2
template <typename hb> __device__ __forceinline__ V8<hb> pack2(const f4_t& x, const f4_t& y) {
  return V8<hb>{(hb)x[0], (hb)x[1], (hb)x[2], (hb)x[3], (hb)y[0], (hb)y[1], (hb)y[2], (hb)y[3]};
}

// cooperative block loads: rows [r0, r0+64) of a [T, ld] matrix slice (D columns at col0) into LDS
template <int D, typename hb>
__device__ __forceinline__ void stage_rows(hb* dst, int dld, const hb* src, long long src_ld, int r0, int T) {
  constexpr int CPR = D / 8;                                  // 16-byte chunks per row
  for (int i = threadIdx.x; i < BLK * CPR; i += blockDim.x) {
    const int r = i / CPR, c = i - r * CPR;
    V8<hb> v;
    if (r0 + r < T) v = *reinterpret_cast<const V8<hb>*>(src + (long long)(r0 + r) * src_ld + c * 8);
    else v = V8<hb>{0, 0, 0, 0, 0, 0, 0, 0};
    *reinterpret_cast<V8<hb>*>(dst + r * dld + c * 8) = v;
  }
}
template <int D, typename hb>
__device__ __forceinline__ void stage_rows_t(hb* dst, int dld, const hb* src, long long src_ld, int r0, int T) {
  constexpr int CPR = D / 8;                                  // transposed: dst[d][row]
  for (int i = threadIdx.x; i < BLK * CPR; i += blockDim.x) {
    const int r = i % BLK, c = i / BLK;
    V8<hb> v;
    if (r0 + r < T) v = *reinterpret_cast<const V8<hb>*>(src + (long long)(r0 + r) * src_ld + c * 8);
    else v = V8<hb>{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[(c * 8 + k) * dld + r] = v[k];
  }
}

__device__ __forceinline__ float wmax16(float v) {            // max over the 4 lane groups (l>>4)
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float wsum16(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// ------------------------------------------------------------------------------------------------ forward
// NB key blocks are staged per round (NB = 2 for D = 64: a T = 128 sequence is one round, one global round trip and
// one barrier pair instead of two); every thread issues all of the round's K and V loads before any LDS store.
template <int D, typename hb, int NB>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const hb* __restrict__ qkv, const float* __restrict__ mask,
                                                       hb* __restrict__ out, float* __restrict__ lse, int T, int H,
                                                       float scale2, int causal) {
  constexpr int KS = D / 32, DT = D / 16;
  constexpr int LDK = D + 8, LDV = NB * BLK + 8;
  constexpr int CPR = D / 8, PER = BLK * CPR / 256;              // 16-byte chunks per row / per thread per block
  __shared__ __attribute__((aligned(16))) hb Ks[NB * BLK * LDK];
  __shared__ __attribute__((aligned(16))) hb Vt[D * LDV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int E = H * D;
  const long long ld3 = 3LL * E;
  const hb* base = qkv + (long long)b * T * ld3;
  const int q = blockIdx.x * BLK + wave * 16 + col;
  const int qc = min(q, T - 1);
  V8<hb> qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qf[ks] = ld8(base + (long long)qc * ld3 + h * D + ks * 32 + 8 * hgrp);
  f4_t acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = f4_t{0.f, 0.f, 0.f, 0.f};
  float m = kNegInf, l = 0.f;
  const float* mrow = mask ? mask + (long long)b * T : nullptr;
  const int nkb = causal ? min((blockIdx.x * BLK + BLK + BLK - 1) / BLK, (T + BLK - 1) / BLK) : (T + BLK - 1) / BLK;
  for (int kb0 = 0; kb0 < nkb; kb0 += NB) {
    __syncthreads();
    V8<hb> kr[NB][PER], vr[NB][PER];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const int i = threadIdx.x + it * 256, r = i / CPR, c = i - r * CPR;
        const int row = (kb0 + j) * BLK + r;
        const bool ok = kb0 + j < nkb && row < T;
        const hb* src = base + (long long)(ok ? row : 0) * ld3 + h * D + c * 8;
        kr[j][it] = ok ? ld8(src + E) : V8<hb>{0, 0, 0, 0, 0, 0, 0, 0};
        vr[j][it] = ok ? ld8(src + 2 * E) : V8<hb>{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int it = 0; it < PER; ++it) {
        const int i = threadIdx.x + it * 256, r = i / CPR, c = i - r * CPR;
        *reinterpret_cast<V8<hb>*>(Ks + (j * BLK + r) * LDK + c * 8) = kr[j][it];
#pragma unroll
        for (int k = 0; k < 8; ++k) Vt[(c * 8 + k) * LDV + j * BLK + r] = vr[j][it][k];
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int kb = kb0 + j;
      if (kb >= nkb) break;
      const hb* Kj = Ks + j * BLK * LDK;
      f4_t s[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        s[mt] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[mt] = mma(ld8(Kj + (mt * 16 + col) * LDK + ks * 32 + 8 * hgrp), qf[ks], s[mt]);
      }
      float bm = kNegInf;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * BLK + mt * 16 + hgrp * 4 + r;
          bool ok = key < T && (!causal || key <= q);
          if (ok && mrow) ok = mrow[key] != 0.f;
          const float v = ok ? s[mt][r] * scale2 : kNegInf;
          s[mt][r] = v;
          bm = fmaxf(bm, v);
        }
      bm = wmax16(bm);
      const float mn = fmaxf(m, bm);
      const float alpha = (mn == kNegInf) ? 1.f : exp2f(m - mn);
      float ps = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = (mn == kNegInf) ? 0.f : exp2f(s[mt][r] - mn);
          s[mt][r] = p;
          ps += p;
        }
      l = l * alpha + wsum16(ps);
      m = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc[dt] *= alpha;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const V8<hb> pb = pack2<hb>(s[2 * k2], s[2 * k2 + 1]);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          acc[dt] = mma(ld4x2(Vt + (dt * 16 + col) * LDV + j * BLK + 32 * k2, hgrp), pb, acc[dt]);
      }
    }
  }
  if (q < T) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    hb* orow = out + ((long long)b * T + q) * E + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const V4<hb> v{tobf<hb>(acc[dt][0] * inv), tobf<hb>(acc[dt][1] * inv), tobf<hb>(acc[dt][2] * inv), tobf<hb>(acc[dt][3] * inv)};
      *reinterpret_cast<V4<hb>*>(orow + dt * 16 + hgrp * 4) = v;
    }
    if (hgrp == 0) lse[(long long)bh * T + q] = l > 0.f ? m + log2f(l) : 1e30f;
  }
}

// ------------------------------------------------------------------------------------------------ backward
// Dq[b,h,q] = sum_d dO[q,d] * O[q,d]
template <int D, typename hb>
__global__ void __launch_bounds__(256) attn_bwd_pre_kernel(const hb* __restrict__ o, const hb* __restrict__ dout,
                                                           float* __restrict__ dq_dot, int B, int T, int H) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // over B*H*T
  if (i >= (long long)B * H * T) return;
  const int q = (int)(i % T);
  const long long bh = i / T;
  const int h = (int)(bh % H), b = (int)(bh / H);
  const long long off = ((long long)b * T + q) * H * D + h * D;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    const V8<hb> a = ld8(o + off + c * 8), g = ld8(dout + off + c * 8);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += (float)a[k] * (float)g[k];
  }
  dq_dot[i] = s;
}

// dQ per query block (forward orientation: query on the lane)
template <int D, typename hb>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(const hb* __restrict__ qkv, const hb* __restrict__ dout,
                                                          const float* __restrict__ mask, const float* __restrict__ lse,
                                                          const float* __restrict__ dq_dot, hb* __restrict__ dqkv,
                                                          int T, int H, float scale2, float scale, int causal) {
  constexpr int KS = D / 32, DT = D / 16;
  constexpr int LDK = D + 8, LDT = BLK + 8;
  __shared__ __attribute__((aligned(16))) hb Ks[BLK * LDK];
  __shared__ __attribute__((aligned(16))) hb Vs[BLK * LDK];
  __shared__ __attribute__((aligned(16))) hb Kt[D * LDT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int E = H * D;
  const long long ld3 = 3LL * E;
  const hb* base = qkv + (long long)b * T * ld3;
  const int q = blockIdx.x * BLK + wave * 16 + col;
  const int qc = min(q, T - 1);
  V8<hb> qf[KS], df[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = ld8(base + (long long)qc * ld3 + h * D + ks * 32 + 8 * hgrp);
    df[ks] = ld8(dout + ((long long)b * T + qc) * E + h * D + ks * 32 + 8 * hgrp);
  }
  const float l2 = lse[(long long)bh * T + qc];
  const float dd = dq_dot[(long long)bh * T + qc];
  f4_t acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = f4_t{0.f, 0.f, 0.f, 0.f};
  const float* mrow = mask ? mask + (long long)b * T : nullptr;
  const int nkb = causal ? min((blockIdx.x * BLK + BLK + BLK - 1) / BLK, (T + BLK - 1) / BLK) : (T + BLK - 1) / BLK;
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    stage_rows<D>(Ks, LDK, base + E + h * D, ld3, kb * BLK, T);
    stage_rows<D>(Vs, LDK, base + 2 * E + h * D, ld3, kb * BLK, T);
    stage_rows_t<D>(Kt, LDT, base + E + h * D, ld3, kb * BLK, T);
    __syncthreads();
    f4_t s[4], dp[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      s[mt] = f4_t{0.f, 0.f, 0.f, 0.f};
      dp[mt] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s[mt] = mma(ld8(Ks + (mt * 16 + col) * LDK + ks * 32 + 8 * hgrp), qf[ks], s[mt]);
        dp[mt] = mma(ld8(Vs + (mt * 16 + col) * LDK + ks * 32 + 8 * hgrp), df[ks], dp[mt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb * BLK + mt * 16 + hgrp * 4 + r;
        bool ok = key < T && q < T && (!causal || key <= q);
        if (ok && mrow) ok = mrow[key] != 0.f;
        const float p = ok ? exp2f(s[mt][r] * scale2 - l2) : 0.f;
        s[mt][r] = p * (dp[mt][r] - dd);                       // dS (w.r.t. the scaled scores)
      }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const V8<hb> sb = pack2<hb>(s[2 * k2], s[2 * k2 + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc[dt] = mma(ld4x2(Kt + (dt * 16 + col) * LDT + 32 * k2, hgrp), sb, acc[dt]);
    }
  }
  if (q < T) {
    hb* dst = dqkv + ((long long)b * T + q) * ld3 + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const V4<hb> v{tobf<hb>(acc[dt][0] * scale), tobf<hb>(acc[dt][1] * scale), tobf<hb>(acc[dt][2] * scale),
                       tobf<hb>(acc[dt][3] * scale)};
      *reinterpret_cast<V4<hb>*>(dst + dt * 16 + hgrp * 4) = v;
    }
  }
}

// dK, dV per key block (key on the lane)
template <int D, typename hb>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(const hb* __restrict__ qkv,
                                                            const hb* __restrict__ dout,
                                                            const float* __restrict__ mask,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ dq_dot,
                                                            hb* __restrict__ dqkv, int T, int H, float scale2,
                                                            float scale, int causal) {
  constexpr int KS = D / 32, DT = D / 16;
  constexpr int LDQ = D + 8, LDT = BLK + 8;
  __shared__ __attribute__((aligned(16))) hb Qs[BLK * LDQ];
  __shared__ __attribute__((aligned(16))) hb Ds[BLK * LDQ];
  __shared__ __attribute__((aligned(16))) hb Qt[D * LDT];
  __shared__ __attribute__((aligned(16))) hb Dt[D * LDT];
  __shared__ float Ls[BLK], Dd[BLK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, hgrp = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int E = H * D;
  const long long ld3 = 3LL * E;
  const hb* base = qkv + (long long)b * T * ld3;
  const hb* dbase = dout + (long long)b * T * E;
  const int key = blockIdx.x * BLK + wave * 16 + col;
  const int kc = min(key, T - 1);
  bool kvalid = key < T;
  if (kvalid && mask) kvalid = mask[(long long)b * T + key] != 0.f;
  V8<hb> kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    kf[ks] = ld8(base + (long long)kc * ld3 + E + h * D + ks * 32 + 8 * hgrp);
    vf[ks] = ld8(base + (long long)kc * ld3 + 2 * E + h * D + ks * 32 + 8 * hgrp);
  }
  f4_t dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dk[dt] = dv[dt] = f4_t{0.f, 0.f, 0.f, 0.f};
  const int nqb = (T + BLK - 1) / BLK;
  const int qb0 = causal ? blockIdx.x : 0;                     // queries before the key block see none of it
  for (int qb = qb0; qb < nqb; ++qb) {
    __syncthreads();
    stage_rows<D>(Qs, LDQ, base + h * D, ld3, qb * BLK, T);
    stage_rows<D>(Ds, LDQ, dbase + h * D, E, qb * BLK, T);
    stage_rows_t<D>(Qt, LDT, base + h * D, ld3, qb * BLK, T);
    stage_rows_t<D>(Dt, LDT, dbase + h * D, E, qb * BLK, T);
    if (threadIdx.x < BLK) {
      const int qq = min(qb * BLK + (int)threadIdx.x, T - 1);
      Ls[threadIdx.x] = lse[(long long)bh * T + qq];
      Dd[threadIdx.x] = dq_dot[(long long)bh * T + qq];
    }
    __syncthreads();
    f4_t s[4], dp[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      s[mt] = f4_t{0.f, 0.f, 0.f, 0.f};
      dp[mt] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s[mt] = mma(ld8(Qs + (mt * 16 + col) * LDQ + ks * 32 + 8 * hgrp), kf[ks], s[mt]);
        dp[mt] = mma(ld8(Ds + (mt * 16 + col) * LDQ + ks * 32 + 8 * hgrp), vf[ks], dp[mt]);
      }
    }
    f4_t ds[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = mt * 16 + hgrp * 4 + r, q = qb * BLK + qi;
        const bool ok = kvalid && q < T && (!causal || key <= q);
        const float p = ok ? exp2f(s[mt][r] * scale2 - Ls[qi]) : 0.f;
        s[mt][r] = p;
        ds[mt][r] = p * (dp[mt][r] - Dd[qi]);
      }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const V8<hb> pb = pack2<hb>(s[2 * k2], s[2 * k2 + 1]);
      const V8<hb> sb = pack2<hb>(ds[2 * k2], ds[2 * k2 + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dv[dt] = mma(ld4x2(Dt + (dt * 16 + col) * LDT + 32 * k2, hgrp), pb, dv[dt]);
        dk[dt] = mma(ld4x2(Qt + (dt * 16 + col) * LDT + 32 * k2, hgrp), sb, dk[dt]);
      }
    }
  }
  if (key < T) {
    hb* dst = dqkv + ((long long)b * T + key) * ld3 + h * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const V4<hb> kv{tobf<hb>(dk[dt][0] * scale), tobf<hb>(dk[dt][1] * scale), tobf<hb>(dk[dt][2] * scale),
                        tobf<hb>(dk[dt][3] * scale)};
      const V4<hb> vv{tobf<hb>(dv[dt][0]), tobf<hb>(dv[dt][1]), tobf<hb>(dv[dt][2]), tobf<hb>(dv[dt][3])};
      *reinterpret_cast<V4<hb>*>(dst + E + dt * 16 + hgrp * 4) = kv;
      *reinterpret_cast<V4<hb>*>(dst + 2 * E + dt * 16 + hgrp * 4) = vv;
    }
  }
}

// ------------------------------------------------------------------------------------------------ launch
template <int D, typename hb>
static int fwd_l(const void* qkv, const float* mask, void* out, float* lse, int B, int T, int H, float scale,
                 int causal, hipStream_t s) {
  const dim3 grid((T + BLK - 1) / BLK, B * H);
  constexpr int NB = D == 64 ? 2 : 1;
  hipLaunchKernelGGL((attn_fwd_kernel<D, hb, NB>), grid, dim3(256), 0, s, (const hb*)qkv, mask, (hb*)out, lse, T, H,
                     scale * kLog2e, causal);
  return (int)hipGetLastError();
}

template <int D, typename hb>
static int bwd_l(const void* qkv, const void* out, const void* dout, const float* mask, const float* lse,
                 float* dq_dot, void* dqkv, int B, int T, int H, float scale, int causal, hipStream_t s) {
  const long long n = (long long)B * H * T;
  hipLaunchKernelGGL((attn_bwd_pre_kernel<D, hb>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const hb*)out,
                     (const hb*)dout, dq_dot, B, T, H);
  const dim3 grid((T + BLK - 1) / BLK, B * H);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, hb>), grid, dim3(256), 0, s, (const hb*)qkv, (const hb*)dout, mask, lse,
                     dq_dot, (hb*)dqkv, T, H, scale * kLog2e, scale, causal);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, hb>), grid, dim3(256), 0, s, (const hb*)qkv, (const hb*)dout, mask, lse,
                     dq_dot, (hb*)dqkv, T, H, scale * kLog2e, scale, causal);
  return (int)hipGetLastError();
}

// dt: 1 = bf16, 2 = fp16. qkv [B,T,3*H*D]; mask [B,T] fp32 or null; out [B,T,H*D]; lse [B,H,T] fp32.
// -1 = unsupported shape / dtype.
DL4J_API int dl4j_attn_fwd_dt(int dt, const void* qkv, const float* mask, void* out, float* lse, int B, int T, int H,
                              int D, float scale, int causal, hipStream_t s) {
  if (B < 1 || T < 1 || H < 1 || (dt != 1 && dt != 2)) return -1;
  if (D == 64) return dt == 1 ? fwd_l<64, __bf16>(qkv, mask, out, lse, B, T, H, scale, causal, s)
                              : fwd_l<64, _Float16>(qkv, mask, out, lse, B, T, H, scale, causal, s);
  if (D == 128) return dt == 1 ? fwd_l<128, __bf16>(qkv, mask, out, lse, B, T, H, scale, causal, s)
                               : fwd_l<128, _Float16>(qkv, mask, out, lse, B, T, H, scale, causal, s);
  return -1;
}

// dout [B,T,H*D]; dq_dot: fp32 workspace [B,H,T]; dqkv [B,T,3*H*D] (fully written).
DL4J_API int dl4j_attn_bwd_dt(int dt, const void* qkv, const void* out, const void* dout, const float* mask,
                              const float* lse, float* dq_dot, void* dqkv, int B, int T, int H, int D, float scale,
                              int causal, hipStream_t s) {
  if (B < 1 || T < 1 || H < 1 || (dt != 1 && dt != 2)) return -1;
  if (D == 64) return dt == 1 ? bwd_l<64, __bf16>(qkv, out, dout, mask, lse, dq_dot, dqkv, B, T, H, scale, causal, s)
                              : bwd_l<64, _Float16>(qkv, out, dout, mask, lse, dq_dot, dqkv, B, T, H, scale, causal, s);
  if (D == 128) return dt == 1 ? bwd_l<128, __bf16>(qkv, out, dout, mask, lse, dq_dot, dqkv, B, T, H, scale, causal, s)
                               : bwd_l<128, _Float16>(qkv, out, dout, mask, lse, dq_dot, dqkv, B, T, H, scale, causal,
                                                      s);
  return -1;
}

DL4J_API int dl4j_attn_fwd(const void* qkv, const float* mask, void* out, float* lse, int B, int T, int H, int D,
                           float scale, int causal, hipStream_t s) {
  return dl4j_attn_fwd_dt(1, qkv, mask, out, lse, B, T, H, D, scale, causal, s);
}

DL4J_API int dl4j_attn_bwd(const void* qkv, const void* out, const void* dout, const float* mask, const float* lse,
                           float* dq_dot, void* dqkv, int B, int T, int H, int D, float scale, int causal,
                           hipStream_t s) {
  return dl4j_attn_bwd_dt(1, qkv, out, dout, mask, lse, dq_dot, dqkv, B, T, H, D, scale, causal, s);
}
