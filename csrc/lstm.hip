// Fused LSTM / GravesLSTM recurrence for gfx950 (the HIP counterpart of the reference's cuDNN LSTMHelper,
// deeplearning4j-cuda/.../recurrent/CudnnLSTMHelper.java; math = nn/layers/recurrent/LSTMHelpers.java
// forward :189-358, backward :392-690).
//
// Work split (MI355X-first): the input projection x·W + b for ALL timesteps and the weight gradients
// (xᵀ·dz, hprevᵀ·dz, Σdz, dz·Wᵀ) are single big library GEMMs outside these kernels. What is left is the
// strictly sequential part, which a per-timestep launch sequence (GEMM + ~8 elementwise kernels per step)
// makes launch-bound. Here ONE launch runs the whole time loop:
//   * one workgroup owns 16 minibatch rows for all T steps (rows are independent in the recurrence, so there is
//     no inter-workgroup communication and nothing to hang on);
//   * each wave owns a slice of 16*NT hidden units for all four gate blocks, so the gate pre-activations of one
//     (row, unit) land in the SAME lane/register of four MFMA accumulators and the gate math, the cell state c
//     and the peephole weights never leave registers;
//   * h_{t-1} (bf16/fp32, the MFMA A operand) lives in a double-buffered LDS tile (rows padded by 16 B: the
//     16 lanes of a ds_read_b128 group hit 16 distinct 4-bank slots); RWᵀ streams from L2 (read-only, shared by
//     every workgroup of the launch) in a FRAGMENT-PACKED layout [n/16][k/KC][lane][FE] built by the caller, so
//     every wave-wide B load is 1 KB contiguous (8 full cache lines). The row-major first version touched 16 rows
//     x 64 B per load and ran at ~30 GB/s per CU (17 us per step at H = 256, time ∝ H²);
//   * per step: z = zx[t] + h_{t-1}·RW on v_mfma_f32_16x16x32_bf16 (fp32: v_mfma_f32_16x16x4_f32), fused
//     gates/peepholes/mask, h_t written to LDS for the next step. One __syncthreads per step.
// Backward mirrors it: per step the gate deltas dz (fp32, kept for the weight GEMMs) are formed in registers,
// staged to LDS, and dh_{t-1} = dz·RWᵀ is one MFMA K-loop over 4H.
// Gate block order in the 4H axis is DL4J's [a | f | o | g] (LSTMHelpers.java:206-316); peepholes (Graves) are
// wFF, wOO, wGG = RW columns 4H, 4H+1, 4H+2.
#include "common.h"

typedef __attribute__((ext_vector_type(4))) float f4_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

template <typename T> struct Mf;
// bf16: one MFMA covers k = 32; lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j = 0..7.
template <> struct Mf<bf16> {
  static constexpr int KC = 32, FE = 8;
  typedef bf16x8_t frag;
  static __device__ __forceinline__ frag load(const bf16* p, int lane) {
    return *reinterpret_cast<const frag*>(p + 8 * (lane >> 4));
  }
  static __device__ __forceinline__ f4_t mma(frag a, frag b, f4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
// fp16: same fragment shapes as bf16 on v_mfma_f32_16x16x32_f16.
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8m_t;
template <> struct Mf<f16> {
  static constexpr int KC = 32, FE = 8;
  typedef f16x8m_t frag;
  static __device__ __forceinline__ frag load(const f16* p, int lane) {
    return *reinterpret_cast<const frag*>(p + 8 * (lane >> 4));
  }
  static __device__ __forceinline__ f4_t mma(frag a, frag b, f4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
// fp32: four 16x16x4 MFMAs cover k = 16; lane group h = l>>4 supplies k = 4h + j for MFMA j (the same permuted
// k order on A and B, so the sum is exact f32 fma chains).
template <> struct Mf<float> {
  static constexpr int KC = 16, FE = 4;
  typedef f4_t frag;
  static __device__ __forceinline__ frag load(const float* p, int lane) {
    return *reinterpret_cast<const frag*>(p + 4 * (lane >> 4));
  }
  static __device__ __forceinline__ f4_t mma(frag a, frag b, f4_t c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
};

template <typename T> __device__ __forceinline__ T cvt(float v);
template <> __device__ __forceinline__ float cvt<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 cvt<bf16>(float v) { return __float2bfloat16(v); }
template <> __device__ __forceinline__ f16 cvt<f16>(float v) { return (f16)v; }

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  // tanh via exp: accurate to a few ulp in fp32, saturates cleanly for |x| large
  const float e = __expf(-2.f * fabsf(x));
  const float r = (1.f - e) / (1.f + e);
  return copysignf(r, x);
}

template <typename T> constexpr int row_pad() { return 16 / (int)sizeof(T); }

// RW fragments (16 B per lane each) are issued together per load batch. 512-thread workgroups (<= 8 waves) leave
// 256 VGPRs per lane for them.
// Register budget (checked with -save-temps: no spills): 16 forward fragments; backward 8 at NT = 1, 4 above.
// At NT = 4 the next step's operands are not prefetched (their registers would be live across the K loop).
#ifndef FWD_FRAGS
#define FWD_FRAGS 16
#endif

// Latency structure (measured: a first version with one 2-deep load chain per k-step and per-row HBM loads in the
// epilogue ran 18 us per timestep): per step a wave now issues its RW fragments in batches of 16 (all in flight
// together, one L2 round trip per batch), and the step's HBM operands (zx / eps / gates / c) are prefetched one
// step ahead into registers so their latency hides behind the previous step's MFMA loop. Loads use a clamped row
// index (no per-row branches); only stores are predicated.

// ------------------------------------------------------------------------------------------------ forward
template <typename T, int NT, bool PEEP>
__global__ void __launch_bounds__(512) lstm_fwd_kernel(
    const T* __restrict__ zx, const T* __restrict__ rwt, const float* __restrict__ peep,
    const float* __restrict__ h0, const float* __restrict__ c0, const float* __restrict__ mask,
    float* __restrict__ out, T* __restrict__ out16, float* __restrict__ gates, float* __restrict__ call,
    float* __restrict__ hT, float* __restrict__ cT, int Tn, int mb, int H) {
  constexpr int KB = FWD_FRAGS / (4 * NT) > 0 ? FWD_FRAGS / (4 * NT) : 1;   // k-steps per load batch
  constexpr bool PF = NT < 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ld = H + row_pad<T>();
  T* hbuf = reinterpret_cast<T*>(smem);                        // [2][16][ld]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int hb = wave * 16 * NT, hw = wave * NT, H16 = H / 16;
  const int col = lane & 15, rg = (lane >> 4) * 4;
  const int H4 = 4 * H;
  const int KS = H / Mf<T>::KC;                                // k-steps per fragment row of the packed RWᵀ

  // h_{-1} into LDS buffer 0 (rows >= mb are zero so they contribute nothing)
  for (int i = threadIdx.x; i < 16 * H; i += blockDim.x) {
    const int r = i / H, j = i - r * H, m = m0 + r;
    hbuf[r * ld + j] = cvt<T>((h0 && m < mb) ? h0[(long long)m * H + j] : 0.f);
  }
  int mrow[4];                                                 // clamped rows: loads never branch
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float c[NT][4], wff[NT], woo[NT], wgg[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int j = hb + nt * 16 + col;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[nt][r] = (c0 && m0 + rg + r < mb) ? c0[(long long)mrow[r] * H + j] : 0.f;
    if (PEEP) {
      wff[nt] = peep[j];
      woo[nt] = peep[H + j];
      wgg[nt] = peep[2 * H + j];
    }
  }
  // zx[t] / mask[t] operands, loaded one step ahead
  float zv[4][NT][4], mv[4];
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long zrow = ((long long)t * mb + mrow[r]) * H4;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int j = hb + nt * 16 + col;
#pragma unroll
        for (int g = 0; g < 4; ++g) zv[g][nt][r] = ld1<T>(zx + zrow + g * H + j);
      }
      mv[r] = mask ? mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  if (PF) load_step(0);
  __syncthreads();

  int cur = 0;
  for (int t = 0; t < Tn; ++t) {
    f4_t acc[4][NT];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[g][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const T* hA = hbuf + cur * 16 * ld + col * ld;
    for (int k0 = 0; k0 < H; k0 += KB * Mf<T>::KC) {
      typename Mf<T>::frag a[KB], b[KB][4][NT];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int k = k0 + kb * Mf<T>::KC;
        if (KB == 1 || k < H) {
          a[kb] = Mf<T>::load(hA + k, lane);
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              b[kb][g][nt] = *reinterpret_cast<const typename Mf<T>::frag*>(
                  rwt + (((long long)(g * H16 + hw + nt) * KS + k / Mf<T>::KC) * 64 + lane) * Mf<T>::FE);
        }
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        if (KB == 1 || k0 + kb * Mf<T>::KC < H) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[g][nt] = Mf<T>::mma(a[kb], b[kb][g][nt], acc[g][nt]);
        }
      }
    }
    if (!PF) load_step(t);
    T* hN = hbuf + (cur ^ 1) * 16 * ld;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int j = hb + nt * 16 + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = rg + r;
        const bool valid = m0 + rr < mb;
        const float za = acc[0][nt][r] + zv[0][nt][r];
        float zf = acc[1][nt][r] + zv[1][nt][r];
        float zo = acc[2][nt][r] + zv[2][nt][r];
        float zg = acc[3][nt][r] + zv[3][nt][r];
        const float cp = c[nt][r];
        if (PEEP) {
          zf += cp * wff[nt];
          zg += cp * wgg[nt];
        }
        const float a = tanh_f(za), f = sigm(zf), g = sigm(zg);
        float cc = f * cp + g * a;
        if (PEEP) zo += cc * woo[nt];
        const float o = sigm(zo);
        float h = o * tanh_f(cc) * mv[r];
        cc *= mv[r];
        c[nt][r] = valid ? cc : 0.f;
        hN[rr * ld + j] = cvt<T>(valid ? h : 0.f);
        if (valid) {
          const long long orow = ((long long)t * mb + m0 + rr) * H;
          out[orow + j] = h;
          if (out16) out16[orow + j] = cvt<T>(h);
          if (call) call[orow + j] = cc;
          if (gates) {
            float* gp = gates + orow * 4 + j;
            gp[0] = a;
            gp[H] = f;
            gp[2 * H] = o;
            gp[3 * H] = g;
          }
        }
      }
    }
    if (PF && t + 1 < Tn) load_step(t + 1);                    // next step's HBM operands in flight now
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int j = hb + nt * 16 + col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + rg + r;
      if (m < mb) {
        if (cT) cT[(long long)m * H + j] = c[nt][r];
        if (hT) hT[(long long)m * H + j] = out[((long long)(Tn - 1) * mb + m) * H + j];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward
template <typename T, int NT, bool PEEP>
__global__ void __launch_bounds__(512) lstm_bwd_kernel(
    const void* __restrict__ eps, int eps_dt, const float* __restrict__ gates, const float* __restrict__ call,
    const float* __restrict__ c0, const T* __restrict__ rw, const float* __restrict__ peep,
    const float* __restrict__ mask, const float* __restrict__ dh_last, const float* __restrict__ dc_last,
    float* __restrict__ dz, float* __restrict__ dh0, float* __restrict__ dc0, int Tn, int mb, int H, int t_end) {
  constexpr int KB = NT == 1 ? 8 : (NT == 2 ? 2 : 1);          // k-steps per load batch
  constexpr bool PF = NT < 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H4 = 4 * H;
  const int ld = H4 + row_pad<T>();
  T* zb = reinterpret_cast<T*>(smem);                          // [16][ld]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int hb = wave * 16 * NT, hw = wave * NT;
  const int col = lane & 15, rg = (lane >> 4) * 4;
  const int KS = H4 / Mf<T>::KC;                               // k-steps per fragment row of the packed RW

  int mrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mrow[r] = min(m0 + rg + r, mb - 1);
  float dhn[NT][4], dcn[NT][4], wff[NT], woo[NT], wgg[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int j = hb + nt * 16 + col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool v = m0 + rg + r < mb;
      dhn[nt][r] = (dh_last && v) ? dh_last[(long long)mrow[r] * H + j] : 0.f;
      dcn[nt][r] = (dc_last && v) ? dc_last[(long long)mrow[r] * H + j] : 0.f;
    }
    if (PEEP) {
      wff[nt] = peep[j];
      woo[nt] = peep[H + j];
      wgg[nt] = peep[2 * H + j];
    }
  }
  // step operands, prefetched one step ahead: eps, a, f, o, g, c_t, c_{t-1}, mask
  float ev[NT][4], av[NT][4], fv[NT][4], ov[NT][4], gv[NT][4], cv[NT][4], pv[NT][4], mv[4];
  auto load_step = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long hrow = ((long long)t * mb + mrow[r]) * H, grow = hrow * 4;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int j = hb + nt * 16 + col;
        ev[nt][r] = ld_any(eps, eps_dt, hrow + j);
        av[nt][r] = gates[grow + j];
        fv[nt][r] = gates[grow + H + j];
        ov[nt][r] = gates[grow + 2 * H + j];
        gv[nt][r] = gates[grow + 3 * H + j];
        cv[nt][r] = call[hrow + j];
        pv[nt][r] = t > 0 ? call[hrow - (long long)mb * H + j] : (c0 ? c0[(long long)mrow[r] * H + j] : 0.f);
      }
      mv[r] = mask ? mask[(long long)mrow[r] * Tn + t] : 1.f;
    }
  };
  if (PF) load_step(Tn - 1);

  for (int t = Tn - 1; t >= t_end; --t) {
    if (!PF) load_step(t);
    float za_[NT][4], zf_[NT][4], zo_[NT][4], zg_[NT][4];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = m0 + rg + r < mb;
        const float dh = (ev[nt][r] + dhn[nt][r]) * mv[r];
        float dc = dcn[nt][r] * mv[r];
        const float a = av[nt][r], f = fv[nt][r], o = ov[nt][r], g = gv[nt][r];
        const float ca = tanh_f(cv[nt][r]);
        const float dzo = dh * ca * o * (1.f - o);
        dc += dh * o * (1.f - ca * ca);
        if (PEEP) dc += dzo * woo[nt];
        const float dzf = dc * pv[nt][r] * f * (1.f - f);
        const float dzg = dc * a * g * (1.f - g);
        const float dza = dc * g * (1.f - a * a);
        float dcp = dc * f;
        if (PEEP) dcp += dzf * wff[nt] + dzg * wgg[nt];
        dcn[nt][r] = valid ? dcp : 0.f;
        za_[nt][r] = valid ? dza : 0.f;
        zf_[nt][r] = valid ? dzf : 0.f;
        zo_[nt][r] = valid ? dzo : 0.f;
        zg_[nt][r] = valid ? dzg : 0.f;
      }
    }
    if (PF && t - 1 >= t_end) load_step(t - 1);                // next step's HBM operands in flight now
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int j = hb + nt * 16 + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = rg + r;
        zb[rr * ld + j] = cvt<T>(za_[nt][r]);
        zb[rr * ld + H + j] = cvt<T>(zf_[nt][r]);
        zb[rr * ld + 2 * H + j] = cvt<T>(zo_[nt][r]);
        zb[rr * ld + 3 * H + j] = cvt<T>(zg_[nt][r]);
        if (m0 + rr < mb) {
          float* dp = dz + ((long long)t * mb + m0 + rr) * H4 + j;
          dp[0] = za_[nt][r];
          dp[H] = zf_[nt][r];
          dp[2 * H] = zo_[nt][r];
          dp[3 * H] = zg_[nt][r];
        }
      }
    }
    __syncthreads();
    f4_t acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const T* zA = zb + col * ld;
    for (int k0 = 0; k0 < H4; k0 += KB * Mf<T>::KC) {
      typename Mf<T>::frag a[KB], b[KB][NT];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int k = k0 + kb * Mf<T>::KC;
        if (k < H4) {
          a[kb] = Mf<T>::load(zA + k, lane);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            b[kb][nt] = *reinterpret_cast<const typename Mf<T>::frag*>(
                rw + (((long long)(hw + nt) * KS + k / Mf<T>::KC) * 64 + lane) * Mf<T>::FE);
        }
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
        if (k0 + kb * Mf<T>::KC < H4) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[nt] = Mf<T>::mma(a[kb], b[kb][nt], acc[nt]);
        }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dhn[nt][r] = acc[nt][r];
    __syncthreads();
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int j = hb + nt * 16 + col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + rg + r;
      if (m < mb) {
        if (dh0) dh0[(long long)m * H + j] = dhn[nt][r];
        if (dc0) dc0[(long long)m * H + j] = dcn[nt][r];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ launch
// NT = 16-unit tiles per wave, <= 8 waves per workgroup (H <= 512)
static int pick_nt(int H) {
  if (H % 16 != 0) return 0;
  if (H / 16 <= 8) return 1;
  if (H % 32 == 0 && H / 32 <= 8) return 2;
  if (H % 64 == 0 && H / 64 <= 8) return 4;
  return 0;
}

static constexpr size_t kMaxLds = 160 * 1024;

template <typename K>
static bool set_lds(K kern, size_t bytes) {
  if (bytes > kMaxLds) return false;
  if (bytes > 64 * 1024)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes) == hipSuccess;
  return true;
}

template <typename T, int NT, bool PEEP>
static int fwd_launch(const void* zx, const void* rwt, const float* peep, const float* h0, const float* c0,
                      const float* mask, float* out, void* out16, float* gates, float* call, float* hT, float* cT,
                      int Tn, int mb, int H, hipStream_t s) {
  const size_t lds = 2ull * 16 * (H + row_pad<T>()) * sizeof(T);
  auto k = lstm_fwd_kernel<T, NT, PEEP>;
  if (!set_lds(k, lds)) return -1;
  const int threads = 64 * (H / (16 * NT));
  hipLaunchKernelGGL(k, dim3((mb + 15) / 16), dim3(threads), lds, s, (const T*)zx, (const T*)rwt, peep, h0, c0, mask,
                     out, (T*)out16, gates, call, hT, cT, Tn, mb, H);
  return (int)hipGetLastError();
}

template <typename T, int NT, bool PEEP>
static int bwd_launch(const void* eps, int eps_dt, const float* gates, const float* call, const float* c0, const void* rw,
                      const float* peep, const float* mask, const float* dhl, const float* dcl, float* dz, float* dh0,
                      float* dc0, int Tn, int mb, int H, int t_end, hipStream_t s) {
  const size_t lds = 16ull * (4 * H + row_pad<T>()) * sizeof(T);
  auto k = lstm_bwd_kernel<T, NT, PEEP>;
  if (!set_lds(k, lds)) return -1;
  const int threads = 64 * (H / (16 * NT));
  hipLaunchKernelGGL(k, dim3((mb + 15) / 16), dim3(threads), lds, s, eps, eps_dt, gates, call, c0, (const T*)rw, peep,
                     mask,
                     dhl, dcl, dz, dh0, dc0, Tn, mb, H, t_end);
  return (int)hipGetLastError();
}

#define LSTM_DISPATCH(FN, ...)                                                              \
  do {                                                                                      \
    const int nt = pick_nt(H);                                                              \
    if (nt == 0) return -1;                                                                 \
    const bool pp = peep != nullptr;                                                        \
    if (dtype == 1) {                                                                       \
      if (nt == 1) return pp ? FN<bf16, 1, true>(__VA_ARGS__) : FN<bf16, 1, false>(__VA_ARGS__);  \
      if (nt == 2) return pp ? FN<bf16, 2, true>(__VA_ARGS__) : FN<bf16, 2, false>(__VA_ARGS__);  \
      return pp ? FN<bf16, 4, true>(__VA_ARGS__) : FN<bf16, 4, false>(__VA_ARGS__);          \
    }                                                                                       \
    if (dtype == 2) {                                                                       \
      if (nt == 1) return pp ? FN<f16, 1, true>(__VA_ARGS__) : FN<f16, 1, false>(__VA_ARGS__);  \
      if (nt == 2) return pp ? FN<f16, 2, true>(__VA_ARGS__) : FN<f16, 2, false>(__VA_ARGS__);  \
      return pp ? FN<f16, 4, true>(__VA_ARGS__) : FN<f16, 4, false>(__VA_ARGS__);           \
    }                                                                                       \
    if (dtype == 0) {                                                                       \
      if (nt == 1) return pp ? FN<float, 1, true>(__VA_ARGS__) : FN<float, 1, false>(__VA_ARGS__); \
      if (nt == 2) return pp ? FN<float, 2, true>(__VA_ARGS__) : FN<float, 2, false>(__VA_ARGS__); \
      return pp ? FN<float, 4, true>(__VA_ARGS__) : FN<float, 4, false>(__VA_ARGS__);        \
    }                                                                                       \
    return -1;                                                                              \
  } while (0)

// Returns 0 on success, -1 when the shape/dtype is outside the kernel (caller uses the per-step path).
DL4J_API int dl4j_lstm_fwd(int dtype, const void* zx, const void* rwt, const float* peep, const float* h0,
                           const float* c0, const float* mask, float* out, void* out16, float* gates, float* call,
                           float* hT, float* cT, int Tn, int mb, int H, hipStream_t s) {
  if (Tn < 1 || mb < 1 || (dtype != 0 && H % 32 != 0)) return -1;
  LSTM_DISPATCH(fwd_launch, zx, rwt, peep, h0, c0, mask, out, out16, gates, call, hT, cT, Tn, mb, H, s);
}

// eps_dt: dtype of eps (0 fp32, 1 bf16, 2 fp16), read directly so the caller needs no conversion pass.
DL4J_API int dl4j_lstm_bwd(int dtype, const void* eps, int eps_dt, const float* gates, const float* call, const float* c0,
                           const void* rw, const float* peep, const float* mask, const float* dh_last,
                           const float* dc_last, float* dz, float* dh0, float* dc0, int Tn, int mb, int H, int t_end,
                           hipStream_t s) {
  if (Tn < 1 || mb < 1 || t_end < 0 || t_end >= Tn) return -1;
  LSTM_DISPATCH(bwd_launch, eps, eps_dt, gates, call, c0, rw, peep, mask, dh_last, dc_last, dz, dh0, dc0, Tn, mb, H, t_end, s);
}
