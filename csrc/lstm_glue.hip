// LSTM backward "prep" pass for gfx950: everything between the sequence backward kernel and the three parameter
// GEMMs in ONE launch (reference LSTMHelpers.java:616-676 computes these with separate ND4J ops):
//   dzb[r, j]   = (T16) dz[r, j]                      operand of dW = xᵀ·dz, dRW = hprevᵀ·dz, dX = dz·Wᵀ
//   hpb[r, j]   = (T16) h_{t-1}[m, j]   (j < H)        rows r = t*mb + m; h_{-1} = h0 (or 0)
//   db[j]      += Σ_r dz[r, j]                        bias gradient (fp32, pre-zeroed by the caller)
//   dpeep[0,j] += Σ_r dz[r, H+j]  * c_{t-1}[m, j]      peephole gradients (GravesLSTM wFF / wOO / wGG columns)
//   dpeep[1,j] += Σ_r dz[r, 2H+j] * c_t[m, j]
//   dpeep[2,j] += Σ_r dz[r, 3H+j] * c_{t-1}[m, j]
// Replaces ~12 elementwise / reduce / concat / convert launches per layer and direction. Threads own a column
// (coalesced rows of dz), a block sweeps ROWS rows, column sums leave through one float atomic per block.
#include "common.h"

static constexpr int ROWS = 8;            // small row chunks: ~800 workgroups for the bench shape (T*mb = 1600)

template <typename T16>
__global__ __launch_bounds__(256) void lstm_bwd_prep_kernel(const float* __restrict__ dz, const float* __restrict__ out,
                                                            const float* __restrict__ h0, const float* __restrict__ call,
                                                            const float* __restrict__ c0, T16* __restrict__ dzb,
                                                            T16* __restrict__ hpb, float* __restrict__ db,
                                                            float* __restrict__ dpeep, int R, int mb, int H,
                                                            int peephole) {
  const int G = 4 * H;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= G) return;
  const int r0 = blockIdx.y * ROWS;
  const int r1 = min(R, r0 + ROWS);
  const int gate = j / H, jj = j - gate * H;
  float sb = 0.f, sp = 0.f;
  for (int r = r0; r < r1; ++r) {
    const float v = dz[(long long)r * G + j];
    st1<T16>(dzb + (long long)r * G + j, v);
    sb += v;
    if (gate == 0) {
      const float hp = r >= mb ? out[(long long)(r - mb) * H + jj] : (h0 ? h0[(long long)r * H + jj] : 0.f);
      st1<T16>(hpb + (long long)r * H + jj, hp);
    } else if (peephole) {
      float c;
      if (gate == 2) c = call[(long long)r * H + jj];
      else c = r >= mb ? call[(long long)(r - mb) * H + jj] : (c0 ? c0[(long long)r * H + jj] : 0.f);
      sp += v * c;
    }
  }
  atomicAdd(db + j, sb);
  if (peephole && gate > 0) atomicAdd(dpeep + (gate - 1) * H + jj, sp);
}

// dt: 1 bf16, 2 fp16 operand copies. h0 / c0 may be null (zero initial state). db [4H] and dpeep [3H] fp32 are
// accumulated into (zero them first).
DL4J_API int dl4j_lstm_bwd_prep(int dt, const float* dz, const float* out, const float* h0, const float* call,
                                const float* c0, void* dzb, void* hpb, float* db, float* dpeep, int R, int mb, int H,
                                int peephole, hipStream_t s) {
  if (R <= 0 || H <= 0) return 0;
  const dim3 grid((4 * H + 255) / 256, (R + ROWS - 1) / ROWS);
  if (dt == 1)
    hipLaunchKernelGGL(lstm_bwd_prep_kernel<bf16>, grid, dim3(256), 0, s, dz, out, h0, call, c0, (bf16*)dzb,
                       (bf16*)hpb, db, dpeep, R, mb, H, peephole);
  else if (dt == 2)
    hipLaunchKernelGGL(lstm_bwd_prep_kernel<f16>, grid, dim3(256), 0, s, dz, out, h0, call, c0, (f16*)dzb, (f16*)hpb,
                       db, dpeep, R, mb, H, peephole);
  else
    return -1;
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------ recurrent weight packing
// One launch per layer per TBPTT window replaces the two permute-copies (forward B = RWᵀ, backward B = RW) and the
// peephole gathers the sequence kernels need (ops/rnn_native.py _pack_b layout): for an [N, K] matrix m the packed
// image is [N/16][K/KC][4][16][FE] with KC = 4*FE (FE = 8 for 16-bit T, 4 for fp32), element
// (n, k) -> ((((n/16)*(K/KC) + k/KC)*4 + (k%KC)/FE)*16 + n%16)*FE + k%FE.
//   forward : m[n][k] = RW[k][n], N = 4H, K = H        backward: m[n][k] = RW[n][k], N = H, K = 4H
// RW is the [H, 4H(+3)] weight view with element strides (s0, s1) (DL4J 'f' order: s0 = 1, s1 = H); peep[i][h] =
// RW[h][4H + i] in fp32. Each thread writes one element of each packed image (reads are strided gathers of a 0.5 MB
// matrix: L2-resident).
template <typename T>
__global__ __launch_bounds__(256) void lstm_pack_rw_kernel(const T* __restrict__ rw, long long s0, long long s1, int H,
                                                           T* __restrict__ fwd, T* __restrict__ bwd,
                                                           float* __restrict__ peep) {
  constexpr int FE = sizeof(T) == 2 ? 8 : 4, KC = 4 * FE;
  const long long total = 4LL * H * H;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (long long)gridDim.x * blockDim.x) {
    // decode the packed position o -> (n, k) for an [N, K] image
    const int e = (int)(o % FE);
    long long q = o / FE;
    const int n16 = (int)(q % 16); q /= 16;
    const int sub = (int)(q % 4); q /= 4;
    if (fwd) {                                            // N = 4H, K = H
      const int KB = H / KC;
      const int kb = (int)(q % KB), nb = (int)(q / KB);
      const int n = nb * 16 + n16, k = kb * KC + sub * FE + e;
      fwd[o] = rw[(long long)k * s0 + (long long)n * s1];
    }
    if (bwd) {                                            // N = H, K = 4H
      const int KB = 4 * H / KC;
      const int kb = (int)(q % KB), nb = (int)(q / KB);
      const int n = nb * 16 + n16, k = kb * KC + sub * FE + e;
      bwd[o] = rw[(long long)n * s0 + (long long)k * s1];
    }
    if (peep && o < 3LL * H) {
      const int i = (int)(o / H), h = (int)(o % H);
      peep[o] = ld1<T>(rw + (long long)h * s0 + (long long)(4 * H + i) * s1);
    }
  }
}

// dt: 0 fp32, 1 bf16, 2 fp16. fwd / bwd / peep may each be null. H % KC == 0 required (KC = 32 / 16).
DL4J_API int dl4j_lstm_pack_rw(int dt, const void* rw, long long s0, long long s1, int H, void* fwd, void* bwd,
                               float* peep, hipStream_t s) {
  if (H <= 0 || H % (dt == 0 ? 16 : 32) != 0) return -1;
  const long long total = 4LL * H * H;
  long long g = (total + 255) / 256;
  if (g > 2048) g = 2048;
  if (dt == 1)
    hipLaunchKernelGGL(lstm_pack_rw_kernel<bf16>, dim3((unsigned)g), dim3(256), 0, s, (const bf16*)rw, s0, s1, H,
                       (bf16*)fwd, (bf16*)bwd, peep);
  else if (dt == 2)
    hipLaunchKernelGGL(lstm_pack_rw_kernel<f16>, dim3((unsigned)g), dim3(256), 0, s, (const f16*)rw, s0, s1, H,
                       (f16*)fwd, (f16*)bwd, peep);
  else if (dt == 0)
    hipLaunchKernelGGL(lstm_pack_rw_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, (const float*)rw, s0, s1, H,
                       (float*)fwd, (float*)bwd, peep);
  else
    return -1;
  return (int)hipGetLastError();
}
