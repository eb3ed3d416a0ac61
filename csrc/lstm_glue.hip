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
