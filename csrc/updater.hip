// Fused multi-tensor updater: ONE launch updates every parameter segment of a network's flat vector.
//
// Per element (reference order: BaseMultiLayerUpdater.java:223-309, UpdaterBlock.java:142-193):
//   u = updater(g, state)            Sgd/Nesterovs/Adam/AdaMax/Nadam/AdaGrad/AdaDelta/RmsProp/NoOp
//   u += l2*p + l1*sign(p)            (post-apply regularisation)
//   u *= 1/minibatch                  (BaseMultiLayerUpdater divi(batchSize))
//   p -= u                            (NegativeGradientStepFunction)
//   shadow = bf16(p)                  (reduced-precision compute copy, optional)
//   g = u                             (DL4J leaves the update in the gradient view, optional)
// Memory-bound: each param is touched once (~22-26 B/param). grid.y = segment, grid.x strides the segment.
#include "common.h"

struct SegDesc {
  long long p_off, n, st_off, in_block, block_n;
  int op, pad;
  float h0, h1, h2, h3, l1, l2;
  // gradient normalization (BaseMultiLayerUpdater.preApply, :322-382), applied to g before the updater:
  //   0 none, 1 RenormalizeL2PerLayer, 2 RenormalizeL2PerParamType, 3 ClipElementWiseAbsoluteValue,
  //   4 ClipL2PerLayer, 5 ClipL2PerParamType. [gn_b0, gn_b1): the update blocks (btab rows) of this segment's norm
  //   group (the layer, or the segment itself); their sum-of-squares partials come from gn_sumsq_kernel.
  int gn_mode, gn_b0, gn_b1;
  float gn_thr;
};

__device__ __forceinline__ bool gn_needs_norm(int m) { return m == 1 || m == 2 || m == 4 || m == 5; }

// pre-pass: partial[b] = sum of g^2 over update block b (0 for blocks whose segment needs no norm); same grid as
// the update kernel, so every partial is one workgroup's chunk (fixed-order, atomic-free)
__global__ __launch_bounds__(256) void gn_sumsq_kernel(const SegDesc* __restrict__ segs, const int2* __restrict__ btab,
                                                       const float* __restrict__ g, float* __restrict__ partial) {
  const int2 bt = btab[blockIdx.x];
  const SegDesc s = segs[bt.x];
  float acc = 0.f;
  if (gn_needs_norm(s.gn_mode)) {
    const long long ibeg = (long long)bt.y * 2048;
    long long iend = ibeg + 2048;
    if (iend > s.n) iend = s.n;
    for (long long i = ibeg + threadIdx.x; i < iend; i += 256) {
      const float v = g[s.p_off + i];
      acc = fmaf(v, v, acc);
    }
  }
  __shared__ float red[4];
  acc = block_reduce<false>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

enum { OP_NOOP = 0, OP_SGD = 1, OP_NESTEROVS = 2, OP_ADAM = 3, OP_ADAMAX = 4, OP_NADAM = 5, OP_ADAGRAD = 6,
       OP_ADADELTA = 7, OP_RMSPROP = 8 };

#define UPD_CHUNK 2048   // elements per workgroup (8 per thread)

// btab[b] = (segment index, chunk index): a flat 1-D grid with exactly the blocks the segments need, so a
// 64-element BN segment and a 2.4M-element conv weight cost one and 1150 workgroups respectively.
template <typename TS>
__global__ __launch_bounds__(256) void fused_update_kernel(const SegDesc* __restrict__ segs,
                                                           const int2* __restrict__ btab, float* __restrict__ p,
                                                           float* __restrict__ g, float* __restrict__ st,
                                                           TS* __restrict__ shadow, float inv_div, int write_update,
                                                           float* __restrict__ reg_out,
                                                           const float* __restrict__ gn_partial,
                                                           const unsigned* __restrict__ guard, int reg_partials) {
  // a cooperative LSTM launch of this step timed out (csrc/lstm_coop.hip step guard): its outputs are invalid, so
  // parameters, updater state and shadow stay as they were; the host reports the failure
  if (guard && __hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  const int2 bt = btab[blockIdx.x];
  const SegDesc s = segs[bt.x];
  float reg = 0.f;   // l1*|p| + 0.5*l2*p^2 of the PRE-update params (the score's regularisation term)
  // gradient normalization factor of this segment's group (block-uniform branch)
  float gscale = 1.f;
  if (gn_needs_norm(s.gn_mode)) {
    __shared__ float gred[4];
    float ss = 0.f;
    for (int b = s.gn_b0 + threadIdx.x; b < s.gn_b1; b += 256) ss += gn_partial[b];
    ss = block_reduce<false>(ss, gred);
    const float nrm = sqrtf(ss);
    gscale = (s.gn_mode == 1 || s.gn_mode == 2) ? 1.f / nrm : fminf(1.f, s.gn_thr / nrm);
  }
  float* s1 = st + s.st_off + s.in_block;
  float* s2 = st + s.st_off + s.block_n + s.in_block;
  const long long ibeg = (long long)bt.y * UPD_CHUNK;
  long long iend = ibeg + UPD_CHUNK;
  if (iend > s.n) iend = s.n;
  // two phases per thread: issue all 8 elements' loads (gradient, parameter, and the state the updater reads),
  // then update and store — 8 independent loads in flight per array instead of one dependent load->store chain
  // per element (the kernel is HBM-bound; the serial form ran at ~60 % of the bandwidth)
  constexpr int PER = UPD_CHUNK / 256;
  const bool need1 = s.op >= OP_NESTEROVS;
  const bool need2 = s.op == OP_ADAM || s.op == OP_ADAMAX || s.op == OP_NADAM || s.op == OP_ADADELTA;
  float gv[PER], pvv[PER], a1[PER], a2[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long long i = ibeg + threadIdx.x + k * 256;
    const bool in = i < iend;
    const long long pi = s.p_off + (in ? i : 0);
    gv[k] = in ? g[pi] : 0.f;
    pvv[k] = in ? p[pi] : 0.f;
    a1[k] = (need1 && in) ? s1[i] : 0.f;
    a2[k] = (need2 && in) ? s2[i] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long long i = ibeg + threadIdx.x + k * 256;
    if (i >= iend) break;
    const long long pi = s.p_off + i;
    float gi = gv[k];
    if (s.gn_mode == 3) gi = fminf(fmaxf(gi, -s.gn_thr), s.gn_thr);
    else gi *= gscale;
    float pv = pvv[k];
    float u;
    switch (s.op) {
      case OP_SGD: u = s.h0 * gi; break;
      case OP_NESTEROVS: {  // v = mu*v - lr*g ; u = mu*v_prev - (1+mu)*v
        const float vp = a1[k];
        const float v = s.h1 * vp - s.h0 * gi;
        s1[i] = v;
        u = s.h1 * vp - (1.f + s.h1) * v;
      } break;
      case OP_ADAM: {       // h0 = alpha_t, h1 = b1, h2 = b2, h3 = eps
        const float m = s.h1 * a1[k] + (1.f - s.h1) * gi;
        const float v = s.h2 * a2[k] + (1.f - s.h2) * gi * gi;
        s1[i] = m; s2[i] = v;
        u = s.h0 * m / (sqrtf(v) + s.h3);
      } break;
      case OP_ADAMAX: {     // h0 = lr/(1-b1^t)
        const float m = s.h1 * a1[k] + (1.f - s.h1) * gi;
        const float uu = fmaxf(s.h2 * a2[k], fabsf(gi));
        s1[i] = m; s2[i] = uu;
        u = s.h0 * m / (uu + s.h3);
      } break;
      case OP_NADAM: {      // h0 = lr/(1-b1^t)
        const float omg = (1.f - s.h1) * gi;
        const float m = s.h1 * a1[k] + omg;
        const float v = s.h2 * a2[k] + (1.f - s.h2) * gi * gi;
        s1[i] = m; s2[i] = v;
        u = (m * s.h1 + omg) * s.h0 / (sqrtf(v) + s.h3);
      } break;
      case OP_ADAGRAD: {    // h0 = lr, h1 = eps
        const float h = a1[k] + gi * gi;
        s1[i] = h;
        u = s.h0 * gi / sqrtf(h + s.h1);
      } break;
      case OP_ADADELTA: {   // h0 = rho, h1 = eps
        const float msg = s.h0 * a1[k] + (1.f - s.h0) * gi * gi;
        const float dx = sqrtf(a2[k] + s.h1) / sqrtf(msg + s.h1) * gi;
        s1[i] = msg;
        s2[i] = s.h0 * a2[k] + (1.f - s.h0) * dx * dx;
        u = dx;
      } break;
      case OP_RMSPROP: {    // h0 = lr, h1 = decay, h2 = eps
        const float c = s.h1 * a1[k] + (1.f - s.h1) * gi * gi;
        s1[i] = c;
        u = s.h0 * gi / sqrtf(c + s.h2);
      } break;
      default: u = gi;    // OP_NOOP: ND4J NoOpUpdater leaves the gradient unchanged
    }
    if (s.l2 > 0.f) u += s.l2 * pv;
    if (s.l1 > 0.f) u += s.l1 * ((pv > 0.f) - (pv < 0.f));
    reg += s.l1 * fabsf(pv) + 0.5f * s.l2 * pv * pv;
    u *= inv_div;
    pv -= u;
    p[pi] = pv;
    if (shadow) st1<TS>(shadow + pi, pv);
    if (write_update) g[pi] = u;
  }
  if (reg_out != nullptr && (s.l1 > 0.f || s.l2 > 0.f)) {
    __shared__ float red[4];
    reg = block_reduce<false>(reg, red);
    if (threadIdx.x == 0) {
      if (reg_partials) reg_out[blockIdx.x] = reg;        // fixed-order sum later (dl4j_score_reduce): deterministic
      else atomicAdd(reg_out, reg);
    }
  } else if (reg_out != nullptr && reg_partials && threadIdx.x == 0) {
    reg_out[blockIdx.x] = 0.f;
  }
}

// segs: device array of SegDesc. shadow_kind: 0 none, 1 bf16, 2 fp16 (reduced-precision compute copy)
// btab: device int2[nblocks] built by the host from the segment sizes (see dl4j_update_chunk).
// gn_partial: nblocks floats of scratch when any segment uses a norm-based gradient normalization (the pre-pass
// writes it), else null.
unsigned* lstm_step_guard_ptr();      // csrc/lstm_coop.hip

static int fused_update_launch(const void* segs, const void* btab, int nblocks, float* p, float* g, float* st,
                               void* shadow, int shadow_kind, float inv_div, int write_update, float* reg_out,
                               float* gn_partial, hipStream_t stream, int reg_partials);

DL4J_API int dl4j_fused_update(const void* segs, const void* btab, int nblocks, float* p, float* g, float* st,
                               void* shadow, int shadow_kind, float inv_div, int write_update, float* reg_out,
                               float* gn_partial, hipStream_t stream) {
  return fused_update_launch(segs, btab, nblocks, p, g, st, shadow, shadow_kind, inv_div, write_update, reg_out,
                             gn_partial, stream, 0);
}

// Same, with the regularisation term written as one partial per block (reg_part: nblocks floats, every block writes
// its slot) instead of a float atomicAdd into one word: the score is then reduced in a fixed order (dl4j_score_reduce)
// and is bitwise reproducible run to run.
DL4J_API int dl4j_fused_update_regpart(const void* segs, const void* btab, int nblocks, float* p, float* g, float* st,
                                       void* shadow, int shadow_kind, float inv_div, int write_update, float* reg_part,
                                       float* gn_partial, hipStream_t stream) {
  return fused_update_launch(segs, btab, nblocks, p, g, st, shadow, shadow_kind, inv_div, write_update, reg_part,
                             gn_partial, stream, 1);
}

static int fused_update_launch(const void* segs, const void* btab, int nblocks, float* p, float* g, float* st,
                               void* shadow, int shadow_kind, float inv_div, int write_update, float* reg_out,
                               float* gn_partial, hipStream_t stream, int reg_partials) {
  if (nblocks <= 0) return 0;
  const unsigned* guard = lstm_step_guard_ptr();
  if (gn_partial)
    hipLaunchKernelGGL(gn_sumsq_kernel, dim3(nblocks), dim3(256), 0, stream, (const SegDesc*)segs, (const int2*)btab,
                       (const float*)g, gn_partial);
  if (shadow_kind == 1)
    hipLaunchKernelGGL(fused_update_kernel<bf16>, dim3(nblocks), dim3(256), 0, stream, (const SegDesc*)segs,
                       (const int2*)btab, p, g, st, (bf16*)shadow, inv_div, write_update, reg_out,
                       (const float*)gn_partial, guard, reg_partials);
  else if (shadow_kind == 2)
    hipLaunchKernelGGL(fused_update_kernel<f16>, dim3(nblocks), dim3(256), 0, stream, (const SegDesc*)segs,
                       (const int2*)btab, p, g, st, (f16*)shadow, inv_div, write_update, reg_out,
                       (const float*)gn_partial, guard, reg_partials);
  else
    hipLaunchKernelGGL(fused_update_kernel<float>, dim3(nblocks), dim3(256), 0, stream, (const SegDesc*)segs,
                       (const int2*)btab, p, g, st, (float*)nullptr, inv_div, write_update, reg_out,
                       (const float*)gn_partial, guard, reg_partials);
  return (int)hipGetLastError();
}

DL4J_API int dl4j_update_chunk() { return UPD_CHUNK; }

DL4J_API int dl4j_segdesc_size() { return (int)sizeof(SegDesc); }
