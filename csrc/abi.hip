// Descriptor-level entry points of the public C ABI (csrc/include/dl4j_amd.h): the pieces a foreign-language binding
// (the JavaCPP preset of SURVEY §7.1 J1) needs without knowing the engine's internal launch structs.
//
//   * dl4j_matmul        — C = alpha * A @ B + beta * C on tensor descriptors (2-D, or 3-D batched with a common
//                          batch stride); picks the LDS-DMA MFMA kernels for 16-bit operands whose layout they can
//                          address (csrc/gemm.hip dl4j_gemm, split-K slabs from the stream-ordered allocator) and the
//                          exact-fp32 MFMA kernel otherwise (dl4j_gemm_simple). Reference call sites:
//                          NN:nn/layers/BaseLayer.java:86,97,334 (Nd4j.gemm / mmul).
//   * dl4j_update_flat   — one updater over one flat [n] parameter / gradient / state triple through the fused
//                          multi-tensor updater (csrc/updater.hip), i.e. the reference's UpdaterBlock.applyUpdater +
//                          l1/l2 + divi(batch) + params.subi(update) (NN:nn/updater/UpdaterBlock.java:142-193,
//                          BaseMultiLayerUpdater.java:223-309).
//   * dl4j_comm_*        — RCCL communicators and collectives over xGMI (ncclCommInitAll for one process driving every
//                          GPU of the node, ncclCommInitRank for one process per GPU), the native counterpart of
//                          Nd4j.averageAndPropagate (PW:ParallelWrapper.java:316-376).
#include "common.h"

#include <rccl/rccl.h>
#include <string.h>

#include "include/dl4j_amd.h"

DL4J_API int dl4j_abi_version() { return DL4J_AMD_ABI_VERSION; }

// ---------------------------------------------------------------------------------------------------- matmul
namespace {

// A [M, K] view: 1 = K-contiguous (row-major), 0 = M-contiguous (column-major), -1 = neither
int kc_layout(const dl4j_tensor_t* t, int rdim, int cdim, long long* ld) {
  const long long sr = t->strides[rdim], sc = t->strides[cdim];
  if (sc == 1) { *ld = sr; return 1; }
  if (sr == 1) { *ld = sc; return 0; }
  return -1;
}

}  // namespace

DL4J_API int dl4j_matmul(const dl4j_tensor_t* A, const dl4j_tensor_t* B, dl4j_tensor_t* C, float alpha, float beta,
                         hipStream_t s) {
  if (!A || !B || !C) return DL4J_ERR_ARG;
  const int nd = A->ndim;
  if (nd < 2 || nd > 3 || B->ndim != nd || C->ndim != nd) return DL4J_ERR_ARG;
  const int r = nd - 2, c = nd - 1;
  const long long M = A->shape[r], K = A->shape[c], N = B->shape[c];
  if (B->shape[r] != K || C->shape[r] != M || C->shape[c] != N) return DL4J_ERR_SHAPE;
  const long long batch = nd == 3 ? A->shape[0] : 1;
  if (nd == 3 && (B->shape[0] != batch || C->shape[0] != batch)) return DL4J_ERR_SHAPE;
  // every kernel behind this entry point reads / writes F32, BF16 or F16 only (an I32 or unknown code would be
  // reinterpreted as fp16 by the fp32 kernel's loader, and any non-F32 C code gets 16-bit stores)
  auto float_code = [](int dt) { return dt == DL4J_F32 || dt == DL4J_BF16 || dt == DL4J_F16; };
  if (A->dtype != B->dtype || !float_code(A->dtype) || !float_code(C->dtype)) return DL4J_ERR_DTYPE;
  if (C->strides[c] != 1) return DL4J_ERR_LAYOUT;                     // row-major destination rows
  const long long sA = nd == 3 ? A->strides[0] : 0, sB = nd == 3 ? B->strides[0] : 0, sC = nd == 3 ? C->strides[0] : 0;
  if (M > 0x7fffffffLL || N > 0x7fffffffLL || K > 0x7fffffffLL || batch > 65535) return DL4J_ERR_SHAPE;
  long long lda = 0, ldb = 0;
  const int akc = kc_layout(A, r, c, &lda);
  // B [K, N]: K-contiguous means column-major B (strides[c] != 1, strides[r] == 1)
  int bkc;
  if (B->strides[r] == 1) { bkc = 1; ldb = B->strides[c]; }
  else if (B->strides[c] == 1) { bkc = 0; ldb = B->strides[r]; }
  else bkc = -1;
  const int in16 = A->dtype == DL4J_BF16 || A->dtype == DL4J_F16;
  if (in16 && akc >= 0 && bkc >= 0) {
    int cfg = -1, splits = 0;
    const long long ws_bytes = dl4j_gemm_plan((int)M, (int)N, (int)K, (int)batch, &cfg, &splits);
    float* ws = nullptr;
    if (ws_bytes > 0 && hipMallocAsync(reinterpret_cast<void**>(&ws), (size_t)ws_bytes, s) != hipSuccess) ws = nullptr;
    int rc = dl4j_gemm(A->dtype, C->dtype, (int)M, (int)N, (int)K, (int)batch, A->data, lda, akc, sA, B->data, ldb, bkc,
                       sB, C->data, C->strides[r], sC, alpha, beta, nullptr, 0, 0, nullptr, ws ? cfg : -1,
                       ws ? splits : 1, ws, nullptr, 0, s);
    if (rc == -2 && !ws) rc = -1;
    if (ws) (void)hipFreeAsync(ws, s);
    if (rc == 0) return 0;
    // any layout the 16-byte DMA kernel cannot address falls through to the exact-fp32 kernel
  }
  int tile = 0, splits = 1;
  const long long wsb = dl4j_gemm_f32_plan((int)M, (int)N, (int)K, (int)batch, &tile, &splits);
  float* ws = nullptr;
  if (wsb > 0 && hipMallocAsync(reinterpret_cast<void**>(&ws), (size_t)wsb, s) != hipSuccess) {
    ws = nullptr;
    splits = 1;
  }
  const int rc = dl4j_gemm_f32(A->dtype, C->dtype, (int)M, (int)N, (int)K, (int)batch, A->data, A->strides[r],
                               A->strides[c], sA, B->data, B->strides[r], B->strides[c], sB, C->data, C->strides[r], sC,
                               alpha, beta, nullptr, 0, 0, nullptr, tile, splits, ws, s);
  if (ws) (void)hipFreeAsync(ws, s);
  return rc == 0 ? 0 : DL4J_ERR_LAUNCH;
}

// ---------------------------------------------------------------------------------------------------- updater
namespace {
// must match csrc/updater.hip SegDesc (checked against dl4j_segdesc_size() at run time)
struct SegDescAbi {
  long long p_off, n, st_off, in_block, block_n;
  int op, pad;
  float h0, h1, h2, h3, l1, l2;
  int gn_mode, gn_b0, gn_b1;
  float gn_thr;
};
}  // namespace

DL4J_API int dl4j_update_flat(int op, float* params, float* grad, float* state, long long n, const float* hp,
                              float l1, float l2, float inv_batch, int write_update, hipStream_t s) {
  if (n <= 0) return 0;
  if (op < DL4J_UPD_NOOP || op > DL4J_UPD_RMSPROP || !params || !grad) return DL4J_ERR_ARG;
  if ((int)sizeof(SegDescAbi) != dl4j_segdesc_size()) return DL4J_ERR_ABI;
  const int chunk = dl4j_update_chunk();
  const long long nb = (n + chunk - 1) / chunk;
  if (nb > 0x7fffffffLL) return DL4J_ERR_SHAPE;
  SegDescAbi d;
  memset(&d, 0, sizeof d);
  d.p_off = 0; d.n = n; d.st_off = 0; d.in_block = 0; d.block_n = n;
  d.op = op;
  d.h0 = hp ? hp[0] : 0.f; d.h1 = hp ? hp[1] : 0.f; d.h2 = hp ? hp[2] : 0.f; d.h3 = hp ? hp[3] : 0.f;
  d.l1 = l1; d.l2 = l2;
  const size_t tab_bytes = (size_t)nb * 2 * sizeof(int);
  int* htab = static_cast<int*>(malloc(tab_bytes));
  if (!htab) return DL4J_ERR_ARG;
  for (long long b = 0; b < nb; ++b) { htab[2 * b] = 0; htab[2 * b + 1] = (int)b; }
  void* dd = nullptr;
  void* dtab = nullptr;
  int rc = DL4J_ERR_LAUNCH;
  if (hipMallocAsync(&dd, sizeof d, s) == hipSuccess && hipMallocAsync(&dtab, tab_bytes, s) == hipSuccess &&
      hipMemcpyAsync(dd, &d, sizeof d, hipMemcpyHostToDevice, s) == hipSuccess &&
      hipMemcpyAsync(dtab, htab, tab_bytes, hipMemcpyHostToDevice, s) == hipSuccess) {
    // the host copies above are staged from pageable memory: keep the host arrays alive until they are consumed
    if (hipStreamSynchronize(s) == hipSuccess)
      rc = dl4j_fused_update(dd, dtab, (int)nb, params, grad, state, nullptr, 0, inv_batch, write_update, nullptr,
                             nullptr, s) == 0 ? 0 : DL4J_ERR_LAUNCH;
  }
  if (dd) (void)hipFreeAsync(dd, s);
  if (dtab) (void)hipFreeAsync(dtab, s);
  free(htab);
  return rc;
}

// ---------------------------------------------------------------------------------------------------- RCCL
namespace {
int nccl_dt(int dt) {
  switch (dt) {
    case DL4J_F32: return ncclFloat32;
    case DL4J_BF16: return ncclBfloat16;
    case DL4J_F16: return ncclFloat16;
    case DL4J_I32: return ncclInt32;
    default: return -1;
  }
}
int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? 0 : DL4J_ERR_COMM; }
}  // namespace

DL4J_API int dl4j_comm_unique_id(void* id_out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r == ncclSuccess) memcpy(id_out, &id, sizeof id);
  return nccl_rc(r);
}

DL4J_API int dl4j_comm_id_bytes() { return (int)sizeof(ncclUniqueId); }

DL4J_API int dl4j_comm_init_rank(dl4j_comm_t* comm, int nranks, const void* id, int rank) {
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t c = nullptr;
  const int rc = nccl_rc(ncclCommInitRank(&c, nranks, u, rank));
  *comm = reinterpret_cast<dl4j_comm_t>(c);
  return rc;
}

DL4J_API int dl4j_comm_init_all(dl4j_comm_t* comms, int ndev, const int* devices) {
  return nccl_rc(ncclCommInitAll(reinterpret_cast<ncclComm_t*>(comms), ndev, devices));
}

DL4J_API int dl4j_comm_all_reduce(dl4j_comm_t comm, const void* send, void* recv, long long count, int dtype, int op,
                                  hipStream_t s) {
  const int dt = nccl_dt(dtype);
  if (dt < 0 || (op != DL4J_SUM && op != DL4J_AVG && op != DL4J_MAX)) return DL4J_ERR_ARG;
  const ncclRedOp_t o = op == DL4J_SUM ? ncclSum : (op == DL4J_AVG ? ncclAvg : ncclMax);
  return nccl_rc(ncclAllReduce(send, recv, (size_t)count, (ncclDataType_t)dt, o, reinterpret_cast<ncclComm_t>(comm), s));
}

DL4J_API int dl4j_comm_broadcast(dl4j_comm_t comm, const void* send, void* recv, long long count, int dtype, int root,
                                 hipStream_t s) {
  const int dt = nccl_dt(dtype);
  if (dt < 0) return DL4J_ERR_ARG;
  return nccl_rc(ncclBroadcast(send, recv, (size_t)count, (ncclDataType_t)dt, root, reinterpret_cast<ncclComm_t>(comm),
                               s));
}

DL4J_API int dl4j_comm_all_gather(dl4j_comm_t comm, const void* send, void* recv, long long count_per_rank, int dtype,
                                  hipStream_t s) {
  const int dt = nccl_dt(dtype);
  if (dt < 0) return DL4J_ERR_ARG;
  return nccl_rc(ncclAllGather(send, recv, (size_t)count_per_rank, (ncclDataType_t)dt,
                               reinterpret_cast<ncclComm_t>(comm), s));
}

DL4J_API int dl4j_comm_reduce_scatter(dl4j_comm_t comm, const void* send, void* recv, long long count_per_rank,
                                      int dtype, int op, hipStream_t s) {
  const int dt = nccl_dt(dtype);
  if (dt < 0 || (op != DL4J_SUM && op != DL4J_AVG && op != DL4J_MAX)) return DL4J_ERR_ARG;
  const ncclRedOp_t o = op == DL4J_SUM ? ncclSum : (op == DL4J_AVG ? ncclAvg : ncclMax);
  return nccl_rc(ncclReduceScatter(send, recv, (size_t)count_per_rank, (ncclDataType_t)dt, o,
                                   reinterpret_cast<ncclComm_t>(comm), s));
}

DL4J_API int dl4j_comm_group_start() { return nccl_rc(ncclGroupStart()); }
DL4J_API int dl4j_comm_group_end() { return nccl_rc(ncclGroupEnd()); }
DL4J_API int dl4j_comm_abort(dl4j_comm_t comm) { return nccl_rc(ncclCommAbort(reinterpret_cast<ncclComm_t>(comm))); }
DL4J_API int dl4j_comm_destroy(dl4j_comm_t comm) {
  return nccl_rc(ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)));
}
