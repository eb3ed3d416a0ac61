/* C-only driver of the public ABI (csrc/include/dl4j_amd.h): runs GEMM, convolution, the flat updater, the
 * workspace arena and an RCCL all-reduce through nothing but the header and the two shared libraries, and checks
 * each against a host reference. Plain C99; the HIP runtime is reached through its C API only (hipMalloc /
 * hipMemcpy / hipStreamSynchronize are declared here, so no HIP header is needed).
 *
 * Build (ops/build.py build_abi_driver): gcc -std=c99 -O2 -I csrc/include tests/native/abi_driver.c
 *   -L deeplearning4j_amd/_lib -ldl4j_amd_kernels -ldl4j_amd_runtime -L/opt/rocm/lib -lamdhip64 -lm
 * Run: ./abi_driver        exit 0 and "ABI OK" when every check passes.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dl4j_amd.h"

/* HIP runtime C API (libamdhip64), declared by hand: enum values are ints, 0 = success */
int hipMalloc(void** p, size_t n);
int hipFree(void* p);
int hipMemcpy(void* dst, const void* src, size_t n, int kind);
int hipDeviceSynchronize(void);
int hipGetDeviceCount(int* n);
#define H2D 1
#define D2H 2

static int failures = 0;
#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                  \
      ++failures;                             \
    }                                         \
  } while (0)

static uint32_t rng = 12345u;
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return ((rng >> 8) & 0xffff) / 32768.0f - 1.0f;
}
static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static void* dev_copy(const void* h, size_t n) {
  void* d = NULL;
  if (hipMalloc(&d, n) != 0 || hipMemcpy(d, h, n, H2D) != 0) {
    fprintf(stderr, "device allocation failed\n");
    exit(2);
  }
  return d;
}
static void set2(dl4j_tensor_t* t, void* data, int dtype, long long r, long long c, long long sr, long long sc) {
  memset(t, 0, sizeof *t);
  t->data = data;
  t->dtype = dtype;
  t->ndim = 2;
  t->shape[0] = r;
  t->shape[1] = c;
  t->strides[0] = sr;
  t->strides[1] = sc;
}

/* C[M,N] = A[M,K] @ B[K,N], bf16 operands (A row-major, B given column-major = K-contiguous), fp32 output */
static void test_matmul_bf16(void) {
  const int M = 256, N = 192, K = 320;
  uint16_t* a = malloc(sizeof(uint16_t) * M * K);
  uint16_t* b = malloc(sizeof(uint16_t) * K * N);  /* column-major: b[n*K + k] */
  float* c = malloc(sizeof(float) * M * N);
  for (int i = 0; i < M * K; ++i) a[i] = f2bf(frand());
  for (int i = 0; i < K * N; ++i) b[i] = f2bf(frand());
  void *da = dev_copy(a, sizeof(uint16_t) * M * K), *db = dev_copy(b, sizeof(uint16_t) * K * N), *dc = NULL;
  hipMalloc(&dc, sizeof(float) * M * N);
  dl4j_tensor_t A, B, C;
  set2(&A, da, DL4J_BF16, M, K, K, 1);
  set2(&B, db, DL4J_BF16, K, N, 1, K);
  set2(&C, dc, DL4J_F32, M, N, N, 1);
  int rc = dl4j_matmul(&A, &B, &C, 1.0f, 0.0f, 0);
  CHECK(rc == 0, "dl4j_matmul bf16 rc=%d", rc);
  hipDeviceSynchronize();
  hipMemcpy(c, dc, sizeof(float) * M * N, D2H);
  double maxerr = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double ref = 0;
      for (int k = 0; k < K; ++k) ref += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]);
      const double e = fabs(ref - c[m * N + n]);
      if (e > maxerr) maxerr = e;
    }
  CHECK(maxerr < 1e-3, "matmul bf16 max abs err %.3g", maxerr);
  printf("matmul bf16 %dx%dx%d: max abs err %.3g\n", M, N, K, maxerr);
  hipFree(da); hipFree(db); hipFree(dc);
  free(a); free(b); free(c);
}

/* exact-fp32 path: fp32 operands, beta accumulation */
static void test_matmul_f32(void) {
  const int M = 70, N = 33, K = 45;
  float *a = malloc(4 * M * K), *b = malloc(4 * K * N), *c = malloc(4 * M * N), *c0 = malloc(4 * M * N);
  for (int i = 0; i < M * K; ++i) a[i] = frand();
  for (int i = 0; i < K * N; ++i) b[i] = frand();
  for (int i = 0; i < M * N; ++i) c0[i] = frand();
  void *da = dev_copy(a, 4 * M * K), *db = dev_copy(b, 4 * K * N), *dc = dev_copy(c0, 4 * M * N);
  dl4j_tensor_t A, B, C;
  set2(&A, da, DL4J_F32, M, K, K, 1);
  set2(&B, db, DL4J_F32, K, N, N, 1);
  set2(&C, dc, DL4J_F32, M, N, N, 1);
  int rc = dl4j_matmul(&A, &B, &C, 0.5f, 2.0f, 0);
  CHECK(rc == 0, "dl4j_matmul f32 rc=%d", rc);
  hipDeviceSynchronize();
  hipMemcpy(c, dc, 4 * M * N, D2H);
  double maxerr = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double ref = 0;
      for (int k = 0; k < K; ++k) ref += (double)a[m * K + k] * b[k * N + n];
      ref = 0.5 * ref + 2.0 * c0[m * N + n];
      const double e = fabs(ref - c[m * N + n]);
      if (e > maxerr) maxerr = e;
    }
  CHECK(maxerr < 1e-4, "matmul f32 max abs err %.3g", maxerr);
  printf("matmul f32 %dx%dx%d (alpha 0.5, beta 2): max abs err %.3g\n", M, N, K, maxerr);
  hipFree(da); hipFree(db); hipFree(dc);
  free(a); free(b); free(c); free(c0);
}

/* dtype validation: int32 operands or an int32 / unknown destination code are refused, nothing is launched */
static void test_matmul_dtype_rejects(void) {
  int32_t dummy[4] = {0, 0, 0, 0};
  dl4j_tensor_t A, B, C;
  set2(&A, dummy, DL4J_I32, 2, 2, 2, 1);
  set2(&B, dummy, DL4J_I32, 2, 2, 2, 1);
  set2(&C, dummy, DL4J_F32, 2, 2, 2, 1);
  int rc = dl4j_matmul(&A, &B, &C, 1.0f, 0.0f, 0);
  CHECK(rc == DL4J_ERR_DTYPE, "dl4j_matmul I32 operands rc=%d", rc);
  set2(&A, dummy, DL4J_F32, 2, 2, 2, 1);
  set2(&B, dummy, DL4J_F32, 2, 2, 2, 1);
  set2(&C, dummy, DL4J_I32, 2, 2, 2, 1);
  rc = dl4j_matmul(&A, &B, &C, 1.0f, 0.0f, 0);
  CHECK(rc == DL4J_ERR_DTYPE, "dl4j_matmul I32 destination rc=%d", rc);
  C.dtype = 77;
  rc = dl4j_matmul(&A, &B, &C, 1.0f, 0.0f, 0);
  CHECK(rc == DL4J_ERR_DTYPE, "dl4j_matmul unknown destination code rc=%d", rc);
  printf("matmul dtype rejects: ok\n");
}

/* 3x3 convolution, NHWC activations, KRSC weights, bf16 in / bf16 out, + bias */
static void test_conv(void) {
  const int N = 2, H = 8, W = 8, C = 64, K = 64, R = 3, S = 3, OH = 8, OW = 8;
  const long long nx = (long long)N * H * W * C, nw = (long long)K * R * S * C, ny = (long long)N * OH * OW * K;
  uint16_t *x = malloc(2 * nx), *w = malloc(2 * nw), *y = malloc(2 * ny);
  float* bias = malloc(4 * K);
  for (long long i = 0; i < nx; ++i) x[i] = f2bf(frand());
  for (long long i = 0; i < nw; ++i) w[i] = f2bf(frand() * 0.1f);
  for (int i = 0; i < K; ++i) bias[i] = frand();
  void *dx = dev_copy(x, 2 * nx), *dw = dev_copy(w, 2 * nw), *dbias = dev_copy(bias, 4 * K), *dy = NULL;
  hipMalloc(&dy, 2 * ny);
  const int variant = dl4j_conv_v3_default_variant((long long)N * OH * OW, K);
  int rc = dl4j_conv_fwd_v3(DL4J_BF16, dx, dw, (const float*)dbias, dy, N, H, W, C, K, R, S, 1, 1, 1, 1, 1, 1, OH, OW,
                            0.0f, NULL, variant, 0);
  CHECK(rc == 0, "dl4j_conv_fwd_v3 rc=%d", rc);
  hipDeviceSynchronize();
  hipMemcpy(y, dy, 2 * ny, D2H);
  double maxrel = 0;
  for (int n = 0; n < N; ++n)
    for (int oh = 0; oh < OH; ++oh)
      for (int ow = 0; ow < OW; ++ow)
        for (int k = 0; k < K; ++k) {
          double ref = bias[k], mag = fabs(bias[k]);
          for (int r = 0; r < R; ++r)
            for (int s = 0; s < S; ++s) {
              const int ih = oh - 1 + r, iw = ow - 1 + s;
              if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
              for (int c = 0; c < C; ++c) {
                const double p = (double)bf2f(x[((long long)(n * H + ih) * W + iw) * C + c]) *
                                 bf2f(w[((long long)(k * R + r) * S + s) * C + c]);
                ref += p;
                mag += fabs(p);
              }
            }
          const double got = bf2f(y[((long long)(n * OH + oh) * OW + ow) * K + k]);
          const double e = fabs(got - ref) / (mag + 1e-3);
          if (e > maxrel) maxrel = e;
        }
  CHECK(maxrel < 8e-3, "conv max rel err %.3g", maxrel);
  printf("conv3x3 NHWC bf16 N%d %dx%d C%d K%d: max err / sum|x*w| %.3g (variant %d)\n", N, H, W, C, K, maxrel, variant);
  hipFree(dx); hipFree(dw); hipFree(dbias); hipFree(dy);
  free(x); free(w); free(y); free(bias);
}

/* Adam step on a flat vector: p -= inv_batch * (lr_t * m / (sqrt(v) + eps) + l2 * p) */
static void test_update_adam(void) {
  const long long n = 5000;
  float *p = malloc(4 * n), *g = malloc(4 * n), *st = calloc(2 * n, 4), *out = malloc(4 * n), *st_out = malloc(8 * n);
  for (long long i = 0; i < n; ++i) { p[i] = frand(); g[i] = frand(); }
  void *dp = dev_copy(p, 4 * n), *dg = dev_copy(g, 4 * n), *ds = dev_copy(st, 8 * n);
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, lr = 1e-2f, l2 = 1e-3f, inv = 0.25f;
  const float alpha_t = lr * sqrtf(1.f - b2) / (1.f - b1);       /* iteration 0 */
  const float hp[4] = {alpha_t, b1, b2, eps};
  int rc = dl4j_update_flat(DL4J_UPD_ADAM, (float*)dp, (float*)dg, (float*)ds, n, hp, 0.0f, l2, inv, 0, 0);
  CHECK(rc == 0, "dl4j_update_flat rc=%d", rc);
  hipDeviceSynchronize();
  hipMemcpy(out, dp, 4 * n, D2H);
  hipMemcpy(st_out, ds, 8 * n, D2H);
  double maxerr = 0, maxst = 0;
  for (long long i = 0; i < n; ++i) {
    const float m = (1.f - b1) * g[i], v = (1.f - b2) * g[i] * g[i];
    const float u = alpha_t * m / (sqrtf(v) + eps) + l2 * p[i];
    const double e = fabs((p[i] - inv * u) - out[i]);
    if (e > maxerr) maxerr = e;
    const double es = fabs(st_out[i] - m) + fabs(st_out[n + i] - v);
    if (es > maxst) maxst = es;
  }
  CHECK(maxerr < 1e-6 && maxst < 1e-7, "adam update err %.3g state err %.3g", maxerr, maxst);
  printf("fused updater (Adam, l2, 1/batch) n=%lld: max abs err %.3g, state err %.3g\n", n, maxerr, maxst);
  hipFree(dp); hipFree(dg); hipFree(ds);
  free(p); free(g); free(st); free(out); free(st_out);
}

/* workspace arena bookkeeping (libdl4j_amd_runtime): aligned bump allocation, spill, cycle reset */
static void test_workspace(void) {
  const long long h = rt_ws_create(1 << 20, 0, 256, 0.0, 0, 0, 0);
  long long off[3], gen;
  int r0 = rt_ws_alloc(h, 1000, &off[0], &gen), r1 = rt_ws_alloc(h, 5000, &off[1], &gen),
      r2 = rt_ws_alloc(h, 2 << 20, &off[2], &gen);
  CHECK(r0 == 0 && r1 == 0 && off[0] == 0 && off[1] == 1024, "arena offsets %lld %lld (rc %d %d)", off[0], off[1], r0,
        r1);
  CHECK(r2 == 1, "oversized request should spill (rc %d)", r2);
  rt_ws_cycle_end(h);
  int r3 = rt_ws_alloc(h, 64, &off[0], &gen);
  CHECK(r3 == 0 && off[0] == 0, "arena not reset after cycle end (off %lld)", off[0]);
  long long stats[16];
  memset(stats, 0, sizeof stats);
  CHECK(rt_ws_stats(h, stats) == 0, "rt_ws_stats");
  rt_ws_destroy(h);
  printf("workspace arena: offsets 0 / 1024, spill, reset ok\n");
}

/* RCCL over the C ABI: a communicator per visible GPU from one thread, all-reduce sum (world 1 on a 1-GPU box:
 * the result equals the input; with more GPUs every rank gets the sum) */
static void test_comm(void) {
  int ndev = 0;
  hipGetDeviceCount(&ndev);
  if (ndev < 1) return;
  const int use = 1;
  dl4j_comm_t comm;
  int dev = 0;
  int rc = dl4j_comm_init_all(&comm, use, &dev);
  CHECK(rc == 0, "dl4j_comm_init_all rc=%d", rc);
  if (rc) return;
  const long long n = 4096;
  float* h = malloc(4 * n);
  for (long long i = 0; i < n; ++i) h[i] = (float)i;
  void* d = dev_copy(h, 4 * n);
  rc = dl4j_comm_all_reduce(comm, d, d, n, DL4J_F32, DL4J_SUM, 0);
  CHECK(rc == 0, "dl4j_comm_all_reduce rc=%d", rc);
  hipDeviceSynchronize();
  float* o = malloc(4 * n);
  hipMemcpy(o, d, 4 * n, D2H);
  int bad = 0;
  for (long long i = 0; i < n; ++i) bad += o[i] != (float)i * use;
  CHECK(bad == 0, "all-reduce: %d wrong elements", bad);
  CHECK(dl4j_comm_destroy(comm) == 0, "dl4j_comm_destroy");
  printf("RCCL all-reduce (world %d) over dl4j_comm_*: ok\n", use);
  hipFree(d);
  free(h); free(o);
}

int main(void) {
  CHECK(dl4j_abi_version() == DL4J_AMD_ABI_VERSION, "ABI version %d != header %d", dl4j_abi_version(),
        DL4J_AMD_ABI_VERSION);
  test_workspace();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != 0 || ndev < 1) {
    printf("no GPU: host-side checks only\n");
  } else {
    test_matmul_bf16();
    test_matmul_f32();
    test_matmul_dtype_rejects();
    test_conv();
    test_update_adam();
    test_comm();
  }
  if (failures) {
    printf("ABI FAILED (%d)\n", failures);
    return 1;
  }
  printf("ABI OK\n");
  return 0;
}
