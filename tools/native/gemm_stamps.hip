// Diagnostic: phase timestamps of the 8-phase GEMM kernel (csrc/gemm.hip built with DL4J_GEMM_STAMPS).
// Prints, over the blocks of the last of R launches: prologue (start -> first K-tile resident), main loop,
// epilogue, in shader cycles (median / max) and the kernel span in real time vs the hipEvent time.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc -DDL4J_GEMM_STAMPS tools/native/gemm_stamps.hip -o gemm_stamps
// Run:   ./gemm_stamps M N K [cfg]
#include "../../csrc/gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_rand(unsigned short* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffffff) / 16777216.0f) * 2.f - 1.f;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 2304, K = argc > 3 ? atoi(argv[3]) : 768;
  const int cfg = argc > 4 ? atoi(argv[4]) : 4;
  unsigned short *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  fill_rand<<<1024, 256>>>(A, (long long)M * K, 1);
  fill_rand<<<1024, 256>>>(B, (long long)N * K, 2);
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  unsigned long long* st;
  CK(hipMalloc(&st, (size_t)tiles * 16 * 8));
  CK(hipMemset(st, 0, (size_t)tiles * 16 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), &st, sizeof(st)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.f;
  for (int r = 0; r < 10; ++r) {
    CK(hipEventRecord(e0, 0));
    // A [M][K] K-contiguous, B [N][K] K-contiguous (akc = bkc = 1), C [M][N] bf16
    int rc = dl4j_gemm(1, 1, M, N, K, 1, A, K, 1, 0, B, K, 1, 0, C, N, 0, 1.f, 0.f, nullptr, 0, 0, nullptr, cfg, 1,
                       nullptr, nullptr, 0, 0);
    if (rc) { printf("dl4j_gemm rc=%d\n", rc); return 1; }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  std::vector<unsigned long long> h((size_t)tiles * 16);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> pro, loop, epi, tot;
  unsigned long long rt_min = ~0ull, rt_max = 0, rt1_max = 0;
  std::vector<double> start_rt;
  for (int b = 0; b < tiles; ++b) {
    const unsigned long long* p = &h[(size_t)b * 16];
    if (!p[0]) continue;
    pro.push_back((double)(p[2] - p[0]));
    loop.push_back((double)(p[4] - p[2]));
    epi.push_back((double)(p[6] - p[4]));
    tot.push_back((double)(p[6] - p[0]));
    rt_min = std::min(rt_min, p[1]);
    rt_max = std::max(rt_max, p[7]);
    start_rt.push_back((double)p[1]);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  auto mx = [](const std::vector<double>& v) { return *std::max_element(v.begin(), v.end()); };
  double smax = 0;
  for (double s : start_rt) smax = std::max(smax, s - (double)rt_min);
  printf("M=%d N=%d K=%d cfg=%d blocks=%zu event %.1f us  span(realtime) %.1f us  last block start +%.2f us\n", M, N, K,
         cfg, pro.size(), ms * 1000.f, (rt_max - rt_min) / 100.0, smax / 100.0);
  printf("  cycles  median / max: prologue %.0f / %.0f   loop %.0f / %.0f   epilogue %.0f / %.0f   total %.0f / %.0f\n",
         med(pro), mx(pro), med(loop), mx(loop), med(epi), mx(epi), med(tot), mx(tot));
  {
    std::vector<double> w0, r0, w1, r1, drain;
    for (int b = 0; b < tiles; ++b) {
      const unsigned long long* p = &h[(size_t)b * 16];
      if (!p[0]) continue;
      w0.push_back((double)(p[8] - p[4]));     // pass 0: LDS image write + barrier
      r0.push_back((double)(p[10] - p[8]));    // pass 0: read-out + stores issued
      w1.push_back((double)(p[12] - p[10]));   // pass 1: barrier + LDS image write + barrier
      r1.push_back((double)(p[14] - p[12]));   // pass 1: read-out
      drain.push_back((double)(p[6] - p[14])); // store drain (vmcnt(0))
    }
    printf("  epilogue medians: pass0 lds-write %.0f readout %.0f | pass1 lds-write %.0f readout %.0f | drain %.0f\n",
           med(w0), med(r0), med(w1), med(r1), med(drain));
  }
  printf("  implied clock %.2f GHz (median total cycles / median block real time)\n",
         med(tot) / 1e3 / ((rt_max - rt_min) / 100.0));
  return 0;
}
