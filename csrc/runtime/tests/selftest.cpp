// Self-test driver for the host runtime (csrc/runtime/*.cpp), built by `python -m deeplearning4j_amd.ops.build
// --sanitize=address|thread|undefined` into a standalone executable so AddressSanitizer / ThreadSanitizer / UBSan
// instrument every runtime translation unit. Exercises each C entry point, multi-threaded where the
// runtime is (workspace arenas from 8 threads, threaded random walks / VP-tree kNN / Barnes-Hut gradient / t-SNE
// row search), and checks results, so a sanitizer report or a wrong answer fails the run (exit status != 0).
// Hogwild embedding updates (rt_glove_apply / rt_w2v_*) race on purpose (as the reference's word2vec does), so
// they run single-threaded here.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {
long long rt_threshold_count(const float*, long long, float);
int rt_threshold_encode(float*, long long, float, int32_t*, int);
void rt_threshold_decode(const int32_t*, float*, float);
int rt_bitmap_encode(float*, long long, float, int32_t*);
void rt_bitmap_decode(const int32_t*, float*, float);
long long rt_ws_create(long long, long long, long long, double, int, int, int);
void rt_ws_destroy(long long);
int rt_ws_alloc(long long, long long, long long*, long long*);
long long rt_ws_cycle_end(long long);
int rt_ws_set_capacity(long long, long long);
int rt_ws_stats(long long, long long*);
int64_t rt_random_walks(const int64_t*, const int32_t*, const float*, const int32_t*, int64_t, int, uint64_t, int,
                        int32_t*, int);
void* rt_vptree_build(const float*, int, int, int, int, uint64_t);
void rt_vptree_free(void*);
void rt_vptree_knn(void*, const float*, int, int, int32_t*, float*, int);
void* rt_sptree_build(const double*, int, int);
void rt_sptree_free(void*);
int rt_sptree_cum(void*);
double rt_bhtsne_gradient(const double*, int, int, const int64_t*, const int32_t*, const double*, double, double*,
                          int);
void rt_tsne_row_probs(const float*, int, int, double, double, float*, int);
void* rt_glove_cooccur_new(const int32_t*, const int64_t*, int64_t, int, int);
int64_t rt_glove_cooccur_size(void*);
int64_t rt_glove_cooccur_fetch(void*, int32_t*, int32_t*, float*, int64_t);
void rt_glove_cooccur_free(void*);
double rt_glove_apply(const int32_t*, const int32_t*, const float*, int64_t, float*, float*, float*, float*, int,
                      float, float, float, int);
}

static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                     \
    }                                                                 \
  } while (0)

static uint64_t g_s = 0x9E3779B97F4A7C15ULL;
static float frand() {
  g_s ^= g_s << 13; g_s ^= g_s >> 7; g_s ^= g_s << 17;
  return float(g_s >> 40) / float(1 << 24) * 2.f - 1.f;
}

static void test_codecs() {
  const long long n = 10007;
  std::vector<float> r(n), r2, acc(n, 0.f), acc2(n, 0.f);
  for (auto& v : r) v = frand();
  r2 = r;
  const float thr = 0.5f;
  const long long cnt = rt_threshold_count(r.data(), n, thr);
  std::vector<int32_t> enc(4 + cnt);
  const int c = rt_threshold_encode(r.data(), n, thr, enc.data(), int(cnt));
  CHECK(c == cnt);
  rt_threshold_decode(enc.data(), acc.data(), 1.f);
  for (long long i = 0; i < n; ++i) CHECK(std::fabs(acc[i] + r[i] - r2[i]) < 1e-6f);   // residual + decoded = input
  std::vector<float> r3 = r2;
  std::vector<int32_t> bm(4 + (n + 15) / 16);
  const int cb = rt_bitmap_encode(r3.data(), n, thr, bm.data());
  CHECK(cb == cnt);
  rt_bitmap_decode(bm.data(), acc2.data(), 1.f);
  for (long long i = 0; i < n; ++i) CHECK(std::fabs(acc2[i] + r3[i] - r2[i]) < 1e-6f);
}

static void test_workspace() {
  const long long h = rt_ws_create(1 << 16, 1 << 24, 256, 0.25, 1, 0, 0);
  std::vector<std::thread> th;
  std::vector<long long> offs(8 * 64, -2);
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < 64; ++k) {
        long long off, gen;
        const int rc = rt_ws_alloc(h, 100 + 7 * k, &off, &gen);
        offs[t * 64 + k] = rc == 0 ? off : -1;
      }
    });
  for (auto& x : th) x.join();
  // carved offsets never overlap (each request rounds up to 256 bytes)
  std::vector<long long> carved;
  for (long long o : offs) if (o >= 0) carved.push_back(o);
  std::vector<char> seen((1 << 16) / 256, 0);
  for (long long o : carved) {
    CHECK(o % 256 == 0);
    CHECK(!seen[o / 256]);
    seen[o / 256] = 1;
  }
  long long st[10];
  CHECK(rt_ws_stats(h, st) == 0);
  CHECK(st[6] == 8 * 64);
  const long long want = rt_ws_cycle_end(h);       // learning: peak * 1.25, rounded to the alignment
  CHECK(want >= st[2]);
  CHECK(rt_ws_set_capacity(h, want) == 0);
  long long off, gen;
  CHECK(rt_ws_alloc(h, 1000, &off, &gen) == 0 && off == 0);
  rt_ws_destroy(h);
  CHECK(rt_ws_alloc(h, 10, &off, &gen) == -1);
}

static void test_walks() {
  // ring of 50 vertices, each with 2 out-edges
  const int V = 50;
  std::vector<int64_t> offs(V + 1);
  std::vector<int32_t> nbr;
  std::vector<float> w;
  for (int v = 0; v < V; ++v) {
    offs[v] = (int64_t)nbr.size();
    nbr.push_back((v + 1) % V); w.push_back(1.f);
    nbr.push_back((v + V - 1) % V); w.push_back(3.f);
  }
  offs[V] = (int64_t)nbr.size();
  std::vector<int32_t> starts(400);
  for (int i = 0; i < 400; ++i) starts[i] = i % V;
  const int L = 20;
  std::vector<int32_t> out(400 * (L + 1)), out2(400 * (L + 1));
  CHECK(rt_random_walks(offs.data(), nbr.data(), w.data(), starts.data(), 400, L, 42, 0, out.data(), 4) == 400);
  CHECK(rt_random_walks(offs.data(), nbr.data(), w.data(), starts.data(), 400, L, 42, 0, out2.data(), 1) == 400);
  CHECK(out == out2);                               // deterministic per walk, independent of thread count
  for (int i = 0; i < 400; ++i)
    for (int k = 1; k <= L; ++k) {
      const int a = out[i * (L + 1) + k - 1], b = out[i * (L + 1) + k];
      CHECK(b == (a + 1) % V || b == (a + V - 1) % V);
    }
}

static void test_trees() {
  const int n = 300, d = 4, k = 5;
  std::vector<float> data(n * d);
  for (auto& v : data) v = frand();
  void* t = rt_vptree_build(data.data(), n, d, 0, 0, 7);
  std::vector<int32_t> idx(n * k);
  std::vector<float> dist(n * k);
  rt_vptree_knn(t, data.data(), n, k, idx.data(), dist.data(), 4);
  for (int q = 0; q < n; ++q) {
    CHECK(idx[q * k] == q);                         // each point is its own nearest neighbour
    for (int j = 1; j < k; ++j) CHECK(dist[q * k + j] >= dist[q * k + j - 1]);
  }
  rt_vptree_free(t);
  std::vector<double> Y(n * 2);
  for (auto& v : Y) v = frand();
  void* sp = rt_sptree_build(Y.data(), n, 2);
  CHECK(sp && rt_sptree_cum(sp) == n);
  rt_sptree_free(sp);
  // sparse symmetric P from the kNN graph
  std::vector<int64_t> rowP(n + 1);
  std::vector<int32_t> colP;
  std::vector<double> valP;
  for (int i = 0; i < n; ++i) {
    rowP[i] = (int64_t)colP.size();
    for (int j = 1; j < k; ++j) { colP.push_back(idx[i * k + j]); valP.push_back(1.0 / (n * (k - 1))); }
  }
  rowP[n] = (int64_t)colP.size();
  std::vector<double> dY1(n * 2), dY4(n * 2);
  rt_bhtsne_gradient(Y.data(), n, 2, rowP.data(), colP.data(), valP.data(), 0.5, dY1.data(), 1);
  rt_bhtsne_gradient(Y.data(), n, 2, rowP.data(), colP.data(), valP.data(), 0.5, dY4.data(), 4);
  for (int i = 0; i < n * 2; ++i) CHECK(std::fabs(dY1[i] - dY4[i]) <= 1e-9 * (1 + std::fabs(dY1[i])));
  std::vector<float> dd(n * (k - 1)), probs(n * (k - 1));
  for (int i = 0; i < n; ++i)
    for (int j = 1; j < k; ++j) dd[i * (k - 1) + j - 1] = dist[i * k + j];
  rt_tsne_row_probs(dd.data(), n, k - 1, 3.0, 1e-5, probs.data(), 4);
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < k - 1; ++j) s += probs[i * (k - 1) + j];
    CHECK(std::fabs(s - 1.0) < 1e-3);
  }
}

static void test_glove() {
  std::vector<int32_t> tokens;
  std::vector<int64_t> offs = {0};
  for (int s = 0; s < 20; ++s) {
    for (int i = 0; i < 30; ++i) tokens.push_back((s * 7 + i * 3) % 40);
    offs.push_back((int64_t)tokens.size());
  }
  void* h = rt_glove_cooccur_new(tokens.data(), offs.data(), 20, 5, 1);
  const int64_t m = rt_glove_cooccur_size(h);
  CHECK(m > 0);
  std::vector<int32_t> ei(m), ej(m);
  std::vector<float> ex(m);
  CHECK(rt_glove_cooccur_fetch(h, ei.data(), ej.data(), ex.data(), m) == m);
  rt_glove_cooccur_free(h);
  const int D = 8;
  std::vector<float> W(40 * D), b(40, 0.f), hW(40 * D, 0.f), hb(40, 0.f);
  for (auto& v : W) v = 0.1f * frand();
  double c0 = rt_glove_apply(ei.data(), ej.data(), ex.data(), m, W.data(), b.data(), hW.data(), hb.data(), D, 0.05f,
                             100.f, 0.75f, 1);
  double c = c0;
  for (int it = 0; it < 20; ++it)
    c = rt_glove_apply(ei.data(), ej.data(), ex.data(), m, W.data(), b.data(), hW.data(), hb.data(), D, 0.05f, 100.f,
                       0.75f, 1);
  CHECK(c < c0);
}

int main() {
  test_codecs();
  test_workspace();
  test_walks();
  test_trees();
  test_glove();
  std::printf(g_fail ? "runtime selftest FAILED\n" : "runtime selftest OK\n");
  return g_fail;
}
