// Spatial trees for nearest neighbours and Barnes-Hut t-SNE.
//
// Reference: nearestneighbor-core clustering/vptree/VPTree.java (vantage-point tree: random vantage point, median
// distance threshold, tau-pruned k-NN search), clustering/sptree/SpTree.java + quadtree/QuadTree.java (2^D-ary
// space-partitioning tree with centre of mass, Barnes-Hut non-edge forces with the theta criterion), and
// deeplearning4j-tsne plot/BarnesHutTsne.java (perplexity binary search over k-NN distances, edge forces).
// Host-side C++ (pointer-chasing trees are CPU work); the dense O(n^2) paths (exact t-SNE, brute-force k-NN) run on
// the GPU through plain GEMMs instead.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <queue>
#include <random>
#include <thread>
#include <vector>

#define RT_API extern "C" __attribute__((visibility("default")))

namespace {

// metric ids: 0 euclidean, 1 manhattan, 2 cosinedistance, 3 cosinesimilarity, 4 dot, 5 hamming, 6 jaccard
double metric(int m, const float* a, const float* b, int d) {
  switch (m) {
    case 1: {
      double s = 0;
      for (int k = 0; k < d; ++k) s += std::fabs(double(a[k]) - b[k]);
      return s;
    }
    case 2:
    case 3: {
      double ab = 0, aa = 0, bb = 0;
      for (int k = 0; k < d; ++k) { ab += double(a[k]) * b[k]; aa += double(a[k]) * a[k]; bb += double(b[k]) * b[k]; }
      double c = ab / std::max(1e-30, std::sqrt(aa) * std::sqrt(bb));
      return m == 2 ? 1.0 - c : c;
    }
    case 4: {
      double s = 0;
      for (int k = 0; k < d; ++k) s += double(a[k]) * b[k];
      return s;
    }
    case 5: {
      double s = 0;
      for (int k = 0; k < d; ++k) s += (a[k] != b[k]);
      return s / d;
    }
    case 6: {
      double mn = 0, mx = 0;
      for (int k = 0; k < d; ++k) { mn += std::min(a[k], b[k]); mx += std::max(a[k], b[k]); }
      return mx > 0 ? 1.0 - mn / mx : 0.0;
    }
    default: {
      double s = 0;
      for (int k = 0; k < d; ++k) { double t = double(a[k]) - b[k]; s += t * t; }
      return std::sqrt(s);
    }
  }
}

struct VPNode {
  int index = -1;
  double threshold = 0;
  int left = -1, right = -1;
};

struct VPTree {
  std::vector<float> data;
  int n = 0, d = 0, m = 0;
  bool invert = false;
  std::vector<VPNode> nodes;
  int root = -1;

  double dist(const float* a, const float* b) const {
    double r = metric(m, a, b, d);
    return invert ? -r : r;
  }
  const float* row(int i) const { return data.data() + size_t(i) * d; }

  int build(std::vector<int>& idx, int lo, int hi, std::mt19937_64& rng) {
    if (lo >= hi) return -1;
    int id = int(nodes.size());
    nodes.emplace_back();
    if (hi - lo == 1) { nodes[id].index = idx[lo]; return id; }
    std::uniform_int_distribution<int> u(lo, hi - 1);
    std::swap(idx[lo], idx[u(rng)]);
    const int vp = idx[lo];
    const int mid = (lo + 1 + hi) / 2;
    std::nth_element(idx.begin() + lo + 1, idx.begin() + mid, idx.begin() + hi, [&](int a, int b) {
      return dist(row(vp), row(a)) < dist(row(vp), row(b));
    });
    nodes[id].index = vp;
    nodes[id].threshold = dist(row(vp), row(idx[mid]));
    int l = build(idx, lo + 1, mid, rng);
    int r = build(idx, mid, hi, rng);
    nodes[id].left = l;
    nodes[id].right = r;
    return id;
  }

  void search(int ni, const float* q, int k, std::priority_queue<std::pair<double, int>>& pq, double& tau) const {
    if (ni < 0) return;
    const VPNode& nd = nodes[ni];
    const double dd = dist(row(nd.index), q);
    if (dd < tau) {
      if (int(pq.size()) == k) pq.pop();
      pq.emplace(dd, nd.index);
      if (int(pq.size()) == k) tau = pq.top().first;
    }
    if (nd.left < 0 && nd.right < 0) return;
    if (dd < nd.threshold) {
      if (dd - tau <= nd.threshold) search(nd.left, q, k, pq, tau);
      if (dd + tau >= nd.threshold) search(nd.right, q, k, pq, tau);
    } else {
      if (dd + tau >= nd.threshold) search(nd.right, q, k, pq, tau);
      if (dd - tau <= nd.threshold) search(nd.left, q, k, pq, tau);
    }
  }
};

template <typename F> void parallel_for(int64_t n, int nthreads, F f) {
  nthreads = std::max(1, std::min<int>(nthreads, int((n + 31) / 32)));
  if (nthreads == 1) { for (int64_t i = 0; i < n; ++i) f(i); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([=] { for (int64_t i = n * t / nthreads; i < n * (t + 1) / nthreads; ++i) f(i); });
  for (auto& x : th) x.join();
}

}  // namespace

RT_API void* rt_vptree_build(const float* data, int n, int d, int metric_id, int invert, uint64_t seed) {
  auto* t = new VPTree();
  t->data.assign(data, data + size_t(n) * d);
  t->n = n; t->d = d; t->m = metric_id; t->invert = invert != 0;
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::mt19937_64 rng(seed);
  t->nodes.reserve(n);
  t->root = t->build(idx, 0, n, rng);
  return t;
}

RT_API void rt_vptree_free(void* h) { delete static_cast<VPTree*>(h); }

// k nearest items for each query, ascending by (possibly inverted) distance; missing slots get index -1.
RT_API void rt_vptree_knn(void* h, const float* queries, int nq, int k, int32_t* out_idx, float* out_dist,
                          int nthreads) {
  const VPTree* t = static_cast<VPTree*>(h);
  parallel_for(nq, nthreads, [&](int64_t qi) {
    std::priority_queue<std::pair<double, int>> pq;
    double tau = DBL_MAX;
    t->search(t->root, queries + size_t(qi) * t->d, k, pq, tau);
    std::vector<std::pair<double, int>> res;
    while (!pq.empty()) { res.push_back(pq.top()); pq.pop(); }
    std::reverse(res.begin(), res.end());
    for (int j = 0; j < k; ++j) {
      out_idx[qi * k + j] = j < int(res.size()) ? res[j].second : -1;
      out_dist[qi * k + j] = j < int(res.size()) ? float(res[j].first) : INFINITY;
    }
  });
}

// ------------------------------------------------------------------------------------------- SpTree
namespace {
struct SpNode {
  double corner[3], width[3];
  double com[3];
  int cum = 0;
  int point = -1;          // leaf payload (capacity 1)
  int child0 = -1;         // first of 2^D children (contiguous)
  bool leaf = true;
};

struct SpTree {
  int D = 2, n = 0;
  const double* Y = nullptr;
  std::vector<SpNode> nodes;

  bool contains(const SpNode& nd, const double* p) const {
    for (int k = 0; k < D; ++k)
      if (p[k] < nd.corner[k] - nd.width[k] || p[k] > nd.corner[k] + nd.width[k]) return false;
    return true;
  }

  void subdivide(int ni) {
    const int nc = 1 << D;
    const int c0 = int(nodes.size());
    for (int c = 0; c < nc; ++c) {
      SpNode ch;
      for (int k = 0; k < D; ++k) {
        ch.width[k] = nodes[ni].width[k] * 0.5;
        ch.corner[k] = nodes[ni].corner[k] + (((c >> k) & 1) ? ch.width[k] : -ch.width[k]);
        ch.com[k] = 0;
      }
      nodes.push_back(ch);
    }
    nodes[ni].child0 = c0;
    nodes[ni].leaf = false;
    const int p = nodes[ni].point;
    nodes[ni].point = -1;
    if (p >= 0) insert_child(ni, p);
  }

  void insert_child(int ni, int p) {
    const double* y = Y + size_t(p) * D;
    int c = 0;
    for (int k = 0; k < D; ++k)
      if (y[k] > nodes[ni].corner[k]) c |= (1 << k);
    insert(nodes[ni].child0 + c, p);
  }

  void insert(int ni, int p) {
    const double* y = Y + size_t(p) * D;
    // online centre of mass
    SpNode& nd = nodes[ni];
    nd.cum += 1;
    const double mult1 = double(nd.cum - 1) / nd.cum, mult2 = 1.0 / nd.cum;
    for (int k = 0; k < D; ++k) nd.com[k] = nd.com[k] * mult1 + mult2 * y[k];
    if (nodes[ni].leaf && nodes[ni].point < 0) { nodes[ni].point = p; return; }
    if (nodes[ni].leaf) {
      // duplicate point: keep as aggregated mass (no infinite subdivision)
      const double* q = Y + size_t(nodes[ni].point) * D;
      bool dup = true;
      for (int k = 0; k < D; ++k) dup = dup && (q[k] == y[k]);
      if (dup) return;
      subdivide(ni);
    }
    insert_child(ni, p);
  }

  void build(const double* y, int n_, int D_) {
    Y = y; n = n_; D = D_;
    nodes.clear();
    nodes.reserve(size_t(4) * n + 16);
    SpNode root;
    double mn[3], mx[3];
    for (int k = 0; k < D; ++k) { mn[k] = DBL_MAX; mx[k] = -DBL_MAX; }
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < D; ++k) { mn[k] = std::min(mn[k], y[i * D + k]); mx[k] = std::max(mx[k], y[i * D + k]); }
    for (int k = 0; k < D; ++k) {
      root.corner[k] = 0.5 * (mn[k] + mx[k]);
      root.width[k] = std::max(0.5 * (mx[k] - mn[k]), 1e-5) + 1e-5;
      root.com[k] = 0;
    }
    nodes.push_back(root);
    for (int i = 0; i < n; ++i) insert(0, i);
  }

  // Barnes-Hut repulsion on point i: accumulates q^2 (y_i - com) * mass into negF; returns sum of q * mass.
  double nonedge(int ni, int i, double theta, double* negF) const {
    const SpNode& nd = nodes[ni];
    if (nd.cum == 0 || (nd.leaf && nd.point == i && nd.cum == 1)) return 0.0;
    const double* y = Y + size_t(i) * D;
    double buf[3], dd = 0, maxw = 0;
    for (int k = 0; k < D; ++k) { buf[k] = y[k] - nd.com[k]; dd += buf[k] * buf[k]; maxw = std::max(maxw, nd.width[k]); }
    if (nd.leaf || maxw / std::sqrt(dd) < theta) {
      int mass = nd.cum;
      if (nd.leaf && nd.point == i) mass -= 1;     // self (aggregated duplicates)
      if (mass <= 0) return 0.0;
      const double q = 1.0 / (1.0 + dd);
      double mult = mass * q;
      const double s = mult;
      mult *= q;
      for (int k = 0; k < D; ++k) negF[k] += mult * buf[k];
      return s;
    }
    double s = 0;
    for (int c = 0; c < (1 << D); ++c) s += nonedge(nd.child0 + c, i, theta, negF);
    return s;
  }

  int depth(int ni) const {
    if (nodes[ni].leaf) return 1;
    int m = 0;
    for (int c = 0; c < (1 << D); ++c) m = std::max(m, depth(nodes[ni].child0 + c));
    return 1 + m;
  }
};
}  // namespace

RT_API void* rt_sptree_build(const double* Y, int n, int D) {
  if (D < 1 || D > 3) return nullptr;
  auto* t = new SpTree();
  t->build(Y, n, D);
  return t;
}
RT_API void rt_sptree_free(void* h) { delete static_cast<SpTree*>(h); }
RT_API int rt_sptree_depth(void* h) { return static_cast<SpTree*>(h)->depth(0); }
RT_API int rt_sptree_cum(void* h) { return static_cast<SpTree*>(h)->nodes[0].cum; }
RT_API void rt_sptree_com(void* h, double* out) {
  auto* t = static_cast<SpTree*>(h);
  for (int k = 0; k < t->D; ++k) out[k] = t->nodes[0].com[k];
}
RT_API double rt_sptree_nonedge(void* h, int i, double theta, double* negF) {
  return static_cast<SpTree*>(h)->nonedge(0, i, theta, negF);
}

// Full Barnes-Hut t-SNE gradient: dY = posF - negF / sumQ (bhtsne / BarnesHutTsne.gradient). Returns sumQ.
RT_API double rt_bhtsne_gradient(const double* Y, int n, int D, const int64_t* rowP, const int32_t* colP,
                                 const double* valP, double theta, double* dY, int nthreads) {
  SpTree t;
  t.build(Y, n, D);
  std::vector<double> negF(size_t(n) * D, 0.0), posF(size_t(n) * D, 0.0);
  nthreads = std::max(1, nthreads);
  std::vector<double> sums(nthreads, 0.0);
  std::vector<std::thread> th;
  for (int tt = 0; tt < nthreads; ++tt)
    th.emplace_back([&, tt] {
      double s = 0;
      for (int64_t i = int64_t(n) * tt / nthreads; i < int64_t(n) * (tt + 1) / nthreads; ++i) {
        s += t.nonedge(0, int(i), theta, negF.data() + i * D);
        const double* yi = Y + i * D;
        double* pf = posF.data() + i * D;
        for (int64_t e = rowP[i]; e < rowP[i + 1]; ++e) {
          const double* yj = Y + size_t(colP[e]) * D;
          double dd = 1.0, buf[3];
          for (int k = 0; k < D; ++k) { buf[k] = yi[k] - yj[k]; dd += buf[k] * buf[k]; }
          const double mult = valP[e] / dd;
          for (int k = 0; k < D; ++k) pf[k] += mult * buf[k];
        }
      }
      sums[tt] = s;
    });
  for (auto& x : th) x.join();
  double sumQ = 0;
  for (double s : sums) sumQ += s;
  for (size_t k = 0; k < size_t(n) * D; ++k) dY[k] = posF[k] - negF[k] / sumQ;
  return sumQ;
}

// Per-row Gaussian conditional probabilities over k-NN distances with a binary search on beta so the row entropy
// matches log(perplexity) (BarnesHutTsne.computeGaussianPerplexity). dist: [n, K] (euclidean); out: [n, K].
RT_API void rt_tsne_row_probs(const float* dist, int n, int K, double perplexity, double tol, float* out,
                              int nthreads) {
  parallel_for(n, nthreads, [&](int64_t i) {
    const float* d = dist + i * K;
    std::vector<double> p(K);
    double beta = 1.0, lo = -DBL_MAX, hi = DBL_MAX;
    const double target = std::log(perplexity);
    for (int it = 0; it < 200; ++it) {
      double sum = 0;
      for (int j = 0; j < K; ++j) { p[j] = std::exp(-beta * double(d[j]) * d[j]); sum += p[j]; }
      sum = std::max(sum, DBL_MIN);
      double H = 0;
      for (int j = 0; j < K; ++j) H += beta * (double(d[j]) * d[j] * p[j]);
      H = H / sum + std::log(sum);
      const double diff = H - target;
      if (std::fabs(diff) < tol) break;
      if (diff > 0) { lo = beta; beta = hi == DBL_MAX ? beta * 2 : 0.5 * (beta + hi); }
      else { hi = beta; beta = lo == -DBL_MAX ? beta / 2 : 0.5 * (beta + lo); }
    }
    double sum = 0;
    for (int j = 0; j < K; ++j) sum += p[j];
    sum = std::max(sum, DBL_MIN);
    for (int j = 0; j < K; ++j) out[i * K + j] = float(p[j] / sum);
  });
}
