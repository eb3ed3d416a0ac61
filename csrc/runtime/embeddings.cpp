// Host runtime for the embedding learners (Word2Vec / ParagraphVectors / DeepWalk / GloVe).
//
// Reference: SequenceVectors + SkipGram/CBOW/DBOW/DM learners (NLP:models/embeddings/learning/impl/elements/
// SkipGram.java:156-287, CBOW.java, sequence/DBOW.java, DM.java) which batch AggregateSkipGram/AggregateCBOW ops
// into libnd4j. Here the work is split in two native stages:
//   1. a batcher (this file) turns token sequences into flat work items — skip-gram pairs or CBOW windows — with
//      the reference's LCG random stream for the dynamic window shrink and frequency subsampling;
//   2. an applier consumes the items: the gfx950 kernels in csrc/embeddings.hip on the GPU, or the multi-threaded
//      (Hogwild, like the reference's worker threads) CPU applier below. Both use identical math: exact sigmoid
//      with word2vec's MAX_EXP=6 clipping, the unigram^0.75 negative table and per-item LCG seeds.
// Also: GloVe co-occurrence counting (NLP:models/glove/AbstractCoOccurrences.java) with 1/distance weighting.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#define RT_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t lcg(uint64_t r) { return r * 25214903917ULL + 11ULL; }

inline uint64_t mix(uint64_t x) {            // splitmix64 — per-item seeds independent of batch layout
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

inline double uniform(uint64_t& r) {
  r = lcg(r);
  return double((r >> 16) & 0xFFFF) / 65536.0;
}

struct Shared {
  float* syn0; float* syn1; float* syn1neg; int D;
  const uint8_t* codes; const int32_t* points; const int32_t* codelen; int maxc;
  const int32_t* table; int64_t tsize; int negative; int flags; uint64_t seed;
};
enum { F_UPD_OUT = 1, F_UPD_IN = 2, F_HS = 4, F_NS = 8 };
constexpr float MAX_EXP = 6.0f;

inline float dotp(const float* a, const float* b, int D) {
  float s = 0.f;
  for (int k = 0; k < D; ++k) s += a[k] * b[k];
  return s;
}

// One (input vector l1, target word) sample: hierarchical softmax over the target's Huffman path and/or negative
// sampling; accumulates the input gradient in neu1e, updates output rows in place. Returns the sample's loss.
inline double learn(const Shared& S, const float* l1, float* neu1e, int tgt, uint64_t rng, float alpha) {
  const int D = S.D;
  double loss = 0;
  if (S.flags & F_HS) {
    const int L = S.codelen[tgt];
    for (int c = 0; c < L; ++c) {
      float* w = S.syn1 + int64_t(S.points[int64_t(tgt) * S.maxc + c]) * D;
      float f = dotp(l1, w, D);
      if (f <= -MAX_EXP || f >= MAX_EXP) continue;
      float sg = 1.f / (1.f + std::exp(-f));
      int code = S.codes[int64_t(tgt) * S.maxc + c];
      float g = (1.f - code - sg) * alpha;
      loss -= std::log(std::max(1e-7f, code ? 1.f - sg : sg));
      for (int k = 0; k < D; ++k) neu1e[k] += g * w[k];
      if (S.flags & F_UPD_OUT)
        for (int k = 0; k < D; ++k) w[k] += g * l1[k];
    }
  }
  if ((S.flags & F_NS) && S.negative > 0) {
    for (int d = 0; d <= S.negative; ++d) {
      int target, label;
      if (d == 0) { target = tgt; label = 1; }
      else {
        rng = lcg(rng);
        target = S.table[(rng >> 16) % uint64_t(S.tsize)];
        if (target == tgt) continue;
        label = 0;
      }
      float* w = S.syn1neg + int64_t(target) * D;
      float f = dotp(l1, w, D);
      float sg = f > MAX_EXP ? 1.f : (f < -MAX_EXP ? 0.f : 1.f / (1.f + std::exp(-f)));
      float g = (float(label) - sg) * alpha;
      loss -= std::log(std::max(1e-7f, label ? sg : 1.f - sg));
      for (int k = 0; k < D; ++k) neu1e[k] += g * w[k];
      if (S.flags & F_UPD_OUT)
        for (int k = 0; k < D; ++k) w[k] += g * l1[k];
    }
  }
  return loss;
}

template <typename F> void parallel(int64_t n, int nthreads, F f) {
  nthreads = std::max(1, std::min<int>(nthreads, int((n + 255) / 256)));
  if (nthreads == 1) { f(0, 0, n); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    int64_t a = n * t / nthreads, b = n * (t + 1) / nthreads;
    th.emplace_back([=] { f(t, a, b); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

// ------------------------------------------------------------------------------------------------ batching
// Skip-gram pairs: for position i (word w) and every context word c inside the randomly shrunk window, one item
// (in_row = c, tgt = w) — the reference's iterateSample(word, lastWord) with syn0[lastWord] the input.
// DBOW pairs: (in_row = label row, tgt = w) for every word and every label of the sequence.
// CBOW / DM items: tgt = w, context = window words (+ labels for DM).
// Sequences are pre-subsampled by the caller-supplied keep probabilities (nullable).
// Returns the number of items written, or -(needed) when a capacity is too small. *words_out = words kept.
RT_API int64_t rt_w2v_batch(const int32_t* tokens, const int64_t* offs, int64_t nseq, const int32_t* labels,
                            const int64_t* label_offs, const float* keep_prob, int window, int mode,
                            uint64_t* seed_io, float alpha0, float alpha_min, int64_t words_before,
                            int64_t total_words, int32_t* item_in, int32_t* item_tgt, float* item_alpha,
                            int32_t* ctx_off, int32_t* ctx, int64_t cap_items, int64_t cap_ctx, int64_t* words_out) {
  // mode bits: 1 skip-gram elements, 2 cbow elements, 4 dbow sequence, 8 dm sequence
  uint64_t r = *seed_io;
  int64_t n = 0, m = 0, words = 0;
  std::vector<int32_t> seq;
  if (ctx_off) ctx_off[0] = 0;
  for (int64_t s = 0; s < nseq; ++s) {
    seq.clear();
    for (int64_t i = offs[s]; i < offs[s + 1]; ++i) {
      int32_t w = tokens[i];
      if (w < 0) continue;
      if (keep_prob) {
        float kp = keep_prob[w];
        if (kp < 1.f && kp < uniform(r)) continue;
      }
      seq.push_back(w);
    }
    const int32_t* lab = labels ? labels + label_offs[s] : nullptr;
    const int nlab = labels ? int(label_offs[s + 1] - label_offs[s]) : 0;
    const int T = int(seq.size());
    const double prog = total_words > 0 ? double(words_before + words) / double(total_words) : 0.0;
    const float alpha = std::max(alpha_min, float(alpha0 * (1.0 - std::min(1.0, prog))));  // SequenceVectors.java
    for (int i = 0; i < T; ++i) {
      r = lcg(r);
      const int b = window > 0 ? int((r >> 16) % uint64_t(window)) : 0;
      const int w = seq[i];
      if (mode & 1) {
        for (int a = b; a < 2 * window + 1 - b; ++a) {
          if (a == window) continue;
          int c = i - window + a;
          if (c < 0 || c >= T || seq[c] == w) continue;
          if (n >= cap_items) return -(n + 1);
          item_in[n] = seq[c]; item_tgt[n] = w; item_alpha[n] = alpha; ++n;
        }
      }
      if (mode & 4) {
        for (int l = 0; l < nlab; ++l) {
          if (n >= cap_items) return -(n + 1);
          item_in[n] = lab[l]; item_tgt[n] = w; item_alpha[n] = alpha; ++n;
        }
      }
      if (mode & 10) {   // cbow / dm
        int64_t m0 = m;
        for (int a = b; a < 2 * window + 1 - b; ++a) {
          if (a == window) continue;
          int c = i - window + a;
          if (c < 0 || c >= T) continue;
          if (m >= cap_ctx) return -(n + 1);
          ctx[m++] = seq[c];
        }
        if (mode & 8)
          for (int l = 0; l < nlab; ++l) {
            if (m >= cap_ctx) return -(n + 1);
            ctx[m++] = lab[l];
          }
        if (m == m0) continue;
        if (n >= cap_items) return -(n + 1);
        item_tgt[n] = w; item_alpha[n] = alpha; item_in[n] = -1; ++n;
        ctx_off[n] = int32_t(m);
      }
    }
    words += T;
  }
  *seed_io = r;
  if (words_out) *words_out = words;
  return n;
}

// ------------------------------------------------------------------------------------------------ CPU appliers
RT_API double rt_w2v_sg_apply(const int32_t* item_in, const int32_t* item_tgt, const float* item_alpha,
                              int64_t n, float* syn0, float* syn1, float* syn1neg, int D, const uint8_t* codes,
                              const int32_t* points, const int32_t* codelen, int maxc, const int32_t* table,
                              int64_t tsize, int negative, int flags, uint64_t seed, int64_t item_base,
                              int nthreads) {
  Shared S{syn0, syn1, syn1neg, D, codes, points, codelen, maxc, table, tsize, negative, flags, seed};
  std::vector<double> losses(std::max(1, nthreads), 0.0);
  parallel(n, nthreads, [&](int t, int64_t a, int64_t b) {
    std::vector<float> neu1e(D), l1(D);
    double loss = 0;
    for (int64_t i = a; i < b; ++i) {
      float* in = S.syn0 + int64_t(item_in[i]) * D;
      const float alpha = item_alpha[i];
      std::fill(neu1e.begin(), neu1e.end(), 0.f);
      std::memcpy(l1.data(), in, sizeof(float) * D);
      loss += learn(S, l1.data(), neu1e.data(), item_tgt[i], mix(seed ^ uint64_t(item_base + i)), alpha);
      if (flags & F_UPD_IN)
        for (int k = 0; k < D; ++k) in[k] += neu1e[k];
    }
    losses[t] = loss;
  });
  double tot = 0;
  for (double l : losses) tot += l;
  return tot;
}

RT_API double rt_w2v_cbow_apply(const int32_t* item_tgt, const float* item_alpha, const int32_t* ctx_off,
                                const int32_t* ctx, int64_t n, float* syn0, float* syn1, float* syn1neg, int D,
                                const uint8_t* codes, const int32_t* points, const int32_t* codelen, int maxc,
                                const int32_t* table, int64_t tsize, int negative, int flags, uint64_t seed,
                                int64_t item_base, int nthreads, const float* extra_in, int n_extra,
                                float* extra_grad) {
  // extra_in (nullable): n_extra additional input vectors averaged into every window — ParagraphVectors DM
  // inference, where the document vector being inferred is not a syn0 row. Its accumulated gradient goes to
  // extra_grad (the caller applies it; run single-threaded for a deterministic result).
  Shared S{syn0, syn1, syn1neg, D, codes, points, codelen, maxc, table, tsize, negative, flags, seed};
  std::vector<double> losses(std::max(1, nthreads), 0.0);
  parallel(n, nthreads, [&](int t, int64_t a, int64_t b) {
    std::vector<float> neu1(D), neu1e(D);
    double loss = 0;
    for (int64_t i = a; i < b; ++i) {
      const int c0 = ctx_off[i], c1 = ctx_off[i + 1];
      const int cw = c1 - c0 + n_extra;
      if (cw <= 0) continue;
      std::fill(neu1.begin(), neu1.end(), 0.f);
      for (int c = c0; c < c1; ++c) {
        const float* v = S.syn0 + int64_t(ctx[c]) * D;
        for (int k = 0; k < D; ++k) neu1[k] += v[k];
      }
      for (int e = 0; e < n_extra; ++e)
        for (int k = 0; k < D; ++k) neu1[k] += extra_in[int64_t(e) * D + k];
      for (int k = 0; k < D; ++k) neu1[k] /= float(cw);
      std::fill(neu1e.begin(), neu1e.end(), 0.f);
      loss += learn(S, neu1.data(), neu1e.data(), item_tgt[i], mix(seed ^ uint64_t(item_base + i)),
                    item_alpha[i]);
      if (flags & F_UPD_IN)
        for (int c = c0; c < c1; ++c) {
          float* v = S.syn0 + int64_t(ctx[c]) * D;
          for (int k = 0; k < D; ++k) v[k] += neu1e[k];
        }
      if (extra_grad)
        for (int e = 0; e < n_extra; ++e)
          for (int k = 0; k < D; ++k) extra_grad[int64_t(e) * D + k] += neu1e[k];
    }
    losses[t] = loss;
  });
  double tot = 0;
  for (double l : losses) tot += l;
  return tot;
}

// ------------------------------------------------------------------------------------------------ GloVe
namespace {
struct PairHash {
  size_t operator()(uint64_t k) const { return size_t(mix(k)); }
};
}  // namespace

// Windowed co-occurrence counts, weight 1/distance, optionally symmetric. Handle protocol: new -> size -> fetch
// (sorted by (i, j)) -> free.
RT_API void* rt_glove_cooccur_new(const int32_t* tokens, const int64_t* offs, int64_t nseq, int window,
                                  int symmetric) {
  auto* M = new std::unordered_map<uint64_t, float, PairHash>();
  for (int64_t s = 0; s < nseq; ++s) {
    const int64_t a = offs[s], b = offs[s + 1];
    for (int64_t i = a; i < b; ++i) {
      const int32_t wi = tokens[i];
      if (wi < 0) continue;
      for (int64_t j = std::max(a, i - window); j < i; ++j) {
        const int32_t wj = tokens[j];
        if (wj < 0 || wj == wi) continue;
        const float w = 1.0f / float(i - j);
        (*M)[(uint64_t(uint32_t(wi)) << 32) | uint32_t(wj)] += w;
        if (symmetric) (*M)[(uint64_t(uint32_t(wj)) << 32) | uint32_t(wi)] += w;
      }
    }
  }
  return M;
}

RT_API int64_t rt_glove_cooccur_size(void* h) {
  return int64_t(static_cast<std::unordered_map<uint64_t, float, PairHash>*>(h)->size());
}

RT_API int64_t rt_glove_cooccur_fetch(void* h, int32_t* out_i, int32_t* out_j, float* out_x, int64_t cap) {
  auto& M = *static_cast<std::unordered_map<uint64_t, float, PairHash>*>(h);
  std::vector<std::pair<uint64_t, float>> v(M.begin(), M.end());
  std::sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  const int64_t n = std::min<int64_t>(cap, int64_t(v.size()));
  for (int64_t k = 0; k < n; ++k) {
    out_i[k] = int32_t(v[k].first >> 32);
    out_j[k] = int32_t(v[k].first & 0xFFFFFFFFu);
    out_x[k] = v[k].second;
  }
  return n;
}

RT_API void rt_glove_cooccur_free(void* h) { delete static_cast<std::unordered_map<uint64_t, float, PairHash>*>(h); }

// AdaGrad GloVe step over entries (tied word/context matrix, as the reference's GloVe learner): returns the
// summed weighted squared error.
RT_API double rt_glove_apply(const int32_t* ei, const int32_t* ej, const float* ex, int64_t n, float* W, float* b,
                             float* hW, float* hb, int D, float lr, float xmax, float alpha, int nthreads) {
  std::vector<double> costs(std::max(1, nthreads), 0.0);
  parallel(n, nthreads, [&](int t, int64_t a, int64_t bb) {
    std::vector<float> gi(D), gj(D);
    double cost = 0;
    for (int64_t k = a; k < bb; ++k) {
      const int i = ei[k], j = ej[k];
      float* wi = W + int64_t(i) * D;
      float* wj = W + int64_t(j) * D;
      const float x = ex[k];
      float pred = dotp(wi, wj, D) + b[i] + b[j] - std::log(x);
      float fd = (x > xmax ? 1.f : std::pow(x / xmax, alpha)) * pred;
      cost += 0.5 * double(fd) * pred;
      for (int d = 0; d < D; ++d) { gi[d] = fd * wj[d]; gj[d] = fd * wi[d]; }
      float* hi = hW + int64_t(i) * D;
      float* hj = hW + int64_t(j) * D;
      for (int d = 0; d < D; ++d) {
        hi[d] += gi[d] * gi[d];
        wi[d] -= lr * gi[d] / std::sqrt(hi[d] + 1e-8f);
        hj[d] += gj[d] * gj[d];
        wj[d] -= lr * gj[d] / std::sqrt(hj[d] + 1e-8f);
      }
      hb[i] += fd * fd;
      b[i] -= lr * fd / std::sqrt(hb[i] + 1e-8f);
      hb[j] += fd * fd;
      b[j] -= lr * fd / std::sqrt(hb[j] + 1e-8f);
    }
    costs[t] = cost;
  });
  double tot = 0;
  for (double c : costs) tot += c;
  return tot;
}
