// GloVe co-occurrence counting under a memory cap (reference NLP:models/glove/AbstractCoOccurrences.java:55-104,
// 185-266, 387-520: a counting map that a "shadow copy" thread flushes to temp files whenever its footprint passes
// maxMemory / 2, merged with the previous file each time, plus count/Binary|ASCIICoOccurrence{Reader,Writer}).
//
// Design here: external sort-and-merge instead of the reference's repeated read-merge-rewrite of one file.
//   * rt_cooc_new(dir, max_entries): a counter whose in-memory hash map holds at most max_entries pairs;
//   * rt_cooc_add(h, tokens, offs, nseq, window, symmetric): counts one CHUNK of sequences (the caller streams the
//     corpus through it), 1/distance weights as the reference (:338). Whenever the map reaches the cap it is sorted
//     by (i, j) and written to a new run file <dir>/cooc_run_<k>.bin, then cleared — memory stays O(cap);
//   * rt_cooc_finish(h, out_path): k-way merge of every run plus the remaining map into ONE sorted file of
//     {int32 i, int32 j, float x} records, equal pairs summed (in run order: deterministic); the run files are
//     deleted. Merge memory is one read buffer per run. Returns the record count (or -1 on an I/O error).
//   * rt_cooc_spills(h): run files written so far (also after the merge).
// The trainer memory-maps the merged file, so neither counting nor training needs the whole table in RAM.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

#define RT_API extern "C" __attribute__((visibility("default")))

namespace {

struct Rec {
  int32_t i, j;
  float x;
};
static_assert(sizeof(Rec) == 12, "record layout");

struct KeyHash {
  size_t operator()(uint64_t k) const {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    return size_t(k);
  }
};

struct Counter {
  std::unordered_map<uint64_t, float, KeyHash> map;
  std::vector<std::string> runs;
  std::string dir;
  int64_t cap;
  int64_t nspills = 0;     // run files written over the counter's life (kept after the merge removes them)
  bool io_error = false;
};

inline uint64_t key(int32_t a, int32_t b) { return (uint64_t(uint32_t(a)) << 32) | uint32_t(b); }

std::vector<Rec> sorted_records(const std::unordered_map<uint64_t, float, KeyHash>& m) {
  std::vector<std::pair<uint64_t, float>> v(m.begin(), m.end());
  std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<Rec> out(v.size());
  for (size_t k = 0; k < v.size(); ++k) out[k] = Rec{int32_t(v[k].first >> 32), int32_t(v[k].first & 0xffffffffu), v[k].second};
  return out;
}

void spill(Counter& c) {
  if (c.map.empty()) return;
  const std::vector<Rec> recs = sorted_records(c.map);
  const std::string path = c.dir + "/cooc_run_" + std::to_string(c.runs.size()) + ".bin";
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f || std::fwrite(recs.data(), sizeof(Rec), recs.size(), f) != recs.size()) c.io_error = true;
  if (f) std::fclose(f);
  c.runs.push_back(path);
  ++c.nspills;
  c.map.clear();
  c.map.rehash(0);
}

// buffered sequential reader of one sorted run (or of the in-memory remainder)
struct Source {
  FILE* f = nullptr;
  const std::vector<Rec>* mem = nullptr;
  std::vector<Rec> buf;
  size_t pos = 0, n = 0, mem_pos = 0;
  bool next(Rec& r) {
    if (mem) {
      if (mem_pos >= mem->size()) return false;
      r = (*mem)[mem_pos++];
      return true;
    }
    if (pos == n) {
      n = std::fread(buf.data(), sizeof(Rec), buf.size(), f);
      pos = 0;
      if (n == 0) return false;
    }
    r = buf[pos++];
    return true;
  }
};

}  // namespace

RT_API void* rt_cooc_new(const char* dir, int64_t max_entries) {
  auto* c = new Counter();
  c->dir = dir ? dir : ".";
  c->cap = max_entries > 0 ? max_entries : (int64_t(1) << 62);
  return c;
}

RT_API int rt_cooc_add(void* h, const int32_t* tokens, const int64_t* offs, int64_t nseq, int window, int symmetric) {
  Counter& c = *static_cast<Counter*>(h);
  for (int64_t s = 0; s < nseq; ++s) {
    const int64_t a = offs[s], b = offs[s + 1];
    for (int64_t i = a; i < b; ++i) {
      const int32_t wi = tokens[i];
      if (wi < 0) continue;
      for (int64_t j = std::max(a, i - window); j < i; ++j) {
        const int32_t wj = tokens[j];
        if (wj < 0 || wj == wi) continue;
        const float w = 1.0f / float(i - j);
        c.map[key(wi, wj)] += w;
        if (symmetric) c.map[key(wj, wi)] += w;
        if (int64_t(c.map.size()) >= c.cap) spill(c);
      }
    }
  }
  return c.io_error ? -1 : 0;
}

RT_API int64_t rt_cooc_spills(void* h) { return static_cast<Counter*>(h)->nspills; }

RT_API int64_t rt_cooc_finish(void* h, const char* out_path) {
  Counter& c = *static_cast<Counter*>(h);
  const std::vector<Rec> rest = sorted_records(c.map);
  c.map.clear();
  std::vector<Source> src(c.runs.size() + 1);
  const size_t per = std::max<size_t>(4096, size_t(1 << 20) / (c.runs.size() + 1));   // ~12 MB of buffers in all
  for (size_t k = 0; k < c.runs.size(); ++k) {
    src[k].f = std::fopen(c.runs[k].c_str(), "rb");
    if (!src[k].f) return -1;
    src[k].buf.resize(per);
  }
  src.back().mem = &rest;
  FILE* out = std::fopen(out_path, "wb");
  if (!out) return -1;
  // min-heap over (key, source index): equal keys pop in source order, so the sum order is fixed
  typedef std::pair<uint64_t, size_t> HK;
  std::priority_queue<HK, std::vector<HK>, std::greater<HK>> heap;
  std::vector<Rec> head(src.size());
  for (size_t k = 0; k < src.size(); ++k)
    if (src[k].next(head[k])) heap.push({key(head[k].i, head[k].j), k});
  std::vector<Rec> obuf;
  obuf.reserve(1 << 16);
  int64_t count = 0;
  bool err = c.io_error;
  while (!heap.empty()) {
    const uint64_t kcur = heap.top().first;
    Rec acc{int32_t(kcur >> 32), int32_t(kcur & 0xffffffffu), 0.f};
    while (!heap.empty() && heap.top().first == kcur) {
      const size_t k = heap.top().second;
      heap.pop();
      acc.x += head[k].x;
      if (src[k].next(head[k])) heap.push({key(head[k].i, head[k].j), k});
    }
    obuf.push_back(acc);
    ++count;
    if (obuf.size() == obuf.capacity()) {
      err |= std::fwrite(obuf.data(), sizeof(Rec), obuf.size(), out) != obuf.size();
      obuf.clear();
    }
  }
  if (!obuf.empty()) err |= std::fwrite(obuf.data(), sizeof(Rec), obuf.size(), out) != obuf.size();
  std::fclose(out);
  for (size_t k = 0; k < c.runs.size(); ++k) {
    std::fclose(src[k].f);
    std::remove(c.runs[k].c_str());
  }
  c.runs.clear();
  return err ? -1 : count;
}

RT_API void rt_cooc_free(void* h) {
  Counter* c = static_cast<Counter*>(h);
  for (const auto& r : c->runs) std::remove(r.c_str());
  delete c;
}
