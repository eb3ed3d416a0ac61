// Workspace arena bookkeeping (the native half of deeplearning4j_amd.memory; ND4J MemoryWorkspace semantics used
// by DL4J, NN:nn/graph/ComputationGraph.java:107-136 and NN:nn/multilayer/MultiLayerNetwork.java:126-144):
//   * bump allocation inside one device buffer, aligned, reset per cycle (policyReset BLOCK_LEFT) or when the end
//     is reached (ENDOFBUFFER_REACHED, cyclic);
//   * learning: FIRST_LOOP sizes the buffer from the first cycle's demand, OVER_TIME from the running peak, each
//     with the overallocation ratio; the Python side reallocates the device buffer when `required` grows;
//   * spills: an allocation that does not fit is reported as a spill (policySpill EXTERNAL / REALLOCATE / FAIL
//     decided by the caller) and counted so learning can absorb it next cycle;
//   * generations: every reset/close increments the generation; arrays record the generation they were carved
//     in, which is what SCOPE_PANIC checks (use of an array after its cycle ended).
// The device memory itself is owned by the Python side (one torch allocation per workspace), so this file stays
// host-only and the buffer participates in HIP-graph capture like any other tensor.
#include <cstdint>
#include <mutex>
#include <unordered_map>

#define RT_API extern "C" __attribute__((visibility("default")))

namespace {
struct Arena {
  long long capacity = 0;      // bytes of the current device buffer
  long long offset = 0;        // bump pointer
  long long cycle_peak = 0;    // demand this cycle (incl. spilled bytes)
  long long max_peak = 0;      // over all cycles
  long long spilled = 0;       // spilled bytes this cycle
  long long spilled_total = 0;
  long long alloc_count = 0;
  long long cycles = 0;
  long long generation = 1;
  long long max_bytes = 0;     // 0 = unlimited
  long long alignment = 256;
  double overalloc = 0.0;
  int learning = 0;            // 0 NONE, 1 FIRST_LOOP, 2 OVER_TIME
  int reset_policy = 0;        // 0 BLOCK_LEFT, 1 ENDOFBUFFER_REACHED
  int cycles_before_init = 0;
  bool learned = false;
};
std::mutex g_mu;
std::unordered_map<long long, Arena> g_arenas;
long long g_next = 1;

long long round_up(long long v, long long a) { return (v + a - 1) / a * a; }
}  // namespace

RT_API long long rt_ws_create(long long initial_bytes, long long max_bytes, long long alignment, double overalloc,
                              int learning, int reset_policy, int cycles_before_init) {
  std::lock_guard<std::mutex> lk(g_mu);
  Arena a;
  a.alignment = alignment > 0 ? alignment : 256;
  a.capacity = round_up(initial_bytes > 0 ? initial_bytes : 0, a.alignment);
  a.max_bytes = max_bytes;
  a.overalloc = overalloc;
  a.learning = learning;
  a.reset_policy = reset_policy;
  a.cycles_before_init = cycles_before_init;
  const long long h = g_next++;
  g_arenas[h] = a;
  return h;
}

RT_API void rt_ws_destroy(long long h) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_arenas.erase(h);
}

// Returns 0 = carved at *off, 1 = does not fit (spill; caller allocates externally), -1 = bad handle.
// For ENDOFBUFFER_REACHED a request that does not fit at the end wraps to offset 0 (new generation) if it fits
// the buffer at all.
RT_API int rt_ws_alloc(long long h, long long bytes, long long* off, long long* generation) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(h);
  if (it == g_arenas.end()) return -1;
  Arena& a = it->second;
  const long long need = round_up(bytes > 0 ? bytes : 1, a.alignment);
  a.alloc_count++;
  a.cycle_peak += need;
  if (a.offset + need > a.capacity && a.reset_policy == 1 && need <= a.capacity) {
    a.offset = 0;                       // cyclic: wrap around, earlier arrays of this buffer become invalid
    a.generation++;
  }
  if (a.offset + need <= a.capacity) {
    *off = a.offset;
    *generation = a.generation;
    a.offset += need;
    return 0;
  }
  a.spilled += need;
  a.spilled_total += need;
  *off = -1;
  *generation = a.generation;
  return 1;
}

// End of a cycle (workspace closed / notifyScopeLeft). Returns the capacity the buffer should have for the next
// cycle (learning + overallocation, capped by max_bytes); the caller reallocates when it differs.
RT_API long long rt_ws_cycle_end(long long h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(h);
  if (it == g_arenas.end()) return -1;
  Arena& a = it->second;
  a.cycles++;
  if (a.cycle_peak > a.max_peak) a.max_peak = a.cycle_peak;
  long long want = a.capacity;
  const bool may_learn = a.cycles > a.cycles_before_init;
  if (may_learn && a.learning == 1 && !a.learned) {
    want = round_up((long long)(a.cycle_peak * (1.0 + a.overalloc)), a.alignment);
    a.learned = true;
  } else if (may_learn && a.learning == 2 && a.max_peak > a.capacity) {
    want = round_up((long long)(a.max_peak * (1.0 + a.overalloc)), a.alignment);
  } else if (a.spilled > 0 && a.learning != 0 && may_learn) {
    want = round_up((long long)(a.cycle_peak * (1.0 + a.overalloc)), a.alignment);
  }
  if (a.max_bytes > 0 && want > a.max_bytes) want = a.max_bytes;
  if (a.reset_policy == 0) a.offset = 0;
  a.cycle_peak = 0;
  a.spilled = 0;
  a.generation++;
  return want;
}

RT_API int rt_ws_set_capacity(long long h, long long bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(h);
  if (it == g_arenas.end()) return -1;
  it->second.capacity = round_up(bytes, it->second.alignment);
  it->second.offset = 0;
  it->second.generation++;
  return 0;
}

RT_API long long rt_ws_generation(long long h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(h);
  return it == g_arenas.end() ? -1 : it->second.generation;
}

// out[10]: capacity, offset, cycle_peak, max_peak, spilled, spilled_total, alloc_count, cycles, generation, learned
RT_API int rt_ws_stats(long long h, long long* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_arenas.find(h);
  if (it == g_arenas.end()) return -1;
  const Arena& a = it->second;
  out[0] = a.capacity; out[1] = a.offset; out[2] = a.cycle_peak; out[3] = a.max_peak; out[4] = a.spilled;
  out[5] = a.spilled_total; out[6] = a.alloc_count; out[7] = a.cycles; out[8] = a.generation; out[9] = a.learned;
  return 0;
}
