// N1 native engine: the device / stream / event / graph manager, a stream-ordered caching device
// allocator and the op registry of the kernel library, as a C ABI over the HIP runtime. This is the layer libnd4j's
// CUDA backend provides to the reference (nd4j-cuda: AffinityManager / CudaContext streams, the AtomicAllocator
// memory handler, the NativeOps op table — SURVEY §2.4), written for one process per MI355X:
//
//  * devices: counts, properties (CUs, XCDs, LDS, HBM, clocks), current device, free/total HBM;
//  * streams (normal / high priority), events (timing or not), stream-event waits;
//  * HIP graphs: capture on a stream (global / thread-local / relaxed), instantiate, launch, destroy;
//  * caching allocator, per device:
//      - sizes rounded to 512 B below 1 MB (carved from 2 MB segments) and to 2 MB above (segments of at least
//        64 MB, sized for a 288 GB HBM3E part: fewer, larger hipMallocs), best-fit with block splitting and
//        coalescing of free neighbours inside a segment;
//      - stream-ordered reuse: a freed block is immediately reusable on the stream it was allocated for; blocks also
//        used on other streams (dl4j_rt_record_stream) carry one event per such stream and return to the pool only
//        once those events have completed;
//      - HIP-graph pools: while a stream captures through dl4j_rt_capture_begin, its allocations come from a private
//        pool of that capture (no hipMalloc inside a capture: blocks are pre-reserved or the capture-time request
//        fails with -2), frees during the capture return to that pool, and the pool stays reserved until the graph
//        is destroyed — a replay never sees its memory handed to someone else;
//      - statistics (allocated / reserved / peak / segments / cache hits) and empty_cache;
//  * op registry: name, C signature and entry point of every kernel entry of this library (dlsym on itself), so a
//    binding layer (JavaCPP / ctypes) can enumerate and call ops without a header.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

#define RT_API extern "C" __attribute__((visibility("default")))

namespace {

inline int rc(hipError_t e) { return e == hipSuccess ? 0 : -(int)e - 1000; }

// ------------------------------------------------------------------------------------------------------- allocator
constexpr size_t kSmall = 1 << 20;            // <= 1 MB: small pool
constexpr size_t kSmallSeg = 2 << 20;         // small segments
constexpr size_t kRound = 512;                // small rounding
constexpr size_t kLargeRound = 2 << 20;       // large rounding
constexpr size_t kLargeSeg = 64ull << 20;     // minimum large segment

struct Block {
  int dev = 0;
  hipStream_t stream = nullptr;
  int pool = 0;                // 0 general; >0 graph pool id
  bool small = false;
  char* ptr = nullptr;
  size_t size = 0;
  size_t requested = 0;
  bool allocated = false;
  Block* prev = nullptr;       // neighbours inside the segment
  Block* next = nullptr;
  std::vector<hipStream_t> uses;     // other streams that used this block (record_stream)
  std::vector<hipEvent_t> pending;   // events to complete before reuse after a free
};

struct BlockLess {
  bool operator()(const Block* a, const Block* b) const {
    if (a->pool != b->pool) return a->pool < b->pool;
    if (a->stream != b->stream) return (uintptr_t)a->stream < (uintptr_t)b->stream;
    if (a->size != b->size) return a->size < b->size;
    return (uintptr_t)a->ptr < (uintptr_t)b->ptr;
  }
};

struct Stats {
  long long allocated = 0, reserved = 0, peak = 0, segments = 0, allocs = 0, hits = 0, frees = 0;
};

struct DevAlloc {
  std::mutex mu;
  std::set<Block*, BlockLess> free_small, free_large;
  std::unordered_map<void*, Block*> live;          // ptr -> allocated block
  std::vector<Block*> deferred;                    // freed, waiting for their events
  std::unordered_map<hipStream_t, int> capturing;  // stream -> graph pool id while it captures
  std::set<int> retained_pools;                    // pools of captured graphs still alive
  Stats st;
};

std::mutex g_mu;
DevAlloc* g_dev[64] = {nullptr};
int g_next_pool = 1;

DevAlloc* dev_alloc(int dev) {
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_dev[dev]) g_dev[dev] = new DevAlloc();
  return g_dev[dev];
}

size_t round_size(size_t n) {
  if (n == 0) n = 1;
  if (n <= kSmall) return (n + kRound - 1) / kRound * kRound;
  return (n + kLargeRound - 1) / kLargeRound * kLargeRound;
}

std::set<Block*, BlockLess>& pool_of(DevAlloc* d, bool small) { return small ? d->free_small : d->free_large; }

// events done? (non-blocking); drops completed ones
bool events_done(Block* b) {
  auto& ev = b->pending;
  for (size_t i = 0; i < ev.size();) {
    if (hipEventQuery(ev[i]) == hipSuccess) {
      (void)hipEventDestroy(ev[i]);
      ev[i] = ev.back();
      ev.pop_back();
    } else {
      ++i;
    }
  }
  return ev.empty();
}

void insert_free(DevAlloc* d, Block* b) {
  // coalesce with free neighbours of the same stream / pool (segment-internal)
  for (Block* nb : {b->prev, b->next}) {
    if (!nb || nb->allocated || !nb->pending.empty() || nb->stream != b->stream || nb->pool != b->pool) continue;
    if (!pool_of(d, nb->small).count(nb)) continue;
    pool_of(d, nb->small).erase(nb);
    if (nb == b->prev) {
      nb->size += b->size;
      nb->next = b->next;
      if (b->next) b->next->prev = nb;
      delete b;
      b = nb;
    } else {
      b->size += nb->size;
      b->next = nb->next;
      if (nb->next) nb->next->prev = b;
      delete nb;
    }
  }
  pool_of(d, b->small).insert(b);
}

void process_deferred(DevAlloc* d) {
  for (size_t i = 0; i < d->deferred.size();) {
    Block* b = d->deferred[i];
    if (events_done(b)) {
      d->deferred[i] = d->deferred.back();
      d->deferred.pop_back();
      insert_free(d, b);
    } else {
      ++i;
    }
  }
}

Block* find_free(DevAlloc* d, bool small, int pool, hipStream_t s, size_t size) {
  auto& p = pool_of(d, small);
  Block key;
  key.pool = pool;
  key.stream = s;
  key.size = size;
  key.ptr = nullptr;
  auto it = p.lower_bound(&key);
  if (it == p.end() || (*it)->pool != pool || (*it)->stream != s) return nullptr;
  // do not carve a small request out of a huge cached block (keeps big segments for big tensors)
  if (!small && (*it)->size > size + (size_t)512 * (1 << 20) && size < (size_t)64 * (1 << 20)) return nullptr;
  Block* b = *it;
  p.erase(it);
  return b;
}

Block* split(DevAlloc* d, Block* b, size_t size) {
  const size_t rem = b->size - size;
  if (rem >= (b->small ? kRound : kLargeRound)) {
    Block* r = new Block(*b);
    r->uses.clear();
    r->pending.clear();
    r->ptr = b->ptr + size;
    r->size = rem;
    r->prev = b;
    r->next = b->next;
    if (b->next) b->next->prev = r;
    b->next = r;
    b->size = size;
    insert_free(d, r);
  }
  return b;
}

}  // namespace

// ------------------------------------------------------------------------------------------------------- devices
struct Dl4jDevProps {
  char name[128];
  char arch[64];
  int cus, xcds, warp, max_threads, lds_per_block, clock_khz, mem_clock_khz, bus_width, pci_bus;
  long long total_mem, l2_bytes, lds_per_cu;
};

RT_API int dl4j_rt_device_count() {
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  return e == hipSuccess ? n : (e == hipErrorNoDevice ? 0 : rc(e));
}

RT_API int dl4j_rt_device_props(int dev, Dl4jDevProps* p) {
  hipDeviceProp_t d;
  const hipError_t e = hipGetDeviceProperties(&d, dev);
  if (e != hipSuccess) return rc(e);
  memset(p, 0, sizeof(*p));
  strncpy(p->name, d.name, sizeof(p->name) - 1);
  strncpy(p->arch, d.gcnArchName, sizeof(p->arch) - 1);
  p->cus = d.multiProcessorCount;
  p->xcds = d.multiProcessorCount >= 256 ? 8 : (d.multiProcessorCount >= 128 ? 4 : 1);   // 32 CUs per XCD
  p->warp = d.warpSize;
  p->max_threads = d.maxThreadsPerBlock;
  p->lds_per_block = (int)d.sharedMemPerBlock;
  p->lds_per_cu = (long long)d.maxSharedMemoryPerMultiProcessor;
  p->clock_khz = d.clockRate;
  p->mem_clock_khz = d.memoryClockRate;
  p->bus_width = d.memoryBusWidth;
  p->pci_bus = d.pciBusID;
  p->total_mem = (long long)d.totalGlobalMem;
  p->l2_bytes = (long long)d.l2CacheSize;
  return 0;
}

RT_API int dl4j_rt_set_device(int dev) { return rc(hipSetDevice(dev)); }
RT_API int dl4j_rt_get_device() {
  int d = -1;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}
RT_API int dl4j_rt_device_sync(int dev) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return -1;
  const int r = rc(hipDeviceSynchronize());
  if (cur != dev) (void)hipSetDevice(cur);
  return r;
}
RT_API int dl4j_rt_mem_info(int dev, long long* free_b, long long* total_b) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return -1;
  size_t f = 0, t = 0;
  const int r = rc(hipMemGetInfo(&f, &t));
  if (cur != dev) (void)hipSetDevice(cur);
  *free_b = (long long)f;
  *total_b = (long long)t;
  return r;
}

// ------------------------------------------------------------------------------------------------ streams / events
RT_API int dl4j_rt_stream_create(int dev, int high_priority, void** out) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return -1;
  int lo = 0, hi = 0;
  hipStream_t s = nullptr;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high_priority ? hi : lo);
  if (cur != dev) (void)hipSetDevice(cur);
  *out = (void*)s;
  return rc(e);
}
// Stream restricted to `ncu` of the device's CUs (hardware queue CU mask), spread evenly over the CU index range so
// every XCD / shader engine keeps the same share whichever way the mask bits map onto them. Used for the
// weight-gradient side stream: its long-running blocks then never occupy the remaining CUs, so the short, latency-
// critical kernels of the main chain (BatchNorm folds, elementwise passes) start at once instead of queueing behind
// them. ncu <= 0 or >= the CU count: an unmasked stream.
RT_API int dl4j_rt_stream_create_cumask(int dev, int ncu, void** out) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return -1;
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  hipStream_t s = nullptr;
  if (e == hipSuccess) {
    const int n = p.multiProcessorCount;
    if (ncu <= 0 || ncu >= n) {
      e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    } else {
      uint32_t mask[64] = {0};
      const int words = (n + 31) / 32 < 64 ? (n + 31) / 32 : 64;
      for (int i = 0; i < n && i < 64 * 32; ++i)
        if ((long long)(i + 1) * ncu / n > (long long)i * ncu / n) mask[i >> 5] |= 1u << (i & 31);
      e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
    }
  }
  if (cur != dev) (void)hipSetDevice(cur);
  *out = (void*)s;
  return rc(e);
}
// number of CUs enabled in a stream's mask (the whole device for an unmasked stream)
RT_API int dl4j_rt_stream_cu_count(void* s) {
  uint32_t mask[64] = {0};
  if (hipExtStreamGetCUMask((hipStream_t)s, 64, mask) != hipSuccess) return -1;
  int c = 0;
  for (int i = 0; i < 64; ++i) c += __builtin_popcount(mask[i]);
  return c;
}
RT_API int dl4j_rt_stream_destroy(void* s) { return rc(hipStreamDestroy((hipStream_t)s)); }
RT_API int dl4j_rt_stream_sync(void* s) { return rc(hipStreamSynchronize((hipStream_t)s)); }
RT_API int dl4j_rt_stream_query(void* s) {
  const hipError_t e = hipStreamQuery((hipStream_t)s);
  return e == hipSuccess ? 1 : (e == hipErrorNotReady ? 0 : rc(e));
}
RT_API int dl4j_rt_stream_wait_event(void* s, void* ev) {
  return rc(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)ev, 0));
}
RT_API int dl4j_rt_event_create(int timing, void** out) {
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming);
  *out = (void*)e;
  return rc(r);
}
RT_API int dl4j_rt_event_destroy(void* e) { return rc(hipEventDestroy((hipEvent_t)e)); }
RT_API int dl4j_rt_event_record(void* e, void* s) { return rc(hipEventRecord((hipEvent_t)e, (hipStream_t)s)); }
RT_API int dl4j_rt_event_sync(void* e) { return rc(hipEventSynchronize((hipEvent_t)e)); }
RT_API int dl4j_rt_event_query(void* e) {
  const hipError_t r = hipEventQuery((hipEvent_t)e);
  return r == hipSuccess ? 1 : (r == hipErrorNotReady ? 0 : rc(r));
}
RT_API int dl4j_rt_event_elapsed(void* a, void* b, float* ms) {
  return rc(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
}

// ------------------------------------------------------------------------------------------------------- graphs
// capture on a stream; allocations from that stream go to a private pool of the capture (see allocator notes)
RT_API int dl4j_rt_capture_begin(void* s, int dev, int mode) {
  const hipStreamCaptureMode m =
      mode == 1 ? hipStreamCaptureModeThreadLocal : (mode == 2 ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal);
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    int id;
    {
      std::lock_guard<std::mutex> lk2(g_mu);
      id = g_next_pool++;
    }
    d->capturing[(hipStream_t)s] = id;
  }
  const hipError_t e = hipStreamBeginCapture((hipStream_t)s, m);
  if (e != hipSuccess) {
    std::lock_guard<std::mutex> lk(d->mu);
    d->capturing.erase((hipStream_t)s);
  }
  return rc(e);
}

struct GraphHandle {
  hipGraphExec_t exec;
  hipGraph_t graph;
  int dev;
  int pool;
};

RT_API int dl4j_rt_capture_end(void* s, int dev, void** out) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture((hipStream_t)s, &g);
  int pool = 0;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    auto it = d->capturing.find((hipStream_t)s);
    if (it != d->capturing.end()) {
      pool = it->second;
      d->capturing.erase(it);
      d->retained_pools.insert(pool);
    }
  }
  if (e != hipSuccess) return rc(e);
  hipGraphExec_t ex = nullptr;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(g);
    return rc(e);
  }
  *out = new GraphHandle{ex, g, dev, pool};
  return 0;
}

RT_API int dl4j_rt_graph_launch(void* h, void* s) {
  return rc(hipGraphLaunch(static_cast<GraphHandle*>(h)->exec, (hipStream_t)s));
}

RT_API long long dl4j_rt_graph_node_count(void* h) {
  size_t n = 0;
  return hipGraphGetNodes(static_cast<GraphHandle*>(h)->graph, nullptr, &n) == hipSuccess ? (long long)n : -1;
}

RT_API int dl4j_rt_free_pool(int dev, int pool);

// destroys the graph and releases its private memory pool
RT_API int dl4j_rt_graph_destroy(void* hp) {
  GraphHandle* h = static_cast<GraphHandle*>(hp);
  int r = rc(hipGraphExecDestroy(h->exec));
  const int r2 = rc(hipGraphDestroy(h->graph));
  if (!r) r = r2;
  if (h->pool) dl4j_rt_free_pool(h->dev, h->pool);
  delete h;
  return r;
}

// ------------------------------------------------------------------------------------------------------- allocator
// Returns 0 and *out, -2 when a capturing stream needs memory the capture pool does not hold, or a HIP error code.
RT_API int dl4j_rt_malloc(int dev, long long nbytes, void* stream, void** out) {
  *out = nullptr;
  DevAlloc* d = dev_alloc(dev);
  if (!d || nbytes < 0) return -1;
  const hipStream_t s = (hipStream_t)stream;
  const size_t size = round_size((size_t)nbytes);
  const bool small = size <= kSmall;
  std::lock_guard<std::mutex> lk(d->mu);
  process_deferred(d);
  auto cap = d->capturing.find(s);
  const int pool = cap == d->capturing.end() ? 0 : cap->second;
  Block* b = find_free(d, small, pool, s, size);
  if (b) {
    d->st.hits++;
  } else {
    if (pool) {
      // a capture may not hipMalloc: move a free general block of this stream into the capture's pool
      b = find_free(d, small, 0, s, size);
      if (!b) return -2;
      b->pool = pool;
      d->st.hits++;
    } else {
      const size_t seg = small ? kSmallSeg : std::max(size, kLargeSeg);
      int cur = 0;
      if (hipGetDevice(&cur) != hipSuccess) return -1;
      if (cur != dev) (void)hipSetDevice(dev);
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, seg);
      if (e != hipSuccess) {
        // out of memory: release cached segments and retry once
        (void)hipGetLastError();
        for (auto* pl : {&d->free_small, &d->free_large}) {
          for (auto it = pl->begin(); it != pl->end();) {
            Block* fb = *it;
            if (!fb->prev && !fb->next && fb->pool == 0) {
              (void)hipFree(fb->ptr);
              d->st.reserved -= (long long)fb->size;
              d->st.segments--;
              delete fb;
              it = pl->erase(it);
            } else {
              ++it;
            }
          }
        }
        e = hipMalloc(&p, seg);
      }
      if (cur != dev) (void)hipSetDevice(cur);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        return rc(e);
      }
      b = new Block();
      b->dev = dev;
      b->stream = s;
      b->pool = 0;
      b->small = small;
      b->ptr = (char*)p;
      b->size = seg;
      d->st.reserved += (long long)seg;
      d->st.segments++;
    }
  }
  b = split(d, b, size);
  b->allocated = true;
  b->requested = (size_t)nbytes;
  b->uses.clear();
  d->live[b->ptr] = b;
  d->st.allocated += (long long)b->size;
  d->st.allocs++;
  if (d->st.allocated > d->st.peak) d->st.peak = d->st.allocated;
  *out = b->ptr;
  return 0;
}

// marks `ptr` as used on stream s too: its free waits for the work queued there
RT_API int dl4j_rt_record_stream(int dev, void* ptr, void* s) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  auto it = d->live.find(ptr);
  if (it == d->live.end()) return -1;
  Block* b = it->second;
  if ((hipStream_t)s != b->stream &&
      std::find(b->uses.begin(), b->uses.end(), (hipStream_t)s) == b->uses.end())
    b->uses.push_back((hipStream_t)s);
  return 0;
}

RT_API int dl4j_rt_free(int dev, void* ptr) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  auto it = d->live.find(ptr);
  if (it == d->live.end()) return -1;
  Block* b = it->second;
  d->live.erase(it);
  b->allocated = false;
  d->st.allocated -= (long long)b->size;
  d->st.frees++;
  for (hipStream_t us : b->uses) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
      if (hipEventRecord(e, us) == hipSuccess) b->pending.push_back(e);
      else (void)hipEventDestroy(e);
    }
  }
  b->uses.clear();
  if (b->pending.empty()) insert_free(d, b);
  else d->deferred.push_back(b);
  return 0;
}

// moves every free block of a destroyed graph's pool back to the general pool (its memory is reusable again)
RT_API int dl4j_rt_free_pool(int dev, int pool) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  d->retained_pools.erase(pool);
  int moved = 0;
  for (auto* pl : {&d->free_small, &d->free_large}) {
    std::vector<Block*> mv;
    for (Block* b : *pl)
      if (b->pool == pool) mv.push_back(b);
    for (Block* b : mv) {
      pl->erase(b);
      b->pool = 0;
      insert_free(d, b);
      ++moved;
    }
  }
  for (auto& kv : d->live)
    if (kv.second->pool == pool) kv.second->pool = 0;     // still-live tensors return to the general pool on free
  return moved;
}

// hipFree of every cached segment that is entirely free (general pool); returns bytes released
RT_API long long dl4j_rt_empty_cache(int dev) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  process_deferred(d);
  long long freed = 0;
  for (auto* pl : {&d->free_small, &d->free_large}) {
    for (auto it = pl->begin(); it != pl->end();) {
      Block* b = *it;
      if (!b->prev && !b->next && b->pool == 0) {
        (void)hipFree(b->ptr);
        freed += (long long)b->size;
        d->st.reserved -= (long long)b->size;
        d->st.segments--;
        delete b;
        it = pl->erase(it);
      } else {
        ++it;
      }
    }
  }
  return freed;
}

// stats[7] = allocated, reserved, peak, segments, allocs, cache hits, frees (bytes / counts)
RT_API int dl4j_rt_alloc_stats(int dev, long long* stats) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  const Stats& s = d->st;
  const long long v[7] = {s.allocated, s.reserved, s.peak, s.segments, s.allocs, s.hits, s.frees};
  memcpy(stats, v, sizeof(v));
  return 0;
}

RT_API int dl4j_rt_reset_peak(int dev) {
  DevAlloc* d = dev_alloc(dev);
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  d->st.peak = d->st.allocated;
  return 0;
}

// ------------------------------------------------------------------------------------------------------ DLPack
// Minimal DLPack v0.x structs (dlpack.h layout) so allocator blocks can back framework tensors (torch.from_dlpack):
// the deleter returns the block to this allocator.
struct DLDevice_ { int32_t device_type; int32_t device_id; };
struct DLDataType_ { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor_ {
  void* data;
  DLDevice_ device;
  int32_t ndim;
  DLDataType_ dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor_ {
  DLTensor_ dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor_*);
};
struct DlpCtx {
  int dev;
  void* ptr;
  int64_t shape[8];
  int64_t strides[8];
};

static void dlp_deleter(DLManagedTensor_* t) {
  DlpCtx* c = static_cast<DlpCtx*>(t->manager_ctx);
  dl4j_rt_free(c->dev, c->ptr);
  delete c;
  delete t;
}

// contiguous tensor over a new allocator block: dtype code (0 int, 1 uint, 2 float, 4 bfloat), bits; device type 10
// = kDLROCM. Returns the DLManagedTensor* (caller wraps it in a "dltensor" capsule) or null (*err set).
RT_API void* dl4j_rt_dlpack_empty(int dev, int ndim, const long long* shape, int code, int bits, void* stream,
                                  int* err) {
  *err = -1;
  if (ndim < 0 || ndim > 8) return nullptr;
  long long n = 1;
  for (int i = 0; i < ndim; ++i) n *= shape[i];
  void* p = nullptr;
  const int r = dl4j_rt_malloc(dev, n * (bits / 8), stream, &p);
  if (r) {
    *err = r;
    return nullptr;
  }
  DlpCtx* c = new DlpCtx();
  c->dev = dev;
  c->ptr = p;
  long long st = 1;
  for (int i = ndim - 1; i >= 0; --i) {
    c->shape[i] = shape[i];
    c->strides[i] = st;
    st *= shape[i];
  }
  DLManagedTensor_* t = new DLManagedTensor_();
  t->dl_tensor.data = p;
  t->dl_tensor.device = {10, dev};
  t->dl_tensor.ndim = ndim;
  t->dl_tensor.dtype = {(uint8_t)code, (uint8_t)bits, 1};
  t->dl_tensor.shape = c->shape;
  t->dl_tensor.strides = c->strides;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = c;
  t->deleter = dlp_deleter;
  *err = 0;
  return t;
}

// ---------------------------------------------------------------------------------------------------- op registry
// Every kernel entry point of this library, with its C signature, looked up by name in the loaded library itself.
namespace {
struct OpEntry {
  const char* name;
  const char* sig;
  const char* what;
};
const OpEntry kOps[] = {
    {"dl4j_gemm", "int(int,int,int,int,int,int,void*,ll,int,ll,void*,ll,int,ll,void*,ll,ll,float,float,float*,int,int,void*,int,int,float*,float*,int,stream)", "MFMA GEMM, fused epilogues, split-K"},
    {"dl4j_gemm_simple", "int(int,int,int,int,int,int,void*,ll,ll,ll,void*,ll,ll,ll,void*,ll,ll,float,float,float*,int,int,void*,stream)", "exact-fp32 MFMA GEMM, any strides"},
    {"dl4j_conv_fwd", "int(...)", "implicit-GEMM convolution forward"},
    {"dl4j_conv_fwd_v3", "int(...)", "LDS-DMA implicit-GEMM convolution forward (tile engine)"},
    {"dl4j_conv_bwd_data_s1", "int(...)", "stride-1 convolution backward-data"},
    {"dl4j_conv_bwd_data_1x1", "int(...)", "1x1 strided convolution backward-data"},
    {"dl4j_conv_wrw_v3", "int(...)", "convolution weight gradient (tile engine, slab reduce)"},
    {"dl4j_conv_wrw_halo", "int(...)", "halo-staged conv weight gradient"},
    {"dl4j_stem_conv_fwd", "int(...)", "7x7/2 stem convolution"},
    {"dl4j_dwconv_fwd", "int(...)", "depthwise convolution"},
    {"dl4j_bn_fwd", "int(int,void*,void*,void*,ll,int,float*,float*,float,float,float*,float*,float,float,int,int,float*,float*,u8*,stream)", "BatchNorm forward (+ReLU, +residual, ReLU bitmask)"},
    {"dl4j_bn_fwd_tiles", "int(...)", "BatchNorm forward from conv-epilogue tile statistics"},
    {"dl4j_bn_bwd", "int(int,void*,void*,void*,void*,void*,ll,int,float*,float*,float*,int,float*,u8*,stream)", "BatchNorm backward"},
    {"dl4j_bn_pool_fwd", "int(...)", "fused BN + ReLU + max pool (stem)"},
    {"dl4j_bn_pool_bwd", "int(...)", "fused stem backward"},
    {"dl4j_pool_fwd", "int(...)", "max / avg pooling"},
    {"dl4j_pool_bwd", "int(...)", "pooling backward"},
    {"dl4j_softmax_xent", "int(int,void*,float*,int,int,void*,float*,float*,float,stream)", "fused softmax + MCXENT"},
    {"dl4j_softmax_xent_strided", "int(...)", "softmax + MCXENT on strided labels, padded gradient"},
    {"dl4j_fused_update", "int(...)", "multi-tensor updaters (Sgd..AdaDelta), L1/L2, grad-norm"},
    {"dl4j_lstm_fwd", "int(...)", "whole-sequence LSTM forward"},
    {"dl4j_lstm_bwd", "int(...)", "whole-sequence LSTM backward"},
    {"dl4j_lstm_fwd_coop", "int(...)", "cooperative LSTM forward (RW resident in LDS)"},
    {"dl4j_lstm_bwd_coop", "int(...)", "cooperative LSTM backward"},
    {"dl4j_lstm_pack_rw", "int(int,void*,ll,ll,int,void*,void*,float*,stream)", "recurrent weight packing"},
    {"dl4j_lstm_bwd_prep", "int(...)", "LSTM backward glue"},
    {"dl4j_ln_fwd", "int(...)", "LayerNorm (+residual) forward"},
    {"dl4j_ln_bwd", "int(...)", "LayerNorm backward (+ producing bias gradient)"},
    {"dl4j_gelu", "int(int,void*,void*,void*,ll,stream)", "exact GELU / backward"},
    {"dl4j_attn_fwd", "int(...)", "flash attention forward"},
    {"dl4j_attn_bwd", "int(...)", "flash attention backward"},
    {"dl4j_transform", "int(int,int,void*,void*,ll,float,float,stream)", "ND4J transform / activation ops"},
    {"dl4j_transform_bp", "int(...)", "activation derivatives"},
    {"dl4j_binary", "int(...)", "N-D broadcast binary ops"},
    {"dl4j_reduce", "int(...)", "dimension reductions (sum/mean/var/norms/argmax)"},
    {"dl4j_strided_copy", "int(int,void*,void*,int,ll*,ll*,ll*,ll*,ll,stream)", "strided / padded copies"},
    {"dl4j_strided_copy2", "int(int,int,void*,void*,int,ll*,ll*,ll*,ll*,ll,stream)", "strided copy with cast"},
    {"dl4j_col2im", "int(...)", "col2im gather"},
    {"dl4j_mergemax", "int(...)", "element-wise max over inputs"},
    {"dl4j_channel_sum", "int(int,void*,ll,int,float*,float*,stream)", "column sums (bias gradients)"},
    {"dl4j_threshold_encode", "int(...)", "threshold gradient codec"},
};
}  // namespace

RT_API int dl4j_rt_op_count() { return (int)(sizeof(kOps) / sizeof(kOps[0])); }

// name / signature / description of op i; *fn = its entry point in this library (null if not exported)
RT_API int dl4j_rt_op_info(int i, const char** name, const char** sig, const char** what, void** fn) {
  if (i < 0 || i >= dl4j_rt_op_count()) return -1;
  *name = kOps[i].name;
  *sig = kOps[i].sig;
  *what = kOps[i].what;
  Dl_info self;
  void* h = nullptr;
  if (dladdr((void*)&dl4j_rt_op_count, &self) && self.dli_fname) h = dlopen(self.dli_fname, RTLD_NOW | RTLD_NOLOAD);
  *fn = h ? dlsym(h, kOps[i].name) : nullptr;
  if (h) dlclose(h);
  return 0;
}
