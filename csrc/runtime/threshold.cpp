// Host (CPU) implementation of the threshold / bitmap update codec, same message format as csrc/threshold.hip:
// [0] count, [1] n, [2] threshold bits, [3] type (0 sparse, 1 bitmap), payload from [4].
// Used for CPU tensors (gloo data-parallel runs, tests) and as the reference for the HIP kernels.
#include <cstdint>
#include <cstring>
#include <cstdlib>

#define RT_API extern "C" __attribute__((visibility("default")))

static inline int32_t fbits(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }
static inline float bitsf(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }

RT_API long long rt_threshold_count(const float* r, long long n, float thr) {
  long long c = 0;
  for (long long i = 0; i < n; ++i) c += (r[i] >= thr || r[i] <= -thr);
  return c;
}

RT_API int rt_threshold_encode(float* r, long long n, float thr, int32_t* out, int capacity) {
  int c = 0;
  for (long long i = 0; i < n && c < capacity; ++i) {
    const float v = r[i];
    if (v >= thr) { out[4 + c++] = (int32_t)(i + 1); r[i] = v - thr; }
    else if (v <= -thr) { out[4 + c++] = -(int32_t)(i + 1); r[i] = v + thr; }
  }
  out[0] = c; out[1] = (int32_t)n; out[2] = fbits(thr); out[3] = 0;
  return c;
}

RT_API void rt_threshold_decode(const int32_t* enc, float* target, float scale) {
  const int c = enc[0];
  const float thr = bitsf(enc[2]) * scale;
  for (int j = 0; j < c; ++j) {
    const int32_t e = enc[4 + j];
    const long long i = (long long)(e > 0 ? e : -e) - 1;
    target[i] += e > 0 ? thr : -thr;
  }
}

RT_API int rt_bitmap_encode(float* r, long long n, float thr, int32_t* out) {
  const long long nw = (n + 15) / 16;
  int c = 0;
  for (long long w = 0; w < nw; ++w) {
    uint32_t word = 0;
    for (int k = 0; k < 16; ++k) {
      const long long i = w * 16 + k;
      if (i >= n) break;
      const float v = r[i];
      if (v >= thr) { word |= 1u << (2 * k); r[i] = v - thr; ++c; }
      else if (v <= -thr) { word |= 2u << (2 * k); r[i] = v + thr; ++c; }
    }
    out[4 + w] = (int32_t)word;
  }
  out[0] = c; out[1] = (int32_t)n; out[2] = fbits(thr); out[3] = 1;
  return c;
}

RT_API void rt_bitmap_decode(const int32_t* enc, float* target, float scale) {
  const long long n = enc[1];
  const float thr = bitsf(enc[2]) * scale;
  const long long nw = (n + 15) / 16;
  for (long long w = 0; w < nw; ++w) {
    const uint32_t word = (uint32_t)enc[4 + w];
    if (!word) continue;
    for (int k = 0; k < 16; ++k) {
      const uint32_t b = (word >> (2 * k)) & 3u;
      if (b) target[w * 16 + k] += b == 1u ? thr : -thr;
    }
  }
}
