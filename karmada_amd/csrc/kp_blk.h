// kp_blk.h — block-execution policies for the kernel bodies in kp_algo.h.
//
// GpuBlk: one HIP workgroup (wave64 x N waves) with wave-shuffle reductions and
// a small LDS scratch for cross-wave combination.
// CpuBlk: a 1-thread "workgroup" used only by the CPU unit-test build of the
// kernel bodies (tests/, libkp_cpusim.so); it is never linked into libkp.so.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define KP_HD __host__ __device__
#define KP_DEV __device__
#define KP_INLINE __device__ __forceinline__
#else
#define KP_HD
#define KP_DEV
#define KP_INLINE inline
#endif
// Forced inlining for the block-parallel helpers: an outlined call in a kernel
// costs a stack frame (scratch) and spills around every call site.
#define KP_FI KP_HD __attribute__((always_inline)) inline
#if defined(__HIPCC__) || defined(__HIP__)
#define KP_UNROLL _Pragma("unroll")
#else
#define KP_UNROLL
#endif

namespace kp {

#if defined(__HIPCC__) || defined(__HIP__)
struct GpuBlk {
  int64_t* red;  // >= 32 int64 of LDS

  KP_INLINE int tid() const { return (int)threadIdx.x; }
  KP_INLINE int nth() const { return (int)blockDim.x; }
  KP_INLINE int lane() const { return (int)(threadIdx.x & 63); }
  KP_INLINE int wid() const { return (int)(threadIdx.x >> 6); }
  KP_INLINE int nwaves() const { return (int)(blockDim.x >> 6); }
  KP_INLINE void sync() const { __syncthreads(); }

  template <class T, class Op>
  KP_INLINE T wave_reduce(T v, Op op) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, (T)__shfl_xor(v, o, 64));
    return v;
  }
  template <class T, class Op>
  KP_INLINE T reduce(T v, Op op) const {
    v = wave_reduce(v, op);
    sync();
    if (lane() == 0) red[wid()] = (int64_t)v;
    sync();
    T r = (T)red[0];
    for (int w = 1; w < nwaves(); w++) r = op(r, (T)red[w]);
    sync();
    return r;
  }
  KP_INLINE int64_t sum64(int64_t v) const { return reduce(v, [](int64_t a, int64_t b) { return a + b; }); }
  KP_INLINE uint64_t minu64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; });
  }
  KP_INLINE int64_t max64(int64_t v) const { return reduce(v, [](int64_t a, int64_t b) { return a > b ? a : b; }); }
  KP_INLINE int64_t min64(int64_t v) const { return reduce(v, [](int64_t a, int64_t b) { return a < b ? a : b; }); }
  KP_INLINE bool any(bool p) const { return sum64(p ? 1 : 0) != 0; }
  // Exclusive prefix sum of per-thread counts in thread order; *total = sum.
  KP_INLINE int32_t excl_scan(int32_t v, int32_t* total) const {
    int32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int32_t y = __shfl_up(x, o, 64);
      if (lane() >= o) x += y;
    }
    sync();
    if (lane() == 63) red[wid()] = x;
    sync();
    int32_t base = 0, tot = 0;
    for (int w = 0; w < nwaves(); w++) {
      int32_t s = (int32_t)red[w];
      if (w < wid()) base += s;
      tot += s;
    }
    sync();
    *total = tot;
    return base + x - v;
  }
  // Histogram search: the first bin i (in ascending index order, or descending
  // when `rev`) whose running sum reaches k (k >= 1); *before = the running sum
  // before it. Wave 0 scans 4 bins per lane. Not found -> the last bin.
  template <class T>
  KP_INLINE int find_bin(const T* hist, int64_t k, int64_t* before, bool rev) const {
    sync();
    if (wid() == 0) {
      const int l = lane();
      int64_t v[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int idx = rev ? 255 - (4 * l + q) : 4 * l + q;
        v[q] = (int64_t)hist[idx];
        s += v[q];
      }
      int64_t incl = s;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(incl, o, 64);
        if (l >= o) incl += y;
      }
      const uint64_t m = __ballot(incl >= k);
      const int first = m ? (int)__builtin_ctzll(m) : 63;
      if (l == first) {
        int64_t c = incl - s;
        int q = 0;
        for (; q < 3; q++) {
          if (c + v[q] >= k) break;
          c += v[q];
        }
        red[0] = rev ? 255 - (4 * l + q) : 4 * l + q;
        red[1] = c;
      }
    }
    sync();
    const int bin = (int)red[0];
    *before = red[1];
    sync();
    return bin;
  }
  KP_INLINE uint64_t and64(uint64_t v) const {
    return (uint64_t)reduce((int64_t)v, [](int64_t a, int64_t b) { return (int64_t)((uint64_t)a & (uint64_t)b); });
  }
  KP_INLINE uint64_t or64(uint64_t v) const {
    return (uint64_t)reduce((int64_t)v, [](int64_t a, int64_t b) { return (int64_t)((uint64_t)a | (uint64_t)b); });
  }
  // Stores the feasibility bit of cluster c (c = wave base + lane) into its u64 word.
  KP_INLINE void mask_store(uint64_t* row, int c, bool bit, int W) const {
    const uint64_t m = __ballot(bit);
    if (lane() == 0 && (c >> 6) < W) row[c >> 6] = m;
  }
  // Value of thread 0 to every thread.
  template <class T>
  KP_INLINE T bcast(T v) const {
    sync();
    if (tid() == 0) red[0] = (int64_t)v;
    sync();
    T r = (T)red[0];
    sync();
    return r;
  }
};
#endif

struct CpuBlk {
  int64_t* red;
  int tid() const { return 0; }
  int nth() const { return 1; }
  int lane() const { return 0; }
  int wid() const { return 0; }
  int nwaves() const { return 1; }
  void sync() const {}
  int64_t sum64(int64_t v) const { return v; }
  uint64_t minu64(uint64_t v) const { return v; }
  int64_t max64(int64_t v) const { return v; }
  int64_t min64(int64_t v) const { return v; }
  bool any(bool p) const { return p; }
  int32_t excl_scan(int32_t v, int32_t* total) const {
    *total = v;
    return 0;
  }
  template <class T>
  T bcast(T v) const {
    return v;
  }
  template <class T>
  int find_bin(const T* hist, int64_t k, int64_t* before, bool rev) const {
    int64_t c = 0;
    for (int i = 0; i < 256; i++) {
      const int idx = rev ? 255 - i : i;
      if (c + (int64_t)hist[idx] >= k || i == 255) {
        *before = c;
        return idx;
      }
      c += (int64_t)hist[idx];
    }
    return 0;
  }
  uint64_t and64(uint64_t v) const { return v; }
  uint64_t or64(uint64_t v) const { return v; }
  void mask_store(uint64_t* row, int c, bool bit, int W) const {
    if ((c >> 6) >= W) return;
    if ((c & 63) == 0) row[c >> 6] = 0;
    if (bit) row[c >> 6] |= 1ull << (c & 63);
  }
};

// Atomics on LDS/global memory, usable from both builds.
template <class T>
KP_HD inline T kp_atomic_add(T* p, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}
KP_HD inline uint32_t kp_atomic_or(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicOr(p, v);
#else
  return __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}
KP_HD inline unsigned long long kp_atomic_min_u64(unsigned long long* p, unsigned long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicMin(p, v);
#else
  unsigned long long o = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < o && !__atomic_compare_exchange_n(p, &o, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
  return o;
#endif
}

}  // namespace kp
