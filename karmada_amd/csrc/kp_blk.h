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

// Bytes of LDS at the start of every workgroup's dynamic shared memory reserved
// for the block primitives' cross-wave scratch (two alternating 64-slot areas).
constexpr int kRedBytes = 1024;

#if defined(__HIPCC__) || defined(__HIP__)
// DPP lane exchange (GFX9 encodings): quad_perm [1,0,3,2] / [2,3,0,1], row
// half-mirror, row mirror, row_shr:n (0x110+n), row_bcast:15 / :31.
template <int CTRL, int ROWS = 0xF, bool BOUND0 = false, class T>
KP_INLINE T kp_dpp(T old, T v) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = (uint64_t)v, o = (uint64_t)old;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)u, CTRL, ROWS, 0xF, BOUND0);
    const uint32_t hi =
        (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(u >> 32), CTRL, ROWS, 0xF, BOUND0);
    return (T)(((uint64_t)hi << 32) | lo);
  } else {
    return (T)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, BOUND0);
  }
}
template <class T>
KP_INLINE T kp_readlane(T v, int l) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = (uint64_t)v;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return (T)(((uint64_t)hi << 32) | lo);
  } else {
    return (T)__builtin_amdgcn_readlane((int)v, l);
  }
}

// Block policy of one HIP workgroup (wave64 x N waves, N <= 16). Wave-level
// reductions and scans run on DPP (no LDS round trips); the cross-wave step
// writes one slot per wave into one of two alternating scratch areas, so each
// primitive needs a single barrier: a thread can only write an area again after
// passing the next primitive's barrier, which every thread reaches only once it
// has read the previous contents. Every primitive must be called in block-
// uniform control flow, in the same sequence by all threads. Workgroup-scope
// barriers also order the workgroup's exchanges through global memory (k_slow's
// scratch slot): its waves share one CU's vector L1, which the stores write through.
struct GpuBlk {
  int64_t* red;  // kRedBytes of LDS
  mutable int ph = 0;

  KP_INLINE int tid() const { return (int)threadIdx.x; }
  KP_INLINE int nth() const { return (int)blockDim.x; }
  KP_INLINE int lane() const { return (int)(threadIdx.x & 63); }
  KP_INLINE int wid() const { return (int)(threadIdx.x >> 6); }
  KP_INLINE int nwaves() const { return (int)(blockDim.x >> 6); }
  KP_INLINE void sync() const { __syncthreads(); }
  KP_INLINE int64_t* area() const {
    int64_t* a = red + (ph ? 64 : 0);
    ph ^= 1;
    return a;
  }

  // Every lane's v combined over the wave (op associative and commutative,
  // id its identity); the result is wave-uniform.
  template <class T, class Op>
  KP_INLINE T wave_reduce(T v, Op op, T id) const {
    v = op(v, kp_dpp<0xB1>(id, v));
    v = op(v, kp_dpp<0x4E>(id, v));
    v = op(v, kp_dpp<0x141>(id, v));
    v = op(v, kp_dpp<0x140>(id, v));
    return op(op(kp_readlane(v, 0), kp_readlane(v, 16)), op(kp_readlane(v, 32), kp_readlane(v, 48)));
  }
  // Inclusive prefix sum over the wave's lanes.
  template <class T>
  KP_INLINE T wave_incl_scan(T x) const {
    x += kp_dpp<0x111, 0xF, true>((T)0, x);
    x += kp_dpp<0x112, 0xF, true>((T)0, x);
    x += kp_dpp<0x114, 0xF, true>((T)0, x);
    x += kp_dpp<0x118, 0xF, true>((T)0, x);
    x += kp_dpp<0x142, 0xA>((T)0, x);
    x += kp_dpp<0x143, 0xC>((T)0, x);
    return x;
  }
  template <class T, class Op>
  KP_INLINE T reduce(T v, Op op, T id) const {
    v = wave_reduce(v, op, id);
    int64_t* a = area();
    if (lane() == 0) a[wid()] = (int64_t)v;
    sync();
    T r = (T)a[0];
    for (int w = 1; w < nwaves(); w++) r = op(r, (T)a[w]);
    return r;
  }
  // Two reductions for one barrier.
  template <class OpA, class OpB>
  KP_INLINE void reduce2(int64_t& x, OpA opa, int64_t ida, int64_t& y, OpB opb, int64_t idb) const {
    x = wave_reduce(x, opa, ida);
    y = wave_reduce(y, opb, idb);
    int64_t* a = area();
    if (lane() == 0) {
      a[wid()] = x;
      a[16 + wid()] = y;
    }
    sync();
    x = a[0];
    y = a[16];
    for (int w = 1; w < nwaves(); w++) {
      x = opa(x, a[w]);
      y = opb(y, a[16 + w]);
    }
  }
  // Four reductions for one barrier.
  template <class OpA, class OpB, class OpC, class OpD>
  KP_INLINE void reduce4(int64_t& x, OpA opa, int64_t ida, int64_t& y, OpB opb, int64_t idb, int64_t& z, OpC opc,
                         int64_t idc, int64_t& u, OpD opd, int64_t idd) const {
    x = wave_reduce(x, opa, ida);
    y = wave_reduce(y, opb, idb);
    z = wave_reduce(z, opc, idc);
    u = wave_reduce(u, opd, idd);
    int64_t* a = area();
    if (lane() == 0) {
      a[wid()] = x;
      a[16 + wid()] = y;
      a[32 + wid()] = z;
      a[48 + wid()] = u;
    }
    sync();
    x = a[0];
    y = a[16];
    z = a[32];
    u = a[48];
    for (int w = 1; w < nwaves(); w++) {
      x = opa(x, a[w]);
      y = opb(y, a[16 + w]);
      z = opc(z, a[32 + w]);
      u = opd(u, a[48 + w]);
    }
  }
  // This thread's slot base for `mine` entries in a list filled by every wave
  // independently: the wave reserves its total with one LDS atomic on *ctr
  // (zeroed beforehand, behind a barrier). No barrier; slot order across
  // waves is not deterministic, within a wave it follows the lanes.
  KP_INLINE int32_t wave_reserve(int32_t mine, uint32_t* ctr) const {
    const int32_t incl = wave_incl_scan(mine);
    const int32_t tot = kp_readlane(incl, 63);
    int32_t base = 0;
    if (lane() == 63 && tot > 0) base = (int32_t)atomicAdd(ctr, (uint32_t)tot);
    base = kp_readlane(base, 63);
    return base + incl - mine;
  }
  KP_INLINE int64_t sum64(int64_t v) const { return reduce(v, [](int64_t a, int64_t b) { return a + b; }, (int64_t)0); }
  KP_INLINE uint64_t minu64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; }, (uint64_t)~0ull);
  }
  KP_INLINE int64_t max64(int64_t v) const {
    return reduce(v, [](int64_t a, int64_t b) { return a > b ? a : b; }, (int64_t)INT64_MIN);
  }
  KP_INLINE int64_t min64(int64_t v) const {
    return reduce(v, [](int64_t a, int64_t b) { return a < b ? a : b; }, (int64_t)INT64_MAX);
  }
  KP_INLINE void sum2(int64_t& x, int64_t& y) const {
    auto add = [](int64_t a, int64_t b) { return a + b; };
    reduce2(x, add, 0, y, add, 0);
  }
  KP_INLINE void maxsum(int64_t& mx, int64_t& sm) const {
    reduce2(mx, [](int64_t a, int64_t b) { return a > b ? a : b; }, INT64_MIN, sm,
            [](int64_t a, int64_t b) { return a + b; }, 0);
  }
  KP_INLINE bool any(bool p) const {
    const bool w = __ballot(p) != 0;
    int64_t* a = area();
    if (lane() == 0) a[wid()] = w ? 1 : 0;
    sync();
    int64_t r = 0;
    for (int i = 0; i < nwaves(); i++) r |= a[i];
    return r != 0;
  }
  // Exclusive prefix sum of per-thread counts in thread order; *total = sum.
  KP_INLINE int32_t excl_scan(int32_t v, int32_t* total) const {
    const int32_t x = wave_incl_scan(v);
    int64_t* a = area();
    if (lane() == 63) a[wid()] = x;
    sync();
    int32_t base = 0, tot = 0;
    for (int w = 0; w < nwaves(); w++) {
      int32_t s = (int32_t)a[w];
      if (w < wid()) base += s;
      tot += s;
    }
    *total = tot;
    return base + x - v;
  }
  // Histogram search: the first bin i (in ascending index order, or descending
  // when `rev`) whose running sum reaches k (k >= 1); *before = the running sum
  // before it. Wave 0 scans 4 bins per lane. Not found -> the last bin.
  template <class T>
  KP_INLINE int find_bin(const T* hist, int64_t k, int64_t* before, bool rev) const {
    sync();
    int64_t* a = area();
    if (wid() == 0) {
      const int l = lane();
      int64_t v[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int idx = rev ? 255 - (4 * l + q) : 4 * l + q;
        v[q] = (int64_t)hist[idx];
        s += v[q];
      }
      const int64_t incl = wave_incl_scan(s);
      const uint64_t m = __ballot(incl >= k);
      const int first = m ? (int)__builtin_ctzll(m) : 63;
      if (l == first) {
        int64_t c = incl - s;
        int q = 0;
        for (; q < 3; q++) {
          if (c + v[q] >= k) break;
          c += v[q];
        }
        a[0] = rev ? 255 - (4 * l + q) : 4 * l + q;
        a[1] = c;
      }
    }
    sync();
    *before = a[1];
    return (int)a[0];
  }
  KP_INLINE uint64_t and64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a & b; }, (uint64_t)~0ull);
  }
  KP_INLINE uint64_t or64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a | b; }, (uint64_t)0);
  }
  KP_INLINE void andor(uint64_t& an, uint64_t& on) const {
    int64_t x = (int64_t)an, y = (int64_t)on;
    reduce2(x, [](int64_t a, int64_t b) { return a & b; }, (int64_t)-1, y, [](int64_t a, int64_t b) { return a | b; },
            (int64_t)0);
    an = (uint64_t)x;
    on = (uint64_t)y;
  }
  // Stores the feasibility bit of cluster c (c = wave base + lane) into its u64 word.
  KP_INLINE void mask_store(uint64_t* row, int c, bool bit, int W) const {
    const uint64_t m = __ballot(bit);
    if (lane() == 0 && (c >> 6) < W) row[c >> 6] = m;
  }
  // Wave-level primitives (the calling wave only; no workgroup barrier).
  KP_INLINE int wwidth() const { return 64; }
  KP_INLINE uint64_t wballot(bool p) const { return __ballot(p); }
  KP_INLINE uint64_t wlt() const { return (1ull << lane()) - 1; }  // lanes below this one
  template <class T>
  KP_INLINE T wread(T v, int l) const {  // lane l's value (l wave-uniform)
    return kp_readlane(v, l);
  }
  KP_INLINE uint64_t wminu64(uint64_t v) const {  // the wave's minimum (no workgroup barrier)
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; }, (uint64_t)~0ull);
  }
  // Orders this wave's LDS/global accesses: writes made by one lane before it
  // are visible to every lane of the wave after it.
  KP_INLINE void wsync() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // Value of thread 0 to every thread.
  template <class T>
  KP_INLINE T bcast(T v) const {
    int64_t* a = area();
    if (tid() == 0) a[0] = (int64_t)v;
    sync();
    return (T)a[0];
  }
};

// Block policy of ONE wave64 working alone (several such "blocks" share a
// workgroup, each on its own binding and LDS slice): every reduction and scan is
// DPP + readlane, and a sync is the wave's own barrier plus a fence, so no
// workgroup barrier ever stalls the other waves. Same interface as GpuBlk.
struct WaveBlk {
  int64_t* red;  // >= 2 int64 of this wave's LDS (find_bin / bcast)
  KP_INLINE int tid() const { return (int)(threadIdx.x & 63); }
  KP_INLINE int nth() const { return 64; }
  KP_INLINE int lane() const { return tid(); }
  KP_INLINE int wid() const { return 0; }
  KP_INLINE int nwaves() const { return 1; }
  KP_INLINE void sync() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  template <class T, class Op>
  KP_INLINE T wave_reduce(T v, Op op, T id) const {
    v = op(v, kp_dpp<0xB1>(id, v));
    v = op(v, kp_dpp<0x4E>(id, v));
    v = op(v, kp_dpp<0x141>(id, v));
    v = op(v, kp_dpp<0x140>(id, v));
    return op(op(kp_readlane(v, 0), kp_readlane(v, 16)), op(kp_readlane(v, 32), kp_readlane(v, 48)));
  }
  template <class T>
  KP_INLINE T wave_incl_scan(T x) const {
    x += kp_dpp<0x111, 0xF, true>((T)0, x);
    x += kp_dpp<0x112, 0xF, true>((T)0, x);
    x += kp_dpp<0x114, 0xF, true>((T)0, x);
    x += kp_dpp<0x118, 0xF, true>((T)0, x);
    x += kp_dpp<0x142, 0xA>((T)0, x);
    x += kp_dpp<0x143, 0xC>((T)0, x);
    return x;
  }
  // The reductions also order the wave's earlier LDS writes before what follows,
  // as GpuBlk's barrier does.
  template <class T, class Op>
  KP_INLINE T reduce(T v, Op op, T id) const {
    sync();
    return wave_reduce(v, op, id);
  }
  template <class OpA, class OpB>
  KP_INLINE void reduce2(int64_t& x, OpA opa, int64_t ida, int64_t& y, OpB opb, int64_t idb) const {
    sync();
    x = wave_reduce(x, opa, ida);
    y = wave_reduce(y, opb, idb);
  }
  template <class OpA, class OpB, class OpC, class OpD>
  KP_INLINE void reduce4(int64_t& x, OpA opa, int64_t ida, int64_t& y, OpB opb, int64_t idb, int64_t& z, OpC opc,
                         int64_t idc, int64_t& u, OpD opd, int64_t idd) const {
    sync();
    x = wave_reduce(x, opa, ida);
    y = wave_reduce(y, opb, idb);
    z = wave_reduce(z, opc, idc);
    u = wave_reduce(u, opd, idd);
  }
  KP_INLINE int32_t wave_reserve(int32_t mine, uint32_t* ctr) const {
    const int32_t incl = wave_incl_scan(mine);
    const int32_t tot = kp_readlane(incl, 63);
    int32_t base = 0;
    if (lane() == 63 && tot > 0) base = (int32_t)atomicAdd(ctr, (uint32_t)tot);
    base = kp_readlane(base, 63);
    return base + incl - mine;
  }
  KP_INLINE int64_t sum64(int64_t v) const { return reduce(v, [](int64_t a, int64_t b) { return a + b; }, (int64_t)0); }
  KP_INLINE uint64_t minu64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; }, (uint64_t)~0ull);
  }
  KP_INLINE int64_t max64(int64_t v) const {
    return reduce(v, [](int64_t a, int64_t b) { return a > b ? a : b; }, (int64_t)INT64_MIN);
  }
  KP_INLINE int64_t min64(int64_t v) const {
    return reduce(v, [](int64_t a, int64_t b) { return a < b ? a : b; }, (int64_t)INT64_MAX);
  }
  KP_INLINE void sum2(int64_t& x, int64_t& y) const {
    auto add = [](int64_t a, int64_t b) { return a + b; };
    reduce2(x, add, 0, y, add, 0);
  }
  KP_INLINE void maxsum(int64_t& mx, int64_t& sm) const {
    reduce2(mx, [](int64_t a, int64_t b) { return a > b ? a : b; }, INT64_MIN, sm,
            [](int64_t a, int64_t b) { return a + b; }, 0);
  }
  KP_INLINE bool any(bool p) const {
    sync();
    return __ballot(p) != 0;
  }
  KP_INLINE int32_t excl_scan(int32_t v, int32_t* total) const {
    sync();
    const int32_t x = wave_incl_scan(v);
    *total = kp_readlane(x, 63);
    return x - v;
  }
  template <class T>
  KP_INLINE int find_bin(const T* hist, int64_t k, int64_t* before, bool rev) const {
    sync();
    const int l = lane();
    int64_t v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int idx = rev ? 255 - (4 * l + q) : 4 * l + q;
      v[q] = (int64_t)hist[idx];
      s += v[q];
    }
    const int64_t incl = wave_incl_scan(s);
    const uint64_t m = __ballot(incl >= k);
    const int first = m ? (int)__builtin_ctzll(m) : 63;
    int64_t c = incl - s;
    int q = 0;
    for (; q < 3; q++) {
      if (c + v[q] >= k) break;
      c += v[q];
    }
    *before = kp_readlane(c, first);
    const int bin = rev ? 255 - (4 * l + q) : 4 * l + q;
    return kp_readlane(bin, first);
  }
  KP_INLINE uint64_t and64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a & b; }, (uint64_t)~0ull);
  }
  KP_INLINE uint64_t or64(uint64_t v) const {
    return reduce(v, [](uint64_t a, uint64_t b) { return a | b; }, (uint64_t)0);
  }
  KP_INLINE void andor(uint64_t& an, uint64_t& on) const {
    int64_t x = (int64_t)an, y = (int64_t)on;
    reduce2(x, [](int64_t a, int64_t b) { return a & b; }, (int64_t)-1, y, [](int64_t a, int64_t b) { return a | b; },
            (int64_t)0);
    an = (uint64_t)x;
    on = (uint64_t)y;
  }
  KP_INLINE void mask_store(uint64_t* row, int c, bool bit, int W) const {
    const uint64_t m = __ballot(bit);
    if (lane() == 0 && (c >> 6) < W) row[c >> 6] = m;
  }
  KP_INLINE int wwidth() const { return 64; }
  KP_INLINE uint64_t wballot(bool p) const { return __ballot(p); }
  KP_INLINE uint64_t wlt() const { return (1ull << lane()) - 1; }
  KP_INLINE uint64_t wminu64(uint64_t v) const {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; }, (uint64_t)~0ull);
  }
  KP_INLINE void wsync() const { sync(); }
  // lane l's value to every lane; the wave's 32-bit sum (no barrier: registers only)
  template <class T>
  KP_INLINE T wread(T v, int l) const {
    return kp_readlane(v, l);
  }
  KP_INLINE int32_t wsum32(int32_t v) const {
    return wave_reduce(v, [](int32_t a, int32_t b) { return a + b; }, (int32_t)0);
  }
  template <class T>
  KP_INLINE T bcast(T v) const {
    sync();
    return kp_readlane(v, 0);
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
  template <class OpA, class OpB>
  void reduce2(int64_t&, OpA, int64_t, int64_t&, OpB, int64_t) const {}
  template <class OpA, class OpB, class OpC, class OpD>
  void reduce4(int64_t&, OpA, int64_t, int64_t&, OpB, int64_t, int64_t&, OpC, int64_t, int64_t&, OpD, int64_t) const {}
  int32_t wave_reserve(int32_t mine, uint32_t* ctr) const {
    const int32_t b = (int32_t)*ctr;
    *ctr += (uint32_t)mine;
    return b;
  }
  void sum2(int64_t&, int64_t&) const {}
  void maxsum(int64_t&, int64_t&) const {}
  void andor(uint64_t&, uint64_t&) const {}
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
  int wwidth() const { return 1; }
  uint64_t wballot(bool p) const { return p ? 1ull : 0ull; }
  uint64_t wlt() const { return 0; }
  uint64_t wminu64(uint64_t v) const { return v; }
  void wsync() const {}
  template <class T>
  T wread(T v, int) const {
    return v;
  }
  int32_t wsum32(int32_t v) const { return v; }
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

// A block-uniform value moved to a scalar register (the first active lane's
// copy): lets the compiler keep per-binding tables in SGPRs. Identity on the host.
KP_HD inline int32_t kp_uniform(int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(v);
#else
  return v;
#endif
}

// A load at a block-uniform address of read-only global memory (batch pools in
// HBM, written before the launch): through the constant address space, so the
// compiler issues a scalar load instead of a vector load plus readfirstlane.
// Never for LDS-staged pools or data the running kernel writes.
template <class T>
KP_HD inline T kp_ldu(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(4))) T*)(p);
#else
  return *p;
#endif
}

// Atomics on LDS/global memory, usable from both builds.
template <class T>
KP_HD inline T kp_atomic_add(T* p, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}
KP_HD inline uint32_t kp_atomic_and(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAnd(p, v);
#else
  return __atomic_fetch_and(p, v, __ATOMIC_RELAXED);
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
