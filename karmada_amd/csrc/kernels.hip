// kernels.hip — CDNA4 (gfx950) kernels of the batched placement engine and the
// HIP implementation of the device interface (kp_dev.h).
//
// k_pair          one workgroup per binding; each wave64 evaluates 64 consecutive
//                 clusters (coalesced SoA columns), emits their feasibility as one
//                 u64 ballot word and the calAvailableReplicas answer per cluster.
// k_select_all    SEL_ALL bindings: block-parallel assignment (Webster threshold
//                 search, Aggregated cut) over the candidates compacted in LDS.
// k_select_cluster / k_region_a / k_region_b   spread-constraint selection.
// k_slow          persistent workgroups: exact serial emulation for flagged bindings.
// k_compact       per-binding results gathered into CSR order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kp_dev.h"
#include "kp_kernels.h"
#include "kp_sets.h"
#include "kp_top.h"

using namespace kp;

// The kernels are compiled in parallel translation units: the Makefile builds this
// file once per group with -DKP_TU=<group>, and each build defines only its group's
// kernels (the others are declared, so the device interface below, built with
// group 1, launches them by their host stubs). KP_TU=0 (or unset) defines all.
#ifndef KP_TU
#define KP_TU 0
#endif
#define KP_K(G) (KP_TU == 0 || KP_TU == (G))
#if KP_K(1)
#define KP_IMPL1(...) __VA_ARGS__
#else
#define KP_IMPL1(...) ;
#endif
#if KP_K(5)
#define KP_IMPL5(...) __VA_ARGS__
#else
#define KP_IMPL5(...) ;
#endif
#if KP_K(9)
#define KP_IMPL9(...) __VA_ARGS__
#else
#define KP_IMPL9(...) ;
#endif
#if KP_K(10)
#define KP_IMPL10(...) __VA_ARGS__
#else
#define KP_IMPL10(...) ;
#endif
#if KP_K(11)
#define KP_IMPL11(...) __VA_ARGS__
#else
#define KP_IMPL11(...) ;
#endif
#if KP_K(12)
#define KP_IMPL12(...) __VA_ARGS__
#else
#define KP_IMPL12(...) ;
#endif
#if KP_K(13)
#define KP_IMPL13(...) __VA_ARGS__
#else
#define KP_IMPL13(...) ;
#endif

#define KP_SMEM extern __shared__ __align__(16) unsigned char smem[]
// k_select_all: workgroup size bound and minimum waves per SIMD. Its LDS (~53 KB at
// C = 5k with KP_ECAP_MAX = 1024) allows 3 workgroups per CU. 256-thread workgroups
// (3 waves per SIMD, 93 VGPRs, no scratch) ran 3.93 ms at config 3 against 4.01-4.02 ms
// for 512 threads at 6 waves per SIMD (80 VGPRs + 60 B/lane scratch): fewer waves wait
// at each of the binding's barriers.
constexpr size_t kLdsPerCu = 160 * 1024;  // gfx950 LDS per CU
#ifndef KP_PAIR_MIN_WAVES
#define KP_PAIR_MIN_WAVES 1
#endif
#ifndef KP_SEL_MAX_THREADS
#define KP_SEL_MAX_THREADS 256
#endif
#ifndef KP_SEL_MIN_WAVES
#define KP_SEL_MIN_WAVES 3
#endif

extern "C" __global__ void __launch_bounds__(kBlock) k_pair(SnapView s, BatchView bv, const int32_t* list, int b0,
                                                            uint64_t* fmask, int32_t* est, int64_t* score,
                                                            int est_mode, int md_cap)
#if KP_K(1)
{
  KP_SMEM;
  body_pair<EST_GENERIC>(GpuBlk{(int64_t*)smem}, (int)blockIdx.x, smem, s, bv, list, b0, fmask, est, score, est_mode,
                         md_cap);
}
#else
;
#endif
#define KP_PAIR_FAST(NAME, KIND)                                                                              \
  extern "C" __global__ void __launch_bounds__(kBlock, KP_PAIR_MIN_WAVES)                                     \
      NAME(SnapView s, BatchView bv, const int32_t* list, int b0, uint64_t* fmask, int32_t* est, int md_cap)   \
      KP_IMPL1({                                                                                              \
        KP_SMEM;                                                                                              \
        body_pair<KIND>(GpuBlk{(int64_t*)smem}, (int)blockIdx.x, smem, s, bv, list, b0, fmask, est, nullptr, 0, \
                        md_cap);                                                                              \
      })
KP_PAIR_FAST(k_pair_fast, EST_MIXED)
KP_PAIR_FAST(k_pair_fast_summary, EST_SUMMARY)
KP_PAIR_FAST(k_pair_fast_m8, EST_MODEL8)
KP_PAIR_FAST(k_pair_fast_m16, EST_MODEL16)
// Estimator-class rows (kp_filter.h), one instance per estimator kind.
#define KP_EST_CLASS(NAME, KIND)                                                                              \
  extern "C" __global__ void __launch_bounds__(kBlock) NAME(SnapView s, BatchView bv, const int32_t* rep,      \
                                                             int32_t* rows, const int32_t* klist,             \
                                                             const uint64_t* fmask)                           \
      KP_IMPL1({                                                                                              \
        KP_SMEM;                                                                                              \
        const int k = klist ? klist[blockIdx.x] : (int)blockIdx.x;                                            \
        body_est_class<KIND>(GpuBlk{(int64_t*)smem}, k, smem, s, bv, rep, rows, fmask);                       \
      })
KP_EST_CLASS(k_est_class, EST_MIXED)
KP_EST_CLASS(k_est_class_summary, EST_SUMMARY)
KP_EST_CLASS(k_est_class_m8, EST_MODEL8)
KP_EST_CLASS(k_est_class_m16, EST_MODEL16)
// Feasibility rows by bitset algebra: one wave64 per binding, kFilterWaves per workgroup.
constexpr int kFilterWaves = 4;
extern "C" __global__ void __launch_bounds__(64 * kFilterWaves) k_filter(SnapView s, BatchView bv, uint64_t* fmask)
#if KP_K(1)
{
  const int b = (int)(blockIdx.x * kFilterWaves + (threadIdx.x >> 6));
  if (b >= bv.B) return;  // wave-uniform
  body_filter(GpuBlk{nullptr}, b, s, bv, fmask);
}
#else
;
#endif
// A launch over a device-appended list (a.n_dev) runs a grid-stride loop; otherwise
// one workgroup per list entry (one iteration).
// A workgroup without an entry returns before anything else: otherwise the body's
// loop-invariant values, hoisted above the loop and spilled (the spread kernels spill),
// are written to scratch by every lane of an idle grid (r05_pmc_config4: 138 MB per
// launch of k_region_b with an empty fallback list).
#define KP_LIST_LOOP(BODY)                                                       \
  const int n_ = a.n_dev ? (int)*a.n_dev : a.n;                                  \
  if ((int)blockIdx.x >= n_) return;                                             \
  for (int blk = (int)blockIdx.x; blk < n_; blk += (int)gridDim.x) {             \
    BODY;                                                                        \
    __syncthreads();                                                             \
  }
extern "C" __global__ void __launch_bounds__(KP_SEL_MAX_THREADS, KP_SEL_MIN_WAVES) k_select_all(KArgs a)
#if KP_K(2)
{
  KP_SMEM;
  KP_LIST_LOOP(body_select_all(GpuBlk{(int64_t*)smem}, blk, smem, a))
}
#else
;
#endif
// SEL_ALL DynamicWeight / Aggregated over the candidates that can matter (kp_top.h):
// kTopWaves independent waves per workgroup, one binding each, no workgroup barrier.
#ifndef KP_TOP_MIN_WAVES
#define KP_TOP_MIN_WAVES 1
#endif
extern "C" __global__ void __launch_bounds__(64 * kTopWaves, KP_TOP_MIN_WAVES) k_select_top(KArgs a, TopArgs t, int slice)
#if KP_K(4)
{
  KP_SMEM;
  const int w = (int)(threadIdx.x >> 6);
  unsigned char* mine = smem + (size_t)w * (size_t)slice;
  const int blk = (int)blockIdx.x * kTopWaves + w;
  if (blk >= a.n) return;  // wave-uniform: the waves never synchronise with each other
  body_select_top(WaveBlk{(int64_t*)mine}, blk, mine, a, t);
}
#else
;
#endif
// k_select_top over a device-appended list (the capacity-overflow list: n_dev holds its
// length, a.n its capacity): a bounded grid whose waves stride over the list
extern "C" __global__ void __launch_bounds__(64 * kTopWaves) k_select_top_list(KArgs a, TopArgs t, int slice)
#if KP_K(4)
{
  KP_SMEM;
  const int w = (int)(threadIdx.x >> 6);
  unsigned char* mine = smem + (size_t)w * (size_t)slice;
  const int n_ = (int)*a.n_dev;
  int blk = (int)blockIdx.x * kTopWaves + w;
  if (blk >= n_) return;  // wave-uniform
  const int step = (int)gridDim.x * kTopWaves;
  for (; blk < n_; blk += step) {
    body_select_top(WaveBlk{(int64_t*)mine}, blk, mine, a, t);
    __builtin_amdgcn_wave_barrier();  // (the next binding re-carves the slice)
  }
}
#else
;
#endif
// The large-subset bindings: one workgroup each, wave 0 walks, the workgroup divides.
extern "C" __global__ void __launch_bounds__(64 * kTopWgWaves) k_select_top_wg(KArgs a, TopArgs t)
#if KP_K(4)
{
  KP_SMEM;
  body_select_top_wg(GpuBlk{(int64_t*)smem}, WaveBlk{(int64_t*)top_wg_slice(smem)}, (int)blockIdx.x, smem, a, t);
}
#else
;
#endif
// StaticWeight SEL_ALL at class level (kp_kernels.h body_select_static): one wave per
// binding, kStaticWaves independent waves per workgroup.
extern "C" __global__ void __launch_bounds__(64 * kStaticWaves) k_select_static(KArgs a, int slice)
#if KP_K(4)
{
  KP_SMEM;
  const int w = (int)(threadIdx.x >> 6);
  unsigned char* mine = smem + (size_t)w * (size_t)slice;
  const int blk = (int)blockIdx.x * kStaticWaves + w;
  if (blk >= a.n) return;  // wave-uniform: the waves never synchronise with each other
  body_select_static(WaveBlk{(int64_t*)mine}, blk, mine, a);
}
#else
;
#endif
// Spread selections over the class orders (kp_kernels.h body_spread_order): one wave
// per binding, kOrderWaves independent waves per workgroup.
extern "C" __global__ void __launch_bounds__(64 * kOrderWaves) k_spread_order(KArgs a, OrderArgs o, int slice)
#if KP_K(6)
{
  KP_SMEM;
  const int w = (int)(threadIdx.x >> 6);
  unsigned char* mine = smem + (size_t)w * (size_t)slice;
  const int blk = (int)blockIdx.x * kOrderWaves + w;
  if (blk >= a.n) return;  // wave-uniform: the waves never synchronise with each other
  body_spread_order(WaveBlk{(int64_t*)mine}, blk, mine, a, o);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(64 * kOrderWaves) k_region_a_order(KArgs a, RegionOut* rout,
                                                                               int32_t* rstat, int32_t* fb,
                                                                               uint32_t* fb_n, int slice)
#if KP_K(6)
{
  KP_SMEM;
  const int w = (int)(threadIdx.x >> 6);
  unsigned char* mine = smem + (size_t)w * (size_t)slice;
  const int blk = (int)blockIdx.x * kOrderWaves + w;
  if (blk >= a.n) return;  // wave-uniform
  body_region_a_order(WaveBlk{(int64_t*)mine}, blk, mine, a, rout, rstat, fb, fb_n);
}
#else
;
#endif
// Each estimator class's row in (estimate desc, rank asc) order: LDS bitonic sort.
extern "C" __global__ void __launch_bounds__(1024) k_class_order(SnapView s, const int32_t* rows, int P, uint64_t* ord,
                                                                int64_t* tot, int32_t* ok)
#if KP_K(4)
{
  KP_SMEM;
  body_class_order(GpuBlk{(int64_t*)smem}, (int)blockIdx.x, (uint64_t*)(smem + kRedBytes), P, s, rows, ord, tot, ok);
}
#else
;
#endif
// SEL_ALL over streamed candidates: ~15 KB LDS at C = 5k, so LDS no longer bounds
// the workgroups per CU; KP_STREAM_MIN_WAVES waves per SIMD bounds the VGPRs.
#ifndef KP_STREAM_THREADS
#define KP_STREAM_THREADS 256
#endif
#ifndef KP_STREAM_MIN_WAVES
#define KP_STREAM_MIN_WAVES 6
#endif
extern "C" __global__ void __launch_bounds__(KP_STREAM_THREADS, KP_STREAM_MIN_WAVES)
    k_select_all_stream(const KArgs* __restrict__ pa)
#if KP_K(3)
{
  const KArgs& a = *pa;
  KP_SMEM;
  KP_LIST_LOOP(body_select_all_stream(GpuBlk{(int64_t*)smem}, blk, smem, a))
}
#else
;
#endif
// Large snapshots (C ~ 10k): the candidate arrays alone take 8 B per cluster, so a
// single workgroup fits a CU; 1024 threads then keep 16 waves in flight instead of 8.
extern "C" __global__ void __launch_bounds__(1024) k_select_all_wide(KArgs a)
#if KP_K(2)
{
  KP_SMEM;
  KP_LIST_LOOP(body_select_all(GpuBlk{(int64_t*)smem}, blk, smem, a))
}
#else
;
#endif
// Spread-constraint selection kernels: workgroup size (their LDS, ~8 B per cluster
// of gathered candidates, bounds the workgroups per CU; wider ones hide latency).
// Two instances each: 256 threads while the LDS leaves several workgroups per CU
// (C up to ~8.6k; fewer waves per barrier), 512 when it leaves one (wider hides
// latency). 4 / 3 waves per SIMD bound the VGPRs at 128 / 168.
#define KP_SPREAD_KERNELS(SUF, T, MINW, IC, IA, IB)                                                                  \
  extern "C" __global__ void __launch_bounds__(T, MINW) k_select_cluster##SUF(const KArgs* __restrict__ pa, int cap) \
      IC({                                                                                                     \
    const KArgs& a = *pa;                                                                                      \
    KP_SMEM;                                                                                                   \
    KP_LIST_LOOP(body_select_cluster(GpuBlk{(int64_t*)smem}, a.sub ? a.sub[blk] : blk, smem, a, cap))         \
  })                                                                                                           \
  extern "C" __global__ void __launch_bounds__(T, MINW) k_region_a##SUF(const KArgs* __restrict__ pa, RegionOut* rout, \
                                                                      int32_t* rstat)                          \
      IA({                                                                                                     \
        const KArgs& a = *pa;                                                                                  \
        KP_SMEM;                                                                                               \
        KP_LIST_LOOP(body_region_a(GpuBlk{(int64_t*)smem}, a.sub ? a.sub[blk] : blk, smem, a, rout, rstat))   \
      })                                                                                                       \
  extern "C" __global__ void __launch_bounds__(T, MINW) k_region_b##SUF(const KArgs* __restrict__ pa,           \
                                                                      const int32_t* rsel,                     \
                                                                      const int32_t* rnsel,                    \
                                                                      const RegionOut* rout, int cap)          \
      IB({                                                                                                     \
        const KArgs& a = *pa;                                                                                  \
        KP_SMEM;                                                                                               \
        KP_LIST_LOOP(body_region_b(GpuBlk{(int64_t*)smem}, a.sub ? a.sub[blk] : blk, smem, a, rsel, rnsel, rout, cap)) \
      })
KP_SPREAD_KERNELS(, 256, 3, KP_IMPL5, KP_IMPL10, KP_IMPL12)
KP_SPREAD_KERNELS(_wide, 512, 4, KP_IMPL9, KP_IMPL11, KP_IMPL13)
// The same with each thread's DFS arrays in LDS (GroupsLds, R planes), 64 threads per
// workgroup: the private arrays (2.3 KB per thread) lived in scratch.
constexpr int kGroupsLdsThreads = 64;
extern "C" __global__ void __launch_bounds__(kGroupsLdsThreads) k_region_groups_lds(
    const RegionOut* rout, const int32_t* rstat, const BindHdr* hdr, const int32_t* list, int n, int R, int32_t* rsel,
    int32_t* rnsel, uint32_t* nhost)
#if KP_K(6)
{
  KP_SMEM;
  const int j = (int)(blockIdx.x * kGroupsLdsThreads + threadIdx.x);
  if (j >= n) return;
  GroupsLds m{(int32_t*)smem + threadIdx.x,
              (int64_t*)(smem + (size_t)7 * R * kGroupsLdsThreads * 4) + threadIdx.x, R, kGroupsLdsThreads};
  const int32_t k = region_groups_one_lds(m, rout + (size_t)j * R, rstat[j], hdr[list[j]], R, rsel + (size_t)j * R);
  if (k == kGroupsHost) atomicAdd(nhost, 1u);
  rnsel[j] = k;
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_region_groups(const RegionOut* rout, const int32_t* rstat,
                                                                  const BindHdr* hdr, const int32_t* list, int n, int R,
                                                                  int32_t* rsel, int32_t* rnsel, uint32_t* nhost)
#if KP_K(6)
{
  const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (j >= n) return;
  const int32_t k = region_groups_one(rout + (size_t)j * R, rstat[j], hdr[list[j]], R, rsel + (size_t)j * R);
  if (k == kGroupsHost) atomicAdd(nhost, 1u);
  rnsel[j] = k;
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(kSlowBlock) k_slow(const KArgs* __restrict__ pa, unsigned char* scratch,
                                                                size_t slot_bytes, int cap, int lds_area, int lds_sort)
#if KP_K(7)
{
  const KArgs& a = *pa;
  KP_SMEM;
  body_slow(GpuBlk{(int64_t*)smem}, (int)blockIdx.x, (int)gridDim.x, smem, a, scratch, slot_bytes, cap, lds_area, lds_sort);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(64) k_sets(SnapView s, const SetsArgs* A, const int32_t* ranks, const int64_t* off,
                                                       uint64_t n, int64_t* scratch, int32_t* out)
#if KP_K(8)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) body_sets(s, A, ranks, off, i, scratch, out);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(64) k_sets_rows(SnapView s, const SetsArgs* A, const int64_t* off,
                                                            int64_t* scratch, int32_t* row, uint32_t* ovf)
#if KP_K(8)
{
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r < s.C) body_sets_row(s, *A, off, r, scratch, row, ovf);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_rows_from_class(SnapView s, BatchView bv, const int32_t* list,
                                                                  const int32_t* bcls, const int32_t* cls_rows,
                                                                  const uint64_t* fmask, int32_t* est)
#if KP_K(1)
{
  body_rows_from_class(GpuBlk{nullptr}, (int)blockIdx.x, s, bv, list, bcls, cls_rows, fmask, est);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_grades(GradesArgs A)
#if KP_K(8)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < A.n) body_grades(A, i);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_node_est(NodeEstArgs A)
#if KP_K(8)
{
  __shared__ int64_t red[128];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const GpuBlk B{red};
  const int64_t s = B.sum64(i < A.v.n ? (int64_t)(uint32_t)node_replicas(A, i) : 0);
  if (threadIdx.x == 0) atomicAdd(A.sum, (uint32_t)(uint64_t)s);  // mod 2^32: Go's wrapping int32 adds
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_node_match(NodeView v, const ClaimProg* P, uint64_t n,
                                                               uint8_t* match)
#if KP_K(8)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) body_node_match(v, P, i, match);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(64) k_node_sets(const NodeSetsArgs* A)
#if KP_K(8)
{
  __shared__ int64_t red[2];
  node_sets(WaveBlk{red}, *A);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(256) k_reasons(SnapView s, BatchView bv, int b0, uint64_t n, uint32_t* out)
#if KP_K(8)
{
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    body_reasons(s, bv, b0, i, out);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(kOffThreads) k_offsets_a(const int32_t* status, const uint32_t* count, int n,
                                                                    uint64_t* offsets, uint64_t* part)
#if KP_K(8)
{
  __shared__ int64_t red[128];
  body_offsets_a(GpuBlk{red}, (int)blockIdx.x, status, count, n, offsets, part);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(kOffThreads) k_offsets_b(int n, uint64_t* offsets, const uint64_t* part)
#if KP_K(8)
{
  __shared__ int64_t red[128];
  body_offsets_b(GpuBlk{red}, (int)blockIdx.x, (int)gridDim.x, n, offsets, part);
}
#else
;
#endif
extern "C" __global__ void __launch_bounds__(64) k_compact(const uint64_t* start, const uint32_t* count,
                                                           const uint64_t* offsets, const uint32_t* in_idx,
                                                           const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep,
                                                           int n, const uint32_t* perm, uint32_t* h_idx,
                                                           int32_t* h_rep, uint64_t h_cap)
#if KP_K(8)
{
  __shared__ int64_t red[8];
  body_compact(GpuBlk{red}, (int)blockIdx.x, start, count, offsets, in_idx, in_rep, out_idx, out_rep, n, perm, h_idx,
               h_rep, h_cap);
}
#else
;
#endif

// ---------------------------------------------------------------------------
// Device interface (HIP)
// ---------------------------------------------------------------------------
#if KP_K(1)
namespace kp {
namespace dev {

namespace {
thread_local hipError_t g_err = hipSuccess;
// Threads per SEL_ALL workgroup (LDS, not threads, bounds the workgroups per CU,
// so wider workgroups add latency hiding). KP_SEL_THREADS overrides for tuning.
int sel_threads() {
  static int n = [] {
    const char* e = getenv("KP_SEL_THREADS");
    int v = e ? atoi(e) : KP_SEL_MAX_THREADS;
    return (v == 128 || v == 256 || v == 512) && v <= KP_SEL_MAX_THREADS ? v : KP_SEL_MAX_THREADS;
  }();
  return n;
}
int chk(hipError_t e) {
  if (e != hipSuccess) {
    g_err = e;
    return -1;
  }
  return 0;
}
}  // namespace

int device_count() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}
int set_device(int d) { return chk(hipSetDevice(d)); }
size_t max_lds_per_block(int d) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, d) != hipSuccess || v <= 0) return 65536;
  return (size_t)v;
}
const char* last_error() { return hipGetErrorString(g_err); }

int stream_create(stream_t* s) {
  hipStream_t h;
  if (chk(hipStreamCreateWithFlags(&h, hipStreamNonBlocking))) return -1;
  *s = h;
  return 0;
}
void stream_destroy(stream_t s) { (void)hipStreamDestroy((hipStream_t)s); }
// KP_SYNC_BLOCK=1: host waits sleep in the driver (hipEventBlockingSync) instead of polling,
// so lane threads waiting on their batches leave the process's CPU quota to the others
static bool blocking_sync() {
  static const bool on = [] {
    const char* v = getenv("KP_SYNC_BLOCK");
    return v && atoi(v) != 0;
  }();
  return on;
}
int sync(stream_t s) {
  if (!blocking_sync()) return chk(hipStreamSynchronize((hipStream_t)s));
  thread_local hipEvent_t ev = nullptr;  // (one per host thread, kept for the process)
  if (!ev && chk(hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming))) return -1;
  if (chk(hipEventRecord(ev, (hipStream_t)s))) return -1;
  return chk(hipEventSynchronize(ev));
}
int event_create(event_t* e) {
  hipEvent_t h;
  if (chk(hipEventCreateWithFlags(&h, blocking_sync() ? hipEventBlockingSync : hipEventDefault))) return -1;
  *e = h;
  return 0;
}
void event_destroy(event_t e) { (void)hipEventDestroy((hipEvent_t)e); }
int event_record(event_t e, stream_t s) { return chk(hipEventRecord((hipEvent_t)e, (hipStream_t)s)); }
int event_sync(event_t e) { return chk(hipEventSynchronize((hipEvent_t)e)); }
int stream_wait(stream_t s, event_t e) { return chk(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0)); }
float event_ms(event_t a, event_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, (hipEvent_t)a, (hipEvent_t)b) != hipSuccess) return -1.f;
  return ms;
}

int alloc(void** p, size_t bytes) { return chk(hipMalloc(p, bytes)); }
void release(void* p) { (void)hipFree(p); }
// (mapped and coherent: the result CSR is written into it by k_compact, uncached, and read
// by the host after the stream's synchronisation)
int host_alloc(void** p, size_t bytes) {
  return chk(hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocCoherent));
}
void host_release(void* p) {
  if (p) (void)hipHostFree(p);
}
int h2d(void* dst, const void* src, size_t bytes, stream_t s) {
  return bytes ? chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)s)) : 0;
}
int d2h(void* dst, const void* src, size_t bytes, stream_t s) {
  return bytes ? chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)s)) : 0;
}
int peer_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, stream_t s) {
  if (!bytes) return 0;
  if (dst_dev == src_dev) return chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s));
  return chk(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, (hipStream_t)s));
}
int fill(void* dst, int value, size_t bytes, stream_t s) {
  return bytes ? chk(hipMemsetAsync(dst, value, bytes, (hipStream_t)s)) : 0;
}

int pair(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* list, int b0, int nb, uint64_t* fmask,
         int32_t* est, int64_t* score, int est_mode, int md_cap, size_t smem, int fast) {
  if (nb <= 0) return 0;
  auto* kf = fast == EST_MIXED     ? k_pair_fast
             : fast == EST_SUMMARY ? k_pair_fast_summary
             : fast == EST_MODEL8  ? k_pair_fast_m8
             : fast == EST_MODEL16 ? k_pair_fast_m16
                                   : nullptr;
  if (fast != EST_GENERIC && !kf) return chk(hipErrorInvalidValue);
  if (kf)
    hipLaunchKernelGGL(kf, dim3(nb), dim3(kBlock), smem, (hipStream_t)st, s, bv, list, b0, fmask, est, md_cap);
  else
    hipLaunchKernelGGL(k_pair, dim3(nb), dim3(kBlock), smem, (hipStream_t)st, s, bv, list, b0, fmask, est, score,
                       est_mode, md_cap);
  return chk(hipGetLastError());
}

int est_class(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* rep, int n_rows, int32_t* rows,
              int fast, const int32_t* klist, const uint64_t* fmask) {
  if (n_rows <= 0) return 0;
  auto* k = fast == EST_MIXED     ? k_est_class
            : fast == EST_SUMMARY ? k_est_class_summary
            : fast == EST_MODEL8  ? k_est_class_m8
            : fast == EST_MODEL16 ? k_est_class_m16
                                  : nullptr;
  if (!k) return chk(hipErrorInvalidValue);
  // (the feasible mode compacts the representative's feasible clusters into LDS)
  const size_t smem = kRedBytes + 4 * kTmplDense + (fmask ? 4 * (size_t)s.Cp : 0);
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  hipLaunchKernelGGL(k, dim3(n_rows), dim3(kBlock), smem, (hipStream_t)st, s, bv, rep, rows, klist, fmask);
  return chk(hipGetLastError());
}

int filter(stream_t st, const SnapView& s, const BatchView& bv, uint64_t* fmask) {
  if (bv.B <= 0 || s.W <= 0) return 0;
  hipLaunchKernelGGL(k_filter, dim3((bv.B + kFilterWaves - 1) / kFilterWaves), dim3(64 * kFilterWaves), 0,
                     (hipStream_t)st, s, bv, fmask);
  return chk(hipGetLastError());
}

// one workgroup per list entry, or over a device-appended list a persistent grid
static int spread_grid(const KArgs& a, const SelectExtra& x) {
  const int g = a.n_dev ? std::min(a.n, 256 * 4) : a.n;
  return a.n_dev && x.list_grid > 0 ? std::min(g, x.list_grid) : g;
}

int select(stream_t st, int which, const KArgs& a, size_t smem, int cap, const SelectExtra& x) {
  if (a.n <= 0) return 0;
  hipStream_t h = (hipStream_t)st;
  const KArgs* pa = x.dargs;  // (the kernels other than k_select_all read their KArgs from it)
  if (!pa && which != SEL_LAUNCH_ALL) return chk(hipErrorInvalidValue);
  switch (which) {
    case SEL_LAUNCH_ALL: {
      // a device-appended list: a persistent grid of a few workgroups per CU
      int g = a.n_dev ? std::min(a.n, 256 * 4) : a.n;
      if (a.n_dev && x.list_grid > 0) g = std::min(g, x.list_grid);
      if (smem > kLdsPerCu / 2 && !getenv("KP_SEL_THREADS"))  // one workgroup per CU: go wide
        hipLaunchKernelGGL(k_select_all_wide, dim3(g), dim3(1024), smem, h, a);
      else
        hipLaunchKernelGGL(k_select_all, dim3(g), dim3(sel_threads()), smem, h, a);
      break;
    }
    case SEL_LAUNCH_ALL_STREAM:
      hipLaunchKernelGGL(k_select_all_stream,
                         dim3(a.n_dev ? std::min(std::min(a.n, 256 * 8), x.list_grid > 0 ? x.list_grid : a.n) : a.n),
                         dim3(KP_STREAM_THREADS),
                         smem, h, pa);
      break;
    case SEL_LAUNCH_CLUSTER:
      if (smem > kLdsPerCu / 2)
        hipLaunchKernelGGL(k_select_cluster_wide, dim3(spread_grid(a, x)), dim3(512), smem, h, pa, cap);
      else
        hipLaunchKernelGGL(k_select_cluster, dim3(spread_grid(a, x)), dim3(256), smem, h, pa, cap);
      break;
    case SEL_LAUNCH_REGION_A:
      if (smem > kLdsPerCu / 2)
        hipLaunchKernelGGL(k_region_a_wide, dim3(spread_grid(a, x)), dim3(512), smem, h, pa, x.rout, x.rstat);
      else
        hipLaunchKernelGGL(k_region_a, dim3(spread_grid(a, x)), dim3(256), smem, h, pa, x.rout, x.rstat);
      break;
    case SEL_LAUNCH_REGION_B:
      if (smem > kLdsPerCu / 2)
        hipLaunchKernelGGL(k_region_b_wide, dim3(spread_grid(a, x)), dim3(512), smem, h, pa, x.rsel, x.rnsel, x.rout, cap);
      else
        hipLaunchKernelGGL(k_region_b, dim3(spread_grid(a, x)), dim3(256), smem, h, pa, x.rsel, x.rnsel, x.rout, cap);
      break;
    case SEL_LAUNCH_SLOW:
      if (smem > 65536 &&
          chk(hipFuncSetAttribute((const void*)k_slow, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
        return -1;
      hipLaunchKernelGGL(k_slow, dim3(x.grid), dim3(kSlowBlock), smem, h, pa, x.scratch, x.slot_bytes, cap, x.lds_area,
                         x.lds_sort);
      break;
    default:
      return chk(hipErrorInvalidValue);
  }
  return chk(hipGetLastError());
}

int class_order(stream_t st, const SnapView& s, const int32_t* rows, int n_rows, uint64_t* ord, int64_t* tot,
                int32_t* ok) {
  if (n_rows <= 0 || s.C <= 0) return 0;
  int P = 1;
  while (P < s.C) P <<= 1;
  const size_t smem = kRedBytes + 8 * (size_t)P;
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k_class_order, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  hipLaunchKernelGGL(k_class_order, dim3(n_rows), dim3(1024), smem, (hipStream_t)st, s, rows, P, ord, tot, ok);
  return chk(hipGetLastError());
}

int select_top(stream_t st, const KArgs& a, const TopArgs& t, size_t slice, int max_grid) {
  if (a.n <= 0) return 0;
  const size_t smem = slice * kTopWaves;
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k_select_top, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  int grid = (a.n + kTopWaves - 1) / kTopWaves;
  if (a.n_dev) {  // the list launch
    if (max_grid > 0 && grid > max_grid) grid = max_grid;
    if (smem > 65536 &&
        chk(hipFuncSetAttribute((const void*)k_select_top_list, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
      return -1;
    hipLaunchKernelGGL(k_select_top_list, dim3(grid), dim3(64 * kTopWaves), smem, (hipStream_t)st, a, t, (int)slice);
    return chk(hipGetLastError());
  }
  hipLaunchKernelGGL(k_select_top, dim3(grid), dim3(64 * kTopWaves), smem,
                     (hipStream_t)st, a, t, (int)slice);
  return chk(hipGetLastError());
}

int select_top_wg(stream_t st, const KArgs& a, const TopArgs& t, size_t smem) {
  if (a.n <= 0) return 0;
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k_select_top_wg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  hipLaunchKernelGGL(k_select_top_wg, dim3(a.n), dim3(64 * kTopWgWaves), smem, (hipStream_t)st, a, t);
  return chk(hipGetLastError());
}

int spread_order(stream_t st, const KArgs& a, const OrderArgs& o, size_t slice) {
  if (a.n <= 0) return 0;
  const size_t smem = slice * kOrderWaves;
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k_spread_order, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  hipLaunchKernelGGL(k_spread_order, dim3((a.n + kOrderWaves - 1) / kOrderWaves), dim3(64 * kOrderWaves), smem,
                     (hipStream_t)st, a, o, (int)slice);
  return chk(hipGetLastError());
}

int region_a_order(stream_t st, const KArgs& a, RegionOut* rout, int32_t* rstat, int32_t* fb, uint32_t* fb_n,
                   size_t slice) {
  if (a.n <= 0) return 0;
  const size_t smem = slice * kOrderWaves;
  hipLaunchKernelGGL(k_region_a_order, dim3((a.n + kOrderWaves - 1) / kOrderWaves), dim3(64 * kOrderWaves), smem,
                     (hipStream_t)st, a, rout, rstat, fb, fb_n, (int)slice);
  return chk(hipGetLastError());
}

int select_static(stream_t st, const KArgs& a, size_t slice) {
  if (a.n <= 0) return 0;
  const size_t smem = slice * kStaticWaves;
  if (smem > 65536 &&
      chk(hipFuncSetAttribute((const void*)k_select_static, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)))
    return -1;
  hipLaunchKernelGGL(k_select_static, dim3((a.n + kStaticWaves - 1) / kStaticWaves), dim3(64 * kStaticWaves), smem,
                     (hipStream_t)st, a, (int)slice);
  return chk(hipGetLastError());
}

int region_groups(stream_t st, const RegionOut* rout, const int32_t* rstat, const BindHdr* hdr, const int32_t* list,
                  int n, int R, int32_t* rsel, int32_t* rnsel, uint32_t* nhost) {
  if (n <= 0) return 0;
  const size_t lds = groups_lds_bytes(R, kGroupsLdsThreads);
  if (R >= 1 && lds <= 65536 && !getenv("KP_GROUPS_PRIV"))
    hipLaunchKernelGGL(k_region_groups_lds, dim3((n + kGroupsLdsThreads - 1) / kGroupsLdsThreads), dim3(kGroupsLdsThreads),
                       lds, (hipStream_t)st, rout, rstat, hdr, list, n, R, rsel, rnsel, nhost);
  else
    hipLaunchKernelGGL(k_region_groups, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)st, rout, rstat, hdr, list, n,
                       R, rsel, rnsel, nhost);
  return chk(hipGetLastError());
}

int component_sets(stream_t st, const SnapView& s, const SetsArgs* A, const int32_t* ranks, const int64_t* off,
                   uint64_t n, int64_t* scratch, int32_t* out) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_sets, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)st, s, A, ranks, off, n, scratch, out);
  return chk(hipGetLastError());
}

int sets_rows(stream_t st, const SnapView& s, const SetsArgs* A, const int64_t* off, int64_t* scratch, int32_t* row,
              uint32_t* ovf) {
  if (s.C <= 0) return 0;
  hipLaunchKernelGGL(k_sets_rows, dim3((unsigned)((s.C + 63) / 64)), dim3(64), 0, (hipStream_t)st, s, A, off, scratch,
                     row, ovf);
  return chk(hipGetLastError());
}

int rows_from_class(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* list, int n,
                    const int32_t* bcls, const int32_t* cls_rows, const uint64_t* fmask, int32_t* est) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_rows_from_class, dim3(n), dim3(256), 0, (hipStream_t)st, s, bv, list, bcls, cls_rows, fmask,
                     est);
  return chk(hipGetLastError());
}

int grades(stream_t st, const GradesArgs& A) {
  if (A.n == 0) return 0;
  hipLaunchKernelGGL(k_grades, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, (hipStream_t)st, A);
  return chk(hipGetLastError());
}

int node_est(stream_t st, const NodeEstArgs& A) {
  if (A.v.n == 0) return 0;
  hipLaunchKernelGGL(k_node_est, dim3((unsigned)((A.v.n + 255) / 256)), dim3(256), 0, (hipStream_t)st, A);
  return chk(hipGetLastError());
}

int node_match(stream_t st, const NodeView& v, const ClaimProg* P, int K, uint8_t* match) {
  const uint64_t n = v.n * (uint64_t)K;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_node_match, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st, v, P, n, match);
  return chk(hipGetLastError());
}

int node_sets(stream_t st, const NodeSetsArgs* A) {
  hipLaunchKernelGGL(k_node_sets, dim3(1), dim3(64), 0, (hipStream_t)st, A);
  return chk(hipGetLastError());
}

int reasons(stream_t st, const SnapView& s, const BatchView& bv, int b0, int nb, uint32_t* out) {
  const uint64_t n = (uint64_t)nb * (uint64_t)s.C;
  if (n == 0) return 0;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_reasons, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)st, s, bv, b0, n, out);
  return chk(hipGetLastError());
}

int offsets(stream_t st, const int32_t* status, const uint32_t* count, int n, uint64_t* off, uint64_t* part) {
  if (n <= 0) return 0;
  const int nb = (n + kOffChunk - 1) / kOffChunk;
  hipLaunchKernelGGL(k_offsets_a, dim3(nb), dim3(kOffThreads), 0, (hipStream_t)st, status, count, n, off, part);
  hipLaunchKernelGGL(k_offsets_b, dim3(nb), dim3(kOffThreads), 0, (hipStream_t)st, n, off, (const uint64_t*)part);
  return chk(hipGetLastError());
}

int compact(stream_t st, const uint64_t* start, const uint32_t* count, const uint64_t* offsets, const uint32_t* in_idx,
            const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n, const uint32_t* perm, uint32_t* h_idx,
            int32_t* h_rep, uint64_t h_cap) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_compact, dim3(n), dim3(64), 0, (hipStream_t)st, start, count, offsets, in_idx, in_rep, out_idx,
                     out_rep, n, perm, h_idx, h_rep, h_cap);
  return chk(hipGetLastError());
}
int host_device_ptr(void* host, void** dev) { return chk(hipHostGetDevicePointer(dev, host, 0)); }

}  // namespace dev
}  // namespace kp
#endif  // KP_K(1)
