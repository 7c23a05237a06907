// kp_launch.h — arguments shared by the kernels and their launchers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "kp_layout.h"
#include "kp_paths.h"

namespace kp {

struct KArgs {
  SnapView s;
  BatchView bv;
  const int32_t* list;    // binding ids handled by this launch
  int32_t n;
  const uint64_t* fmask;  // [B][W]
  // calAvailableReplicas rows: [B][Cp] merged per binding (bcls == nullptr), or
  // [n_classes][Cp] raw GeneralEstimator rows of the estimator classes, binding b
  // reading row bcls[b] (row 0: non-workload bindings, MaxInt32).
  const int32_t* est;
  const int32_t* bcls;
  Sink sink;
  int32_t* slow;          // [B] SLOW_* reason the binding needs k_slow for (0: none)
  int32_t* slow_ids;      // bindings flagged for k_slow, [0, stats[0]) (append order)
  uint32_t* stats;        // [0]: bindings flagged for the serial path, [SLOW_*]: by reason
  unsigned long long* dbg;  // diagnostic build only: phase cycle sums (nullptr otherwise)
  // set: the launch covers list[0, *n_dev) with a grid-stride loop (a list another
  // kernel appended to, e.g. k_select_top's fallback list); n is its capacity
  const uint32_t* n_dev = nullptr;
  // k_class_order's per-class orders and walkability (bits mode; nullptr when the
  // batch did not compute them): the spread kernels' class-order shortcut
  const uint64_t* ord = nullptr;
  const int32_t* cok = nullptr;
  uint32_t* n_order = nullptr;  // count of the bindings that took it
  // set (with n_dev): loop index j stands for list position sub[j] (a device-appended
  // fallback list of positions, so per-position arrays such as rsel stay aligned)
  const int32_t* sub = nullptr;
  // set: the estimator class of list[i] (k_select_top loads it with the list entry, so the
  // class order and class flags load one dependent global load earlier)
  const int32_t* lcls = nullptr;
};

enum : int {
  SEL_LAUNCH_ALL = 0,
  SEL_LAUNCH_CLUSTER,
  SEL_LAUNCH_REGION_A,
  SEL_LAUNCH_REGION_B,
  SEL_LAUNCH_SLOW,
  SEL_LAUNCH_ALL_STREAM  // SEL_ALL over streamed candidates (bits mode)
};

struct SelectExtra {
  RegionOut* rout = nullptr;         // region A output [n][n_regions]
  int32_t* rstat = nullptr;          // region A status [n]
  const int32_t* rsel = nullptr;     // region B input [n][n_regions]
  const int32_t* rnsel = nullptr;    // region B input [n]
  unsigned char* scratch = nullptr;  // slow path global scratch
  size_t slot_bytes = 0;
  int grid = 0;                      // slow path persistent grid
  int list_grid = 0;                 // > 0: caps the grid of a launch over a device-appended list
                                     // (its count read back by the host: no idle workgroups)
  int lds_area = 0;                  // slow path: LDS bytes for the small serial problems
  int lds_sort = 0;                  // slow path: LDS bytes for the candidate sorts (0: global slot)
  // the launch's KArgs in device memory: the kernels whose bodies keep pointers into
  // their arguments (SelCtx: &a.s, &a.bv) across calls take them by pointer, since a
  // by-value kernel argument would be copied to scratch by every wave (~34 KB per wave)
  const KArgs* dargs = nullptr;
};
// device KArgs slots per batch (one per such launch in a schedule call)
constexpr int kArgSlots = 16;

constexpr int kBlock = 256;
constexpr int kSlowBlock = 512;  // k_slow: wider for the LDS bitonic sort
// waves per workgroup of the one-wave-per-binding kernels (each wave its own LDS slice)
// Waves per workgroup of the one-wave-per-binding kernels. LDS is granted per workgroup and
// held until its last wave ends, so a finished binding's slice waits for its neighbours':
// k_select_top at 1 / 2 / 4 waves per workgroup 0.751 / 0.819 / 0.935 ms (same box,
// profiles/r06_ab/waves_*.json).
#ifndef KP_TOP_WAVES
#define KP_TOP_WAVES 1
#endif
#ifndef KP_STATIC_WAVES
#define KP_STATIC_WAVES 4
#endif
#ifndef KP_ORDER_WAVES
#define KP_ORDER_WAVES 4
#endif
constexpr int kTopWaves = KP_TOP_WAVES;        // k_select_top
constexpr int kTopWgWaves = 4;                 // k_select_top_wg: one binding per workgroup of this many waves
constexpr int kStaticWaves = KP_STATIC_WAVES;  // k_select_static
constexpr int kOrderWaves = KP_ORDER_WAVES;    // k_spread_order, k_region_a_order
constexpr int kPairStage = 4096;  // bytes of per-binding predicate data staged in LDS
constexpr int kTsetMax = 4096;    // distinct taint lists answered once per binding (LDS bits)


constexpr int kOffThreads = 256, kOffChunk = 4 * kOffThreads;  // CSR offsets scan (body_offsets_a/b)
constexpr int kSwRules = 4;  // StaticWeight rules kept as LDS bitsets (more: per-cluster static_vote)
// Dynamic LDS of k_select_all_stream (kp_kernels.h body_select_all_stream).
KP_HD inline size_t sel_stream_lds_bytes(int Cp) {
  const int words = (Cp + 31) >> 5, W = Cp / 64;
  return kRedBytes + 4 * (size_t)((words + 3) & ~3) + 8 * (size_t)kSwRules * W + 3072 + 8 * (size_t)sel_all_ecap(Cp) +
         64;
}
}  // namespace kp
