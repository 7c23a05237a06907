// kp_launch.h — host-callable launchers for the kernels in kernels.hip, so the
// engine (engine.cpp) stays plain host C++.
#pragma once
#include <hip/hip_runtime_api.h>
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
  const int32_t* est;     // [B][Cp]
  Sink sink;
  int32_t* slow;          // [B] flag: needs k_slow
};

enum : int { SEL_LAUNCH_ALL = 0, SEL_LAUNCH_CLUSTER, SEL_LAUNCH_REGION_A, SEL_LAUNCH_REGION_B, SEL_LAUNCH_SLOW };

struct SelectExtra {
  RegionOut* rout = nullptr;    // region A output [n][n_regions]
  int32_t* rstat = nullptr;     // region A status [n]
  const int32_t* rsel = nullptr;   // region B input [n][n_regions]
  const int32_t* rnsel = nullptr;  // region B input [n]
  unsigned char* scratch = nullptr;  // slow path global scratch
  size_t slot_bytes = 0;
  int grid = 0;                 // slow path persistent grid
};

constexpr int kBlock = 256;

hipError_t launch_pair(hipStream_t st, const SnapView& s, const BatchView& bv, int b0, int nb, uint64_t* fmask,
                       int32_t* est, int64_t* score, int est_mode, int md_cap, size_t smem);
hipError_t launch_select(hipStream_t st, int which, const KArgs& a, size_t smem, int cap, const SelectExtra& x);
hipError_t launch_compact(hipStream_t st, const uint64_t* start, const uint32_t* count, const uint64_t* offsets,
                          const uint32_t* in_idx, const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n);

}  // namespace kp
