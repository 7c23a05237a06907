// kp_sets.h — GeneralEstimator.MaxAvailableComponentSets (estimator/client/general.go:
// 154-292) on the device: one thread per cluster of the request.
//
//   summary bound   podsInSet / podBound / perSetRequirement / resourceBoundedSets
//                   over the snapshot's quantityAsInt64 availability column (qa)
//   model bound     SchedulingSimulator.SimulateScheduling (scheduling_simulator_
//                   components.go:51-131) over the cluster's model-grade nodes, as
//                   runs of identical nodes: a run of cnt nodes that each absorb m
//                   replicas is one step, a partial fill splits it into at most three
//                   runs, equal neighbours merge again, and a component's scan resumes
//                   at the first run that may still hold it (capacity only drops), so
//                   the first-fit order is kept without visiting single nodes.
#pragma once
#include "kp_algo.h"

namespace kp {

constexpr int kSetsComp = 16;   // components per set
constexpr int kSetsSlots = 8;   // resource slots (the requested model resources + pods)
constexpr int kSetsPer = 16;    // perSetRequirement entries
constexpr int kSetsRunsMax = 4096;  // node runs per cluster (global scratch; a run holds >= 1 node)
constexpr int kSetsOverflow = INT32_MIN;  // a cluster's simulation needed more runs

// One component list, resolved against the snapshot's resource dictionary (host).
struct SetsArgs {
  int32_t K, NS, nper, per_nonzero;
  int64_t pods_per_set;
  int32_t replicas[kSetsComp];
  int32_t slot_rid[kSetsSlots];            // resource id; -1 none of the clusters has it; -2 pods
  int64_t req[kSetsComp][kSetsSlots];      // requiredPerReplica (util.NewResource units, pods = 1)
  int64_t pos[kSetsComp][kSetsSlots];      // its positive part (Resource.ResourceList, MaxDivided)
  int32_t per_rid[kSetsPer];               // -1: no cluster allocates it
  int64_t per_req[kSetsPer];               // sum over components of quantityAsInt64 * replicas
};

KP_HD inline int32_t i32_of(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }  // Go int32(x)

// Resource.MaxDivided (util/resource.go:221-248) of one run's node for component k.
KP_HD inline int64_t sets_maxdiv(const SetsArgs& A, const int64_t* cap, int k) {
  int64_t res = INT64_MAX;
  for (int j = 0; j < A.NS; j++) {
    if (A.slot_rid[j] == -2) {
      res = cap[j] < res ? cap[j] : res;  // min with AllowedPodNumber
    } else if (A.pos[k][j] > 0) {
      const int64_t q = cap[j] / A.pos[k][j];
      res = q < res ? q : res;
    }
  }
  return res;
}
// SubResource(requiredPerReplica.Clone().Multiply(f)) (util/resource.go:77-115): clamp at 0.
KP_HD inline void sets_sub(const SetsArgs& A, int64_t* cap, int k, int64_t f) {
  for (int j = 0; j < A.NS; j++) {
    const int64_t d = (int64_t)((uint64_t)A.req[k][j] * (uint64_t)f);
    const int64_t v = (int64_t)((uint64_t)cap[j] - (uint64_t)d);
    cap[j] = v > 0 ? v : 0;
  }
}

// maxAvailableComponentSets (general.go:163-199) for cluster rank c. runs: this
// thread's rcap x (1 + kSetsSlots) int64 scratch (rcap = the cluster's model node
// count, capped at kSetsRunsMax). kSetsOverflow when the run list outgrew it.
KP_HD inline int32_t sets_one(const SnapView& s, const SetsArgs& A, int c, int64_t* runs, int rcap) {
  const uint32_t f = s.flags[c];
  if (!(f & CF_HAS_SUMMARY)) return 0;
  const int64_t allowed = s.allowed[c];  // getAllowedPodNumber
  if (allowed <= 0) return 0;
  if (A.pods_per_set <= 0) return i32_of(allowed);
  int32_t maxSets = i32_of(allowed / A.pods_per_set);
  if (A.per_nonzero) {  // resourceBoundedSets (general.go:218-236)
    for (int j = 0; j < A.nper; j++) {
      if (A.per_req[j] <= 0) continue;
      const int64_t av = A.per_rid[j] < 0 ? kQaAbsent : s.qa[(size_t)A.per_rid[j] * s.Cp + c];
      if (av == kQaAbsent || av <= 0) return 0;
      const int32_t rb = i32_of(av / A.per_req[j]);
      if (rb < maxSets) maxSets = rb;
    }
  }
  // applyResourceModelBound: models present and buildModelNodes without error
  if (!(f & CF_MODEL_OK)) return maxSets;
  constexpr int kStride = 1 + kSetsSlots;
  int nr = 0;
  for (int k = 0; k < s.kmax; k++) {  // buildModelNodes: grades ascending
    const int32_t cnt = s.mg_cnt[(size_t)k * s.Cp + c];
    if (cnt <= 0) continue;
    if (nr == rcap) return kSetsOverflow;
    const int32_t tid = s.mg_tid[(size_t)k * s.Cp + c];
    int64_t* r = runs + (size_t)nr * kStride;
    r[0] = cnt;
    for (int j = 0; j < A.NS; j++) {
      const int32_t rid = A.slot_rid[j];
      r[1 + j] = rid == -2 ? 110 : (rid >= 0 ? s.tmpl[(size_t)tid * s.n_res + rid] : 0);  // pods: maxPodsCountPerNode
    }
    nr++;
  }
  auto same = [&](int a, int b) {
    for (int j = 0; j < A.NS; j++)
      if (runs[(size_t)a * kStride + 1 + j] != runs[(size_t)b * kStride + 1 + j]) return false;
    return true;
  };
  auto move_runs = [&](int from, int to) {  // runs[from..nr) -> runs[to..), to != from
    const int n = nr - from;
    if (to > from)
      for (int i = n - 1; i >= 0; i--)
        for (int j = 0; j < kStride; j++) runs[(size_t)(to + i) * kStride + j] = runs[(size_t)(from + i) * kStride + j];
    else
      for (int i = 0; i < n; i++)
        for (int j = 0; j < kStride; j++) runs[(size_t)(to + i) * kStride + j] = runs[(size_t)(from + i) * kStride + j];
  };
  int ptr[kSetsComp];
  for (int k = 0; k < A.K; k++) ptr[k] = 0;
  // merges run i into i - 1 when their capacities are equal (keeps the list short)
  auto merge_left = [&](int i) {
    if (i <= 0 || i >= nr || !same(i - 1, i)) return;
    runs[(size_t)(i - 1) * kStride] += runs[(size_t)i * kStride];
    move_runs(i + 1, i);
    nr--;
    for (int k = 0; k < A.K; k++)
      if (ptr[k] >= i) ptr[k] = ptr[k] - 1 > 0 ? ptr[k] - 1 : 0;
  };
  int32_t complete = 0;
  while (complete < maxSets) {
    bool ok = true;
    for (int k = 0; k < A.K && ok; k++) {  // scheduleComponentSet
      int64_t rem = A.replicas[k];
      if (rem == 0) continue;  // succeeds at the first node that fits, or at the end
      bool lead = true;
      for (int i = ptr[k]; i < nr && rem > 0; i++) {  // scheduleComponent, first fit
        int64_t* r = runs + (size_t)i * kStride;
        const int64_t m = sets_maxdiv(A, r + 1, k);
        if (m <= 0) {
          if (lead) ptr[k] = i + 1;
          continue;
        }
        lead = false;
        const __int128 all = (__int128)m * r[0];
        if ((__int128)rem >= all) {  // every node of the run takes m
          sets_sub(A, r + 1, k, m);
          rem -= (int64_t)all;
          const int before = nr;
          merge_left(i);
          if (nr < before) i--;
          continue;
        }
        // partial: q nodes take m, one takes rem % m, the rest keep their capacity
        const int64_t q = rem / m, rr = rem % m, rest = r[0] - q - (rr > 0 ? 1 : 0);
        const int parts = (q > 0) + (rr > 0) + (rest > 0);
        if (nr + parts - 1 > rcap) return kSetsOverflow;
        if (parts > 1) move_runs(i + 1, i + parts);
        int64_t base[kSetsSlots];
        for (int j = 0; j < A.NS; j++) base[j] = r[1 + j];
        int at = i;
        auto put = [&](int64_t cnt, int64_t take) {
          int64_t* w = runs + (size_t)at * kStride;
          w[0] = cnt;
          for (int j = 0; j < A.NS; j++) w[1 + j] = base[j];
          if (take > 0) sets_sub(A, w + 1, k, take);
          at++;
        };
        if (q > 0) put(q, m);
        if (rr > 0) put(1, rr);
        if (rest > 0) put(rest, 0);
        nr += parts - 1;
        for (int j = 0; j < A.K; j++)
          if (j != k && ptr[j] > i) ptr[j] += parts - 1;
        merge_left(i);
        rem = 0;
      }
      if (rem > 0) ok = false;
    }
    if (!ok) break;
    complete++;
  }
  return complete < maxSets ? complete : maxSets;
}

// off[i] / off[i + 1]: cluster i's runs in the scratch (units of runs).
KP_HD inline void body_sets(const SnapView& s, const SetsArgs* A, const int32_t* ranks, const int64_t* off, uint64_t i,
                            int64_t* scratch, int32_t* out) {
  out[i] = sets_one(s, *A, ranks[i], scratch + (size_t)off[i] * (1 + kSetsSlots), (int)(off[i + 1] - off[i]));
}

// Component-set class row (kp_schedule_batch, BF_SETS bindings): cluster rank r's
// answer; a simulation that outgrew its runs raises *ovf (the batch then fails with
// KP_ENOTSUP) instead of leaving kSetsOverflow in the row.
KP_HD inline void body_sets_row(const SnapView& s, const SetsArgs& A, const int64_t* off, int r, int64_t* scratch,
                                int32_t* row, uint32_t* ovf) {
  const int32_t v = sets_one(s, A, r, scratch + (size_t)off[r] * (1 + kSetsSlots), (int)(off[r + 1] - off[r]));
  if (v == kSetsOverflow) {
    *ovf = (uint32_t)r + 1u;  // (any overflowing cluster's rank + 1)
    row[r] = 0;
  } else {
    row[r] = v;
  }
}

}  // namespace kp
