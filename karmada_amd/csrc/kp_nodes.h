// kp_nodes.h — member-cluster node kernels: the resource-model
// grade histogram (modeling.AddToResourceSummary) and the accurate estimator's
// per-node MaxDivided sum (noderesource.nodeResourceEstimator.Estimate). The host
// (engine.cpp) resolves names and exact Quantities; the device classifies and
// divides one node per thread.
#pragma once
#include "kp_layout.h"

namespace kp {

// ---- grades ----------------------------------------------------------------------
// Quantities as exact 128-bit nano-unit integers split into (hi, lo).
struct GradesArgs {
  int32_t K, NR;             // grades, resource names (modelSortingResourceNames)
  const int64_t* min_hi;     // [NR][K] modelSortings
  const uint64_t* min_lo;
  const int64_t* val_hi;     // [n][NR] the node's available quantity of each name (0 if absent)
  const uint64_t* val_lo;
  uint64_t n;                // nodes before the walk's stop
  unsigned long long* counts;  // [K]
};
KP_HD inline int q128_cmp(int64_t ah, uint64_t al, int64_t bh, uint64_t bl) {
  if (ah != bh) return ah < bh ? -1 : 1;
  if (al != bl) return al < bl ? -1 : 1;
  return 0;
}
// searchLastLessElement (modeling.go:123-145), literally (its answer on unsorted
// input is the bisection's).
KP_HD inline int search_last_less(const int64_t* hi, const uint64_t* lo, int K, int64_t th, uint64_t tl) {
  int low = 0, high = K - 1;
  while (low <= high) {
    const int mid = low + ((high - low) >> 1);
    const int d1 = q128_cmp(hi[mid], lo[mid], th, tl);
    const int d2 = mid != K - 1 ? q128_cmp(hi[mid + 1], lo[mid + 1], th, tl) : 0;
    if (d1 < 1) {
      if (mid == K - 1 || d2 == 1) return mid;
      low = mid + 1;
    } else {
      high = mid - 1;
    }
  }
  return -1;
}
// getIndex (modeling.go:112-121): the minimum over resource names (NR >= 1).
KP_HD inline int node_grade(const GradesArgs& A, uint64_t i) {
  int idx = 0x7fffffff;
  for (int r = 0; r < A.NR; r++) {
    const size_t o = (size_t)i * A.NR + r;
    const int t = search_last_less(A.min_hi + (size_t)r * A.K, A.min_lo + (size_t)r * A.K, A.K, A.val_hi[o], A.val_lo[o]);
    idx = t < idx ? t : idx;
  }
  return idx;
}
KP_HD inline void body_grades(const GradesArgs& A, uint64_t i) {
  const int g = node_grade(A, i);
  if (g >= 0) kp_atomic_add(&A.counts[g], 1ull);  // AddToResourceSummary: Quantity += 1 (index -1: skipped)
}

// ---- per-node estimate ---------------------------------------------------------------
struct NodeEstArgs {
  uint64_t n;
  int32_t NQ;                // requested resources that divide (cpu milli, memory, ephemeral, scalars)
  const int64_t* avail;      // [n][NQ] available per request entry, clamped at 0 (SubResource)
  const int64_t* q;          // [NQ] request per entry (> 0)
  const int64_t* pods;       // [n] AllowedPodNumber - len(pods), clamped at 0
  const uint32_t* flags;     // [n] bit 0 unschedulable
  const int32_t* lbl_off;    // [n + 1] node label (key, value) ids, CSR
  const int64_t* lbl;        // key << 32 | value
  const int32_t* tnt_off;    // [n + 1] NoSchedule/NoExecute taints, CSR
  const int32_t* tnt;        // [3 * k] key, value, effect
  const int64_t* sel;        // [n_sel] nodeSelector pairs (key << 32 | value); -1: a pair no node has
  int32_t n_sel;
  const Tol* tols;
  int32_t n_tols;
  int32_t tol_unsched;       // the tolerations tolerate node.kubernetes.io/unschedulable:NoSchedule
  uint32_t* sum;             // int32 sum (wrapping), as Go's atomic.AddInt32
};
// MatchNode (scheduling_simulator_components.go:149-153; filter.go:60-90): the
// nodeSelector as an equality set, the unschedulable taint, then every
// NoSchedule/NoExecute taint tolerated (ToleratesTaint, comparison operators off).
KP_HD inline bool node_matches(const NodeEstArgs& A, uint64_t i) {
  const int l0 = A.lbl_off[i], l1 = A.lbl_off[i + 1];
  for (int s = 0; s < A.n_sel; s++) {
    bool f = false;
    for (int l = l0; l < l1 && !f; l++) f = A.lbl[l] == A.sel[s];
    if (!f) return false;
  }
  if ((A.flags[i] & 1u) && !A.tol_unsched) return false;
  for (int t = A.tnt_off[i]; t < A.tnt_off[i + 1]; t++) {
    const int32_t k = A.tnt[3 * t], v = A.tnt[3 * t + 1], e = A.tnt[3 * t + 2];
    bool tol = false;
    for (int j = 0; j < A.n_tols && !tol; j++) {
      const Tol tl = A.tols[j];
      tol = (tl.eff == EFF_ANY || tl.eff == e) && (tl.key < 0 || tl.key == k) && (tl.op == TOL_EXISTS || tl.val == v);
    }
    if (!tol) return false;
  }
  return true;
}
// int32(MaxDivided) of node i (util/resource.go:221-248); 0 when it does not match.
KP_HD inline int32_t node_replicas(const NodeEstArgs& A, uint64_t i) {
  if (!node_matches(A, i)) return 0;
  int64_t res = INT64_MAX;
  for (int j = 0; j < A.NQ; j++) {
    const int64_t d = A.avail[(size_t)i * A.NQ + j] / A.q[j];
    res = d < res ? d : res;
  }
  res = A.pods[i] < res ? A.pods[i] : res;
  return (int32_t)(uint32_t)(uint64_t)res;  // int32(int64): two's-complement truncation
}

}  // namespace kp
