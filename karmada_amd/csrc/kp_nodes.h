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

// ---- node claims (estimator/server/nodes/filter.go:38-99) ------------------------
// A member cluster's nodes as the device sees them: interned (key, value) label
// pairs with each value's base-10 parse, the NoSchedule/NoExecute taints, and the
// interned metadata.name.
struct NodeView {
  uint64_t n;
  const uint32_t* flags;     // [n] bit 0 unschedulable
  const int32_t* name;       // [n] metadata.name id, -1 when empty (extractNodeFields)
  const int32_t* lbl_off;    // [n + 1] node label (key, value) ids, CSR
  const int64_t* lbl;        // key << 32 | value
  const int64_t* lbl_int;    // strconv.ParseInt(value, 10, 64) ...
  const uint8_t* lbl_int_ok; // ... and whether it parsed
  const int32_t* tnt_off;    // [n + 1] NoSchedule/NoExecute taints, CSR
  const int32_t* tnt;        // [3 * k] key, value, effect
};
// One compiled requirement of a required node-affinity term.
enum : int32_t {
  NA_IN = 0,         // labels In (values: ids)
  NA_NOTIN = 1,
  NA_EXISTS = 2,
  NA_DNE = 3,
  NA_GT = 4,         // label value parsed > x
  NA_LT = 5,
  NA_NAME_IN = 6,    // matchFields metadata.name == value id
  NA_NAME_NOTIN = 7,
  NA_FIELD_TRUE = 8,   // matchFields on a field the node does not carry ("" vs the value)
  NA_FIELD_FALSE = 9
};
struct NodeReq {
  int32_t op, key, voff, nv;
  int64_t x;
};
// pb.NodeClaim compiled against the call's dictionary: SelectorFromSet pairs,
// tolerations, and the required node affinity as usable terms (empty and
// unparsable terms dropped, nodeaffinity.go:39-170).
struct ClaimProg {
  const int64_t* sel;        // nodeSelector pairs (key << 32 | value)
  int32_t n_sel;
  const Tol* tols;
  int32_t n_tols;
  int32_t tol_unsched;       // the tolerations tolerate node.kubernetes.io/unschedulable:NoSchedule
  int32_t has_aff;           // RequiredDuringSchedulingIgnoredDuringExecution != nil
  int32_t n_terms;
  const int32_t* term_off;   // [n_terms + 1] into reqs
  const NodeReq* reqs;
  const int32_t* vals;       // In / NotIn value ids
};
KP_HD inline int node_label(const NodeView& v, uint64_t i, int32_t key) {
  for (int l = v.lbl_off[i]; l < v.lbl_off[i + 1]; l++)
    if ((int32_t)(v.lbl[l] >> 32) == key) return l;
  return -1;
}
// nodeSelectorTerm.match (nodeaffinity.go:179-190) for a parsed term: every label
// requirement (labels.Requirement.Matches, selector.go:247-292); the field
// requirements only when the node has fields (a non-empty name).
KP_HD inline bool node_term(const NodeView& v, const ClaimProg& p, int t, uint64_t i) {
  const int32_t nm = v.name[i];
  for (int q = p.term_off[t]; q < p.term_off[t + 1]; q++) {
    const NodeReq r = p.reqs[q];
    bool ok;
    if (r.op >= NA_NAME_IN) {
      if (nm < 0) continue;
      if (r.op == NA_NAME_IN) ok = nm == r.voff;
      else if (r.op == NA_NAME_NOTIN) ok = nm != r.voff;
      else ok = r.op == NA_FIELD_TRUE;
    } else {
      const int l = node_label(v, i, r.key);
      if (r.op == NA_EXISTS) {
        ok = l >= 0;
      } else if (r.op == NA_DNE) {
        ok = l < 0;
      } else if (r.op == NA_GT || r.op == NA_LT) {
        ok = l >= 0 && v.lbl_int_ok[l] && (r.op == NA_GT ? v.lbl_int[l] > r.x : v.lbl_int[l] < r.x);
      } else {
        bool has = false;
        if (l >= 0) {
          const int32_t val = (int32_t)(v.lbl[l] & 0xffffffff);
          for (int j = 0; j < r.nv && !has; j++) has = p.vals[r.voff + j] == val;
        }
        ok = r.op == NA_IN ? (l >= 0 && has) : !has;
      }
    }
    if (!ok) return false;
  }
  return true;
}
// MatchNode (scheduling_simulator_components.go:149-156; filter.go:60-90):
// RequiredNodeAffinity.Match (the nodeSelector as an equality set, then any usable
// term), the unschedulable taint, then every NoSchedule/NoExecute taint tolerated
// (ToleratesTaint, comparison operators off).
KP_HD inline bool node_matches(const NodeView& v, const ClaimProg& p, uint64_t i) {
  const int l0 = v.lbl_off[i], l1 = v.lbl_off[i + 1];
  for (int s = 0; s < p.n_sel; s++) {
    bool f = false;
    for (int l = l0; l < l1 && !f; l++) f = v.lbl[l] == p.sel[s];
    if (!f) return false;
  }
  if (p.has_aff) {
    bool any = false;
    for (int t = 0; t < p.n_terms && !any; t++) any = node_term(v, p, t, i);
    if (!any) return false;
  }
  if ((v.flags[i] & 1u) && !p.tol_unsched) return false;
  for (int t = v.tnt_off[i]; t < v.tnt_off[i + 1]; t++) {
    const int32_t k = v.tnt[3 * t], val = v.tnt[3 * t + 1], e = v.tnt[3 * t + 2];
    bool tol = false;
    for (int j = 0; j < p.n_tols && !tol; j++) {
      const Tol tl = p.tols[j];
      tol = (tl.eff == EFF_ANY || tl.eff == e) && (tl.key < 0 || tl.key == k) && (tl.op == TOL_EXISTS || tl.val == val);
    }
    if (!tol) return false;
  }
  return true;
}

// ---- node resources -------------------------------------------------------------------
// A node's util.Resource as slots: 0 = AllowedPodNumber, then the resources some
// request names (cpu milli, memory, ephemeral-storage, scalar resources).
constexpr int kNodeRes = 8;
constexpr int kNodeComp = 16;      // components of one set
constexpr int kNodeCompAll = 64;   // over every phase (assumed workloads + the request)
constexpr int kNodePhase = 17;

// ---- per-node estimate ---------------------------------------------------------------
struct NodeEstArgs {
  NodeView v;
  ClaimProg p;
  int32_t NU;
  const int64_t* avail;      // [n][NU] available resources (after any assumed-workload deduction)
  int64_t q[kNodeRes];       // the request's MaxDivided entries (> 0; 0 = not divided by); slot 0 unused
  uint32_t* sum;             // int32 sum (wrapping), as Go's atomic.AddInt32
};
// int32(MaxDivided) of node i (util/resource.go:221-248); 0 when it does not match.
KP_HD inline int32_t node_replicas(const NodeEstArgs& A, uint64_t i) {
  if (!node_matches(A.v, A.p, i)) return 0;
  const int64_t* a = A.avail + i * A.NU;
  int64_t res = INT64_MAX;
  for (int u = 1; u < A.NU; u++) {
    if (A.q[u] <= 0) continue;
    const int64_t d = a[u] / A.q[u];
    res = d < res ? d : res;
  }
  res = a[0] < res ? a[0] : res;
  return (int32_t)(uint32_t)(uint64_t)res;  // int32(int64): two's-complement truncation
}

// ---- component sets over nodes (noderesource.go:70-190) -----------------------------
// Phases run in order on one node state: each assumed workload with upper bound 1
// (the deduction, noderesource.go:95-113,166-185), then the request's components
// with upper bound MaxInt32, whose set count is the answer.
struct NodeSetsArgs {
  uint64_t n;
  int32_t NU;
  int32_t mono;              // every request entry >= 0 and every Replicas >= 0: capacities only drop
  int64_t max_steps;         // literal set simulations before giving up (*ovf)
  int32_t n_phase;
  int32_t last_upper;        // upper bound of the last phase (MaxInt32; 1 when it is a deduction too)
  int32_t ph_k0[kNodePhase + 1];        // phase p: components [ph_k0[p], ph_k0[p + 1])
  int32_t replicas[kNodeCompAll];
  int64_t req[kNodeCompAll][kNodeRes];  // requiredPerReplica (util.NewResource, AllowedPodNumber = 1)
  int64_t pos[kNodeCompAll][kNodeRes];  // its positive part (Resource.ResourceList, what MaxDivided reads)
  int64_t* avail;            // [n][NU] node.Allocatable after getNodeAvailableResource; consumed in place
  const uint32_t* present;   // [n] bit u: the node's Resource carries slot u (scalars: in its allocatable)
  const uint8_t* match;      // [components][n] MatchNode of each component's NodeClaim
  int32_t* out;              // sets of the last phase
  uint32_t* ovf;             // 1: the simulation needed more than max_steps literal sets
};
KP_HD inline int64_t nsets_maxdiv(const NodeSetsArgs& A, const int64_t* a, int k) {
  int64_t res = INT64_MAX;
  for (int u = 0; u < A.NU; u++) {
    const int64_t q = A.pos[k][u];
    if (q > 0) {
      const int64_t d = a[u] / q;
      res = d < res ? d : res;
    }
  }
  return res;
}
// node.Allocatable.SubResource(requiredPerReplica.Clone().Multiply(f)): Go's
// wrapping int64 products and differences, clamped at 0, absent scalars untouched.
KP_HD inline void nsets_sub(const NodeSetsArgs& A, int64_t* a, uint32_t pres, int k, int64_t f) {
  for (int u = 0; u < A.NU; u++) {
    if (!((pres >> u) & 1u)) continue;
    const int64_t d = (int64_t)((uint64_t)A.req[k][u] * (uint64_t)f);
    const int64_t v = (int64_t)((uint64_t)a[u] - (uint64_t)d);
    a[u] = v > 0 ? v : 0;
  }
}
// Orders one lane's global stores before the other lanes' loads (same wave).
KP_HD inline void kp_fence_wg() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
#endif
}
// match[k * n + j] = MatchNode of node j for component k's claim.
KP_HD inline void body_node_match(const NodeView& v, const ClaimProg* P, uint64_t i, uint8_t* match) {
  const uint64_t k = i / v.n, j = i - k * v.n;
  match[i] = node_matches(v, P[k], j) ? 1 : 0;
}
// SchedulingSimulator.SimulateScheduling(components [k0, k0 + K), upper)
// (scheduling_simulator_components.go:51-131) run by one block policy (a wave64 on
// the device, one thread on the host). Each component's first-fit scan resumes at
// the first node that may still hold it (capacities only drop when every request
// entry is >= 0), the next candidate node is found W nodes at a time by ballot, and
// a set in which every component fit whole on one node is repeated in closed form:
// the same placement holds for the next j sets while each component's node keeps
// A - j*D - P >= r*q on every entry it divides by (D: the set's use of that node,
// P: the earlier components' use within the set), so k = min floor((A-P-rq)/D) + 1
// further sets are applied at once. Every batch ends with some (component, node)
// pair exhausted, so the literal sets number O(K * n).
template <class Blk>
KP_HD inline int32_t node_sets_phase(const Blk& b, const NodeSetsArgs& A, int k0, int K, int32_t upper,
                                     int64_t* steps, bool* over) {
  const int W = b.wwidth();
  const int lane = b.lane();
  int64_t ptr[kNodeComp];
  int64_t at[kNodeComp];
  for (int k = 0; k < K; k++) ptr[k] = 0;
  int32_t sets = 0;
  while (sets < upper) {
    if (++*steps > A.max_steps) {
      *over = true;
      break;
    }
    bool ok = true, whole = A.mono != 0;
    for (int k = 0; k < K && ok; k++) {  // scheduleComponentSet
      const int g = k0 + k;
      int64_t rem = A.replicas[g];
      at[k] = -1;
      if (rem == 0) continue;  // returns true at the first fitting node, or after the scan
      bool first = true;
      uint64_t base = A.mono ? (uint64_t)ptr[k] : 0;
      const uint8_t* m = A.match + (size_t)g * A.n;
      for (;;) {  // scheduleComponent: the next matching node with MaxDivided > 0
        int64_t node = -1, cap = 0;
        for (; base < A.n; base += (uint64_t)W) {
          const uint64_t i = base + (uint64_t)lane;
          int64_t c = 0;
          if (i < A.n && m[i]) c = nsets_maxdiv(A, A.avail + i * A.NU, g);
          const uint64_t bal = b.wballot(c > 0);
          if (bal) {
            const int f = __builtin_ctzll(bal);
            node = (int64_t)base + f;
            cap = b.wread(c, f);
            break;
          }
        }
        if (node < 0) break;
        if (A.mono && first) ptr[k] = node;  // every node before it holds none of k
        const int64_t take = rem < cap ? rem : cap;
        if (lane == 0) nsets_sub(A, A.avail + (uint64_t)node * A.NU, A.present[node], g, take);
        kp_fence_wg();
        rem = (int64_t)(int32_t)(uint32_t)(uint64_t)(rem - take);  // remaining -= int32(allocatable)
        if (rem == 0) {
          if (first && take == A.replicas[g]) at[k] = node;
          else whole = false;
          break;
        }
        whole = false;
        if (A.mono) ptr[k] = node + 1;  // take == cap: node exhausted for k
        first = false;
        base = (uint64_t)node + 1;
      }
      if (rem != 0) ok = false;
    }
    if (!ok) break;
    sets++;
    if (!whole || sets >= upper) continue;
    // closed-form repeat of this set's placement
    __int128 kmax = (__int128)(upper - sets);
    for (int k = 0; k < K && kmax > 0; k++) {
      if (at[k] < 0) continue;
      const int g = k0 + k;
      const int64_t* a = A.avail + (uint64_t)at[k] * A.NU;
      for (int u = 0; u < A.NU; u++) {
        if (A.pos[g][u] <= 0) continue;
        __int128 P = 0, D = 0;
        for (int j = 0; j < K; j++) {
          if (at[j] != at[k]) continue;
          const __int128 use = (__int128)A.replicas[k0 + j] * A.req[k0 + j][u];
          D += use;
          if (j < k) P += use;
        }
        const __int128 num = (__int128)a[u] - P - (__int128)A.replicas[g] * A.pos[g][u];
        const __int128 lim = num < 0 ? 0 : num / D + 1;
        if (lim < kmax) kmax = lim;
      }
    }
    if (kmax <= 0) continue;
    if (lane == 0) {
      for (int k = 0; k < K; k++) {
        if (at[k] < 0) continue;
        const int g = k0 + k;
        int64_t* a = A.avail + (uint64_t)at[k] * A.NU;
        const uint32_t pres = A.present[at[k]];
        for (int u = 0; u < A.NU; u++)
          if ((pres >> u) & 1u) a[u] = (int64_t)((__int128)a[u] - kmax * ((__int128)A.replicas[g] * A.req[g][u]));
      }
    }
    kp_fence_wg();
    sets += (int32_t)kmax;
  }
  return sets;
}
template <class Blk>
KP_HD inline void node_sets(const Blk& b, const NodeSetsArgs& A) {
  int64_t steps = 0;
  bool over = false;
  int32_t sets = 0;
  for (int p = 0; p < A.n_phase && !over; p++)
    sets = node_sets_phase(b, A, A.ph_k0[p], A.ph_k0[p + 1] - A.ph_k0[p], p + 1 == A.n_phase ? A.last_upper : 1,
                           &steps, &over);
  if (b.lane() == 0) {
    *A.out = sets;
    *A.ovf = over ? 1u : 0u;
  }
}

}  // namespace kp
