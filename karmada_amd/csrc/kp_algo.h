// kp_algo.h — kernel bodies of the placement engine, written once as
// __host__ __device__ templates over a block policy (kp_blk.h).
//
// Stage map (reference functions, /root/reference):
//   pair stage   findClustersThatFit + RunFilterPlugins  core/generic_scheduler.go:119-163
//                GeneralEstimator.maxAvailableReplicas   estimator/client/general.go:66-108
//                calAvailableReplicas                    core/util.go:57-110
//   select stage GroupClustersWithScore / sortClusters   spreadconstraint/group_clusters.go:103-378, util.go:43-61
//                SelectBestClusters                      spreadconstraint/select_clusters*.go
//                AssignReplicas + strategies             core/common.go:51-170, assignment.go, division_algorithm.go
//                Dispenser / AllocateWebsterSeats        util/helper/binding.go:51-183, webstermethod.go:112-161
#pragma once
#include <stdint.h>

#include "kp_blk.h"
#include "kp_layout.h"

namespace kp {

// ============================================================================
// small helpers
// ============================================================================
KP_HD inline bool list_has(const int32_t* p, int n, int32_t x) {
  for (int i = 0; i < n; i++)
    if (p[i] == x) return true;
  return false;
}
// col[c] with a 32-bit byte offset (c < 2^28): with a uniform column base the
// load takes the scalar-base + vector-offset form, no 64-bit address math per lane.
template <class T>
KP_HD inline T ldcol(const T* col, int c) {
  return *(const T*)((const char*)col + (uint32_t)c * (uint32_t)sizeof(T));
}
KP_HD inline bool bit_test(const uint32_t* bits, int c) { return (bits[c >> 5] >> (c & 31)) & 1u; }
KP_HD inline bool mask_test(const uint64_t* row, int c) { return (row[c >> 6] >> (c & 63)) & 1ull; }
KP_HD inline int32_t wrap32(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }
KP_HD inline int32_t add32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
KP_HD inline int32_t sub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
KP_HD inline int64_t add64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
KP_HD inline int64_t mul64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
KP_HD inline int popc64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(x);
#else
  return __builtin_popcountll(x);
#endif
}
KP_HD inline int ctz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll((unsigned long long)x) - 1;
#else
  return __builtin_ctzll(x);
#endif
}
KP_HD inline uint64_t dbits(double d) {
  union {
    double d;
    uint64_t u;
  } x;
  x.d = d;
  return x.u;
}
KP_HD inline double bitsd(uint64_t u) {
  union {
    double d;
    uint64_t u;
  } x;
  x.u = u;
  return x.d;
}
KP_HD inline double kp_floor(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return floor(x);
#else
  return __builtin_floor(x);
#endif
}
KP_HD inline double kp_ceil(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ceil(x);
#else
  return __builtin_ceil(x);
#endif
}

// ============================================================================
// Sort key of sortClusters (spreadconstraint/util.go:43-61): ascending u64 order ==
// (OverflowOrder asc, Score desc, AvailableReplicas desc, Name asc).
// [63:58] overflow (6b, 63 = 1000 / beyond) | [57:51] 127 - score (7b) |
// [50:18] ~(avail + 2^32) (33b) | [17:0] rank
// Scores are framework scores in [0, 100] (MaxClusterScore, framework/interface.go:
// 39-42); the in-tree sum is {0, 100}. AvailableReplicas = estimate + assigned, two
// int32s, so it lies in [-2^32, 2^32). OverflowOrder is a term index below
// kMaxOvfTerms or 1000 (getClusterOverflowOrder); the packer limits the terms.
// ============================================================================
constexpr int kMaxOvfTerms = 63;  // affinity term + overflow terms a key orders
KP_HD inline uint64_t sort_key(int32_t ovf, int64_t score, int64_t avail, uint32_t rank) {
  const uint64_t o = (uint64_t)(ovf >= kMaxOvfTerms ? kMaxOvfTerms : (ovf < 0 ? 0 : ovf)) << 58;
  const uint64_t sc = (uint64_t)(127 - (score > 127 ? 127 : (score < 0 ? 0 : score))) << 51;
  const uint64_t a = ((1ull << 33) - 1) - (uint64_t)(avail + (1ll << 32));
  return o | sc | ((a & ((1ull << 33) - 1)) << 18) | (uint64_t)(rank & 0x3ffff);
}
KP_HD inline uint32_t key_rank(uint64_t k) { return (uint32_t)(k & 0x3ffff); }
KP_HD inline int64_t key_avail(uint64_t k) {
  const uint64_t a = (k >> 18) & ((1ull << 33) - 1);
  return (int64_t)(((1ull << 33) - 1) - a) - (1ll << 32);
}
KP_HD inline int64_t key_score(uint64_t k) { return 127 - (int64_t)((k >> 51) & 127); }
KP_HD inline int32_t key_ovf(uint64_t k) {
  const int32_t o = (int32_t)(k >> 58);
  return o == kMaxOvfTerms ? 1000 : o;
}
// (AvailableReplicas desc, then sortClusters position) for the swap step of
// selectClustersByAvailableResource (select_clusters_by_cluster.go:55-78).
KP_HD inline uint64_t avail_key(uint64_t k) {
  const uint64_t a = (k >> 18) & ((1ull << 33) - 1);
  return (a << 31) | ((k >> 58) << 25) | (((k >> 51) & 127) << 18) | (k & 0x3ffff);
}

// ============================================================================
// Selector programs: util.ClusterMatches compiled (pkg/util/selector.go:97-155)
// ============================================================================
KP_HD inline bool prog_match(const SnapView& s, const BatchView& bv, int32_t prog_id, int c) {
  const Prog p = bv.progs[prog_id];
  for (int i = 0; i < p.ins_cnt; i++) {
    const Instr in = bv.instrs[p.ins_off + i];
    bool ok = true;
    switch (in.op) {
      case OP_FALSE:
        return false;
      case OP_TRUE:
        break;
      case OP_EXCLUDE:
        ok = !list_has(bv.ipool + in.a, in.b, c);
        break;
      case OP_NAMES:
        ok = list_has(bv.ipool + in.a, in.b, c);
        break;
      case OP_LBL_IN:
      case OP_LBL_NOTIN:
      case OP_LBL_EXISTS:
      case OP_LBL_DNE: {
        int32_t v = s.label_val[(size_t)in.a * s.Cp + c];
        if (in.op == OP_LBL_IN) ok = v >= 0 && list_has(bv.ipool + in.b, in.c, v);
        else if (in.op == OP_LBL_NOTIN) ok = v < 0 || !list_has(bv.ipool + in.b, in.c, v);
        else if (in.op == OP_LBL_EXISTS) ok = v >= 0;
        else ok = v < 0;
        break;
      }
      case OP_FLD_IN:
      case OP_FLD_NOTIN:
      case OP_FLD_EXISTS:
      case OP_FLD_DNE: {
        int32_t v = in.a == 0 ? s.provider[c] : s.region[c];
        if (in.op == OP_FLD_IN) ok = v >= 0 && list_has(bv.ipool + in.b, in.c, v);
        else if (in.op == OP_FLD_NOTIN) ok = v < 0 || !list_has(bv.ipool + in.b, in.c, v);
        else if (in.op == OP_FLD_EXISTS) ok = v >= 0;
        else ok = v < 0;
        break;
      }
      case OP_FLD_GT:
      case OP_FLD_LT: {
        uint32_t f = s.flags[c];
        bool has = in.a == 0 ? (f & CF_PROVIDER_INT) : (f & CF_REGION_INT);
        int64_t x = in.a == 0 ? s.provider_int[c] : s.region_int[c];
        ok = has && (in.op == OP_FLD_GT ? x > in.v : x < in.v);
        break;
      }
      case OP_ZONE_IN:
      case OP_ZONE_NOTIN: {
        int z0 = s.zone_off[c], z1 = s.zone_off[c + 1];
        bool hit = false;
        for (int z = z0; z < z1 && !hit; z++) hit = list_has(bv.ipool + in.b, in.c, s.zone_ids[z]);
        ok = in.op == OP_ZONE_IN ? (z1 > z0 && hit) : !hit;
        break;
      }
      case OP_ZONE_EXISTS:
        ok = s.zone_off[c + 1] > s.zone_off[c];
        break;
      case OP_ZONE_DNE:
        ok = s.zone_off[c + 1] == s.zone_off[c];
        break;
      default:
        return false;
    }
    if (!ok) return false;
  }
  return true;
}

// The same program evaluated with block-uniform control flow, for the fast pair
// kernels: the program text is read at uniform addresses (scalar loads from the
// batch pools in HBM), every lane runs every instruction (no per-lane early
// exit, so the loops stay uniform), and list membership is an OR over the
// uniform list. Same answer as prog_match for c < C; lanes C <= c < Cp read
// in-bounds padding and are masked out by the caller. Requires C >= 1.
// U clusters per lane (c[0..U)): every instruction issues its loads for all U
// clusters before comparing, so a wave has U memory round trips in flight.
template <int U>
KP_HD inline void prog_eval_u(const SnapView& s, const BatchView& bv, int32_t prog_id, const int (&c)[U],
                              bool (&res)[U]) {
  const Prog p = kp_ldu(bv.progs + prog_id);
  bool ok[U];
KP_UNROLL
  for (int u = 0; u < U; u++) ok[u] = true;
  for (int i = 0; i < p.ins_cnt; i++) {
    const Instr in = kp_ldu(bv.instrs + p.ins_off + i);
    const int32_t* lst = bv.ipool + (in.op == OP_EXCLUDE || in.op == OP_NAMES ? in.a : in.b);
    const int nl = in.op == OP_EXCLUDE || in.op == OP_NAMES ? in.b : in.c;
    switch (in.op) {
      case OP_FALSE:
KP_UNROLL
        for (int u = 0; u < U; u++) ok[u] = false;
        break;
      case OP_TRUE:
        break;
      case OP_EXCLUDE:
      case OP_NAMES: {
        bool hit[U];
KP_UNROLL
        for (int u = 0; u < U; u++) hit[u] = false;
        for (int k = 0; k < nl; k++) {
          const int32_t x = kp_ldu(lst + k);
KP_UNROLL
          for (int u = 0; u < U; u++) hit[u] = hit[u] | (x == c[u]);
        }
KP_UNROLL
        for (int u = 0; u < U; u++) ok[u] = ok[u] & (in.op == OP_NAMES ? hit[u] : !hit[u]);
        break;
      }
      case OP_LBL_IN:
      case OP_LBL_NOTIN:
      case OP_FLD_IN:
      case OP_FLD_NOTIN: {
        const bool lbl = in.op == OP_LBL_IN || in.op == OP_LBL_NOTIN;
        const int32_t* col = lbl ? s.label_val + (size_t)in.a * s.Cp : (in.a == 0 ? s.provider : s.region);
        int32_t v[U];
        bool hit[U];
KP_UNROLL
        for (int u = 0; u < U; u++) {
          v[u] = ldcol(col, c[u]);
          hit[u] = false;
        }
        for (int k = 0; k < nl; k++) {
          const int32_t x = kp_ldu(lst + k);
KP_UNROLL
          for (int u = 0; u < U; u++) hit[u] = hit[u] | (x == v[u]);
        }
        const bool isin = in.op == OP_LBL_IN || in.op == OP_FLD_IN;
KP_UNROLL
        for (int u = 0; u < U; u++) ok[u] = ok[u] & (isin ? ((v[u] >= 0) & hit[u]) : ((v[u] < 0) | !hit[u]));
        break;
      }
      case OP_LBL_EXISTS:
      case OP_LBL_DNE:
      case OP_FLD_EXISTS:
      case OP_FLD_DNE: {
        const bool lbl = in.op == OP_LBL_EXISTS || in.op == OP_LBL_DNE;
        const int32_t* col = lbl ? s.label_val + (size_t)in.a * s.Cp : (in.a == 0 ? s.provider : s.region);
        const bool ex = in.op == OP_LBL_EXISTS || in.op == OP_FLD_EXISTS;
KP_UNROLL
        for (int u = 0; u < U; u++) {
          const int32_t v = ldcol(col, c[u]);
          ok[u] = ok[u] & (ex ? v >= 0 : v < 0);
        }
        break;
      }
      case OP_FLD_GT:
      case OP_FLD_LT:
KP_UNROLL
        for (int u = 0; u < U; u++) {
          const uint32_t f = s.flags[c[u]];
          const bool has = (in.a == 0 ? (f & CF_PROVIDER_INT) : (f & CF_REGION_INT)) != 0;
          const int64_t x = in.a == 0 ? s.provider_int[c[u]] : s.region_int[c[u]];
          ok[u] = ok[u] & has & (in.op == OP_FLD_GT ? x > in.v : x < in.v);
        }
        break;
      case OP_ZONE_IN:
      case OP_ZONE_NOTIN:
      case OP_ZONE_EXISTS:
      case OP_ZONE_DNE:
KP_UNROLL
        for (int u = 0; u < U; u++) {
          const int cc = c[u] < s.C ? c[u] : s.C - 1;  // zone_off has C + 1 entries
          const int z0 = s.zone_off[cc], z1 = s.zone_off[cc + 1];
          if (in.op == OP_ZONE_EXISTS || in.op == OP_ZONE_DNE) {
            ok[u] = ok[u] & (in.op == OP_ZONE_EXISTS ? z1 > z0 : z1 == z0);
          } else {
            bool hit = false;
            for (int z = z0; z < z1; z++)
              for (int k = 0; k < nl; k++) hit = hit | (kp_ldu(lst + k) == s.zone_ids[z]);
            ok[u] = ok[u] & (in.op == OP_ZONE_IN ? ((z1 > z0) & hit) : !hit);
          }
        }
        break;
      default:
KP_UNROLL
        for (int u = 0; u < U; u++) ok[u] = false;
    }
  }
KP_UNROLL
  for (int u = 0; u < U; u++) res[u] = ok[u];
}
KP_HD inline bool prog_eval_u(const SnapView& s, const BatchView& bv, int32_t prog_id, int c) {
  const int cc[1] = {c};
  bool r[1];
  prog_eval_u<1>(s, bv, prog_id, cc, r);
  return r[0];
}

// ============================================================================
// Pair stage
// ============================================================================
// TaintToleration.Filter (taint_toleration.go:53-84), FindMatchingUntoleratedTaint
// (component-helpers/scheduling/corev1/helpers.go:79-102), ToleratesTaint with
// comparison operators disabled (core/v1/toleration.go:52-77). Only
// NoSchedule/NoExecute taints are packed.
KP_HD inline bool taints_tolerated(const SnapView& s, const BatchView& bv, const BindHdr& h, int c) {
  int t0 = s.taint_off[c], t1 = s.taint_off[c + 1];
  for (int t = t0; t < t1; t++) {
    int32_t k = s.taint_key[t], v = s.taint_val[t], e = s.taint_eff[t];
    bool tol = false;
    for (int j = 0; j < h.tol_cnt && !tol; j++) {
      const Tol tl = bv.tols[h.tol_off + j];
      tol = (tl.eff == EFF_ANY || tl.eff == e) && (tl.key < 0 || tl.key == k) && (tl.op == TOL_EXISTS || tl.val == v);
    }
    if (!tol) return false;
  }
  return true;
}

// FitError diagnosis of one pair (kp_filter_reasons): findClustersThatFit's skip of
// deleting clusters, then the Result of the first failing plugin of RunFilterPlugins
// (runtime/framework.go:93-105) as KP_REASON_* | arg << 8. Reads spec.Clusters and
// the eviction list from the pools (no LDS bitsets): a diagnosis path, not the hot one.
KP_HD inline uint32_t pair_reason(const SnapView& s, const BatchView& bv, const BindHdr& h, int c) {
  const uint32_t f = s.flags[c];
  if (f & CF_DELETING) return 255u;  // KP_REASON_DELETING
  const int en = h.enabled;
  bool in_t = false;  // TargetContains (binding_types_helper.go:102-110)
  for (int j = 0; j < h.tgt_cnt && !in_t; j++) in_t = bv.ipool[h.tgt_off + 2 * j] == c;
  if ((en & 1) && !in_t) {  // APIEnablement (api_enablement.go:51-78)
    if (h.gvk < 0 || !((s.api_bits[(size_t)(h.gvk >> 6) * s.Cp + c] >> (h.gvk & 63)) & 1ull)) return 1u;
  }
  if ((en & 2) && !in_t) {  // TaintToleration: FindMatchingUntoleratedTaint (taint_toleration.go:65-83)
    const int t0 = s.taint_off[c], t1 = s.taint_off[c + 1];
    for (int t = t0; t < t1; t++) {
      const int32_t k = s.taint_key[t], v = s.taint_val[t], e = s.taint_eff[t];
      bool tol = false;
      for (int j = 0; j < h.tol_cnt && !tol; j++) {
        const Tol tl = bv.tols[h.tol_off + j];
        tol = (tl.eff == EFF_ANY || tl.eff == e) && (tl.key < 0 || tl.key == k) && (tl.op == TOL_EXISTS || tl.val == v);
      }
      if (!tol) return 2u | (uint32_t)(t - t0) << 8;
    }
  }
  if ((en & 4) && !(h.flags & BF_AFF_ALL)) {  // ClusterAffinity (cluster_affinity.go:51-94)
    bool m = false;
    for (int j = 0; j < h.filt_cnt && !m; j++) m = prog_match(s, bv, bv.ipool[h.filt_off + j], c);
    if (!m) return 3u;
  }
  if (en & 8) {  // SpreadConstraint (spread_constraint.go:49-66): constraints in spec order
    for (int k = 0; k < 3; k++) {
      const int fld = (h.spread_order >> (2 * k)) & 3;
      if (fld == 1 && !(f & CF_HAS_PROVIDER)) return 4u;
      if (fld == 2 && !(f & CF_HAS_REGION)) return 5u;
      if (fld == 3 && !(f & CF_HAS_ZONES)) return 6u;
    }
  }
  if (en & 32) {  // ClusterEviction (cluster_eviction.go:50-57)
    for (int j = 0; j < h.evict_cnt; j++)
      if (bv.ipool[h.evict_off + j] == c) return 7u;
  }
  return 0u;
}

// findClustersThatFit skip-deleting + RunFilterPlugins over the enabled plugins.
KP_HD inline bool pair_feasible(const SnapView& s, const BatchView& bv, const BindHdr& h, int c,
                                const uint32_t* tgt_bits, const uint32_t* evict_bits) {
  if (c >= s.C) return false;
  uint32_t f = s.flags[c];
  if (f & CF_DELETING) return false;
  int en = h.enabled;
  bool in_t = h.tgt_cnt > 0 && bit_test(tgt_bits, c);
  if ((en & 1) && !in_t) {  // APIEnablement (api_enablement.go:51-78)
    if (h.gvk < 0) return false;
    uint64_t w = s.api_bits[(size_t)(h.gvk >> 6) * s.Cp + c];
    if (!((w >> (h.gvk & 63)) & 1ull)) return false;
  }
  if ((en & 2) && !in_t && !taints_tolerated(s, bv, h, c)) return false;
  if ((en & 4) && !(h.flags & BF_AFF_ALL)) {  // ClusterAffinity (cluster_affinity.go:51-94)
    bool m = false;
    for (int j = 0; j < h.filt_cnt && !m; j++) m = prog_match(s, bv, bv.ipool[h.filt_off + j], c);
    if (!m) return false;
  }
  if (en & 8) {  // SpreadConstraint (spread_constraint.go:49-66)
    if ((h.flags & BF_NEED_PROVIDER) && !(f & CF_HAS_PROVIDER)) return false;
    if ((h.flags & BF_NEED_REGION) && !(f & CF_HAS_REGION)) return false;
    if ((h.flags & BF_NEED_ZONES) && !(f & CF_HAS_ZONES)) return false;
  }
  if ((en & 32) && h.evict_cnt > 0 && bit_test(evict_bits, c)) return false;  // ClusterEviction
  return true;
}

// MaxDivided of one model template for this binding's request (resource.go:191-220),
// pods capped at 110 (general.go:318-330).
KP_HD inline int32_t template_md(const SnapView& s, const BatchView& bv, const BindHdr& h, int tid) {
  int64_t res = kMaxPodsPerNode;
  for (int j = 0; j < h.mreq_cnt; j++) {
    int32_t rid = bv.ipool[h.mreq_off + j];
    int64_t q = bv.lpool[h.mreq_q_off + j];
    int64_t have = rid < 0 ? 0 : s.tmpl[(size_t)tid * s.n_res + rid];
    int64_t d = have / q;
    if (d < res) res = d;
  }
  return (int32_t)res;
}

// Estimator instances of the pair kernel (the template argument `Fast`):
//   EST_GENERIC  every fallback compiled in;
//   EST_MIXED    pair_fast_ok: dense node counts, <= kReqUnroll requests, no cold paths;
//   EST_SUMMARY  as MIXED, and no cluster of the snapshot has resource models;
//   EST_MODEL8 / EST_MODEL16  as MIXED, and every cluster with a summary has
//                models: only the <= 8 / 16 zero-padded template rows are loaded
//                (the summary columns are read late, on a path these snapshots
//                never take).
enum : int { EST_GENERIC = 0, EST_MIXED = 1, EST_SUMMARY = 2, EST_MODEL8 = 8, EST_MODEL16 = 16 };

// min(a / q, lim) for a >= 0, q >= 1, lim >= 0 without a 64-bit integer divide:
// a double estimate decides "quotient >= lim" when it is far from the limit,
// otherwise the quotient (< lim + 2 <= 2^31 + 2) is corrected exactly.
template <int Fast = EST_GENERIC>
KP_HD inline int64_t floor_div_below(int64_t a, int64_t q, int64_t lim) {
  if (a < q) return 0;
  if (Fast == EST_GENERIC && q > ((int64_t)1 << 60)) {  // enormous request: the quotient is tiny, divide exactly
    const int64_t d = a / q;
    return d < lim ? d : lim;
  }
  const double est = kp_floor((double)a / (double)q);
  if (est >= (double)lim + 2.0) return lim;
  uint64_t e = (uint64_t)est;
  const uint64_t ua = (uint64_t)a, uq = (uint64_t)q;  // e*uq <= a + uq < 2^64
  while (e > 0 && e * uq > ua) e--;
  while ((e + 1) * uq <= ua) e++;
  return (int64_t)e < lim ? (int64_t)e : lim;
}

// Per-cluster operands of the GeneralEstimator, loaded before any is used: the
// grade walk and the per-resource minimum then cost one memory latency per
// cluster, not one per grade or resource (the loads are independent; only the
// uniform binding fields decide which are issued).
constexpr int kEstUnroll = 8;   // model node groups per cluster (generic path)
constexpr int kReqUnroll = 4;   // summary-path resource requests per binding
constexpr int kTmplDense = 16;  // templates of the dense node-count matrix (fast path)

struct EstOps {
  uint32_t f;
  int64_t allowed;
  int32_t gc[kEstUnroll], gt[kEstUnroll];  // generic: model node groups k < kEstUnroll
  int32_t mt[kTmplDense];                  // fast: nodes of template t (SnapView::mt_cnt)
  int64_t av[kReqUnroll];                  // summary available of request j < kReqUnroll
};
template <int Fast = EST_GENERIC>
// md (the binding's MaxDivided per template, uniform; estimator-class rows only): the
// model-node counts of templates whose MaxDivided is 0 are not loaded (their product is 0)
KP_HD inline EstOps est_load(const SnapView& s, const BatchView& bv, const BindHdr& h, int c, uint32_t f,
                             const int32_t* md = nullptr) {
  EstOps o;
  o.f = f;
  o.allowed = ldcol(s.allowed, c);
  const bool rr = (h.flags & BF_HAS_RR) != 0;
  const bool model = rr;
  const int jh = rr && Fast < EST_MODEL8 ? (h.sreq_cnt < kReqUnroll ? h.sreq_cnt : kReqUnroll) : 0;
  if (Fast >= EST_MODEL8) {  // zero-padded rows: no per-template guard
KP_UNROLL
    for (int t = 0; t < kTmplDense; t++) {
      o.mt[t] = 0;
      if (t < Fast && model && (!md || kp_uniform(md[t]) != 0)) o.mt[t] = ldcol(s.mt_cnt + (size_t)t * s.Cp, c);
    }
  } else if (Fast == EST_SUMMARY) {
  } else if (Fast == EST_MIXED) {
    const int th = model ? s.n_tmpl : 0;
KP_UNROLL
    for (int t = 0; t < kTmplDense; t++) {
      o.mt[t] = 0;
      if (t < th) o.mt[t] = ldcol(s.mt_cnt + (size_t)t * s.Cp, c);
    }
  } else {
    const int kh = model ? (s.kmax < kEstUnroll ? s.kmax : kEstUnroll) : 0;
KP_UNROLL
    for (int k = 0; k < kEstUnroll; k++) {
      o.gc[k] = 0;
      o.gt[k] = 0;
      if (k < kh) {
        o.gc[k] = s.mg_cnt[(size_t)k * s.Cp + c];
        o.gt[k] = s.mg_tid[(size_t)k * s.Cp + c];
      }
    }
  }
KP_UNROLL
  for (int j = 0; j < kReqUnroll; j++) {
    o.av[j] = 0;
    if (j < jh) {
      const int32_t rid = Fast != EST_GENERIC ? kp_ldu(bv.ipool + h.sreq_off + j) : bv.ipool[h.sreq_off + j];
      if (rid >= 0) o.av[j] = ldcol(s.avail + (size_t)rid * s.Cp, c);
    }
  }
  return o;
}

// GeneralEstimator.maxAvailableReplicas (general.go:66-108), assumed workloads empty.
// md: per-template MaxDivided table (LDS) or nullptr to compute per pair.
// Fast != EST_GENERIC: the launch guarantees md != nullptr (zero past n_tmpl),
// the dense node-count matrix (n_tmpl <= kTmplDense, every template value >= 0
// so every MaxDivided is >= 0), every sreq_cnt <= kReqUnroll and every divisor
// <= 2^60 (pair_fast_ok, engine.cpp), so the cold fallbacks are compiled out.
template <int Fast = EST_GENERIC>
KP_HD inline int32_t est_compute(const SnapView& s, const BatchView& bv, const BindHdr& h, int c, const int32_t* md,
                                 const EstOps& o) {
  const uint32_t f = o.f;
  if (!(f & CF_HAS_SUMMARY)) return 0;
  int64_t m = o.allowed;
  if (m <= 0) return 0;
  if (!(h.flags & BF_HAS_RR)) return (int32_t)m;
  // A NodeClaim never diverts a binding from the model path: it converts without
  // error and every model node matches it (accurate.go:155-177,
  // scheduling_simulator_components.go:149-153).
  if (f & CF_MODEL_OK) {
    // getMaximumReplicasBasedOnResourceModels: each identical model node absorbs
    // exactly its initial MaxDivided, capped at MaxInt32.
    // d <= 110 (MaxPodsPerNode) and cnt <= MaxInt32: d*cnt < 2^38, and the
    // sum stops growing at MaxInt32 (Go's break), so int64 cannot overflow.
    int64_t total = 0;
    if (Fast != EST_GENERIC) {
      // Groups of one template merged: sum_t MaxDivided_t * nodes_t, each term
      // >= 0, so Go's stop at MaxInt32 is the clamp below; a node count
      // clamped at MaxInt32 only matters when its MaxDivided >= 1, where the
      // sum saturates either way.
KP_UNROLL
      for (int t = 0; t < kTmplDense; t++)
        if (Fast >= EST_MODEL8 ? t < Fast : t < s.n_tmpl) total += (int64_t)md[t] * (int64_t)o.mt[t];
    }
KP_UNROLL
    for (int k = 0; Fast == EST_GENERIC && k < kEstUnroll; k++)
      if (k < s.kmax && o.gc[k] != 0 && total < kInt32Max)
        total += (int64_t)(md ? md[o.gt[k]] : template_md(s, bv, h, o.gt[k])) * o.gc[k];
    for (int k = kEstUnroll; Fast == EST_GENERIC && k < s.kmax && total < kInt32Max; k++) {
      const int64_t cnt = s.mg_cnt[(size_t)k * s.Cp + c];
      if (cnt == 0) continue;
      const int32_t tid = s.mg_tid[(size_t)k * s.Cp + c];
      total += (int64_t)(md ? md[tid] : template_md(s, bv, h, tid)) * cnt;
    }
    if (total >= kInt32Max) total = kInt32Max;
    if (total < m) m = total;
    return (int32_t)m;
  }
  // getMaximumReplicasBasedOnClusterSummary (general.go:465-505)
  int64_t num = INT64_MAX;
  bool zero = false;
  if (Fast >= EST_MODEL8) {  // not preloaded: these snapshots give every summary cluster models
    for (int j = 0; j < h.sreq_cnt; j++) {
      const int32_t rid = bv.ipool[h.sreq_off + j];
      if (rid < 0) return 0;
      const int64_t a = s.avail[(size_t)rid * s.Cp + c];
      if (a <= 0) return 0;
      const int64_t lim = num < m ? num : m;
      const int64_t d = floor_div_below<Fast>(a, bv.lpool[h.sreq_q_off + j], lim);
      if (d < num) num = d;
    }
    if (num < m) m = num;
    return (int32_t)m;
  }
KP_UNROLL
  for (int j = 0; j < kReqUnroll; j++) {
    if (j < h.sreq_cnt && !zero) {
      if (bv.ipool[h.sreq_off + j] < 0 || o.av[j] <= 0) {
        zero = true;
      } else {
        const int64_t lim = num < m ? num : m;  // only quotients below min(num, allowed) matter
        const int64_t d = floor_div_below<Fast>(o.av[j], bv.lpool[h.sreq_q_off + j], lim);
        if (d < num) num = d;
      }
    }
  }
  if (zero) return 0;
  for (int j = kReqUnroll; Fast == EST_GENERIC && j < h.sreq_cnt; j++) {
    int32_t rid = bv.ipool[h.sreq_off + j];
    if (rid < 0) return 0;
    int64_t a = s.avail[(size_t)rid * s.Cp + c];
    if (a <= 0) return 0;
    const int64_t lim = num < m ? num : m;
    const int64_t d = floor_div_below(a, bv.lpool[h.sreq_q_off + j], lim);
    if (d < num) num = d;
  }
  if (num < m) m = num;
  return (int32_t)m;
}
KP_HD inline int32_t general_estimate(const SnapView& s, const BatchView& bv, const BindHdr& h, int c,
                                      const int32_t* md) {
  return est_compute(s, bv, h, c, md, est_load(s, bv, h, c, s.flags[c]));
}

// Branch-free forms of est_compute / cal_merge for the fast instances (the
// same answers; per-lane conditions become selects, so a wave's lanes never
// diverge inside the pair loop). floor_div_bf: min(a / q, lim) for a >= 1,
// 1 <= q <= 2^60, 0 <= lim < 2^31 + 2: the double quotient is within 1 of the
// true one below 2^33 (three roundings of relative 2^-53), so two selects fix it.
KP_HD inline int64_t floor_div_bf(int64_t a, int64_t q, int64_t lim) {
  const double est = kp_floor((double)a / (double)q);
  const bool big = est >= (double)lim + 2.0;
  uint64_t e = big ? 0ull : (uint64_t)est;
  const uint64_t ua = (uint64_t)a, uq = (uint64_t)q;
  e = (e > 0 && e * uq > ua) ? e - 1 : e;
  e = ((e + 1) * uq <= ua) ? e + 1 : e;
  const int64_t d = (int64_t)e < lim ? (int64_t)e : lim;
  return big ? lim : (a < q ? 0 : d);
}
template <int Fast>
KP_HD inline int32_t est_compute_bf(const SnapView& s, const BatchView& bv, const BindHdr& h, int c,
                                    const int32_t* md, const EstOps& o) {
  const uint32_t f = o.f;
  const int64_t allowed = o.allowed;
  int64_t m = allowed;
  const bool rr = (h.flags & BF_HAS_RR) != 0;  // uniform
  // model path: sum_t MaxDivided_t * nodes_t, clamped at MaxInt32
  int64_t total = 0;
KP_UNROLL
  for (int t = 0; t < kTmplDense; t++)
    if (Fast >= EST_MODEL8 ? t < Fast : (Fast == EST_MIXED && t < s.n_tmpl)) total += (int64_t)md[t] * (int64_t)o.mt[t];
  total = total >= kInt32Max ? (int64_t)kInt32Max : total;
  const int64_t mod = total < m ? total : m;
  // summary path (general.go:465-505), requests j < kReqUnroll (pair_fast_ok)
  int64_t sum = m;
  if (Fast == EST_MIXED || Fast == EST_SUMMARY) {
    int64_t num = INT64_MAX;
    bool zero = false;
KP_UNROLL
    for (int j = 0; j < kReqUnroll; j++) {
      if (j < h.sreq_cnt) {  // uniform
        const bool z = kp_ldu(bv.ipool + h.sreq_off + j) < 0 || o.av[j] <= 0;
        const int64_t lim = num < m ? num : m;
        const int64_t d = floor_div_bf(z ? 1 : o.av[j], kp_ldu(bv.lpool + h.sreq_q_off + j), lim);
        zero = zero | z;
        num = d < num ? d : num;
      }
    }
    sum = zero ? 0 : (num < m ? num : m);
  } else if (rr) {  // (model-only snapshots: every summary cluster has models; exact fallback)
    if (!(f & CF_MODEL_OK) && (f & CF_HAS_SUMMARY) && allowed > 0) sum = est_compute<Fast>(s, bv, h, c, md, o);
  }
  int64_t r = !rr ? m : ((f & CF_MODEL_OK) ? mod : sum);
  r = ((f & CF_HAS_SUMMARY) && allowed > 0) ? r : 0;
  return (int32_t)r;
}
KP_HD inline int32_t cal_merge_bf(int32_t replicas, int32_t r) {
  const int32_t v = (r != -1 && r < kInt32Max) ? r : kInt32Max;
  return v == kInt32Max ? replicas : v;
}

// calAvailableReplicas over an estimate: MaxInt32 init, min with the
// GeneralEstimator answer (-1 = UnauthenticReplica is skipped, core/util.go:86-99),
// leftover MaxInt32 -> spec.Replicas.
KP_HD inline int32_t cal_merge(const BindHdr& h, int32_t r) {
  int32_t v = kInt32Max;
  if (r != -1 && v > r) v = r;
  if (v == kInt32Max) v = h.replicas;
  return v;
}

// calAvailableReplicas (core/util.go:57-110) with the GeneralEstimator only.
KP_HD inline int32_t cal_available(const SnapView& s, const BatchView& bv, const BindHdr& h, int c,
                                   const int32_t* md) {
  if (h.flags & BF_NONWORKLOAD_EST) return kInt32Max;
  return cal_merge(h, general_estimate(s, bv, h, c, md));
}

// Filter + calAvailableReplicas of one (binding, cluster) pair for the pair
// kernel: every snapshot column the pair can need is loaded first, so the
// filter's and the estimator's memory latencies overlap. tol_bits: per taint
// set "tolerated" bits of this binding (LDS), or nullptr for the per-taint
// loop. Returns the estimate (0 when infeasible); *fit = feasibility.
template <int Fast = EST_GENERIC>
KP_HD inline int32_t pair_eval(const SnapView& s, const BatchView& bv, const BindHdr& h, int c,
                               const uint32_t* tgt_bits, const uint32_t* evict_bits, const uint32_t* tol_bits,
                               const int32_t* md, bool* fit) {
  const int en = h.enabled;
  const uint32_t f = s.flags[c];
  const bool api_on = (en & 1) && h.gvk >= 0;
  uint64_t aw = 0;
  if (api_on) aw = s.api_bits[(size_t)(h.gvk >> 6) * s.Cp + c];
  const bool tset_on = (en & 2) && (Fast != EST_GENERIC || tol_bits != nullptr);
  int32_t ts = 0;
  if (tset_on) ts = s.taint_set[c];
#ifdef KP_EXP_NOEST  // timing experiments only (tuning variants, wrong answers)
  const bool est_on = false;
#else
  const bool est_on = !(h.flags & BF_NONWORKLOAD_EST);
#endif
  EstOps o;
  if (est_on) o = est_load<Fast>(s, bv, h, c, f);
  // ClusterAffinity first: its selector loads then issue while the loads above
  // are still in flight (it reads none of them).
  bool aff = true;
#ifdef KP_EXP_NOAFF  // timing experiments only (tuning variants, wrong answers)
  if (false) {
#else
  if (Fast != EST_GENERIC) {
#endif
    // uniform loop over the affinity terms (scalar program loads), no early exit
    if ((en & 4) && !(h.flags & BF_AFF_ALL) && s.C > 0) {
      aff = false;
      for (int j = 0; j < h.filt_cnt; j++) aff = aff | prog_eval_u(s, bv, kp_ldu(bv.ipool + h.filt_off + j), c);
    }
  } else if ((en & 4) && !(h.flags & BF_AFF_ALL) && c < s.C) {  // (zone lists are [C+1])
    aff = false;
    for (int j = 0; j < h.filt_cnt && !aff; j++) aff = prog_match(s, bv, bv.ipool[h.filt_off + j], c);
  }
  // findClustersThatFit skip-deleting + RunFilterPlugins (same predicates as pair_feasible)
  bool ok = c < s.C && !(f & CF_DELETING) && aff;
  const bool in_t = h.tgt_cnt > 0 && bit_test(tgt_bits, c);
  if ((en & 1) && !in_t) ok = ok && api_on && ((aw >> (h.gvk & 63)) & 1ull);
  if ((en & 2) && !in_t)
    ok = ok && ((Fast != EST_GENERIC || tset_on) ? bit_test(tol_bits, ts) : taints_tolerated(s, bv, h, c));
  if (en & 8) {
    if ((h.flags & BF_NEED_PROVIDER) && !(f & CF_HAS_PROVIDER)) ok = false;
    if ((h.flags & BF_NEED_REGION) && !(f & CF_HAS_REGION)) ok = false;
    if ((h.flags & BF_NEED_ZONES) && !(f & CF_HAS_ZONES)) ok = false;
  }
  if ((en & 32) && h.evict_cnt > 0 && bit_test(evict_bits, c)) ok = false;
  *fit = ok;
  if (!ok) return 0;
  return est_on ? cal_merge(h, est_compute<Fast>(s, bv, h, c, md, o)) : kInt32Max;
}

// pair_eval of the fast instances for U clusters per lane (c[u] < Cp): every
// column load of all U clusters issues before the first use, so a wave keeps U
// memory round trips in flight per loop step instead of one.
template <int Fast, int U>
KP_HD inline void pair_eval_fast(const SnapView& s, const BatchView& bv, const BindHdr& h, const int (&c)[U],
                                 const uint32_t* tgt_bits, const uint32_t* evict_bits, const uint32_t* tol_bits,
                                 const int32_t* md, bool (&fit)[U], int32_t (&out)[U]) {
  static_assert(Fast != EST_GENERIC, "fast instances only");
  const int en = h.enabled;
  const bool api_on = (en & 1) && h.gvk >= 0;
#ifdef KP_EXP_NOEST  // timing experiments only (tuning variants, wrong answers)
  const bool est_on = false;
#else
  const bool est_on = !(h.flags & BF_NONWORKLOAD_EST);
#endif
  uint32_t f[U];
  uint64_t aw[U];
  int32_t ts[U];
  EstOps o[U];
KP_UNROLL
  for (int u = 0; u < U; u++) {
    f[u] = ldcol(s.flags, c[u]);
    aw[u] = 0;
    if (api_on) aw[u] = ldcol(s.api_bits + (size_t)(h.gvk >> 6) * s.Cp, c[u]);
    ts[u] = 0;
    if (en & 2) ts[u] = ldcol(s.taint_set, c[u]);
    if (est_on) o[u] = est_load<Fast>(s, bv, h, c[u], f[u]);
  }
  bool aff[U];
KP_UNROLL
  for (int u = 0; u < U; u++) aff[u] = true;
#ifndef KP_EXP_NOAFF
  if ((en & 4) && !(h.flags & BF_AFF_ALL) && s.C > 0) {  // uniform loop over the terms, no early exit
KP_UNROLL
    for (int u = 0; u < U; u++) aff[u] = false;
    for (int j = 0; j < h.filt_cnt; j++) {
      bool m[U];
      prog_eval_u<U>(s, bv, kp_ldu(bv.ipool + h.filt_off + j), c, m);
KP_UNROLL
      for (int u = 0; u < U; u++) aff[u] = aff[u] | m[u];
    }
  }
#endif
  // the filter plugins as one bitwise expression per lane (uniform parts fold
  // into scalar masks): no divergent branch in the loop
  const uint32_t need = (en & 8) ? (((h.flags & BF_NEED_PROVIDER) ? CF_HAS_PROVIDER : 0u) |
                                    ((h.flags & BF_NEED_REGION) ? CF_HAS_REGION : 0u) |
                                    ((h.flags & BF_NEED_ZONES) ? CF_HAS_ZONES : 0u))
                                 : 0u;
  const bool chk_api = (en & 1) != 0, chk_tol = (en & 2) != 0;
  const bool chk_ev = (en & 32) && h.evict_cnt > 0, any_t = h.tgt_cnt > 0;
KP_UNROLL
  for (int u = 0; u < U; u++) {
    const bool in_t = any_t & bit_test(tgt_bits, c[u]);
    const bool api_ok = api_on & (((aw[u] >> (h.gvk & 63)) & 1ull) != 0);
    const bool ok = (c[u] < s.C) & ((f[u] & CF_DELETING) == 0) & aff[u] & (!chk_api | in_t | api_ok) &
                    (!chk_tol | in_t | bit_test(tol_bits, ts[u])) & ((f[u] & need) == need) &
                    !(chk_ev & bit_test(evict_bits, c[u]));
    fit[u] = ok;
    const int32_t e = est_on ? cal_merge_bf(h.replicas, est_compute_bf<Fast>(s, bv, h, c[u], md, o[u])) : kInt32Max;
    out[u] = ok ? e : 0;
  }
}

// getClusterOverflowOrder (group_clusters.go:517-543)
KP_HD inline int32_t overflow_order(const SnapView& s, const BatchView& bv, const BindHdr& h, int c) {
  if (h.ovf_mode == OVF_ZERO) return 0;
  if (h.ovf_mode == OVF_1000) return 1000;
  for (int j = 0; j < h.ovf_cnt; j++)
    if (prog_match(s, bv, bv.ipool[h.ovf_off + j], c)) return j;
  return 1000;
}

// ============================================================================
// Per-binding candidate view
// ============================================================================
struct Cands {
  uint32_t* r;  // rank | overflow << kRankBits
  int32_t* v;   // AllocatableReplicas (or static weight for SEL_ALL StaticWeight)
  int32_t F;
  int16_t* g = nullptr;  // region-spread kernels: region index of candidate i (LDS; -1 none)
};
KP_HD inline uint32_t c_rank(const Cands& cd, int i) { return cd.r[i] & kRankMask; }
KP_HD inline int32_t c_ovf(const Cands& cd, int i) { return (int32_t)(cd.r[i] >> kRankBits); }

// AssignedReplicasForCluster (binding_types_helper.go:124-132): first spec.Clusters entry.
KP_HD inline int32_t assigned_of(const BatchView& bv, const BindHdr& h, const uint32_t* tgt_bits, uint32_t rank) {
  if (h.tgt_cnt == 0 || !bit_test(tgt_bits, (int)rank)) return 0;
  for (int j = 0; j < h.tgt_cnt; j++)
    if ((uint32_t)bv.ipool[h.tgt_off + 2 * j] == rank) return bv.ipool[h.tgt_off + 2 * j + 1];
  return 0;
}
KP_HD inline int64_t locality_score(const BindHdr& h, const uint32_t* tgt_bits, uint32_t rank) {
  return ((h.flags & BF_SCORE_LOCALITY) && h.tgt_cnt > 0 && bit_test(tgt_bits, (int)rank)) ? 100 : 0;
}

// ============================================================================
// Result sink
// ============================================================================
struct Sink {
  uint32_t* out_idx;   // snapshot rank (k_compact maps it through perm to the caller's index)
  int32_t* out_rep;
  unsigned long long* counter;
  int32_t* status;
  int32_t* err;
  int64_t* arg;
  uint64_t* start;
  uint32_t* count;
  uint64_t cap_end;  // entries of out_idx/out_rep: the slots [0, out_cap) + the shared area
};

// ============================================================================
// Go sort.Sort (pdqsort) on TargetClustersList (division_algorithm.go:31-36),
// restated from the structure of sort/zsortinterface.go (go1.26). Parity for
// n > 12 is unpinned by reference tests (SURVEY hazard H2).
// ============================================================================
struct TCL {
  uint32_t* name;
  int32_t* rep;
  KP_HD bool Less(int i, int j) const { return rep[i] > rep[j]; }
  KP_HD void Swap(int i, int j) const {
    uint32_t a = name[i];
    name[i] = name[j];
    name[j] = a;
    int32_t b = rep[i];
    rep[i] = rep[j];
    rep[j] = b;
  }
};
KP_HD inline int bits_len(uint64_t x) {
  int n = 0;
  while (x) {
    n++;
    x >>= 1;
  }
  return n;
}
template <class D>
KP_HD void pdq_insertion(const D& d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
}
template <class D>
KP_HD void pdq_sift(const D& d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
    if (!d.Less(first + root, first + child)) return;
    d.Swap(first + root, first + child);
    root = child;
  }
}
template <class D>
KP_HD void pdq_heapsort(const D& d, int a, int b) {
  int first = a, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) pdq_sift(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) {
    d.Swap(first, first + i);
    pdq_sift(d, 0, i, first);
  }
}
template <class D>
KP_HD int pdq_median(const D& d, int a, int b, int c, int& swaps) {
  if (d.Less(b, a)) {
    swaps++;
    int t = a;
    a = b;
    b = t;
  }
  if (d.Less(c, b)) {
    swaps++;
    int t = b;
    b = c;
    c = t;
  }
  if (d.Less(b, a)) {
    swaps++;
    int t = a;
    a = b;
    b = t;
  }
  return b;
}
// breakPatterns: three xorshift-chosen swaps around the middle.
template <class D>
KP_HD void pdq_break_patterns(const D& d, int a, int b) {
  const int length = b - a;
  if (length >= 8) {
    uint64_t r = (uint64_t)length;
    uint64_t modulus = 1ull << bits_len((uint64_t)length);
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13;
      r ^= r >> 7;
      r ^= r << 17;
      int other = (int)((unsigned)r & (modulus - 1));
      if (other >= length) other -= length;
      d.Swap(idx - 1 + i, a + other);
    }
  }
}
// choosePivot (read-only): median of three, Tukey ninther from 50 elements.
// *hint: 0 unknown, 1 increasing, 2 decreasing.
template <class D>
KP_HD int pdq_choose_pivot(const D& d, int a, int b, int* hint) {
  const int length = b - a;
  int swaps = 0;
  int pi = a + length / 4 * 1, pj = a + length / 4 * 2, pk = a + length / 4 * 3;
  if (length >= 8) {
    if (length >= 50) {
      pi = pdq_median(d, pi - 1, pi, pi + 1, swaps);
      pj = pdq_median(d, pj - 1, pj, pj + 1, swaps);
      pk = pdq_median(d, pk - 1, pk, pk + 1, swaps);
    }
    pj = pdq_median(d, pi, pj, pk, swaps);
  }
  *hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
  return pj;
}
// The loop state (wasBalanced, wasPartitioned) is a parameter so that a
// segment handed over mid-loop (pdq_wave) resumes exactly where Go would.
//
// Go recurses into the smaller side and loops on the larger one. Here the larger
// side's continuation goes on an explicit stack and the loop descends into the
// smaller side, so the depth stays <= log2(n) + 1 and, above all, the function does
// not recurse: a recursive device function gives its kernel a dynamic call stack the
// runtime does not size, and k_slow's thread 0 (the serial emulation) overran its
// stack into the next wave's scratch, corrupting threads 64-65's spilled state
// (round 4: config 8 seed 6). Disjoint segments are independent (the
// only read outside a segment, a[-1] in partitionEqual, is a placed pivot), so the
// order in which they are finished does not change the permutation.
struct PdqTaskGo {
  int a, b, limit;
  bool wasBalanced, wasPartitioned;
};
constexpr int kPdqGoStack = 40;  // > log2(2^31) + 1 pending continuations
template <class D>
KP_HD void pdqsort_go(const D& d, int a, int b, int limit, bool wasBalanced = true, bool wasPartitioned = true) {
  PdqTaskGo st[kPdqGoStack];
  int sp = 0;
  for (;;) {
    int length = b - a;
    bool done = length <= 12 || limit == 0;  // (Go: return from this segment)
    if (done) {
      if (length <= 12) pdq_insertion(d, a, b);
      else pdq_heapsort(d, a, b);
    }
    if (!done && !wasBalanced) {
      pdq_break_patterns(d, a, b);
      limit--;
    }
    int hint = 0, pivot = 0;
    if (!done) pivot = pdq_choose_pivot(d, a, b, &hint);
    if (hint == 2) {
      int i = a, j = b - 1;
      while (i < j) {
        d.Swap(i, j);
        i++;
        j--;
      }
      pivot = (b - 1) - (pivot - a);
      hint = 1;
    }
    if (!done && wasBalanced && wasPartitioned && hint == 1) {  // partialInsertionSort
      int i = a + 1;
      bool sorted = false;
      for (int step = 0; step < 5; step++) {
        while (i < b && !d.Less(i, i - 1)) i++;
        if (i == b) {
          sorted = true;
          break;
        }
        if (b - a < 50) break;
        d.Swap(i, i - 1);
        if (i - a >= 2) {
          for (int j = i - 1; j >= 1; j--) {
            if (!d.Less(j, j - 1)) break;
            d.Swap(j, j - 1);
          }
        }
        if (b - i >= 2) {
          for (int j = i + 1; j < b; j++) {
            if (!d.Less(j, j - 1)) break;
            d.Swap(j, j - 1);
          }
        }
      }
      done = sorted;
    }
    if (done) {  // the segment is sorted: resume the innermost pending continuation
      if (sp == 0) return;
      const PdqTaskGo& t = st[--sp];
      a = t.a, b = t.b, limit = t.limit, wasBalanced = t.wasBalanced, wasPartitioned = t.wasPartitioned;
      continue;
    }
    if (a > 0 && !d.Less(a - 1, pivot)) {  // partitionEqual
      d.Swap(a, pivot);
      int i = a + 1, j = b - 1;
      for (;;) {
        while (i <= j && !d.Less(a, i)) i++;
        while (i <= j && d.Less(a, j)) j--;
        if (i > j) break;
        d.Swap(i, j);
        i++;
        j--;
      }
      a = i;
      continue;
    }
    // partition
    d.Swap(a, pivot);
    int i = a + 1, j = b - 1;
    bool already = false;
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    int mid;
    if (i > j) {
      d.Swap(j, a);
      mid = j;
      already = true;
    } else {
      d.Swap(i, j);
      i++;
      j--;
      for (;;) {
        while (i <= j && d.Less(i, a)) i++;
        while (i <= j && !d.Less(j, a)) j--;
        if (i > j) break;
        d.Swap(i, j);
        i++;
        j--;
      }
      d.Swap(j, a);
      mid = j;
    }
    wasPartitioned = already;
    int leftLen = mid - a, rightLen = b - mid;
    int balanceThreshold = length / 8;
    // Go: recurse into the smaller side with fresh state, then loop on the larger one
    if (leftLen < rightLen) {
      wasBalanced = leftLen >= balanceThreshold;
      if (sp < kPdqGoStack) st[sp++] = PdqTaskGo{mid + 1, b, limit, wasBalanced, wasPartitioned};
      b = mid;
    } else {
      wasBalanced = rightLen >= balanceThreshold;
      if (sp < kPdqGoStack) st[sp++] = PdqTaskGo{a, mid, limit, wasBalanced, wasPartitioned};
      a = mid + 1;
    }
    wasBalanced = true;  // the smaller side starts as Go's recursive call does
    wasPartitioned = true;
  }
}
KP_HD inline void sort_tcl(uint32_t* name, int32_t* rep, int n) {
  if (n <= 1) return;
  TCL d{name, rep};
  pdqsort_go(d, 0, n, bits_len((uint64_t)n));
}

// ============================================================================
// Webster / Sainte-Lague priorities (webstermethod.go:57-85)
// ============================================================================
// float64(Votes) / float64(2*Seats+1) with Seats < 2^30 (no int32 wrap). From 2^30
// seats on, 2*Seats+1 wraps negative in Go's int32: the block-parallel paths hand
// targets of 2^30 seats or more to the serial emulation (webster_serial).
constexpr int64_t kSeatWrap = (int64_t)1 << 30;
KP_HD inline double w_prio(int64_t v, int64_t k) { return (double)v / (double)(2 * k + 1); }
// Bit pattern of a double and back (positive doubles order as their patterns do).
KP_HD inline uint64_t kp_dbits(double d) {
  uint64_t u;
  __builtin_memcpy(&u, &d, 8);
  return u;
}
KP_HD inline double kp_bitsd(uint64_t u) {
  double d;
  __builtin_memcpy(&d, &u, 8);
  return d;
}

// #{k >= 0 : prio(v,k) >= t} (ge) or > t, for v >= 0, t > 0, saturating at cap.
KP_HD inline int64_t w_count(int64_t v, double t, int64_t cap, bool ge) {
  if (v <= 0) return 0;
  double r = (double)v / t;
  const double y = (r - 1.0) * 0.5;
  double kf = r < 1.0 ? 0.0 : kp_floor(y) + 1.0;
  // Exact without further divisions when y = (v/t - 1)/2 is far from every
  // integer: y's error is below r*2^-51, and fl(v/(2k+1)) can only compare
  // with t differently from the real v/(2k+1) when v/t lies within a relative
  // 2^-52 of 2k+1 (|y - k| < r*2^-52). Outside tol = r*2^-44 neither happens,
  // so the count is floor(y)+1 for >= and > alike.
  if (r >= 1.0) {
    const double fr = y - kp_floor(y), tol = r * 0x1p-44;
    if (fr > tol && fr < 1.0 - tol) return kf > (double)cap ? cap : (int64_t)kf;
  }
  int64_t k = kf > (double)cap ? cap : (int64_t)kf;
  while (k > 0) {
    double p = w_prio(v, k - 1);
    if (ge ? p >= t : p > t) break;
    k--;
  }
  while (k < cap) {
    double p = w_prio(v, k);
    if (!(ge ? p >= t : p > t)) break;
    k++;
  }
  return k;
}

// w_count with r = v * rt, rt = fl(1/t) computed once per pass (no division per
// party): r's relative error stays below 2^-52 (two roundings), so y's error
// stays below r*2^-52, far inside the same tol band, and every count the fast
// path returns is the exact one; the band itself takes the exact divisions.
KP_HD inline int64_t w_count_r(int64_t v, double t, double rt, int64_t cap, bool ge) {
  if (v <= 0) return 0;
  const double r = (double)v * rt;
  const double y = (r - 1.0) * 0.5;
  if (r >= 1.0) {
    const double fy = kp_floor(y);
    const double fr = y - fy, tol = r * 0x1p-44;
    if (fr > tol && fr < 1.0 - tol) {
      const double kf = fy + 1.0;
      return kf > (double)cap ? cap : (int64_t)kf;
    }
  }
  return w_count(v, t, cap, ge);
}

// Serial exact AllocateWebsterSeats for parties with unique names and votes >= 0
// (dispenser with nil init): result seats[] per party. Names order: rank asc,
// `desc` flips the name tie-break (tieBreakerByUID, binding.go:117-144).
// Works from a count threshold t0 with cnt_gt(t0) <= N (every element above t0
// is in the top-N), then continues with Go's heap order for the rest.
struct WHeap {
  const uint32_t* name;
  const int64_t* votes;
  int32_t* seats;
  int32_t* h;  // heap of party indices
  bool desc;
  KP_HD double pr(int i) const { return (double)votes[i] / (double)add32((int32_t)(2u * (uint32_t)seats[i]), 1); }
  KP_HD bool less(int a, int b) const {  // a before b
    double pa = pr(a), pb = pr(b);
    if (pa == pb) {
      if (seats[a] != seats[b]) return seats[a] < seats[b];
      return desc ? name[a] > name[b] : name[a] < name[b];
    }
    return pa > pb;
  }
  KP_HD void down(int i0, int n) {
    int i = i0;
    for (;;) {
      int j1 = 2 * i + 1;
      if (j1 >= n || j1 < 0) break;
      int j = j1;
      if (j1 + 1 < n && less(h[j1 + 1], h[j1])) j = j1 + 1;
      if (!less(h[j], h[i])) break;
      int t = h[i];
      h[i] = h[j];
      h[j] = t;
      i = j;
    }
  }
};
KP_HD inline void webster_serial(const uint32_t* name, const int64_t* votes, int32_t* seats, int32_t* heap, int n,
                                 int32_t N, bool desc) {
  for (int i = 0; i < n; i++) seats[i] = 0;
  if (n == 0 || N <= 0) return;
  int npos = 0, nzero = 0, ipos = -1;
  int64_t V = 0;
  for (int i = 0; i < n; i++) {
    V += votes[i] > 0 ? votes[i] : 0;
    if (votes[i] > 0) npos++, ipos = i;
    if (votes[i] == 0) nzero++;
  }
  auto before = [&](int j, int i) { return desc ? name[j] > name[i] : name[j] < name[i]; };  // name tie-break
  // Party i's k-th seat has priority v_i / int32(2k+1) (webstermethod.go:60-61): for
  // v > 0 positive and falling while k < 2^30, then negative (2k+1 wraps) and
  // falling; for v = 0 always 0; for v < 0 negative and RISING. Every positive
  // element comes first, so while npos * 2^30 >= N the seats are the top N of the
  // positive parties' elements (below); otherwise the positive parties take 2^30
  // each and the rest R goes, in heap order, to: the zero-vote parties (priority 0
  // beats every negative one; ties by seats then name: a round robin in name
  // order); else to the positive party's wrapped seats while they stay above the
  // best negative head v_j (a tie goes to the fewer seats, j), and then to j, whose
  // priority only rises once it has a seat.
  if (npos <= 1 && (int64_t)N > (int64_t)npos * kSeatWrap) {
    if (ipos >= 0) seats[ipos] = (int32_t)kSeatWrap;
    int64_t R = (int64_t)N - (int64_t)npos * kSeatWrap;
    if (nzero > 0) {
      const int64_t q = R / nzero, rem = R % nzero;
      for (int i = 0; i < n; i++) {
        if (votes[i] != 0) continue;
        int64_t ahead = 0;
        for (int j = 0; j < n; j++) ahead += (votes[j] == 0 && before(j, i)) ? 1 : 0;
        seats[i] = (int32_t)(q + (ahead < rem ? 1 : 0));
      }
      return;
    }
    int jn = -1;  // the best negative head: largest v, then the name order
    for (int j = 0; j < n; j++)
      if (votes[j] < 0 && (jn < 0 || votes[j] > votes[jn] || (votes[j] == votes[jn] && before(j, jn)))) jn = j;
    if (ipos >= 0) {
      // wrapped seats of the positive party: k = 2^30 + m, priority v / (2k+1 - 2^32), falling in m
      const double vj = jn >= 0 ? (double)votes[jn] : 0.0;
      auto above = [&](int64_t m) {
        const int64_t k = kSeatWrap + m;
        return jn < 0 || (double)votes[ipos] / (double)(int32_t)(uint32_t)(2 * k + 1) > vj;
      };
      int64_t lo = 0, hi = R;  // m seats taken: the first m with !above(m), or R
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (above(mid)) lo = mid + 1;
        else hi = mid;
      }
      seats[ipos] = (int32_t)((int64_t)seats[ipos] + lo);
      R -= lo;
    }
    if (R > 0 && jn >= 0) seats[jn] = (int32_t)R;
    return;
  }
  int32_t done = 0;
  if (npos > 0) {
    // Count threshold t over the positive parties: every element with priority > t
    // is in the top N when the count is <= N. Bisected while the heap's share
    // would be large, so the heap below orders about the tie group at the N-th
    // priority. A party's count stops at 2^30 (its later priorities are negative).
    const int64_t cap = (int64_t)N + 1 < kSeatWrap ? (int64_t)N + 1 : kSeatWrap;
    auto total = [&](double t) {
      int64_t S = 0;
      for (int i = 0; i < n; i++) S += votes[i] > 0 ? w_count(votes[i], t, cap, false) : 0;
      return S;
    };
    double hi = (double)V / (2.0 * (double)N), lo = 0;
    int64_t S = total(hi);
    for (int it = 0; it < 200 && S > (int64_t)N; it++) {
      lo = hi;
      hi *= 2.0;
      S = total(hi);
    }
    for (int it = 0; it < 64 && S <= (int64_t)N && (int64_t)N - S > 4 * (int64_t)n + 64; it++) {
      const double mid = lo + (hi - lo) * 0.5;
      if (!(mid > lo && mid < hi)) break;
      const int64_t Sm = total(mid);
      if (Sm <= (int64_t)N) hi = mid, S = Sm;
      else lo = mid;
    }
    if (S <= (int64_t)N)
      for (int i = 0; i < n; i++) {
        seats[i] = votes[i] > 0 ? (int32_t)w_count(votes[i], hi, cap, false) : 0;
        done += seats[i];
      }
  }
  WHeap w{name, votes, seats, heap, desc};
  for (int i = 0; i < n; i++) heap[i] = i;
  for (int i = n / 2 - 1; i >= 0; i--) w.down(i, n);
  for (int32_t rem = N - done; rem > 0; rem--) {
    // heap.Pop + Seats++ + heap.Push == increase the top's key and sift down
    int top = heap[0];
    seats[top] = add32(seats[top], 1);
    w.down(0, n);
  }
}

}  // namespace kp
