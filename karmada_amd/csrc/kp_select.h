// kp_select.h — per-binding select/assign bodies (one workgroup per binding).
#pragma once
#include "kp_algo.h"

namespace kp {

constexpr int kSmallMax = 256;   // selected-list capacity of the small (serial) path
constexpr int kTgtSmallMax = 256;

struct Item {
  uint32_t rank;
  int32_t alloc;   // AllocatableReplicas
  int64_t avail;   // AvailableReplicas
  int32_t ovf;
  int32_t pad;
};

struct SerialScratch {
  int cap;
  Item* tier;                    // overflow tier list
  uint32_t* en;  int64_t* ew;    // dispense input entries (name, weight)
  uint32_t* pn;  int64_t* pv;    // parties (name, votes)
  int32_t* ps;   int32_t* ph;    // seats, heap
  uint32_t* an;  int32_t* ar;    // available list (TargetClustersList)
  uint32_t* xn;  int32_t* xr;    // temp (resort, merge map names/values)
  int32_t* xf;                   // merge map presence
  uint32_t* tn;  int32_t* tr;    // one strategy call's result
  uint32_t* sn;  int32_t* sr;    // scheduledClusters
  uint32_t* rn;  int32_t* rr;    // final result
  int32_t* pos;                  // optional rank-indexed scratch (all -1 between uses)
  int presorted;                 // an/ar already hold the sorted TargetClustersList (body_slow)
};
// Bytes serial_scratch_carve takes: 2 i64 arrays, the tier list and 15 u32 arrays of
// `cap` entries, each rounded up to 16 B. (This once counted 14 u32 arrays: the last
// one, rr, ran 4*cap bytes past a k_slow slot into the next workgroup's.)
KP_HD inline size_t serial_scratch_bytes(int cap) {
  const size_t c = (size_t)cap;
  auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  return 2 * r16(c * sizeof(int64_t)) + r16(c * sizeof(Item)) + 15 * r16(c * sizeof(uint32_t)) + 16;
}
KP_HD inline SerialScratch serial_scratch_carve(void* mem, int cap) {
  SerialScratch s;
  s.cap = cap;
  char* p = (char*)mem;
  auto take = [&](size_t bytes) {
    char* q = p;
    p += (bytes + 15) & ~(size_t)15;
    return q;
  };
  s.ew = (int64_t*)take((size_t)cap * 8);
  s.pv = (int64_t*)take((size_t)cap * 8);
  s.tier = (Item*)take((size_t)cap * sizeof(Item));
  s.en = (uint32_t*)take((size_t)cap * 4);
  s.pn = (uint32_t*)take((size_t)cap * 4);
  s.ps = (int32_t*)take((size_t)cap * 4);
  s.ph = (int32_t*)take((size_t)cap * 4);
  s.an = (uint32_t*)take((size_t)cap * 4);
  s.ar = (int32_t*)take((size_t)cap * 4);
  s.xn = (uint32_t*)take((size_t)cap * 4);
  s.xr = (int32_t*)take((size_t)cap * 4);
  s.xf = (int32_t*)take((size_t)cap * 4);
  s.tn = (uint32_t*)take((size_t)cap * 4);
  s.tr = (int32_t*)take((size_t)cap * 4);
  s.sn = (uint32_t*)take((size_t)cap * 4);
  s.sr = (int32_t*)take((size_t)cap * 4);
  s.rn = (uint32_t*)take((size_t)cap * 4);
  s.rr = (int32_t*)take((size_t)cap * 4);
  s.pos = nullptr;
  s.presorted = 0;
  return s;
}

struct SelCtx {
  const SnapView* s;
  const BatchView* bv;
  const BindHdr* h;
  int b;
  const uint64_t* frow;
  // calAvailableReplicas of cluster c = est_at(x, c): erow is either the binding's
  // own merged row (merge == false) or its estimator class's raw GeneralEstimator
  // row, merged here with spec.Replicas (mrep) as cal_merge_bf does.
  const int32_t* erow;
  int32_t mrep;
  bool merge;
  const uint32_t* tgt_bits;
  Sink sink;
  unsigned long long* dbg;  // diagnostic build only (KP_STAMPS): per-phase cycle sums
};

KP_HD inline int32_t est_merge(const SelCtx& x, int32_t r) { return x.merge ? cal_merge_bf(x.mrep, r) : r; }
KP_HD inline int32_t est_at(const SelCtx& x, int c) { return est_merge(x, x.erow[c]); }

// Diagnostic phase stamps (a separate -DKP_STAMPS build; never in libkp.so). Each
// workgroup adds into one of kDbgSpread copies of the kDbgSlots counters (by its index),
// so the atomics of concurrent waves do not contend for one address (a contended atomic
// holds back every later load of its wave, which the stamps would then count); the host
// sums the copies.
constexpr int kDbgSlots = 96;
#if defined(KP_STAMPS)
constexpr int kDbgSpread = 256;
#else
constexpr int kDbgSpread = 1;
#endif
#define KP_DBG_AT(i) ((i) + kDbgSlots * (int)(blockIdx.x & (kDbgSpread - 1)))
#if defined(KP_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define KP_STAMP_INIT unsigned long long kp_t0 = __builtin_amdgcn_s_memtime();
#define KP_STAMP(ctx_, i)                                                \
  do {                                                                   \
    if (threadIdx.x == 0 && (ctx_).dbg) {                                \
      unsigned long long t = __builtin_amdgcn_s_memtime();               \
      atomicAdd(&(ctx_).dbg[KP_DBG_AT(i)], t - kp_t0);                   \
      kp_t0 = t;                                                         \
    }                                                                    \
  } while (0)
#define KP_COUNT(ctx_, i, v)                                             \
  do {                                                                   \
    if (threadIdx.x == 0 && (ctx_).dbg) atomicAdd(&(ctx_).dbg[KP_DBG_AT(i)], (unsigned long long)(v)); \
  } while (0)
#define KP_STAMPD(dbg, i)                                                \
  do {                                                                   \
    if (threadIdx.x == 0 && (dbg)) {                                     \
      unsigned long long t = __builtin_amdgcn_s_memtime();               \
      atomicAdd(&(dbg)[KP_DBG_AT(i)], t - kp_t0);                        \
      kp_t0 = t;                                                         \
    }                                                                    \
  } while (0)
#else
#define KP_STAMP_INIT
#define KP_STAMP(x, i) \
  do {                 \
  } while (0)
#define KP_STAMPD(dbg, i) \
  do {                    \
  } while (0)
#if defined(KP_STAMPS)  // host build with -DKP_STAMPS: the counters only (one thread per block)
#define KP_COUNT(ctx_, i, v)                                                                        \
  do {                                                                                              \
    if ((ctx_).dbg) __atomic_fetch_add(&(ctx_).dbg[i], (unsigned long long)(v), __ATOMIC_RELAXED); \
  } while (0)
#else
#define KP_COUNT(x, i, v) \
  do {                    \
  } while (0)
#endif
#endif

struct SerialOut {
  int status = 0;
  int err = 0;
  int64_t arg = 0;
  int n = 0;
};

// ----------------------------------------------------------------------------
// Serial exact emulation (thread 0) of AssignReplicas over an explicit list.
// ----------------------------------------------------------------------------
struct SerialAssign {
  const SelCtx& x;
  SerialScratch& sc;
  bool desc;

  KP_HD int tgt_cnt() const { return x.h->tgt_cnt; }
  KP_HD uint32_t tgt_rank(int j) const { return (uint32_t)x.bv->ipool[x.h->tgt_off + 2 * j]; }
  KP_HD int32_t tgt_rep(int j) const { return x.bv->ipool[x.h->tgt_off + 2 * j + 1]; }

  // Dispenser(num, nil, uid).AllocateByWeight over entries en/ew[0..ne)
  // (binding.go:94-115, webstermethod.go:112-161); all parties with their seats
  // (name order) into tn/tr; returns the count.
  KP_HD int dispense(int32_t num, int ne) {
    int64_t sum = 0;
    for (int i = 0; i < ne; i++) sum = add64(sum, sc.ew[i]);
    if (sum == 0) return 0;
    int np = 0;
    for (int i = 0; i < ne; i++) {  // partyVotes map: later entries overwrite
      int k = -1;
      if (sc.pos) {
        k = sc.pos[sc.en[i]];
      } else {
        for (int j = 0; j < np; j++)
          if (sc.pn[j] == sc.en[i]) {
            k = j;
            break;
          }
      }
      if (k < 0) {
        k = np++;
        sc.pn[k] = sc.en[i];
        if (sc.pos) sc.pos[sc.en[i]] = k;
      }
      sc.pv[k] = sc.ew[i];
    }
    if (sc.pos)
      for (int k = 0; k < np; k++) sc.pos[sc.pn[k]] = -1;
    // Parties keep list order: the heap compares names itself and the result is
    // compared as a multiset, so the final sort by name is not materialised.
    webster_serial(sc.pn, sc.pv, sc.ps, sc.ph, np, num, desc);
    for (int i = 0; i < np; i++) {
      sc.tn[i] = sc.pn[i];
      sc.tr[i] = sc.ps[i];
    }
    return np;
  }

  // util.MergeTargetClusters (pkg/util/binding.go:91-115) of old=(sn,sr,ns)
  // with new=(tn,tr,nt) into (tn,tr); returns the count.
  KP_HD int merge(int ns, int nt) {
    if (ns == 0) return nt;
    if (nt == 0) {
      for (int i = 0; i < ns; i++) {
        sc.tn[i] = sc.sn[i];
        sc.tr[i] = sc.sr[i];
      }
      return ns;
    }
    int nu = 0;  // oldMap, last value wins
    for (int i = 0; i < ns; i++) {
      int k = -1;
      if (sc.pos) {
        k = sc.pos[sc.sn[i]];
      } else {
        for (int j = 0; j < nu; j++)
          if (sc.xn[j] == sc.sn[i]) k = j;
      }
      if (k < 0) {
        k = nu++;
        sc.xn[k] = sc.sn[i];
        if (sc.pos) sc.pos[sc.sn[i]] = k;
      }
      sc.xr[k] = sc.sr[i];
      sc.xf[k] = 1;
    }
    for (int i = 0; i < nt; i++) {
      int k = -1;
      if (sc.pos) {
        k = sc.pos[sc.tn[i]];
      } else {
        for (int j = 0; j < nu; j++)
          if (sc.xn[j] == sc.tn[i]) {
            k = j;
            break;
          }
      }
      if (k >= 0 && sc.xf[k]) {
        sc.tr[i] = add32(sc.tr[i], sc.xr[k]);
        sc.xf[k] = 0;
      }
    }
    for (int j = 0; j < nu; j++) {
      if (sc.pos) sc.pos[sc.xn[j]] = -1;
      if (sc.xf[j]) {
        sc.tn[nt] = sc.xn[j];
        sc.tr[nt] = sc.xr[j];
        nt++;
      }
    }
    return nt;
  }

  // dynamicDivideReplicas (division_algorithm.go:75-101); available list in
  // an/ar[0..na); scheduled (for merge) in sn/sr[0..ns).
  KP_HD bool divide(int na, int32_t target, int ns, int code, SerialOut& o, int* nt_out) {
    int32_t availableReplicas = 0;
    for (int i = 0; i < na; i++) availableReplicas = add32(availableReplicas, sc.ar[i]);
    if (availableReplicas < target) {
      o.status = KP_STATUS_UNSCHEDULABLE;
      o.err = code;
      o.arg = availableReplicas;
      return false;
    }
    int st = x.h->strategy;
    if (st == ST_AGGREGATED) {
      // resortAvailableClusters (assignment.go:151-178): prior = scheduled with replicas > 0
      bool anyPrior = false;
      for (int j = 0; j < ns; j++)
        if (sc.sr[j] > 0) anyPrior = true;
      if (anyPrior) {
        int k = 0;
        if (sc.pos)
          for (int j = 0; j < ns; j++)
            if (sc.sr[j] > 0) sc.pos[sc.sn[j]] = 1;
        for (int pass = 0; pass < 2; pass++)
          for (int i = 0; i < na; i++) {
            bool pr = false;
            if (sc.pos) pr = sc.pos[sc.an[i]] == 1;
            else
              for (int j = 0; j < ns && !pr; j++) pr = sc.sr[j] > 0 && sc.sn[j] == sc.an[i];
            if (pr == (pass == 0)) {
              sc.xn[k] = sc.an[i];
              sc.xr[k] = sc.ar[i];
              k++;
            }
          }
        for (int i = 0; i < na; i++) {
          sc.an[i] = sc.xn[i];
          sc.ar[i] = sc.xr[i];
        }
        if (sc.pos)
          for (int j = 0; j < ns; j++) sc.pos[sc.sn[j]] = -1;
      }
      int32_t sum = 0;
      for (int i = 0; i < na; i++) {
        sum = add32(sum, sc.ar[i]);
        if (sum >= target) {
          na = i + 1;
          break;
        }
      }
    } else if (st != ST_DYNAMIC) {
      o.status = KP_STATUS_ERROR;
      o.err = KP_ERR_UNDEFINED_STRATEGY;
      return false;
    }
    // SpreadReplicasByTargetClusters: weights = int64(Replicas) (binding.go:157-183)
    for (int i = 0; i < na; i++) {
      sc.en[i] = sc.an[i];
      sc.ew[i] = (int64_t)sc.ar[i];
    }
    int nt = dispense(target, na);
    *nt_out = merge(ns, nt);
    return true;
  }

  // assignFuncMap strategies (assignment.go:181-244) over list[0..m) with `rep`
  // replicas; result in tn/tr, count in *nt. Returns false on error.
  KP_HD bool strategy(const Item* list, int m, int32_t rep, SerialOut& o, int* nt) {
    const BindHdr& h = *x.h;
    int st = h.strategy;
    if (st == ST_NONE) {
      o.status = KP_STATUS_ERROR;
      o.err = KP_ERR_UNSUPPORTED_STRATEGY;
      return false;
    }
    if (st == ST_DUPLICATED) {
      for (int i = 0; i < m; i++) {
        sc.tn[i] = list[i].rank;
        sc.tr[i] = rep;
      }
      *nt = m;
      return true;
    }
    if (st == ST_STATIC) {
      // getStaticWeightInfoList (division_algorithm.go:38-72)
      int ne = 0;
      for (int i = 0; i < m; i++) {
        int64_t w = 0;
        if (!(h.flags & BF_HAS_WP)) {
          w = 1;  // getDefaultWeightPreference: {ClusterNames:[name]} weight 1
        } else {
          for (int j = 0; j < h.sw_cnt; j++)
            if (prog_match(*x.s, *x.bv, x.bv->ipool[h.sw_off + j], (int)list[i].rank)) {
              int64_t rw = x.bv->lpool[h.sw_w_off + j];
              if (rw > w) w = rw;
            }
        }
        if (w > 0) {
          sc.en[ne] = list[i].rank;
          sc.ew[ne] = w;
          ne++;
        }
      }
      int64_t sum = 0;
      for (int i = 0; i < ne; i++) sum = add64(sum, sc.ew[i]);
      if (sum == 0)
        for (int i = 0; i < m; i++) {
          sc.en[ne] = list[i].rank;
          sc.ew[ne] = 1;
          ne++;
        }
      *nt = dispense(rep, ne);
      return true;
    }
    // assignByDynamicStrategy
    int ns = 0;
    if (sc.pos)
      for (int i = 0; i < m; i++) sc.pos[list[i].rank] = 1;
    for (int j = 0; j < tgt_cnt(); j++) {  // buildScheduledClusters (assignment.go:125-142)
      uint32_t r = tgt_rank(j);
      bool cand = false;
      if (sc.pos) cand = sc.pos[r] == 1;
      else
        for (int i = 0; i < m && !cand; i++) cand = list[i].rank == r;
      if (cand) {
        sc.sn[ns] = r;
        sc.sr[ns] = tgt_rep(j);
        ns++;
      }
    }
    if (sc.pos)
      for (int i = 0; i < m; i++) sc.pos[list[i].rank] = -1;
    int32_t assigned = 0;
    for (int j = 0; j < ns; j++) assigned = add32(assigned, sc.sr[j]);
    if ((h.flags & BF_FRESH) && sc.presorted) return divide(m, rep, 0, KP_ERR_FRESH_NOT_ENOUGH, o, nt);
    if (h.flags & BF_FRESH) {  // dynamicFreshScale (division_algorithm.go:139-166)
      for (int i = 0; i < m; i++) {
        sc.an[i] = list[i].rank;
        sc.ar[i] = list[i].alloc;
      }
      if (sc.pos) {
        for (int i = m - 1; i >= 0; i--) sc.pos[sc.an[i]] = i;  // first occurrence
        for (int j = 0; j < ns; j++) {
          int i = sc.pos[sc.sn[j]];
          if (i >= 0) sc.ar[i] = add32(sc.ar[i], sc.sr[j]);
        }
        for (int i = 0; i < m; i++) sc.pos[sc.an[i]] = -1;
      } else {
        for (int j = 0; j < ns; j++)
          for (int i = 0; i < m; i++)
            if (sc.an[i] == sc.sn[j]) {
              sc.ar[i] = add32(sc.ar[i], sc.sr[j]);
              break;
            }
      }
      sort_tcl(sc.an, sc.ar, m);
      return divide(m, rep, 0, KP_ERR_FRESH_NOT_ENOUGH, o, nt);
    }
    if (assigned > rep) {  // dynamicScaleDown (:103-119)
      for (int j = 0; j < ns; j++) {
        sc.an[j] = sc.sn[j];
        sc.ar[j] = sc.sr[j];
      }
      sort_tcl(sc.an, sc.ar, ns);
      return divide(ns, rep, 0, KP_ERR_SCALE_DOWN_NOT_ENOUGH, o, nt);
    }
    if (assigned < rep && sc.presorted) return divide(m, sub32(rep, assigned), ns, KP_ERR_SCALE_UP_NOT_ENOUGH, o, nt);
    if (assigned < rep) {  // dynamicScaleUp (:121-136)
      for (int i = 0; i < m; i++) {
        sc.an[i] = list[i].rank;
        sc.ar[i] = list[i].alloc;
      }
      sort_tcl(sc.an, sc.ar, m);
      return divide(m, sub32(rep, assigned), ns, KP_ERR_SCALE_UP_NOT_ENOUGH, o, nt);
    }
    for (int j = 0; j < ns; j++) {
      sc.tn[j] = sc.sn[j];
      sc.tr[j] = sc.sr[j];
    }
    *nt = ns;
    return true;
  }

  // assignReplicasToClusters (common.go:141-154): strategy + removeZeroReplicasCluster,
  // appended to rn/rr at o.n.
  KP_HD bool to_clusters(const Item* list, int m, int32_t rep, SerialOut& o) {
    int nt = 0;
    if (!strategy(list, m, rep, o, &nt)) return false;
    for (int i = 0; i < nt; i++)
      if (sc.tr[i] > 0) {
        sc.rn[o.n] = sc.tn[i];
        sc.rr[o.n] = sc.tr[i];
        o.n++;
      }
    return true;
  }

  // AssignReplicas (common.go:51-83) + assignWorkloadReplicas (:97-139) +
  // attachZeroReplicasCluster (util.go:174-186).
  KP_HD SerialOut run(const Item* items, int n) {
    SerialOut o;
    const BindHdr& h = *x.h;
    if (n == 0) {
      o.status = KP_STATUS_ERROR;
      o.err = KP_ERR_NO_CLUSTERS;
      return o;
    }
    if (!(h.flags & BF_WORKLOAD_ASSIGN)) {
      for (int i = 0; i < n; i++) {
        sc.rn[i] = items[i].rank;
        sc.rr[i] = 0;
      }
      o.n = n;
    } else if (h.flags & BF_OVERFLOW) {
      int maxOrder = 0;
      for (int i = 0; i < n; i++)
        if (items[i].ovf > maxOrder) maxOrder = items[i].ovf;
      int32_t remaining = h.replicas;
      for (int t = 0; t <= maxOrder; t++) {
        int m = 0;
        int64_t tierAvail = 0;
        for (int i = 0; i < n; i++)
          if (items[i].ovf == t) {
            sc.tier[m++] = items[i];
            tierAvail += items[i].avail;
          }
        if (m == 0) continue;
        int32_t rep_t = (int32_t)((int64_t)remaining < tierAvail ? (int64_t)remaining : tierAvail);
        if (!to_clusters(sc.tier, m, rep_t, o)) {
          o.n = 0;
          return o;
        }
        remaining = sub32(remaining, rep_t);
        if (remaining <= 0) break;
      }
      if (remaining > 0) {
        o.status = KP_STATUS_UNSCHEDULABLE;
        o.err = KP_ERR_OVERFLOW_NOT_ENOUGH;
        o.n = 0;
        return o;
      }
    } else {
      if (!to_clusters(items, n, h.replicas, o)) {
        o.n = 0;
        return o;
      }
    }
    if (h.flags & BF_EMPTY_PROP) {
      int base = o.n;
      if (sc.pos)
        for (int j = 0; j < base; j++) sc.pos[sc.rn[j]] = 1;
      for (int i = 0; i < n; i++) {
        bool have = false;
        if (sc.pos) have = sc.pos[items[i].rank] == 1;
        else
          for (int j = 0; j < base && !have; j++) have = sc.rn[j] == items[i].rank;
        if (!have) {
          sc.rn[o.n] = items[i].rank;
          sc.rr[o.n] = 0;
          o.n++;
        }
      }
      if (sc.pos)
        for (int j = 0; j < base; j++) sc.pos[sc.rn[j]] = -1;
    }
    return o;
  }
};

// Writes a serial result (thread 0 only).
KP_HD inline void sink_serial(const SelCtx& x, const SerialScratch& sc, const SerialOut& o) {
  const Sink& k = x.sink;
  int b = x.b;
  k.status[b] = o.status;
  k.err[b] = o.err;
  k.arg[b] = o.arg;
  if (o.status != KP_STATUS_OK || o.n == 0) {
    k.start[b] = 0;
    k.count[b] = 0;
    return;
  }
  // The binding's own slot when the list fits it (out_cap = min(C, Replicas) +
  // len(spec.Clusters) bounds every AssignReplicas result: the positive new entries
  // of all overflow tiers hold at most Replicas seats on distinct candidates, and
  // MergeTargetClusters adds only scheduled clusters, each in one tier); else the
  // shared area past every slot, checked against its end so a wrong bound reports
  // an error instead of writing past the allocation.
  unsigned long long base = (uint64_t)o.n <= x.h->out_cap ? (unsigned long long)x.h->out_off
                                                          : kp_atomic_add(k.counter, (unsigned long long)o.n);
  if (base + (uint64_t)o.n > k.cap_end) {
    k.status[b] = KP_STATUS_ERROR;
    k.err[b] = KP_ERR_RESULT_CAPACITY;
    k.arg[b] = o.n;
    k.start[b] = 0;
    k.count[b] = 0;
    return;
  }
  k.start[b] = base;
  k.count[b] = (uint32_t)o.n;
  for (int i = 0; i < o.n; i++) {
    k.out_idx[base + i] = sc.rn[i];  // (rank: k_compact maps it)
    k.out_rep[base + i] = sc.rr[i];
  }
}
KP_HD inline void sink_error(const SelCtx& x, int status, int err, int64_t arg) {
  const Sink& k = x.sink;
  k.status[x.b] = status;
  k.err[x.b] = err;
  k.arg[x.b] = arg;
  k.start[x.b] = 0;
  k.count[x.b] = 0;
}

// StaticWeight vote of cluster c: the largest matching rule weight, saturated at
// MaxInt32 (getStaticWeightInfoList, division_algorithm.go:41-48).
KP_HD inline int32_t static_vote(const SelCtx& x, int c) {
  const BindHdr& h = *x.h;
  int64_t wt = 0;
  if (!(h.flags & BF_HAS_WP)) {
    wt = 1;
  } else {
    for (int j = 0; j < h.sw_cnt; j++)
      if (prog_match(*x.s, *x.bv, x.bv->ipool[h.sw_off + j], c)) {
        int64_t rw = x.bv->lpool[h.sw_w_off + j];
        if (rw > wt) wt = rw;
      }
  }
  return (int32_t)(wt > kInt32Max ? kInt32Max : wt);
}

// ----------------------------------------------------------------------------
// Candidate gather: feasible clusters of the binding in rank order.
// ----------------------------------------------------------------------------
struct alignas(16) I32x4 {
  int32_t v[4];
};
// `between()` runs after the vector form has issued its row loads and before it
// uses them (block-uniform; it may contain barriers), so independent setup
// work overlaps the row's memory latency.
template <class BLK, class Between>
KP_FI int gather(const BLK& B, const SelCtx& x, Cands cd, bool weights, Between between) {
  // Vector form (no overflow tiers, AllocatableReplicas votes): thread t owns
  // the 4-cluster units t + nth*j and issues every 16-B row load before the
  // first use, so a binding's row costs one memory latency, not one per unit.
  constexpr int kJ = 8;
  const int nu = (x.s->Cp + 3) >> 2;
  if (!weights && x.h->ovf_mode == OVF_ZERO && nu <= kJ * B.nth()) {
    const int tid = B.tid(), nth = B.nth();
    const I32x4* e4 = (const I32x4*)x.erow;
    uint32_t fm[kJ];
    I32x4 ev[kJ];
    int32_t mine = 0;
KP_UNROLL
    for (int j = 0; j < kJ; j++) {
      const int u = tid + nth * j;
      fm[j] = u < nu ? (uint32_t)(x.frow[u >> 4] >> ((u & 15) * 4)) & 0xFu : 0u;
      if (u < nu) ev[j] = e4[u];  // not behind the mask: one memory latency for both
      mine += popc64(fm[j]);
    }
    between();
    int32_t F;
    int32_t pos = B.excl_scan(mine, &F);
KP_UNROLL
    for (int j = 0; j < kJ; j++)
      for (int q = 0; q < 4; q++)
        if ((fm[j] >> q) & 1u) {
          cd.r[pos] = (uint32_t)(4 * (tid + nth * j) + q);
          cd.v[pos] = est_merge(x, ev[j].v[q]);
          pos++;
        }
    B.sync();
    return F;
  }
  // Thread t owns clusters t + nth*j: one pass counts them (the feasibility word
  // is a broadcast load per wave), one scan places them, and the second pass
  // reads erow fully coalesced with no barrier between iterations. Candidate
  // order is thread-major; nothing downstream depends on it (keys carry ranks).
  between();
  const SnapView& s = *x.s;
  const BindHdr& h = *x.h;
  const int tid = B.tid(), nth = B.nth();
  int32_t mine = 0;
  for (int c = tid; c < s.C; c += nth) mine += mask_test(x.frow, c) ? 1 : 0;
  int32_t F;
  int32_t pos = B.excl_scan(mine, &F);
  for (int c = tid; c < s.C; c += nth)
    if (mask_test(x.frow, c)) {
      cd.r[pos] = (uint32_t)c | ((uint32_t)overflow_order(s, *x.bv, h, c) << kRankBits);
      cd.v[pos] = weights ? static_vote(x, c) : est_at(x, c);
      pos++;
    }
  B.sync();
  return F;
}

template <class BLK>
KP_FI int gather(const BLK& B, const SelCtx& x, Cands cd, bool weights) {
  return gather(B, x, cd, weights, [] {});
}

// ----------------------------------------------------------------------------
// Block-parallel exact Webster over a candidate subset with int32 votes >= 0.
// ----------------------------------------------------------------------------
struct WebRes {
  int mode;       // 0 no parties, 1 all zero seats, 2 normal
  double t;       // t*
  double rt = 0;  // fl(1 / t*) (w_count_r)
  uint64_t tie;   // tie-key threshold (inclusive)
  int32_t N;
  bool desc;
  // mode 2 with compact: every party with a seat is among the np entries of pl
  // ((rank << 32) | votes, votes >= Lb); the list stays valid after the return.
  bool compact = false;
  int32_t np = 0;
  int64_t Lb = 1;
  const uint64_t* pl = nullptr;
};
KP_HD inline uint64_t tie_key(int64_t base, uint32_t rank, bool desc) {
  return ((uint64_t)base << kRankBits) | (desc ? (uint64_t)(kRankMask - rank) : (uint64_t)rank);
}
KP_HD inline int32_t web_seats(const WebRes& w, int64_t v, uint32_t rank) {
  if (w.mode != 2 || (double)v < w.t) return 0;  // every priority of v is below t*
  int64_t base = w_count_r(v, w.t, w.rt, (int64_t)w.N + 1, false);
  if (base < w.N && w_prio(v, base) == w.t && tie_key(base, rank, w.desc) <= w.tie) base++;
  return (int32_t)base;
}

// Scratch for the exact selection steps (LDS): a 256-bin histogram and a key
// buffer of `cap` u64 entries. cap == 0 -> bisection only.
struct SelScratch {
  uint32_t* hist;
  unsigned long long* whist;  // 256 u64 bins (weighted selection); may alias hist storage
  uint64_t* buf;
  int cap;
  unsigned long long* dbg = nullptr;  // diagnostic build only (KP_STAMPS)
};

// Enumeration capacity (u64 entries) of the SEL_ALL selection buffer.
// 1024 entries (8 KB) keep k_select_all's LDS under a third of the CU's 160 KB at
// C = 5k; larger party sets fall back to the uncompacted (exact) Webster passes.
#ifndef KP_ECAP_MAX
#define KP_ECAP_MAX 1024
#endif
KP_HD inline int sel_all_ecap(int Cp) { return Cp / 2 < 64 ? 64 : (Cp / 2 > KP_ECAP_MAX ? KP_ECAP_MAX : Cp / 2); }
KP_HD inline SelScratch carve_sel_scratch(unsigned char* p, int Cp) {
  SelScratch ss;
  ss.whist = (unsigned long long*)p;
  ss.hist = (uint32_t*)(ss.whist + 256);
  ss.buf = (uint64_t*)(ss.hist + 256);
  ss.cap = sel_all_ecap(Cp);
  return ss;
}

template <class BLK, class Pred, class Key>
KP_FI uint64_t radix_select(const BLK& B, uint32_t* hist, int F, Pred pred, Key key, int64_t k);

// k-th largest (1-based) vote over the parties with votes in [1, 2^31), counted
// with multiplicity (k <= #parties with v > 0): 8-bit radix descent over the
// bytes in which the votes differ.
template <class BLK, class Parties>
KP_FI int64_t kth_largest_vote(const BLK& B, uint32_t* hist, Parties parties, int64_t k) {
  uint64_t an = ~0ull, on = 0;
  parties([&](uint32_t, int64_t v) {
    if (v > 0) {
      an &= (uint64_t)v;
      on |= (uint64_t)v;
    }
  });
  B.andor(an, on);
  const uint64_t diff = an ^ on;
  if (diff == 0) return (int64_t)an;
  int top = 31;
  while (!((diff >> top) & 1)) top--;
  const int start = (top / 8) * 8;
  uint32_t prefix = start >= 24 ? 0u : (uint32_t)(an & (~0ull << (start + 8)));
  for (int shift = start; shift >= 0; shift -= 8) {
    for (int i = B.tid(); i < 256; i += B.nth()) hist[i] = 0;
    B.sync();
    const uint32_t hm = shift >= 24 ? 0u : (~0u << (shift + 8));
    parties([&](uint32_t, int64_t v64) {
      const uint32_t v = (uint32_t)v64;
      if (v64 > 0 && (v & hm) == (prefix & hm)) kp_atomic_add(&hist[(v >> shift) & 255], 1u);
    });
    int64_t before;
    const int bin = B.find_bin(hist, k, &before, true);
    k -= before;
    prefix |= (uint32_t)bin << shift;
  }
  return (int64_t)prefix;
}

// Octave bins of a vote in [1, 2^31): (floor(log2 v), next 3 bits), monotone
// in v; vote_bin_floor(b) is the smallest vote in bin b.
KP_HD inline int vote_bin(uint32_t v) {
  const int e = 31 - __builtin_clz(v);
  const uint32_t m = e >= 3 ? (v >> (e - 3)) & 7u : (v << (3 - e)) & 7u;
  return e * 8 + (int)m;
}
KP_HD inline int64_t vote_bin_floor(int b) { return ((int64_t)(8 + (b & 7)) << (b >> 3)) >> 3; }

// k-th largest (1-based) of E <= 64 * (waves) u64 keys in LDS by rank counting:
// the key x with #(> x) < k <= #(>= x). desc = false selects the k-th smallest.
// Every thread gets the answer (one barrier).
template <class BLK>
KP_FI uint64_t rank_select(const BLK& B, const uint64_t* keys, int E, int64_t k, bool largest, uint64_t* slot) {
  for (int i = B.tid(); i < E; i += B.nth()) {
    const uint64_t x = keys[i];
    int64_t before = 0, upto = 0;
    for (int j = 0; j < E; j++) {
      const uint64_t y = keys[j];
      before += largest ? (y > x) : (y < x);
      upto += y == x ? 1 : 0;
    }
    upto += before;
    if (before < k && k <= upto) *slot = x;  // every writer writes the same value
  }
  B.sync();
  return *slot;
}

// AllocateWebsterSeats (webstermethod.go:112-161) for parties with int32 votes
// >= 0 and no initial seats, block-parallel. `parties(fn)` calls fn(rank, votes)
// for every party the calling thread owns. The N-th largest seat priority
// t* = max{t : cnt_ge(t) >= N} is bracketed by the divisor-method bounds
//   V/(2N+P) <= t* < V/(2N-P-1)   (P = parties with votes > 0)
// and by t* >= the N-th largest vote >= Lb (every party's first priority is its
// vote). Parties below Lb take no seat: the rest are compacted into LDS (when
// they fit) so every later pass walks only them. The bracket is verified with
// exact counts and bisected over the double's bit pattern until at most 64
// priorities remain, which are enumerated and rank-selected.
// Seats strictly above t* are exact per party; the tie group at t* is ordered
// by (seats asc, name) as the heap's tie-breaker orders it (tie_key).
// Totals of the party votes a caller already took in its own pass (with the octave
// histogram in sc.hist and the party-list counter zeroed): webster_par skips its first pass.
struct WebPre {
  int64_t V, vmax, P;
};
// webster_par's last steps from t*: the seats strictly above t*, then the tie group
// at t* ordered by (seats asc, name) as the heap's tie-breaker orders it.
constexpr int kWebFirstMax = 128;  // compacted lists rank-selected for the first-seat case
template <class BLK, class Parties>
KP_FI WebRes webster_tail(const BLK& B, WebRes r, Parties parties, double tstar, int32_t N, bool desc,
                          const SelScratch& sc, int ecap, bool compact, int32_t np, int64_t Lb, uint64_t* pl) {
  r.t = tstar;
  r.rt = 1.0 / tstar;
  r.compact = compact;
  r.np = np;
  r.Lb = Lb;
  r.pl = pl;
  KP_STAMP_INIT
  KP_STAMPD(sc.dbg, 67);
  // seats strictly above t*, then the tie group at t* ordered by (k asc, name)
  int64_t S = 0, T = 0;
  const double rts = 1.0 / tstar;
  parties([&](uint32_t, int64_t v) {
    int64_t base = w_count_r(v, tstar, rts, (int64_t)N + 1, false);
    S += base;
    if (w_prio(v, base) == tstar) T++;
  });
  B.sum2(S, T);
  const int64_t M = (int64_t)N - S;
  KP_STAMPD(sc.dbg, 68);
  if (M >= T) {
    r.tie = ~0ull;
  } else if (T <= (int64_t)ecap) {
    int32_t mine = 0;
    parties([&](uint32_t, int64_t v) {
      int64_t base = w_count_r(v, tstar, rts, (int64_t)N + 1, false);
      if (w_prio(v, base) == tstar) mine++;
    });
    int32_t n;
    int32_t pos = B.excl_scan(mine, &n);
    parties([&](uint32_t rk, int64_t v) {
      int64_t base = w_count_r(v, tstar, rts, (int64_t)N + 1, false);
      if (w_prio(v, base) == tstar) sc.buf[pos++] = tie_key(base, rk, desc);
    });
    B.sync();
    r.tie = rank_select(B, sc.buf, n, M, false, (uint64_t*)sc.whist);
  } else {
    uint64_t tlo = 0, thi = (uint64_t)1 << 62;  // smallest x with count(tk <= x) >= M
    while (tlo < thi) {
      uint64_t mid = tlo + (thi - tlo) / 2;
      int64_t c = 0;
      parties([&](uint32_t rk, int64_t v) {
        int64_t base = w_count_r(v, tstar, rts, (int64_t)N + 1, false);
        if (w_prio(v, base) == tstar && tie_key(base, rk, desc) <= mid) c++;
      });
      c = B.sum64(c);
      if (c >= M) thi = mid;
      else tlo = mid + 1;
    }
    r.tie = tlo;
  }
  KP_STAMPD(sc.dbg, 69);
  B.sync();  // buf[0, 64) / whist are free again for the caller; pl stays
  return r;
}

KP_HD inline uint32_t* web_ctr(const SelScratch& sc) { return (uint32_t*)sc.whist + 511; }  // party list fill counter
template <class BLK>
KP_FI WebRes webster_reg(const BLK& B, bool party, uint32_t rk, int64_t v, int32_t N, bool desc, int64_t V, bool* ok,
                         int* nsteps = nullptr);
template <class BLK, class Parties>
KP_FI WebRes webster_par(const BLK& B, Parties all_parties, int32_t N, bool desc, const SelScratch& sc,
                         const WebPre* pre = nullptr) {
  KP_STAMP_INIT
  WebRes r;
  r.N = N;
  r.desc = desc;
  r.t = 0;
  r.tie = 0;
  uint32_t* ctr = web_ctr(sc);
  int64_t V = 0, vmax = 0, P = 0, none = 0;
  if (pre) {
    V = pre->V;
    vmax = pre->vmax;
    P = pre->P;
  } else {
    // One pass: totals and the octave histogram of the votes (kth_vote_floor).
    for (int i = B.tid(); i < 256; i += B.nth()) sc.hist[i] = 0;
    if (B.tid() == 0) *ctr = 0;
    B.sync();
    all_parties([&](uint32_t, int64_t v) {
      V += v;
      if (v > vmax) vmax = v;
      if (v > 0) {
        P++;
        kp_atomic_add(&sc.hist[vote_bin((uint32_t)v)], 1u);
      }
    });
    auto add = [](int64_t p, int64_t q) { return p + q; };
    B.reduce4(V, add, 0, P, add, 0, vmax, [](int64_t p, int64_t q) { return p > q ? p : q; }, INT64_MIN, none, add, 0);
  }
  if (V == 0) {
    r.mode = 0;
    return r;
  }
  if (N <= 0) {
    r.mode = 1;
    return r;
  }
  r.mode = 2;
  // LDS areas of sc.buf: [0, ecap) enumeration / rank selection, [64, cap) parties
  const int ecap = sc.cap < 64 ? sc.cap : 64;
  const int pcap = sc.cap > 64 ? sc.cap - 64 : 0;
  uint64_t* pl = sc.buf + 64;
  int64_t Lb = 1;
  // (few parties: all of them go to the list, where the quota search below needs no Lb)
  if (P > (int64_t)N && (P > (int64_t)ecap || pcap < ecap)) {  // lower edge of the octave bin holding the N-th largest vote
    int64_t before;
    Lb = vote_bin_floor(B.find_bin(sc.hist, (int64_t)N, &before, true));
  }
  int32_t np = 0;
  bool compact = false;
  for (int attempt = 0; attempt < 2 && pcap > 0; attempt++) {
    // parties with v >= Lb into pl: per-wave slot reservation, one barrier
    int32_t mine = 0;
    all_parties([&](uint32_t, int64_t v) { mine += v >= Lb ? 1 : 0; });
    int32_t pos = B.wave_reserve(mine, ctr);
    all_parties([&](uint32_t rk, int64_t v) {
      if (v >= Lb) {
        if (pos < pcap) pl[pos] = ((uint64_t)rk << 32) | (uint64_t)(uint32_t)v;
        pos++;
      }
    });
    B.sync();
    np = (int32_t)*ctr;
    if (np <= pcap) {
      compact = true;
      break;
    }
    // the octave bin was crowded: the exact N-th largest vote, then retry once
    if (attempt == 0 && P > (int64_t)N) {
      Lb = kth_largest_vote(B, sc.hist, all_parties, (int64_t)N);  // (barriers: every thread read ctr)
      if (B.tid() == 0) *ctr = 0;
      B.sync();
    } else {
      break;
    }
  }
  auto parties = [&](auto fn) {
    if (compact) {
      for (int i = B.tid(); i < np; i += B.nth()) {
        const uint64_t e = pl[i];
        fn((uint32_t)(e >> 32), (int64_t)(uint32_t)e);
      }
    } else {
      all_parties([&](uint32_t rk, int64_t v) {
        if (v >= Lb) fn(rk, v);
      });
    }
  };
  KP_STAMPD(sc.dbg, 64);
  const int64_t capN = (int64_t)N;
  // Few parties (the compacted list fits the enumeration area): t* by adjusting the
  // quota counts. At t0 = V / 2N each party holds s = #{k : prio(v, k) >= t0} =
  // floor(N v / V + 1/2) <= N priorities, within np/2 of N in total. With C of them,
  // t* (the N-th largest priority) is found by dropping the C - N smallest held ones
  // (each party's smallest held priority is prio(v, s - 1)) or adding the N - C
  // largest next ones (prio(v, s)), one block-wide min or max per step. Parties
  // below Lb hold no priority >= t* (t* >= the N-th largest vote >= Lb, or Lb = 1),
  // so the list decides t*. The held counts live in buf[0, np) until webster_tail.
  // One wave (k_select_top's subsets past 64 candidates): the list holds one party per lane,
  // so webster_reg runs the same adjustment in registers (the winner alone recomputes its
  // priority; no pass over the list per step) and the same tie selection.
  if (B.nwaves() == 1 && compact && np > 0 && np <= ecap && np <= B.nth()) {
    const bool party = B.tid() < np;
    const uint64_t e = party ? pl[B.tid()] : 0ull;
    bool ok = false;
    WebRes w = webster_reg(B, party, (uint32_t)(e >> 32), (int64_t)(uint32_t)e, N, desc, V, &ok);
    if (ok) {
      KP_COUNT(sc, 80, 1);
      w.compact = true;
      w.np = np;
      w.Lb = Lb;
      w.pl = pl;
      return w;
    }
  } else if (compact && np > 0 && np <= ecap) {
    constexpr int64_t kAdjMax = 64;
    const double t0 = (double)V / (2.0 * (double)N);
    int64_t C = 0;
    for (int i = B.tid(); i < np; i += B.nth()) {
      const int64_t s = w_count((int64_t)(uint32_t)pl[i], t0, capN + 1, true);
      sc.buf[i] = (uint64_t)s;
      C += s;
    }
    C = B.sum64(C);  // (its barrier also orders the counts before the steps read them)
    const int64_t steps = C >= (int64_t)N ? C - (int64_t)N : (int64_t)N - C;
    if (steps <= kAdjMax) {
      const bool drop = C >= (int64_t)N;
      double tstar = 0;
      for (int64_t left = steps;; left--) {
        // this thread's best held (drop: smallest) or next (add: largest) priority
        uint64_t best = drop ? ~0ull : 0ull;
        int64_t bi = INT64_MAX;
        for (int i = B.tid(); i < np; i += B.nth()) {
          const int64_t v = (int64_t)(uint32_t)pl[i], s = (int64_t)sc.buf[i];
          if (drop && s == 0) continue;
          const uint64_t p = kp_dbits(w_prio(v, drop ? s - 1 : s));  // positive doubles order as their bits
          if (drop ? p < best : p > best) {
            best = p;
            bi = i;
          }
        }
        const uint64_t ext = drop ? B.minu64(best) : (uint64_t)B.max64((int64_t)best);
        if (drop && left == 0) {
          tstar = kp_bitsd(ext);
          break;
        }
        const int64_t win = B.min64(best == ext ? bi : INT64_MAX);  // one party holding it
        if (win != INT64_MAX && win % B.nth() == B.tid()) sc.buf[win] += drop ? ~0ull : 1ull;
        if (!drop && left == 1) {
          tstar = kp_bitsd(ext);
          break;
        }
      }
      B.sync();  // every step's reads of buf precede webster_tail's use of it
      return webster_tail(B, r, parties, tstar, N, desc, sc, ecap, compact, np, Lb, pl);
    }
  }
  KP_STAMPD(sc.dbg, 76);  // (stamps build: [76] the quota adjustment, [77] the first-seat rank, [78] enumeration)
  // Every seat a first seat: with P >= N parties of positive votes and the largest
  // vote below 3 v_N (v_N = the N-th largest vote), every second priority vmax/3 is
  // below v_N (exactly: fl(vmax/3) < v_N by far more than its rounding), so the N
  // largest priorities are first priorities and t* = v_N. v_N is rank-selected from
  // the compacted list (every vote >= v_N is in it: Lb <= v_N).
  if (compact && P >= (int64_t)N && np <= kWebFirstMax) {
    int64_t* slot = (int64_t*)sc.whist;
    for (int i = B.tid(); i < np; i += B.nth()) {
      const int64_t v = (int64_t)(uint32_t)pl[i];
      int64_t before = 0, upto = 0;
      for (int j = 0; j < np; j++) {
        const int64_t y = (int64_t)(uint32_t)pl[j];
        before += y > v ? 1 : 0;
        upto += y == v ? 1 : 0;
      }
      upto += before;
      if (before < (int64_t)N && (int64_t)N <= upto) *slot = v;  // every writer writes the same value
    }
    B.sync();
    const int64_t vN = *slot;
    B.sync();
    KP_STAMPD(sc.dbg, 77);
    if (vmax < 3 * vN) {
      KP_COUNT(sc, 79, 1);
      return webster_tail(B, r, parties, (double)vN, N, desc, sc, ecap, compact, np, Lb, pl);
    }
  }
  auto cnt2 = [&](double ta, double tb, int64_t* ca, int64_t* cb) {
    int64_t a = 0, b = 0;
    const double ra = 1.0 / ta, rb = 1.0 / tb;
    parties([&](uint32_t, int64_t v) {
      a += w_count_r(v, ta, ra, capN, true);
      b += w_count_r(v, tb, rb, capN, true);
    });
    B.sum2(a, b);
    *ca = a;
    *cb = b;
  };
  auto cnt1 = [&](double t) {
    int64_t c = 0;
    const double rt = 1.0 / t;
    parties([&](uint32_t, int64_t v) { c += w_count_r(v, t, rt, capN, true); });
    return B.sum64(c);
  };
  // invariant: cnt_ge(lo) >= N > cnt_ge(hi), lo < hi (as bit patterns)
  uint64_t lo = 1, hi = dbits((double)vmax) + 1;
  int64_t clo = -1, chi = 0;
  {
    double l0 = (double)V / (double)(2 * (int64_t)N + P);
    uint64_t lb = dbits(l0) > 64 ? dbits(l0) - 64 : 1;  // a few ulps below the bound
    double h0 = 2 * (int64_t)N - P - 1 > 0 ? (double)V / (double)(2 * (int64_t)N - P - 1) : (double)vmax;
    uint64_t hb = dbits(h0) + 64;
    if (hb > hi) hb = hi;
    if (Lb > 1) {  // t* >= Lb (every count below is taken at t >= Lb, where it is exact)
      const uint64_t lL = dbits((double)Lb);
      if (lL > lb) lb = lL;
      if (hb <= lb) hb = lb + 1;
    }
    int64_t cl, ch;
    cnt2(bitsd(lb), bitsd(hb), &cl, &ch);
    if (cl >= N) {
      lo = lb;
      clo = cl;
    }
    if (ch < N) {
      hi = hb;
      chi = ch;
    }
    if (clo < 0) clo = cnt1(bitsd(lo));
  }
  KP_STAMPD(sc.dbg, 65);
  while (hi - lo > 1 && clo - chi > (int64_t)ecap) {
    uint64_t mid = lo + (hi - lo) / 2;
    int64_t c = cnt1(bitsd(mid));
    if (c >= N) {
      lo = mid;
      clo = c;
    } else {
      hi = mid;
      chi = c;
    }
  }
  KP_STAMPD(sc.dbg, 66);
  double tstar;
  if (hi - lo <= 1) {
    tstar = bitsd(lo);
  } else {
    // enumerate the <= 64 priorities in [lo, hi); t* is the (N - chi)-th largest
    const double tl = bitsd(lo), th = bitsd(hi);
    const double rl = 1.0 / tl, rh = 1.0 / th;  // (w_count_r: the same counts, no division per party)
    int32_t mine = 0;
    parties([&](uint32_t, int64_t v) {
      mine += (int32_t)(w_count_r(v, tl, rl, capN, true) - w_count_r(v, th, rh, capN, true));
    });
    int32_t E;
    int32_t pos = B.excl_scan(mine, &E);
    parties([&](uint32_t, int64_t v) {
      int64_t k0 = w_count_r(v, th, rh, capN, true), k1 = w_count_r(v, tl, rl, capN, true);
      for (int64_t k = k0; k < k1; k++) sc.buf[pos++] = dbits(w_prio(v, k));
    });
    B.sync();
    tstar = bitsd(rank_select(B, sc.buf, E, (int64_t)N - chi, true, (uint64_t*)sc.whist));
  }
  KP_STAMPD(sc.dbg, 78);
  KP_COUNT(sc, 81, 1);
  KP_COUNT(sc, 82, np);
  return webster_tail(B, r, parties, tstar, N, desc, sc, ecap, compact, np, Lb, pl);
}

// webster_par for a single-wave block holding at most one party per lane in registers
// (k_select_top's subsets of <= 64 candidates, RegCands): the same t* and tie threshold,
// with no LDS. At t0 = V/2N each party holds s = #{k : prio(v, k) >= t0} = round(Nv/V)
// priorities, within one party per lane / 2 of N in total (so at most 32 steps); the
// smallest held priority is dropped (or the largest next one added) one at a time by a
// wave min / max, and only the lane that gave it recomputes its next one. The tie group
// at t* is ordered by tie_key as webster_tail orders it: each tied lane counts the tied
// keys below its own (the keys are distinct: one party per cluster rank). V: the parties'
// vote total. `ok` is false (nothing decided) when the count is off by more than the
// step bound, which the rounding argument excludes: the caller runs webster_par then.
template <class BLK>
KP_FI WebRes webster_reg(const BLK& B, bool party, uint32_t rk, int64_t v, int32_t N, bool desc, int64_t V, bool* ok,
                         int* nsteps) {
  WebRes r;
  r.N = N;
  r.desc = desc;
  r.t = 0;
  r.tie = 0;
  *ok = true;
  if (V == 0) {
    r.mode = 0;
    return r;
  }
  if (N <= 0) {
    r.mode = 1;
    return r;
  }
  r.mode = 2;
  const int64_t capN = (int64_t)N;
  const double t0 = (double)V / (2.0 * (double)N);
  int64_t s = party ? w_count(v, t0, capN + 1, true) : 0;
  const int64_t C = B.sum64(s);
  const int64_t steps = C >= capN ? C - capN : capN - C;
  if (nsteps) *nsteps = (int)steps;
  if (steps > 64) {
    *ok = false;
    return r;
  }
  const int lane = B.lane();
  double tstar;
  if (C >= capN) {  // drop the smallest held priorities: t* is the smallest one left
    uint64_t cand = party && s > 0 ? kp_dbits(w_prio(v, s - 1)) : ~0ull;
    for (int64_t left = steps;; left--) {
      const uint64_t m = B.minu64(cand);
      if (left == 0) {
        tstar = kp_bitsd(m);
        break;
      }
      const int win = __builtin_ctzll(B.wballot(cand == m));
      if (lane == win) {
        s--;
        cand = s > 0 ? kp_dbits(w_prio(v, s - 1)) : ~0ull;
      }
    }
  } else {  // add the largest next priorities: t* is the last one added
    uint64_t cand = party ? kp_dbits(w_prio(v, s)) : 0ull;
    for (int64_t left = steps;; left--) {
      const uint64_t m = (uint64_t)B.max64((int64_t)cand);  // (positive doubles: below 2^63)
      if (left == 1) {
        tstar = kp_bitsd(m);
        break;
      }
      const int win = __builtin_ctzll(B.wballot(cand == m));
      if (lane == win) {
        s++;
        cand = kp_dbits(w_prio(v, s));
      }
    }
  }
  r.t = tstar;
  r.rt = 1.0 / tstar;
  // seats strictly above t*, then the tie group at t* (webster_tail)
  const int64_t base = party ? w_count_r(v, tstar, r.rt, capN + 1, false) : 0;
  const bool tie = party && w_prio(v, base) == tstar;
  int64_t S = base, T = tie ? 1 : 0;
  B.sum2(S, T);
  const int64_t M = capN - S;
  if (M >= T) {
    r.tie = ~0ull;
  } else {
    // the M-th smallest tie key (1-based): the tied lane with M - 1 tied keys below its own
    const uint64_t key = tie ? tie_key(base, rk, desc) : ~0ull;
    const uint64_t tmask = B.wballot(tie);
    int64_t below = 0;
    for (uint64_t m = tmask; m; m &= m - 1) below += B.wread(key, __builtin_ctzll(m)) < key ? 1 : 0;
    const uint64_t sel = B.wballot(tie && below == M - 1);
    r.tie = B.wread(key, sel ? __builtin_ctzll(sel) : 0);
  }
  return r;
}

// Largest value v* over a value set (values in [0, 2^31)) such that the values
// >= v* sum to at least `target` (>= 1; the caller guarantees the total reaches
// it): an 8-bit radix descent with value-weighted bins. `vals(fn)` calls fn(v)
// for every value the calling thread owns.
// sum{v_i > v*} and #{v_i == v*} of wsel_max's answer, read off its last histogram
// (cnt_eq = -1 when v* = 0: the caller counts).
struct WselTail {
  int64_t sum_gt = 0, cnt_eq = -1;
};
template <class BLK, class Vals>
KP_FI int64_t wsel_max(const BLK& B, unsigned long long* wh, Vals vals, int64_t target, int64_t vmax = -1,
                       WselTail* tail = nullptr) {
  // the highest set bit of the OR of the values is the maximum's: a known maximum
  // spares the OR pass
  uint64_t on = 0;
  if (vmax >= 0) {
    on = (uint64_t)vmax;
  } else {
    vals([&](int64_t v) { on |= (uint64_t)v; });
    on = B.or64(on);
  }
  int start = 24;
  while (start > 0 && !(on >> start)) start -= 8;
  uint32_t prefix = 0;
  int64_t above = 0;
  for (int shift = start; shift >= 0; shift -= 8) {
    for (int i = B.tid(); i < 256; i += B.nth()) wh[i] = 0;
    B.sync();
    const uint32_t hm = shift == 24 ? 0u : (~0u << (shift + 8));
    vals([&](int64_t v64) {
      uint32_t v = (uint32_t)v64;
      if ((v & hm) == (prefix & hm) && v) kp_atomic_add(&wh[(v >> shift) & 255], (unsigned long long)v);
    });
    int64_t before;
    const int bin = B.find_bin(wh, target - above, &before, true);
    above += before;
    prefix |= (uint32_t)bin << shift;
    if (shift == 0 && tail) {  // the last round's bins are single values: bin = v*
      tail->sum_gt = above;
      tail->cnt_eq = prefix ? (int64_t)(wh[bin] / prefix) : -1;
    }
  }
  return (int64_t)prefix;
}

// ----------------------------------------------------------------------------
// k-th smallest (1-based) 64-bit key over a predicate set: 8-bit radix select.
// ----------------------------------------------------------------------------
// keys(fn) calls fn(key) for every key of the set the calling thread owns.
template <class BLK, class Keys>
KP_FI uint64_t radix_select_each(const BLK& B, uint32_t* hist, Keys keys, int64_t k) {
  // bytes shared by every key are skipped: start at the highest differing byte
  uint64_t an = ~0ull, on = 0;
  keys([&](uint64_t kk) {
    an &= kk;
    on |= kk;
  });
  B.andor(an, on);
  const uint64_t diff = an ^ on;
  if (diff == 0) return an;  // all keys equal
  int top = 63;
  while (!((diff >> top) & 1)) top--;
  const int start = (top / 8) * 8;
  uint64_t prefix = start == 56 ? 0ull : (an & (~0ull << (start + 8)));
  for (int shift = start; shift >= 0; shift -= 8) {
    for (int i = B.tid(); i < 256; i += B.nth()) hist[i] = 0;
    B.sync();
    const uint64_t hm = shift == 56 ? 0ull : (~0ull << (shift + 8));
    keys([&](uint64_t kk) {
      if ((kk & hm) == (prefix & hm)) kp_atomic_add(&hist[(kk >> shift) & 255], 1u);
    });
    int64_t before;
    const int bin = B.find_bin(hist, k, &before, false);
    k -= before;
    prefix |= (uint64_t)bin << shift;
  }
  return prefix;
}
template <class BLK, class Pred, class Key>
KP_FI uint64_t radix_select(const BLK& B, uint32_t* hist, int F, Pred pred, Key key, int64_t k) {
  return radix_select_each(
      B, hist,
      [&](auto fn) {
        for (int i = B.tid(); i < F; i += B.nth())
          if (pred(i)) fn(key(i));
      },
      k);
}

}  // namespace kp
