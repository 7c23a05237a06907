// kp_paths.h — per-binding select/assign paths (one workgroup per binding).
//
//   sel_all_fast      SelectBestClusters "select all" + AssignReplicas, block-parallel
//                     (Duplicated, StaticWeight, DynamicWeight, Aggregated).
//   sel_cluster_fast  selectBestClustersByCluster: top-MaxGroups + swap step, then
//                     the serial AssignReplicas on the selected list.
//   region_a/_b       generateRegionInfo/calcGroupScore on device; selectGroups DFS
//                     on the host; region heads + top-up + AssignReplicas on device.
//   slow_path         exact serial emulation over the fully sorted candidate list
//                     for the rare hazards the fast paths refuse (Aggregated ties
//                     at the prefix cut, int32 wrap risk, overflow tiers, ...).
#pragma once
#include "kp_select.h"

#include <type_traits>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <vector>
#endif

namespace kp {

constexpr int kRegionMax = 256;

// Reasons a binding leaves the fast paths for the exact serial path (stats[reason]).
enum : int { SLOW_NONE = 0, SLOW_OVERFLOW_DUP = 1, SLOW_SCALE_DOWN = 2, SLOW_WRAP = 3, SLOW_TIE = 4, SLOW_WEIGHT = 5,
             SLOW_CLUSTER = 6,
             SLOW_TOP_FULL = 100 };  // k_select_top only: the binding needs the full candidate set (not a k_slow reason)

KP_HD inline uint64_t cand_key(const SelCtx& x, const Cands& cd, int i, int32_t est) {
  uint32_t rank = c_rank(cd, i);
  int64_t avail = (int64_t)est + (int64_t)assigned_of(*x.bv, *x.h, x.tgt_bits, rank);
  return sort_key(c_ovf(cd, i), locality_score(*x.h, x.tgt_bits, rank), avail, rank);
}
// A candidate's sortClusters key kept in place of its (rank, estimate) pair (the
// spread kernels compute it once after the gather).
KP_HD inline uint64_t ckey(const Cands& cd, int i) { return ((uint64_t)cd.r[i] << 32) | (uint64_t)(uint32_t)cd.v[i]; }
KP_HD inline void put_ckey(const Cands& cd, int i, uint64_t k) {
  cd.r[i] = (uint32_t)(k >> 32);
  cd.v[i] = (int32_t)(uint32_t)k;
}
KP_HD inline Item item_from_key(const SelCtx& x, uint64_t k) {
  Item it;
  it.rank = key_rank(k);
  it.alloc = est_at(x, (int)it.rank);
  it.avail = key_avail(k);
  it.ovf = key_ovf(k);
  it.pad = 0;
  return it;
}
// #{j < m : keys[j] < k}: four independent chains so the LDS reads (the same
// address in every lane) overlap instead of waiting one by one.
KP_FI int count_less(const uint64_t* keys, int m, uint64_t k) {
  int p0 = 0, p1 = 0, p2 = 0, p3 = 0, j = 0;
  for (; j + 4 <= m; j += 4) {
    p0 += keys[j] < k ? 1 : 0;
    p1 += keys[j + 1] < k ? 1 : 0;
    p2 += keys[j + 2] < k ? 1 : 0;
    p3 += keys[j + 3] < k ? 1 : 0;
  }
  for (; j < m; j++) p0 += keys[j] < k ? 1 : 0;
  return p0 + p1 + p2 + p3;
}
// Distinct keys[0..m) (the rank sits in the low bits) as items in ascending key
// order: each key's position is the count of smaller keys (block-parallel; the
// list is at most 2 * kSmallMax long).
template <class BLK>
KP_FI void place_sorted(const BLK& B, const SelCtx& x, const uint64_t* keys, int m, Item* dst) {
  for (int i = B.tid(); i < m; i += B.nth()) {
    const uint64_t k = keys[i];
    dst[count_less(keys, m, k)] = item_from_key(x, k);
  }
  B.sync();
}

// scheduledClusters helpers: spec.Clusters entries whose cluster is a candidate
// (assignment.go:125-142). Targets are unique here (BF_DUP_TARGETS goes slow).
KP_HD inline int32_t sched_rep_of(const SelCtx& x, uint32_t rank) {
  return assigned_of(*x.bv, *x.h, x.tgt_bits, rank);
}
KP_HD inline bool in_sched(const SelCtx& x, uint32_t rank) {
  return x.h->tgt_cnt > 0 && bit_test(x.tgt_bits, (int)rank) && mask_test(x.frow, (int)rank);
}

// sortClusters key of a SEL_ALL candidate (no overflow tiers on the fast path).
KP_HD inline uint64_t cand_order_key(const SelCtx& x, uint32_t rk, int32_t est) {
  const int64_t avail = (int64_t)est + (int64_t)assigned_of(*x.bv, *x.h, x.tgt_bits, rk);
  return sort_key(0, locality_score(*x.h, x.tgt_bits, rk), avail, rk);
}

// Candidate sets for the SEL_ALL path. each(fn) calls fn(rank, v) for every
// candidate the calling thread owns, always in the same per-thread order.
struct LdsCands {  // candidates compacted in LDS (gather)
  const Cands* cd;
  int tid, nth;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) fn(c_rank(*cd, i), cd->v[i]);
  }
  // v := fn(rank, v) for every candidate the thread owns (same order as each).
  template <class Fn>
  KP_FI void each_set(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) cd->v[i] = fn(c_rank(*cd, i), cd->v[i]);
  }
  static constexpr bool kSettable = true;
  // Position key of a candidate in the sort.Sort input (sortClusters order).
  KP_FI uint64_t okey(const SelCtx& x, uint32_t rk, int32_t v0) const { return cand_order_key(x, rk, v0); }
  static constexpr bool kExact = false;  // okey is sort.Sort's output order only for <= 12 (stable insertion)
};
// At most one candidate per lane, held in registers (k_select_top's subsets of at most
// 64 on one wave): every pass of the division reads it without an LDS round trip.
struct RegCands {
  bool has;
  uint32_t rk;
  mutable int32_t v;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    if (has) fn(rk, v);
  }
  template <class Fn>
  KP_FI void each_set(Fn fn) const {
    if (has) v = fn(rk, v);
  }
  static constexpr bool kSettable = true;
  KP_FI uint64_t okey(const SelCtx& x, uint32_t r, int32_t v0) const { return cand_order_key(x, r, v0); }
  static constexpr bool kExact = false;
};
// Gathered candidates (any memory) whose sort.Sort output order is known:
// pos[rank] = position after the emulated sort (k_slow, kp_pdq.h).
struct PosCands {
  const Cands* cd;
  const int32_t* pos;
  int tid, nth;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) fn(c_rank(*cd, i), cd->v[i]);
  }
  template <class Fn>
  KP_FI void each_set(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) cd->v[i] = fn(c_rank(*cd, i), cd->v[i]);
  }
  static constexpr bool kSettable = true;
  KP_FI uint64_t okey(const SelCtx&, uint32_t rk, int32_t) const { return (uint64_t)(uint32_t)pos[rk]; }
  static constexpr bool kExact = true;
};

// The binding's spec.Clusters entries that are candidates (scheduledClusters,
// assignment.go:125-142), v = their scheduled replicas: the parties of
// dynamicScaleDown (division_algorithm.go:103-119).
struct TgtCands {
  const SelCtx* x;
  int tid, nth;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    const BindHdr& h = *x->h;
    for (int j = tid; j < h.tgt_cnt; j += nth) {
      const uint32_t r = (uint32_t)x->bv->ipool[h.tgt_off + 2 * j];
      if (mask_test(x->frow, (int)r)) fn(r, x->bv->ipool[h.tgt_off + 2 * j + 1]);
    }
  }
  // Position in scheduledClusters = position in spec.Clusters (targets unique).
  KP_FI uint64_t okey(const SelCtx&, uint32_t rk, int32_t) const {
    const BindHdr& h = *x->h;
    for (int j = 0; j < h.tgt_cnt; j++)
      if ((uint32_t)x->bv->ipool[h.tgt_off + 2 * j] == rk) return (uint64_t)j;
    return ~0ull;
  }
  static constexpr bool kExact = false;
  static constexpr bool kSettable = false;
};

// Block-parallel emission of per-candidate results. rep(rank, v) gives the
// replicas of a candidate; `keep_all` emits every candidate (non-workload /
// EnableEmptyWorkloadPropagation), otherwise only rep > 0 (removeZeroReplicasCluster).
// Candidate sets that can store a value per candidate (CS::kSettable) keep the
// replicas from the counting pass, so rep runs once per candidate; the votes
// are dead after this.
template <class BLK, class CS, class RepFn>
KP_FI void emit_each(const BLK& B, const SelCtx& x, const CS& cs, RepFn rep, bool keep_all) {
  int32_t mine = 0;
  if constexpr (CS::kSettable) {
    cs.each_set([&](uint32_t rk, int32_t v) {
      const int32_t r = rep(rk, v);
      if (keep_all || r > 0) mine++;
      return r;
    });
  } else {
    cs.each([&](uint32_t rk, int32_t v) {
      if (keep_all || rep(rk, v) > 0) mine++;
    });
  }
  int32_t tot;
  const int32_t off = B.excl_scan(mine, &tot);
  // the binding's own slot of out_cap entries (the fast paths never exceed it)
  const uint64_t base = x.h->out_off;
  if (B.tid() == 0) {
    x.sink.status[x.b] = KP_STATUS_OK;
    x.sink.err[x.b] = KP_ERR_NONE;
    x.sink.arg[x.b] = 0;
    x.sink.start[x.b] = base;
    x.sink.count[x.b] = (uint32_t)tot;
  }
  uint64_t o = base + (uint64_t)off;
  cs.each([&](uint32_t rk, int32_t v) {
    const int32_t r = CS::kSettable ? v : rep(rk, v);
    if (keep_all || r > 0) {
      x.sink.out_idx[o] = rk;  // (snapshot rank: k_compact maps it through perm)
      x.sink.out_rep[o] = r < 0 ? 0 : r;
      o++;
    }
  });
}

// Block-parallel emission from a compacted party list pl[0, np) ((rank << 32) |
// votes; rep(rank, votes) gives the replicas, emitted when > 0) plus, when
// `targets`, the binding's spec.Clusters entries that are candidates with
// trep(rank) > 0 (0 for those the list already holds).
template <class BLK, class RepFn, class TRepFn>
KP_FI void emit_lists(const BLK& B, const SelCtx& x, uint64_t* pl, int np, RepFn rep, bool targets, TRepFn trep) {
  const BindHdr& h = *x.h;
  const int nt = targets ? h.tgt_cnt : 0;
  auto trank = [&](int j) { return (uint32_t)x.bv->ipool[h.tgt_off + 2 * j]; };
  int32_t mine = 0;
  for (int i = B.tid(); i < np; i += B.nth()) {  // replicas replace the votes (same thread, both passes)
    const int32_t r = rep((uint32_t)(pl[i] >> 32), (int64_t)(uint32_t)pl[i]);
    pl[i] = (pl[i] & ~0xffffffffull) | (uint64_t)(uint32_t)r;
    if (r > 0) mine++;
  }
  for (int j = B.tid(); j < nt; j += B.nth())
    if (mask_test(x.frow, (int)trank(j)) && trep(trank(j)) > 0) mine++;
  int32_t tot;
  const int32_t off = B.excl_scan(mine, &tot);
  // the binding's own slot of out_cap entries (the fast paths never exceed it)
  const uint64_t base = x.h->out_off;
  if (B.tid() == 0) {
    x.sink.status[x.b] = KP_STATUS_OK;
    x.sink.err[x.b] = KP_ERR_NONE;
    x.sink.arg[x.b] = 0;
    x.sink.start[x.b] = base;
    x.sink.count[x.b] = (uint32_t)tot;
  }
  uint64_t o = base + (uint64_t)off;
  for (int i = B.tid(); i < np; i += B.nth()) {
    const uint32_t rk = (uint32_t)(pl[i] >> 32);
    const int32_t r = (int32_t)(uint32_t)pl[i];
    if (r > 0) {
      x.sink.out_idx[o] = rk;  // (snapshot rank: k_compact maps it through perm)
      x.sink.out_rep[o] = r;
      o++;
    }
  }
  for (int j = B.tid(); j < nt; j += B.nth()) {
    const uint32_t rk = trank(j);
    if (!mask_test(x.frow, (int)rk)) continue;
    const int32_t r = trep(rk);
    if (r > 0) {
      x.sink.out_idx[o] = rk;  // (snapshot rank: k_compact maps it through perm)
      x.sink.out_rep[o] = r;
      o++;
    }
  }
}

// dynamicScaleDown (division_algorithm.go:103-119) for SEL_ALL bindings: the
// parties are the scheduled clusters only, so the serial answer needs no
// candidate sort. Thread 0; `mem` holds Items[tgt_cnt] + serial scratch.
// Returns false when the binding needs the general serial path instead.
KP_HD inline bool scale_down_targets(const SelCtx& x, unsigned char* mem, size_t mem_bytes) {
  const BindHdr& h = *x.h;
  if (h.sel != SEL_ALL || !(h.flags & BF_WORKLOAD_ASSIGN)) return false;
  if (h.flags & (BF_OVERFLOW | BF_DUP_TARGETS | BF_EMPTY_PROP | BF_FRESH)) return false;
  if (h.strategy != ST_DYNAMIC && h.strategy != ST_AGGREGATED) return false;
  const int nt = h.tgt_cnt;
  const int cap = 2 * nt + 16;
  if (sizeof(Item) * (size_t)nt + serial_scratch_bytes(cap) + 16 > mem_bytes) return false;
  Item* items = (Item*)mem;
  int n = 0;
  int32_t assigned = 0;
  for (int j = 0; j < nt; j++) {
    uint32_t r = (uint32_t)x.bv->ipool[h.tgt_off + 2 * j];
    if (!mask_test(x.frow, (int)r)) continue;
    assigned = add32(assigned, x.bv->ipool[h.tgt_off + 2 * j + 1]);
    items[n].rank = r;
    items[n].alloc = est_at(x, (int)r);
    items[n].avail = 0;
    items[n].ovf = 0;
    items[n].pad = 0;
    n++;
  }
  if (!(assigned > h.replicas)) return false;
  SerialScratch sc = serial_scratch_carve(items + nt, cap);
  SerialAssign sa{x, sc, (h.flags & BF_UID_DESC) != 0};
  SerialOut o = sa.run(items, n);
  sink_serial(x, sc, o);
  return true;
}

// divide_par's reductions over the candidate votes, when the caller already took
// them in its own pass: |votes|, min, total, count, and over the targets with
// scheduled replicas > 0 (the prior clusters, if merging) their sum and count.
struct DivSums {
  int64_t sabs = 0, vmin = 0, vtot = 0, nparty = 0, sp = 0, np = 0;
  int64_t vmax = 0, P = 0;  // largest vote, votes > 0 (with the octave histogram in ss.hist: WebPre)
  bool valid = false;
};

// sel_all_fast over a SUBSET of the candidates (k_select_top, kp_top.h): `cs` holds
// every scheduled cluster among the candidates and the non-scheduled ones with the
// largest votes (enough to decide the Webster top-N or the Aggregated cut exactly);
// F is the full candidate count (sort.Sort's list length); complete: cs is every
// candidate. A subset whose votes cannot cover the target returns SLOW_TOP_FULL.
struct TopInfo {
  int64_t F = 0;
  bool complete = false;
};

// ----------------------------------------------------------------------------
// SEL_ALL: every feasible cluster is selected (select_clusters.go:29-32) and
// AssignReplicas runs block-parallel over the candidate set `cs` (F members).
// Returns SLOW_NONE when the result (or error) is written, else the reason the
// binding needs the exact serial path (nothing written).
// ----------------------------------------------------------------------------
// kDynOnly: the caller's bindings are DynamicWeight / Aggregated workloads (k_select_top,
// k_slow's tie route); anything else returns SLOW_TOP_FULL without writing, and the
// other strategies' code is not instantiated (k_select_top: 46k -> 20k instructions).
template <bool kDynOnly = false, class BLK, class CS>
KP_FI int sel_all_fast(const BLK& B, const SelCtx& x, const CS& cs, const SelScratch& ss,
                       const TopInfo* top = nullptr) {
  KP_STAMP_INIT
  const BindHdr& h = *x.h;
  const bool desc = (h.flags & BF_UID_DESC) != 0;
  const bool prop = (h.flags & BF_EMPTY_PROP) != 0;
  const int st = h.strategy;
  if constexpr (kDynOnly) {
    if (!(h.flags & BF_WORKLOAD_ASSIGN) || (h.flags & (BF_OVERFLOW | BF_DUP_TARGETS)) ||
        (st != ST_DYNAMIC && st != ST_AGGREGATED))
      return SLOW_TOP_FULL;
  } else {
  if (!(h.flags & BF_WORKLOAD_ASSIGN)) {  // non-workload: all candidates, 0 replicas (common.go:72-82)
    emit_each(B, x, cs, [&](uint32_t, int32_t) { return (int32_t)0; }, true);
    return SLOW_NONE;
  }
  if (h.flags & (BF_OVERFLOW | BF_DUP_TARGETS)) return SLOW_OVERFLOW_DUP;
  if (st == ST_NONE) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_UNSUPPORTED_STRATEGY, 0);
    return SLOW_NONE;
  }
  if (st == ST_DUPLICATED) {
    const int32_t rep = h.replicas > 0 ? h.replicas : 0;
    emit_each(B, x, cs, [&](uint32_t, int32_t) { return rep; }, prop);
    return SLOW_NONE;
  }
  if (st == ST_STATIC) {  // v = max matching rule weight (gather)
    int64_t wmax = 0, wsum = 0;
    cs.each([&](uint32_t, int32_t w) {
      if (w > wmax) wmax = w;
      wsum += w > 0 ? w : 0;
    });
    B.maxsum(wmax, wsum);
    if (wmax >= kInt32Max) return SLOW_WEIGHT;
    if ((int64_t)h.replicas >= kSeatWrap) return SLOW_WRAP;  // seats past 2^30 (w_prio)
    const bool all1 = wsum == 0;  // getStaticWeightInfoList: every candidate weight 1
    auto parties = [&](auto fn) {
      cs.each([&](uint32_t rk, int32_t w) {
        if (all1 || w > 0) fn(rk, all1 ? (int64_t)1 : (int64_t)w);
      });
    };
    WebRes w = webster_par(B, parties, h.replicas, desc, ss);
    emit_each(
        B, x, cs,
        [&](uint32_t rk, int32_t wt) {
          return (all1 || wt > 0) ? web_seats(w, all1 ? (int64_t)1 : (int64_t)wt, rk) : (int32_t)0;
        },
        prop);
    return SLOW_NONE;
  }
  }
  // Dynamic / Aggregated (assignment.go:213-244)
  // GetSumOfReplicas(scheduledClusters) wraps in int32; the int64 sum taken
  // mod 2^32 is the same value. One pass also takes divide_par's vote sums
  // for the fresh / scale-up modes (the vote formula depends only on
  // BF_FRESH; the prior-cluster sum is 0 unless some prior has replicas).
  const bool fresh = (h.flags & BF_FRESH) != 0;
  auto tgt = [&](uint32_t rk) { return h.tgt_cnt > 0 && bit_test(x.tgt_bits, (int)rk); };
  // this pass also takes Webster's vote totals and octave histogram (WebPre); one
  // candidate per lane of one wave (RegCands) takes webster_reg instead, which needs no
  // histogram
  const bool reg = std::is_same<CS, RegCands>::value && B.nwaves() == 1;
  if (!reg) {
    for (int i = B.tid(); i < 256; i += B.nth()) ss.hist[i] = 0;
    if (B.tid() == 0) *web_ctr(ss) = 0;
  }
  int64_t asum = 0, apos = 0;
  TgtCands{&x, B.tid(), B.nth()}.each([&](uint32_t, int32_t v) {
    asum += v;
    apos += v > 0 ? 1 : 0;
  });
  B.sync();
  DivSums ds;
  cs.each([&](uint32_t rk, int32_t v0) {
    int32_t v32 = v0;
    bool pr = false;
    if (tgt(rk)) {
      const int32_t sr = sched_rep_of(x, rk);
      if (fresh) v32 = add32(v32, sr);
      pr = sr > 0;
    }
    const int64_t v = v32;
    ds.sabs += v < 0 ? -v : v;
    if (v < ds.vmin) ds.vmin = v;
    if (v > ds.vmax) ds.vmax = v;
    ds.vtot += v;
    ds.nparty++;
    if (v > 0) {
      ds.P++;
      if (!reg) kp_atomic_add(&ss.hist[vote_bin((uint32_t)v)], 1u);
    }
    if (pr) {
      ds.sp += v;
      ds.np++;
    }
  });
  {
    // counts < 2^32 share a slot: (apos | P << 32), (nparty | np << 32)
    auto add = [](int64_t p, int64_t q) { return p + q; };
    int64_t ap = apos + (ds.P << 32), pn = ds.nparty + (ds.np << 32);
    B.reduce4(asum, add, 0, ap, add, 0, ds.sabs, add, 0, ds.vtot, add, 0);
    B.reduce4(ds.vmin, [](int64_t p, int64_t q) { return p < q ? p : q; }, 0, pn, add, 0, ds.sp, add, 0, ds.vmax,
              [](int64_t p, int64_t q) { return p > q ? p : q; }, 0);
    apos = ap & 0xffffffffll;
    ds.P = ap >> 32;
    ds.nparty = pn & 0xffffffffll;
    ds.np = pn >> 32;
  }
  ds.valid = true;
#if defined(KP_TOP_EXIT) && KP_TOP_EXIT == 3  // timing experiments only (wrong results)
  if (top) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, ds.vtot);
    return SLOW_NONE;
  }
#endif
  if (top) ds.nparty = top->F;  // the whole TargetClustersList (SLOW_TIE's n > 12 test)
  const int32_t assigned = wrap32(asum);
  const bool anyPriorPos = apos != 0;
  int mode;  // 0 fresh, 1 scale up, 2 unchanged, 3 scale down
  if (fresh) mode = 0;
  else if (assigned > h.replicas) mode = 3;
  else if (assigned < h.replicas) mode = 1;
  else mode = 2;
  if (mode == 3) {  // dynamicScaleDown: parties = scheduledClusters, no merge
    if (prop) return SLOW_SCALE_DOWN;  // attachZeroReplicasCluster over all candidates: serial
    TgtCands tc{&x, B.tid(), B.nth()};
    return divide_par(B, x, tc, h.replicas, false, false, false, KP_ERR_SCALE_DOWN_NOT_ENOUGH, ss);
  }
  if (mode == 2) {  // unchanged: scheduledClusters, removeZero
    emit_each(B, x, cs, [&](uint32_t rk, int32_t) { return tgt(rk) ? sched_rep_of(x, rk) : (int32_t)0; }, prop);
    return SLOW_NONE;
  }
  const int32_t target = mode == 0 ? h.replicas : sub32(h.replicas, assigned);
  // a subset that does not cover the target cannot report the availability error
  if (top && !top->complete && (int32_t)ds.vtot < target) return SLOW_TOP_FULL;
  return divide_par(B, x, cs, target, mode == 0, mode == 1, anyPriorPos,
                    mode == 0 ? KP_ERR_FRESH_NOT_ENOUGH : KP_ERR_SCALE_UP_NOT_ENOUGH, ss, &ds);
}

// dynamicDivideReplicas (division_algorithm.go:75-101) for DynamicWeight and
// Aggregated, block-parallel over the candidate set: votes (fresh: + scheduled
// replicas), the availability check, the Aggregated prefix cut, Webster
// (SpreadReplicasByTargetClusters) and MergeTargetClusters (scale-up).
template <class BLK, class CS>
KP_FI int divide_par(const BLK& B, const SelCtx& x, const CS& cs, int32_t target, bool fresh, bool merge,
                     bool anyPriorPos, int not_enough, const SelScratch& ss, const DivSums* pre = nullptr) {
  KP_STAMP_INIT
  const BindHdr& h = *x.h;
  const int st = h.strategy;
  const bool desc = (h.flags & BF_UID_DESC) != 0;
  const bool prop = (h.flags & BF_EMPTY_PROP) != 0;
  auto tgt = [&](uint32_t rk) { return h.tgt_cnt > 0 && bit_test(x.tgt_bits, (int)rk); };
  auto vote32 = [&](uint32_t rk, int32_t v) -> int32_t {
    if (fresh && tgt(rk)) v = add32(v, sched_rep_of(x, rk));
    return v;
  };
  int64_t sabs = 0, vmin = 0, vtot = 0, nparty = 0;
  if (pre) {
    sabs = pre->sabs;
    vmin = pre->vmin;
    vtot = pre->vtot;
    nparty = pre->nparty;
  } else {
    cs.each([&](uint32_t rk, int32_t v0) {
      int64_t v = vote32(rk, v0);
      sabs += v < 0 ? -v : v;
      if (v < vmin) vmin = v;
      vtot += v;
      nparty++;
    });
    B.sum2(sabs, vtot);
    B.reduce2(vmin, [](int64_t p, int64_t q) { return p < q ? p : q; }, (int64_t)0, nparty,
              [](int64_t p, int64_t q) { return p + q; }, (int64_t)0);
  }
  // int32 wrap hazards: vote sums, and seats past 2^30 (w_prio)
  if (vmin < 0 || sabs >= (int64_t)kInt32Max || (int64_t)target >= kSeatWrap) return SLOW_WRAP;
  KP_STAMP(x, 2);
  if ((int32_t)vtot < target) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_UNSCHEDULABLE, not_enough, vtot);
    return SLOW_NONE;
  }
  auto prior = [&](uint32_t rk) { return merge && anyPriorPos && tgt(rk) && sched_rep_of(x, rk) > 0; };
  // Aggregated prefix cut (division_algorithm.go:81-89) over sort.Sort order
  // (Replicas desc) with prior clusters first: membership is exact unless a
  // tie group straddles the cut (then the pdqsort permutation matters).
  int64_t vstar = -1;  // members: X elements with v > vstar, plus the whole tie group
  bool xIsPrior = false, noCut = false, straddle = false;
  uint64_t tieCut = 0;  // straddle: tie-group members with okey <= tieCut are taken
  if (st == ST_AGGREGATED) {
    int64_t SP = 0, nP = 0;
    if (pre) {  // prior = merge && anyPriorPos && (target with replicas > 0)
      SP = merge && anyPriorPos ? pre->sp : 0;
      nP = merge && anyPriorPos ? pre->np : 0;
    } else {
      cs.each([&](uint32_t rk, int32_t v0) {
        if (prior(rk)) {
          SP += vote32(rk, v0);
          nP++;
        }
      });
      B.sum2(SP, nP);
    }
    xIsPrior = nP > 0 && SP >= target;
    const int64_t tX = xIsPrior ? (int64_t)target : (int64_t)target - SP;
    auto xvals = [&](auto fn) {
      cs.each([&](uint32_t rk, int32_t v0) {
        if (prior(rk) == xIsPrior) fn((int64_t)vote32(rk, v0));
      });
    };
    int64_t xmax = -1, xsum = 0;
    const bool all_x = pre && nP == 0;  // no prior cluster: X is every candidate, sel_all_fast's sums hold
    if (all_x) {
      xmax = pre->vmax;
      xsum = pre->vtot;
    } else {
      xvals([&](int64_t v) {
        if (v > xmax) xmax = v;
        xsum += v;
      });
      B.maxsum(xmax, xsum);
    }
    if (xmax < 0 || xsum < tX) {
      noCut = true;  // every element of X is taken
    } else {
      WselTail wt;
      if (tX <= 0) vstar = xmax;  // the first element alone reaches the target
      else vstar = wsel_max(B, ss.whist, xvals, tX, xmax, &wt);  // largest v with sum{v_i >= v} >= tX
      int64_t sgt = wt.sum_gt, ceq = wt.cnt_eq;
      if (ceq < 0) {  // (not read off the radix: v* from the maximum, or v* = 0)
        sgt = 0;
        ceq = 0;
        xvals([&](int64_t v) {
          if (v > vstar) sgt += v;
          if (v == vstar) ceq++;
        });
        B.sum2(sgt, ceq);
      }
      const int64_t need = tX - sgt;
      const int64_t j = need <= 0 ? 1 : (vstar > 0 ? (need + vstar - 1) / vstar : ceq);
      if (j < ceq) {  // the tie group straddles the cut
        // Only sort.Sort's permutation of equal keys decides: the first j tie
        // members in its output order are taken. Lists of at most 12 are
        // insertion-sorted (stable), so input order is output order; longer
        // lists need the emulated permutation (CS::kExact, k_slow).
        if (!CS::kExact && nparty > 12) return SLOW_TIE;
        tieCut = radix_select_each(
            B, ss.hist,
            [&](auto fn) {
              cs.each([&](uint32_t rk, int32_t v0) {
                if (prior(rk) == xIsPrior && (int64_t)vote32(rk, v0) == vstar) fn(cs.okey(x, rk, v0));
              });
            },
            j);
        straddle = true;
      }
    }
  }
  KP_STAMP(x, 3);
#if defined(KP_TOP_EXIT) && KP_TOP_EXIT == 5  // timing experiments only (wrong results)
  if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, vstar);
  return SLOW_NONE;
#endif
  auto member = [&](uint32_t rk, int64_t v, int32_t v0) {
    if (st != ST_AGGREGATED) return true;
    const bool p = prior(rk);
    if (!xIsPrior && p) return true;  // X = non-prior: every prior cluster precedes the cut
    if (p != xIsPrior) return false;
    if (noCut || v > vstar) return true;
    return v == vstar && (!straddle || cs.okey(x, rk, v0) <= tieCut);
  };
  auto parties = [&](auto fn) {
    cs.each([&](uint32_t rk, int32_t v0) {
      const int64_t v = vote32(rk, v0);
      if (member(rk, v, v0)) fn(rk, v);
    });
  };
  // DynamicWeight: the parties are every candidate with the votes sel_all_fast's pass
  // summed (vote32), so its totals and histogram stand in for Webster's first pass
  const WebPre wp{pre ? pre->vtot : 0, pre ? pre->vmax : 0, pre ? pre->P : 0};
  WebRes w;
  bool reg_ok = false;
  if constexpr (std::is_same<CS, RegCands>::value) {
    if (B.nwaves() == 1) {  // one party per lane in registers (sel_all_fast skipped the histogram)
      bool party = false;
      uint32_t prk = 0;
      int64_t pv = 0;
      parties([&](uint32_t rk, int64_t v) {
        party = true;
        prk = rk;
        pv = v;
      });
      const int64_t V = pre && st != ST_AGGREGATED ? pre->vtot : B.sum64(party ? pv : 0);
      KP_STAMP(x, 56);  // (stamps build: [56] the party pass, [57] webster_reg, [4] webster_par after a refusal)
      int nsteps = 0;
      w = webster_reg(B, party, prk, pv, target, desc, V, &reg_ok, &nsteps);
      KP_STAMP(x, 57);
      KP_COUNT(x, 58, nsteps);
      KP_COUNT(x, 59, 1);
      KP_COUNT(x, 60, reg_ok ? 0 : 1);
      if (!reg_ok) w = webster_par(B, parties, target, desc, ss, nullptr);
    }
  }
  if constexpr (!std::is_same<CS, RegCands>::value) w = webster_par(B, parties, target, desc, ss, pre && st != ST_AGGREGATED ? &wp : nullptr);
  else if (B.nwaves() != 1) w = webster_par(B, parties, target, desc, ss, pre && st != ST_AGGREGATED ? &wp : nullptr);
  KP_STAMP(x, 4);
#if defined(KP_TOP_EXIT) && KP_TOP_EXIT == 4
  if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, (int64_t)w.tie);
  return SLOW_NONE;
#endif
  if (w.mode == 2 && w.compact && !prop) {
    // Only parties take seats, and every party with a seat is in Webster's compacted
    // list (votes >= Lb <= t*): emit from it, plus the prior targets outside it
    // whose merged replicas are > 0 (MergeTargetClusters), instead of walking every
    // candidate. Same multiset as the full walk below.
    auto in_list = [&](uint32_t rk) {
      const int32_t v0 = est_at(x, (int)rk);
      const int64_t v = vote32(rk, v0);
      return member(rk, v, v0) && v >= w.Lb;
    };
    emit_lists(
        B, x, const_cast<uint64_t*>(w.pl), w.np,
        [&](uint32_t rk, int64_t v) {
          int32_t r = web_seats(w, v, rk);
          if (merge && tgt(rk)) r = add32(r, sched_rep_of(x, rk));
          return r;
        },
        merge, [&](uint32_t rk) { return in_list(rk) ? (int32_t)0 : sched_rep_of(x, rk); });
    KP_STAMP(x, 5);
    return SLOW_NONE;
  }
  emit_each(
      B, x, cs,
      [&](uint32_t rk, int32_t v0) {
        const int64_t v = vote32(rk, v0);
        int32_t r = member(rk, v, v0) ? web_seats(w, v, rk) : 0;
        if (merge && tgt(rk)) r = add32(r, sched_rep_of(x, rk));
        return r;
      },
      prop);
  KP_STAMP(x, 5);
  return SLOW_NONE;
}

// ----------------------------------------------------------------------------
// Small selected list -> AssignReplicas -> sink.
// The selected clusters (spread selection's output, in the order AssignReplicas
// receives them) as a candidate set for the block-parallel assignment
// (sel_all_fast): v = AllocatableReplicas, or the StaticWeight vote; sort.Sort's
// input position is the position in the list.
// ----------------------------------------------------------------------------
struct ItemCands {
  const Item* it;
  int n, tid, nth;
  const SelCtx* x;
  bool weights;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    for (int i = tid; i < n; i += nth) fn(it[i].rank, weights ? static_vote(*x, (int)it[i].rank) : it[i].alloc);
  }
  static constexpr bool kSettable = false;
  KP_FI uint64_t okey(const SelCtx&, uint32_t rk, int32_t) const {
    for (int i = 0; i < n; i++)
      if (it[i].rank == rk) return (uint64_t)i;
    return ~0ull;
  }
  static constexpr bool kExact = false;
};
// The block-parallel AssignReplicas over the selected list, with the candidate
// bitset (scheduledClusters = spec.Clusters entries among the selected ones) in
// scratch; the exact serial emulation (thread 0) for what it refuses (Aggregated
// ties at the cut in lists > 12, overflow tiers, wrap hazards, ...).
// scratch: at least area_bytes of LDS.
template <class BLK>
KP_FI void assign_small(const BLK& B, const SelCtx& x, const Item* items, int n, void* scratch, int cap,
                        size_t area_bytes) {
  const int W = x.s->W;
  if (n > 0 && 8 * (size_t)W + 3072 + 8 * (size_t)sel_all_ecap(x.s->Cp) + 64 <= area_bytes) {
    uint64_t* selb = (uint64_t*)scratch;
    uint32_t* sel32 = (uint32_t*)scratch;
    for (int w = B.tid(); w < W; w += B.nth()) selb[w] = 0;
    B.sync();
    for (int i = B.tid(); i < n; i += B.nth()) kp_atomic_or(&sel32[items[i].rank >> 5], 1u << (items[i].rank & 31));
    B.sync();
    SelCtx y = x;
    y.frow = selb;
    const SelScratch ss = carve_sel_scratch((unsigned char*)(selb + W), x.s->Cp);
    const bool weights = x.h->strategy == ST_STATIC;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (std::is_same<BLK, GpuBlk>::value) {
      // a list of at most 64: one wave runs the division, so its passes meet at
      // wave barriers instead of the workgroup's; the other waves wait below
      if (n <= 64 && B.nwaves() > 1) {
        int32_t* whyp = (int32_t*)(B.red + 126);
        if (B.wid() == 0) {
          const WaveBlk wb{B.red};
          const int w = sel_all_fast(wb, y, ItemCands{items, n, wb.tid(), 64, &y, weights}, ss);
          if (wb.tid() == 0) *whyp = w;
        }
        B.sync();
        const int why = *whyp;
        B.sync();
        if (why == SLOW_NONE) return;
        goto serial;
      }
    }
#endif
    {
      const int why = sel_all_fast(B, y, ItemCands{items, n, B.tid(), B.nth(), &y, weights}, ss);
      B.sync();
      if (why == SLOW_NONE) return;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
serial:
#endif
  if (B.tid() == 0) {
    SerialScratch sc = serial_scratch_carve(scratch, cap);
    SerialAssign sa{x, sc, (x.h->flags & BF_UID_DESC) != 0};
    SerialOut o = sa.run(items, n);
    sink_serial(x, sc, o);
  }
  B.sync();
}

// ----------------------------------------------------------------------------
// SEL_CLUSTER: selectBestClustersByCluster (select_clusters_by_cluster.go:25-102)
// items: LDS buffer of kSmallMax*2 Items. Returns false -> slow path.
// kKeyed: the candidates already hold their sortClusters keys in place (put_ckey).
// n_sel: when set, the selection only: *n_sel = the selected count (items[0, n)),
// -1 when a status was written; no assignment (the spread self-test, kp_spread_test).
// ----------------------------------------------------------------------------
template <class BLK, bool kKeyed = false>
KP_FI bool sel_cluster_fast(const BLK& B, const SelCtx& x, const Cands& cd, uint32_t* hist, Item* items,
                            uint64_t* keys, void* scratch, int cap, size_t area_bytes, int* n_sel = nullptr) {
  const BindHdr& h = *x.h;
  const int F = cd.F;
  if (n_sel) *n_sel = -1;
  if ((int64_t)F < h.cluster_min) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_MIN_GROUPS, 0);
    return true;
  }
  int64_t needCnt = (int64_t)F < h.cluster_max ? (int64_t)F : h.cluster_max;
  if (needCnt < 0) needCnt = 0;
  if (needCnt > kSmallMax || h.tgt_cnt > kTgtSmallMax) return false;
  const int32_t need = h.need_replicas;
  if (needCnt == 0) {
    if (B.tid() == 0) {
      if (need == -1) sink_error(x, KP_STATUS_ERROR, KP_ERR_NO_CLUSTERS, 0);
      else sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, 0);
    }
    return true;
  }
  KP_STAMP_INIT
  // every candidate's sortClusters key once, in place of its (rank, estimate) pair
  if (!kKeyed) {
    for (int i = B.tid(); i < F; i += B.nth()) put_ckey(cd, i, cand_key(x, cd, i, cd.v[i]));
    B.sync();
  }
  auto key = [&](int i) { return ckey(cd, i); };
  auto all = [&](int) { return true; };
  uint64_t kth = radix_select(B, hist, F, all, key, needCnt);
  KP_STAMP(x, 28);
  // compact the selected keys
  int n = 0;
  for (int t0 = 0; t0 < F; t0 += B.nth()) {
    int i = t0 + B.tid();
    uint64_t k = 0;
    bool e = false;
    if (i < F) {
      k = key(i);
      e = k <= kth;
    }
    int32_t tot;
    int32_t off = B.excl_scan(e ? 1 : 0, &tot);
    if (e) keys[n + off] = k;
    n += tot;
  }
  B.sync();
  place_sorted(B, x, keys, n, items);  // sorted order (sortClusters)
  if (need != -1) {
    int64_t tot = 0;
    for (int i = 0; i < n; i++) tot += items[i].avail;
    if (tot < (int64_t)need) {
      // candidates for the swap step: the best rest clusters by (avail desc, position)
      int64_t m2 = (int64_t)F - needCnt;
      if (m2 > needCnt) m2 = needCnt;
      int nr = 0;
      Item* rest = items + kSmallMax;
      uint64_t* rkeys = keys + kSmallMax;
      if (m2 > 0) {
        auto isrest = [&](int i) { return key(i) > kth; };
        auto akey = [&](int i) { return avail_key(key(i)); };
        uint64_t kth2 = radix_select(B, hist, F, isrest, akey, m2);
        for (int t0 = 0; t0 < F; t0 += B.nth()) {
          int i = t0 + B.tid();
          uint64_t k = 0;
          bool e = false;
          if (i < F) {
            k = key(i);
            e = k > kth && avail_key(k) <= kth2;
          }
          int32_t tt;
          int32_t off = B.excl_scan(e ? 1 : 0, &tt);
          if (e) rkeys[nr + off] = k;
          nr += tt;
        }
        B.sync();
        // position in the rest slice = #{candidates with smaller key} - needCnt
        for (int z = 0; z < nr; z++) {
          uint64_t kz = rkeys[z];
          int64_t c = 0;
          for (int i = B.tid(); i < F; i += B.nth())
            if (key(i) < kz) c++;
          c = B.sum64(c);
          if (B.tid() == 0) {
            rest[z] = item_from_key(x, kz);
            rest[z].pad = (int32_t)(c - needCnt);  // position
          }
        }
        B.sync();
      }
      int ok = 1;
      if (B.tid() == 0) {
        // selectClustersByAvailableResource swap loop with explicit positions
        for (int i = 0; i < n; i++) items[i].pad = -1;
        int64_t upd = needCnt - 1;
        auto check = [&]() {
          int64_t s = 0;
          for (int i = 0; i < n; i++) s += items[i].avail;
          return s >= (int64_t)need;
        };
        while (!check() && upd >= 0) {
          // GetClusterWithMaxAvailableResource: first (by position) maximum above the
          // slot's AvailableReplicas
          int64_t bv = items[upd].avail;
          int best = -1;
          for (int z = 0; z < nr; z++) {
            if (rest[z].avail > bv) {
              best = z;
              bv = rest[z].avail;
            } else if (best >= 0 && rest[z].avail == bv && rest[z].pad < rest[best].pad) {
              best = z;
            }
          }
          if (best < 0) {
            upd--;
            continue;
          }
          Item out = items[upd];
          out.pad = rest[best].pad;  // the swapped-out cluster takes the taken slot's position
          items[upd] = rest[best];
          items[upd].pad = -1;
          rest[best] = out;
          upd--;
        }
        ok = check() ? 1 : 0;
        if (!ok) sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, needCnt);
      }
      ok = B.bcast(ok);
      if (!ok) return true;
    }
  }
  KP_STAMP(x, 29);
  if (n_sel) {
    *n_sel = n;
    return true;
  }
  assign_small(B, x, items, n, scratch, cap, area_bytes);
  KP_STAMP(x, 30);
  return true;
}

// ----------------------------------------------------------------------------
// Region stage A: generateRegionInfo + calcGroupScore (group_clusters.go:156-351,
// 418-457) for every region; out[r] = {count, score}.
// ----------------------------------------------------------------------------
struct RegionOut {
  int32_t count;
  int32_t pad;
  int64_t score;
};
// ----------------------------------------------------------------------------
// selectGroups (select_groups.go:102-224) on the device, one thread per binding.
// Groups are the regions with clusters: value = #clusters, weight = group score.
// Same answer as the host DFS (engine.cpp select_groups) without storing the
// feasible paths:
//  - pass 1 runs the DFS and keeps the best path by (weight desc, value desc),
//    the first found winning ties (= the smallest id);
//  - prioritizePaths then only ever moves to a proper subpath of the current
//    path, i.e. to a prefix (in weight order) of the best path. A prefix Q of
//    the current path F sorts after F exactly when Q.weight <= F.weight (group
//    values are >= 1, so Q.value < F.value), and the first such Q in sorted
//    order has the largest weight, then value. A prefix is a feasible path iff
//    it is feasible and none of its proper prefixes in DFS (value) order is.
// Returns the number of selected regions (ids in sel, best-path order),
// -KP_ERR_* for the reference's errors, or kGroupsHost when the DFS exceeds
// kGroupNodes nodes (the host DFS answers those).
// ----------------------------------------------------------------------------
constexpr int kGroupMax = 64;         // regions per snapshot on the device path
constexpr int64_t kGroupNodes = 1 << 20;
constexpr int32_t kGroupsHost = -2000;
KP_HD inline int32_t select_groups_dev(const struct RegionOut* ro, int R, int64_t minC, int64_t maxC, int64_t target,
                                       int32_t* sel);

struct RegionLds {
  int32_t* cnt;
  int32_t* dvalid;
  int32_t* wcnt;
  int32_t* done;
  int64_t* sumAvail;
  int64_t* sumScore;
  int64_t* dscore;
  int64_t* wsum;
  int64_t* wscore;
  int64_t* amin;
  unsigned long long* minkey;
  unsigned long long* last;
};

// The DFS's per-binding arrays: in private memory (GroupsPriv), or one thread's slice
// of a workgroup's LDS (GroupsLds: k_region_groups, one thread per binding, whose
// 2.3 KB of private arrays per thread went to scratch and moved 11x its compulsory
// bytes at config 4). Both give the same answers (the same code over either).
struct GroupsPriv {
  int32_t a[7][kGroupMax];
  int64_t b[kGroupMax];
};
// [7 int32 planes of G][G int64] per thread, strided by the workgroup width: entry i of
// plane k of thread t at (k * G + i) * nth + t (consecutive threads, consecutive banks).
struct GroupsLds {
  int32_t* p32;  // (already offset by the thread)
  int64_t* p64;
  int G, nth;
};
KP_HD inline size_t groups_lds_bytes(int G, int nth) { return (size_t)nth * (size_t)G * (7 * 4 + 8); }
KP_HD inline int32_t& garr(GroupsPriv& m, int k, int i) { return m.a[k][i]; }
KP_HD inline int64_t& garr64(GroupsPriv& m, int i) { return m.b[i]; }
KP_HD inline int32_t& garr(GroupsLds& m, int k, int i) { return m.p32[((size_t)k * m.G + i) * m.nth]; }
KP_HD inline int64_t& garr64(GroupsLds& m, int i) { return m.p64[(size_t)i * m.nth]; }
template <class M>
KP_HD inline int32_t select_groups_in(M& m, const RegionOut* ro, int R, int64_t minC, int64_t maxC, int64_t target,
                                      int32_t* sel) {
#define sid(i) garr(m, 0, (i))
#define sv(i) garr(m, 1, (i))
#define st(i) garr(m, 2, (i))
#define nx(i) garr(m, 3, (i))
#define best(i) garr(m, 4, (i))
#define w(i) garr(m, 5, (i))
#define idx(i) garr(m, 6, (i))
#define sw(i) garr64(m, (i))
  int n = 0;
  for (int r = 0; r < R; r++)
    if (ro[r].count > 0) {
      int j = n++;  // insertion by (value asc, weight desc, id asc) (select_groups.go:140-151)
      while (j > 0 && (sv(j - 1) > ro[r].count || (sv(j - 1) == ro[r].count && sw(j - 1) < ro[r].score))) {
        sid(j) = sid(j - 1);
        sv(j) = sv(j - 1);
        sw(j) = sw(j - 1);
        j--;
      }
      sid(j) = r;
      sv(j) = ro[r].count;
      sw(j) = ro[r].score;
    }
  if ((int64_t)n < minC) return -KP_ERR_REGION_MIN_GROUPS;  // select_clusters_by_region.go:30-32
  if (n == 0) return -KP_ERR_REGION_CLUSTER_MIN;
  // ---- pass 1: DFS (findFeasiblePaths), best path by (weight desc, value desc, id asc)
  int depth = 0, bl = -1;
  int64_t sum = 0, wsum = 0, bw = 0, bv = 0, nodes = 0;
  const bool nobt = (int64_t)n == minC;  // select_groups.go:179-182: no backtracking
  for (;;) {
    // node entry
    bool down = false;
    if (++nodes > kGroupNodes) return kGroupsHost;
    if (sum >= target && depth >= minC && depth <= maxC) {
      if (bl < 0 || wsum > bw || (wsum == bw && sum > bv)) {
        bl = depth;
        bw = wsum;
        bv = sum;
        for (int k = 0; k < depth; k++) best(k) = st(k);
      }
    } else if (depth < maxC) {
      nx(depth) = depth == 0 ? 0 : st(depth - 1) + 1;
      down = nx(depth) < n;
    }
    if (down) {
      const int i = nx(depth);
      st(depth) = i;
      sum += sv(i);
      wsum += sw(i);
      depth++;
      continue;
    }
    // return to the parent; try its next child
    bool more = false;
    while (depth > 0) {
      depth--;
      if (nobt) break;
      const int i = st(depth);
      sum -= sv(i);
      wsum -= sw(i);
      nx(depth) = i + 1;
      if (nx(depth) < n) {
        st(depth) = nx(depth);
        sum += sv(st(depth));
        wsum += sw(st(depth));
        depth++;
        more = true;
        break;
      }
    }
    if (!more) break;
  }
  if (bl < 0) return -KP_ERR_REGION_CLUSTER_MIN;  // no feasible path (select_clusters_by_region.go:37-39)
  // ---- best path in weight order (sortGroups: weight desc, name asc; ids are name ranks)
  for (int k = 0; k < bl; k++) {
    int j = k;
    const int32_t g = best(k);
    while (j > 0 && (sw(w(j - 1)) < sw(g) || (sw(w(j - 1)) == sw(g) && sid(w(j - 1)) > sid(g)))) {
      w(j) = w(j - 1);
      j--;
    }
    w(j) = g;
  }
  // ---- prioritizePaths: walk to the first later subpath while one exists
  int fl = bl;
  int64_t fw = bw;
  for (;;) {
    int pick = -1;
    int64_t pw = 0, pv = 0;
    int64_t qw = 0, qv = 0;
    for (int j = 1; j < fl; j++) {
      qw += sw(w(j - 1));
      qv += sv(w(j - 1));
      if (qw > fw || !(qv >= target && j >= minC && j <= maxC)) continue;
      // visited by the DFS: no proper prefix in index order is feasible (nor the
      // root); without backtracking only the chain 0,1,2,.. is visited
      for (int k = 0; k < j; k++) {
        int q = k;
        while (q > 0 && idx(q - 1) > w(k)) {
          idx(q) = idx(q - 1);
          q--;
        }
        idx(q) = w(k);
      }
      bool visited = !(0 >= target && 0 >= minC && 0 <= maxC);  // the root returns when feasible
      int64_t ps = 0;
      for (int k = 0; k < j && visited; k++) {
        if (nobt && idx(k) != k) visited = false;
        if (k > 0 && ps >= target && k >= minC && k <= maxC) visited = false;
        ps += sv(idx(k));
      }
      if (!visited) continue;
      if (pick < 0 || qw > pw || (qw == pw && qv > pv)) {
        pick = j;
        pw = qw;
        pv = qv;
      }
    }
    if (pick < 0) break;
    fl = pick;
    fw = pw;
  }
  if (fl == 0) return -KP_ERR_REGION_CLUSTER_MIN;  // the empty root path
  for (int k = 0; k < fl; k++) sel[k] = sid(w(k));
  return fl;
#undef sid
#undef sv
#undef st
#undef nx
#undef best
#undef w
#undef idx
#undef sw
}
KP_HD inline int32_t select_groups_dev(const RegionOut* ro, int R, int64_t minC, int64_t maxC, int64_t target,
                                       int32_t* sel) {
  GroupsPriv m;
  return select_groups_in(m, ro, R, minC, maxC, target, sel);
}


// The group-combination step of one region binding (the host step it replaces:
// engine.cpp kp_schedule_batch). rstat != 0: stage A already finalized it.
KP_HD inline int32_t region_groups_one(const RegionOut* ro, int32_t rstat, const BindHdr& h, int R, int32_t* sel) {
  if (rstat != 0) return -1000;
  for (int r = 0; r < R; r++) sel[r] = -1;
  return select_groups_dev(ro, R, h.region_min, h.region_max, h.cluster_min, sel);
}
// ... with the DFS arrays in the thread's LDS slice (k_region_groups_lds; G = R planes)
KP_HD inline int32_t region_groups_one_lds(GroupsLds& m, const RegionOut* ro, int32_t rstat, const BindHdr& h, int R,
                                           int32_t* sel) {
  if (rstat != 0) return -1000;
  for (int r = 0; r < R; r++) sel[r] = -1;
  return select_groups_in(m, ro, R, h.region_min, h.region_max, h.cluster_min, sel);
}
KP_HD inline int64_t go_ceil_div_i64(int32_t a, int64_t b) {
  double q = kp_ceil((double)a / (double)b);
  if (q != q || q >= 9223372036854775808.0 || q < -9223372036854775808.0) return INT64_MIN;  // amd64 CVTTSD2SQ
  return (int64_t)q;
}
// region_a with the candidates bucketed by region (the same answers): every
// candidate's sortClusters key is computed once and kept in place of its (rank,
// estimate) pair (high word in cd.r, low word in cd.v), the region index array
// cd.g becomes a permutation that lists each region's candidates contiguously,
// and each wave walks whole regions (calcGroupScore's prefix in key order) by
// repeated wave minima: no block barrier and no LDS atomic per walk step.
// Returns false (nothing changed) when the candidates exceed the staging the
// permutation needs (kRegionStage per thread); the caller then runs region_a.
constexpr int kRegionStage = 32;

// calcGroupScore's walk over a region (group_clusters.go:299-351) gives the same
// score as its totals when the region is empty, or when every AvailableReplicas is
// >= 0 (the prefix sums only grow) and either the whole region stays below the
// target (the walk never breaks) or every cluster score is 0 (a break gives
// target*1000 + 0, and so do totals at or above the target).
KP_HD inline bool region_walk_free(int64_t cnt, int64_t negatives, int64_t sum_avail, int64_t sum_score,
                                   int64_t target) {
  return cnt == 0 || (negatives == 0 && (sum_avail < target || sum_score == 0));
}
// The score of a region whose walk is free: its totals.
KP_HD inline int64_t region_score_totals(int64_t cnt, int64_t sum_avail, int64_t sum_score, int64_t target) {
  if (cnt == 0) return 0;
  if (sum_avail < target) return add64(mul64(sum_avail, 1000), sum_score / cnt);
  return add64(mul64(target, 1000), sum_score / cnt);
}

// kKeyed (here and in region_a, region_b): the candidates already hold their
// sortClusters keys in place (put_ckey), e.g. with scores other than the in-tree ones.
template <class BLK, bool kKeyed = false>
KP_FI bool region_a_fast(const BLK& B, const SelCtx& x, const Cands& cd, RegionLds L, RegionOut* out) {
  const int F = cd.F;
#if defined(__HIP_DEVICE_COMPILE__)
  if (F > kRegionStage * B.nth()) return false;
#endif
  const BindHdr& h = *x.h;
  const int R = x.s->n_regions;
  int32_t* off = (int32_t*)L.minkey;  // [R + 1] region segment offsets
  int32_t* cur = (int32_t*)L.last;    // [R] fill cursors
  uint16_t* idx = (uint16_t*)cd.g;    // the permutation, in place of the region indices
  for (int r = B.tid(); r < R; r += B.nth()) {
    L.cnt[r] = 0;
    L.dvalid[r] = 0;
    L.sumAvail[r] = 0;
    L.sumScore[r] = 0;
    L.dscore[r] = 0;
    L.amin[r] = 0;
  }
  B.sync();
  const bool dup = (h.flags & BF_GROUP_DUP) != 0;
  for (int i = B.tid(); i < F; i += B.nth()) {
    const uint64_t k = kKeyed ? ckey(cd, i) : cand_key(x, cd, i, cd.v[i]);
    if (!kKeyed) put_ckey(cd, i, k);
    const int r = cd.g[i];
    if (r < 0) continue;
    const int64_t av = key_avail(k), sc = key_score(k);
    kp_atomic_add(&L.cnt[r], 1);
    kp_atomic_add((unsigned long long*)&L.sumAvail[r], (unsigned long long)av);
    if (sc) kp_atomic_add((unsigned long long*)&L.sumScore[r], (unsigned long long)sc);
    if (av < 0) kp_atomic_add((unsigned long long*)&L.amin[r], 1ull);  // negative count
    if (dup && av >= (int64_t)h.replicas) {
      kp_atomic_add(&L.dvalid[r], 1);
      if (sc) kp_atomic_add((unsigned long long*)&L.dscore[r], (unsigned long long)sc);
    }
  }
  B.sync();
  if (dup) {  // calcGroupScoreForDuplicate
    for (int r = B.tid(); r < R; r += B.nth()) {
      const int64_t v = L.dvalid[r];
      out[r].count = L.cnt[r];
      out[r].score = v == 0 ? 0 : add64(mul64(v, 1000), L.dscore[r] / v);
    }
    B.sync();
    return true;
  }
  // calcGroupScore (divided) needs the walk only where it can stop early with a
  // score that differs from the totals' (region_walk_free)
  const int64_t target = go_ceil_div_i64(h.replicas, h.region_min);
  bool walk = false;
  for (int r = B.tid(); r < R; r += B.nth())
    if (!region_walk_free(L.cnt[r], L.amin[r], L.sumAvail[r], L.sumScore[r], target)) walk = true;
  if (!B.any(walk)) {
    for (int r = B.tid(); r < R; r += B.nth()) {
      out[r].count = L.cnt[r];
      out[r].score = region_score_totals(L.cnt[r], L.sumAvail[r], L.sumScore[r], target);
    }
    B.sync();
    return true;
  }
  if (B.tid() == 0) {
    int32_t o = 0;
    for (int r = 0; r < R; r++) {
      off[r] = o;
      cur[r] = o;
      o += L.cnt[r];
    }
    off[R] = o;
  }
  B.sync();
  // the permutation: region r's candidates at [off[r], off[r + 1])
#if defined(__HIP_DEVICE_COMPILE__)
  int16_t gg[kRegionStage];
#pragma unroll
  for (int j = 0; j < kRegionStage; j++) {
    const int i = B.tid() + j * B.nth();
    gg[j] = i < F ? cd.g[i] : (int16_t)-1;
  }
  B.sync();
#pragma unroll
  for (int j = 0; j < kRegionStage; j++) {
    const int i = B.tid() + j * B.nth();
    if (i < F && gg[j] >= 0) idx[kp_atomic_add(&cur[gg[j]], 1)] = (uint16_t)i;
  }
#else
  {
    std::vector<int16_t> gg(cd.g, cd.g + F);
    for (int i = 0; i < F; i++)
      if (gg[i] >= 0) idx[cur[gg[i]]++] = (uint16_t)i;
  }
#endif
  B.sync();
  // calcGroupScore (divided): each region's clusters in sortClusters order until
  // validClusters >= max(clusterMinGroups, minGroups) and the sum reaches the target
  int64_t m = h.cluster_min;
  if (m < h.region_min) m = h.region_min;
  const int ww = B.wwidth(), lane = B.lane();
  auto key = [&](int j) { return ckey(cd, j); };
  for (int r = B.wid(); r < R; r += B.nwaves()) {
    const int64_t cnt = L.cnt[r];
    int64_t sa = L.sumAvail[r], ss = L.sumScore[r], valid = cnt;
    if (!region_walk_free(cnt, L.amin[r], sa, ss, target)) {
      uint64_t last = 0;
      int64_t wcnt = 0, wsum = 0, wscore = 0;
      for (;;) {
        uint64_t mn = ~0ull;
        for (int j = off[r] + lane; j < off[r + 1]; j += ww) {
          const uint64_t k = key(idx[j]);
          if ((wcnt == 0 || k > last) && k < mn) mn = k;
        }
        mn = B.wminu64(mn);
        if (mn == ~0ull) break;  // walked the whole region: the totals
        last = mn;
        wcnt++;
        wsum = add64(wsum, key_avail(mn));
        wscore = add64(wscore, key_score(mn));
        if (wcnt >= m && wsum >= target) {
          sa = wsum;
          ss = wscore;
          valid = wcnt;
          break;
        }
      }
      KP_COUNT(x, 25, wcnt);
    }
    if (lane == 0) {
      out[r].count = (int32_t)cnt;
      if (cnt == 0) out[r].score = 0;
      else if (sa < target) out[r].score = add64(mul64(sa, 1000), ss / cnt);
      else out[r].score = add64(mul64(target, 1000), ss / valid);
    }
  }
  B.sync();
  return true;
}

template <class BLK, bool kKeyed = false>
KP_FI void region_a(const BLK& B, const SelCtx& x, const Cands& cd, RegionLds L, RegionOut* out) {
  const BindHdr& h = *x.h;
  const int R = x.s->n_regions;
  for (int r = B.tid(); r < R; r += B.nth()) {
    L.cnt[r] = 0;
    L.dvalid[r] = 0;
    L.wcnt[r] = 0;
    L.done[r] = 0;
    L.sumAvail[r] = 0;
    L.sumScore[r] = 0;
    L.dscore[r] = 0;
    L.wsum[r] = 0;
    L.wscore[r] = 0;
    L.amin[r] = 0;
    L.last[r] = 0;
  }
  B.sync();
  const bool dup = (h.flags & BF_GROUP_DUP) != 0;
  for (int i = B.tid(); i < cd.F; i += B.nth()) {
    int r = cd.g[i];
    if (r < 0) continue;
    uint64_t k = kKeyed ? ckey(cd, i) : cand_key(x, cd, i, cd.v[i]);
    int64_t av = key_avail(k), sc = key_score(k);
    kp_atomic_add(&L.cnt[r], 1);
    kp_atomic_add((unsigned long long*)&L.sumAvail[r], (unsigned long long)av);
    kp_atomic_add((unsigned long long*)&L.sumScore[r], (unsigned long long)sc);
    if (av < 0) kp_atomic_add((unsigned long long*)&L.amin[r], 1ull);  // negative count
    if (dup && av >= (int64_t)h.replicas) {
      kp_atomic_add(&L.dvalid[r], 1);
      kp_atomic_add((unsigned long long*)&L.dscore[r], (unsigned long long)sc);
    }
  }
  B.sync();
  if (dup) {  // calcGroupScoreForDuplicate
    for (int r = B.tid(); r < R; r += B.nth()) {
      int64_t v = L.dvalid[r];
      out[r].count = L.cnt[r];
      out[r].score = v == 0 ? 0 : add64(mul64(v, 1000), L.dscore[r] / v);
    }
    B.sync();
    return;
  }
  // calcGroupScore (divided): walk each region's clusters in sortClusters order
  const int64_t target = go_ceil_div_i64(h.replicas, h.region_min);
  int64_t m = h.cluster_min;  // clusterMinGroups (last cluster constraint)
  if (m < h.region_min) m = h.region_min;
  for (int r = B.tid(); r < R; r += B.nth())
    if (region_walk_free(L.cnt[r], L.amin[r], L.sumAvail[r], L.sumScore[r], target)) L.done[r] = 1;  // totals
  B.sync();
  KP_COUNT(x, 21, 1);
  for (;;) {
    bool any = false;
    for (int r = B.tid(); r < R; r += B.nth()) {
      if (!L.done[r]) any = true;
      L.minkey[r] = ~0ull;
    }
    if (!B.any(any)) break;
    KP_COUNT(x, 25, 1);
    for (int i = B.tid(); i < cd.F; i += B.nth()) {
      int r = cd.g[i];
      if (r < 0 || L.done[r]) continue;
      uint64_t k = kKeyed ? ckey(cd, i) : cand_key(x, cd, i, cd.v[i]);
      if (L.wcnt[r] > 0 && k <= L.last[r]) continue;
      kp_atomic_min_u64(&L.minkey[r], k);
    }
    B.sync();
    for (int r = B.tid(); r < R; r += B.nth()) {
      if (L.done[r]) continue;
      uint64_t k = L.minkey[r];
      if (k == ~0ull) {
        L.done[r] = 1;
        continue;
      }
      L.last[r] = k;
      L.wcnt[r]++;
      L.wsum[r] = add64(L.wsum[r], key_avail(k));
      L.wscore[r] = add64(L.wscore[r], key_score(k));
      if ((int64_t)L.wcnt[r] >= m && L.wsum[r] >= target) L.done[r] = 2;
    }
    B.sync();
  }
  for (int r = B.tid(); r < R; r += B.nth()) {
    out[r].count = L.cnt[r];
    if (L.cnt[r] == 0) {
      out[r].score = 0;
      continue;
    }
    int64_t sa, ss, valid;
    if (L.done[r] == 2) {
      sa = L.wsum[r];
      ss = L.wscore[r];
      valid = L.wcnt[r];
    } else {  // walked (or skipped) the whole region
      sa = L.sumAvail[r];
      ss = L.sumScore[r];
      valid = L.cnt[r];
    }
    if (sa < target) out[r].score = add64(mul64(sa, 1000), ss / (int64_t)L.cnt[r]);
    else out[r].score = add64(mul64(target, 1000), ss / valid);
  }
  B.sync();
}

// ----------------------------------------------------------------------------
// Region stage B: selectBestClustersByRegion after the host group selection
// (select_clusters_by_region.go:41-63). sel: selected region ids in path order.
// ----------------------------------------------------------------------------
// n_sel: as sel_cluster_fast's (the selection only, no assignment).
template <class BLK, bool kKeyed = false>
KP_FI void region_b(const BLK& B, const SelCtx& x, const Cands& cd, const int32_t* sel, int nsel, uint32_t* hist,
                    unsigned long long* heads, int32_t* rsel, Item* items, uint64_t* keys, void* scratch, int cap,
                    size_t area_bytes, int* n_sel = nullptr) {
  if (n_sel) *n_sel = -1;
  KP_STAMP_INIT
  const BindHdr& h = *x.h;
  const int R = x.s->n_regions;
  for (int r = B.tid(); r < R; r += B.nth()) {
    heads[r] = ~0ull;
    rsel[r] = -1;
  }
  B.sync();
  uint32_t* ctr = hist + 255;
  if (B.tid() == 0) *ctr = 0;
  for (int j = B.tid(); j < nsel; j += B.nth()) rsel[sel[j]] = j;
  B.sync();
  // Only the selected regions' candidates matter from here on: each one's
  // sortClusters key is computed once and the list is compacted in place to them
  // (key in place of the (rank, estimate) pair), so every later pass walks only
  // the selected regions (staged through registers on the device; past the
  // staging, every candidate keeps its key in place uncompacted).
  Cands cd2 = cd;
  {
    auto keep_of = [&](int i) {
      const int r = cd.g[i];
      return r >= 0 && rsel[r] >= 0;
    };
#if defined(__HIP_DEVICE_COMPILE__)
    if (cd.F <= kRegionStage * B.nth()) {
      uint64_t kk[kRegionStage];
      int16_t gg[kRegionStage];
      uint32_t keep = 0;
      int32_t mine = 0;
#pragma unroll
      for (int j = 0; j < kRegionStage; j++) {
        const int i = B.tid() + j * B.nth();
        kk[j] = 0;
        gg[j] = -1;
        if (i < cd.F && keep_of(i)) {
          kk[j] = kKeyed ? ckey(cd, i) : cand_key(x, cd, i, cd.v[i]);
          gg[j] = cd.g[i];
          keep |= 1u << j;
          mine++;
        }
      }
      int32_t tot;
      int32_t pos = B.excl_scan(mine, &tot);  // (its barrier: every read precedes every write)
#pragma unroll
      for (int j = 0; j < kRegionStage; j++)
        if ((keep >> j) & 1u) {
          put_ckey(cd, pos, kk[j]);
          cd.g[pos] = gg[j];
          pos++;
        }
      cd2.F = tot;
    } else if (!kKeyed) {
      for (int i = B.tid(); i < cd.F; i += B.nth()) put_ckey(cd, i, cand_key(x, cd, i, cd.v[i]));
    }
#else
    int pos = 0;
    for (int i = 0; i < cd.F; i++)
      if (keep_of(i)) {  // pos <= i: slot pos was read before
        const uint64_t k = kKeyed ? ckey(cd, i) : cand_key(x, cd, i, cd.v[i]);
        const int16_t g = cd.g[i];
        put_ckey(cd, pos, k);
        cd.g[pos] = g;
        pos++;
      }
    cd2.F = pos;
#endif
    B.sync();
  }
  // One pass: each candidate of a selected region gets its sortClusters key
  // once; the region heads take the minimum and the keys are compacted into
  // `keys` (2*kSmallMax entries) when they fit.
  const int kc = 2 * kSmallMax;
  auto in_sel = [&](int i) {
    const int r = cd2.g[i];
    return r >= 0 && rsel[r] >= 0;
  };
  int32_t mine = 0;
  for (int i = B.tid(); i < cd2.F; i += B.nth()) mine += in_sel(i) ? 1 : 0;
  int32_t pos = B.wave_reserve(mine, ctr);
  for (int i = B.tid(); i < cd2.F; i += B.nth()) {
    if (!in_sel(i)) continue;
    const uint64_t k = ckey(cd2, i);
    kp_atomic_min_u64(&heads[cd2.g[i]], k);
    if (pos < kc) keys[pos] = k;
    pos++;
  }
  B.sync();
  KP_STAMP(x, 18);
  const int64_t total = *ctr;
  int64_t needCnt = total < h.cluster_max ? total : h.cluster_max;
  int64_t restCnt = needCnt - nsel;
  if (restCnt > kSmallMax - nsel) {  // engine limit: selected list capacity
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, -1);
    return;
  }
  for (int j = B.tid(); j < nsel; j += B.nth()) items[j] = item_from_key(x, heads[sel[j]]);
  int n = nsel;
  B.sync();
  if (restCnt > 0 && total <= kc) {
    // the restCnt smallest non-head keys, ascending: heads drop out of the list
    // (~0), then each key's position is the count of smaller keys (keys are
    // distinct: the rank is in the low bits)
    for (int i = B.tid(); i < (int)total; i += B.nth())
      if (keys[i] == heads[x.s->region_idx[key_rank(keys[i])]]) keys[i] = ~0ull;
    B.sync();
    for (int i = B.tid(); i < (int)total; i += B.nth()) {
      const uint64_t k = keys[i];
      if (k == ~0ull) continue;
      const int64_t pos = count_less(keys, (int)total, k);
      if (pos < restCnt) items[nsel + pos] = item_from_key(x, k);
    }
    n = nsel + (int)restCnt;
    B.sync();
  } else if (restCnt > 0) {
    KP_COUNT(x, 31, 1);
    auto incand = [&](int i) {
      int r = cd2.g[i];
      return r >= 0 && rsel[r] >= 0 && ckey(cd2, i) != heads[r];
    };
    auto key = [&](int i) { return ckey(cd2, i); };
    uint64_t kth = radix_select(B, hist, cd2.F, incand, key, restCnt);
    int m = 0;
    for (int t0 = 0; t0 < cd2.F; t0 += B.nth()) {
      int i = t0 + B.tid();
      uint64_t k = 0;
      bool e = false;
      if (i < cd2.F && incand(i)) {
        k = key(i);
        e = k <= kth;
      }
      int32_t tt;
      int32_t off = B.excl_scan(e ? 1 : 0, &tt);
      if (e) keys[m + off] = k;
      m += tt;
    }
    B.sync();
    place_sorted(B, x, keys, m, items + nsel);
    n = nsel + m;
  }
  KP_STAMP(x, 19);
  if (n_sel) {
    *n_sel = n;
    return;
  }
  assign_small(B, x, items, n, scratch, cap, area_bytes);
  KP_STAMP(x, 20);
}

}  // namespace kp
