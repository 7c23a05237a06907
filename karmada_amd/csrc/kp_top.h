// kp_top.h — SEL_ALL DynamicWeight / Aggregated assignment over the candidates that
// can matter (k_select_top), one wave64 per binding.
//
// The exact divisions (division_algorithm.go:75-101, webstermethod.go:112-161) only
// look at a few candidates when the target is small against the candidate count:
//   * Webster (DynamicWeight): a party whose vote is below the N-th largest party
//     vote (N = seats) has N elements strictly above its first one, so it takes no
//     seat; the parties with votes >= that N-th vote decide everything.
//   * Aggregated: the cut (sort.Sort by Replicas desc, prior clusters first, prefix
//     until the running sum reaches the target) keeps the prior clusters and the
//     non-prior candidates whose votes are >= the cut value v*.
// Each estimator class's row is sorted once per batch by (estimate desc, rank asc)
// (k_class_order), so a binding walks its class's order, skipping infeasible
// clusters (its k_filter row), and stops once the walked candidates cover the
// target; it then takes the rest of the tie group at the last value. The scheduled
// clusters (spec.Clusters among the candidates) are always in the subset: their
// votes may include their replicas (fresh) and they lead the Aggregated order.
// sel_all_fast then runs unchanged over that subset (kp_paths.h TopInfo), with the
// full candidate count for sort.Sort's n > 12 test. Anything else — other
// strategies, overflow tiers, a subset past its LDS capacity, a class whose
// estimates could wrap int32 sums — goes to the fallback list, which the gathered
// k_select_all then schedules with every candidate.
#pragma once
#include "kp_kernels.h"

namespace kp {

// ---- per-class candidate order ------------------------------------------------
// ord[k][i], i < C: (estimate << 32) | rank of class k's row sorted by estimate
// desc, rank asc; tot[k] = the row's sum over c < C; ok[k] = 0 when the row cannot
// be walked (row 0 = non-workload MaxInt32, or an estimate at MaxInt32 whose merged
// value is spec.Replicas and so differs per binding).
template <class BLK>
KP_FI void body_class_order(const BLK& B, int k, uint64_t* keys, int P, const SnapView& s, const int32_t* rows,
                            uint64_t* ord, int64_t* tot, int32_t* ok) {
  const int32_t* row = rows + (size_t)k * s.Cp;
  int64_t sum = 0, bad = k == 0 ? 1 : 0;
  for (int i = B.tid(); i < P; i += B.nth()) {
    uint64_t key = ~0ull;
    if (i < s.C) {
      const int32_t e = row[i];
      if (e < 0 || e == kInt32Max) bad = 1;
      sum += e;
      key = ((uint64_t)(uint32_t)(kInt32Max - (e < 0 ? 0 : e)) << 32) | (uint32_t)i;  // desc estimate, asc rank
    }
    keys[i] = key;
  }
  B.sync();
  // Bitonic sort, ascending. Thread t owns i = t + nth*q, so a stage whose partner
  // distance j is below the wave width pairs lanes of one wave: its writes need only
  // the wave's own ordering before the next such stage; a workgroup barrier follows the
  // stages with j >= 64 and the last stage of each len >= 64 (the next len starts with
  // j = len). 91 barriers -> 28 at P = 8 192.
  for (int len = 2; len <= P; len <<= 1)
    for (int j = len >> 1; j > 0; j >>= 1) {
      for (int i = B.tid(); i < P; i += B.nth()) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t a = keys[i], b = keys[l];
          const bool up = (i & len) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[l] = a;
          }
        }
      }
      if (j >= 64 || (j == 1 && len >= 64)) B.sync();
      else B.wsync();
    }
  for (int i = B.tid(); i < s.C; i += B.nth()) {
    const uint64_t key = keys[i];
    const uint32_t e = (uint32_t)kInt32Max - (uint32_t)(key >> 32);
    ord[(size_t)k * s.Cp + i] = ((uint64_t)e << 32) | (key & 0xffffffffull);
  }
  int64_t t = sum, b = bad;
  B.reduce2(t, [](int64_t p, int64_t q) { return p + q; }, 0, b, [](int64_t p, int64_t q) { return p > q ? p : q; }, 0);
  if (B.tid() == 0) {
    tot[k] = t;
    ok[k] = b ? 0 : 1;
  }
}

// ---- per-binding subset selection ----------------------------------------------
struct TopArgs {
  const uint64_t* ord;  // [n_classes][Cp]
  const int64_t* tot;   // [n_classes]
  const int32_t* ok;    // [n_classes]
  int32_t* fb;          // fallback list (bindings for the full-candidate kernel)
  uint32_t* fb_n;       // its length
  int cap;              // subset capacity (LDS entries per wave)
  // set: bindings whose subset outgrows cap go here instead (a larger-capacity launch
  // takes them; its own overflow goes to fb)
  int32_t* ofb = nullptr;
  uint32_t* ofb_n = nullptr;
};

// Webster's party list / enumeration buffer of the subset path (u64 entries): larger
// party sets take its uncompacted passes over the subset (exact, kp_select.h).
#ifndef KP_TOP_ECAP
#define KP_TOP_ECAP 160
#endif
constexpr int kTopEcap = KP_TOP_ECAP;
// bindings whose Replicas + len(spec.Clusters) is at most this take the small slice
constexpr int64_t kTopSmallNeed = 160;
// workgroups of the launch over the capacity-overflow list (its length is on the device;
// the waves stride over it): 256 CUs x 4 resident workgroups of the large slice
constexpr int kTopOverGrid = 1024;
KP_HD inline int top_ecap(int cap) { return cap < kTopEcap ? cap : kTopEcap; }
// LDS slice of one binding: [red 64 B | mask W u64 | S votes cap | S ranks cap (u16) | SelScratch]
// (the LDS a wave holds bounds the waves per CU, and this kernel runs as fast as it
// keeps waves in flight: 16-bit ranks, so k_select_top needs Cp <= kTopMaxCp; one
// Cp-bit mask serves as the walk's candidate set and then as the target bits)
KP_HD inline size_t top_lds_bytes(int Cp, int cap) {
  const int W = Cp / 64;
  return 64 + 8 * (size_t)W + 6 * (size_t)cap + 3072 + 8 * (size_t)top_ecap(cap) + 64;
}
constexpr int kTopMaxCp = 1 << 16;

// The subset in LDS: votes and 16-bit ranks (k_select_top's bindings have no overflow
// tiers, so no tier bits ride on the rank).
struct TopSub {
  uint16_t* r;
  int32_t* v;
  int32_t F;
};
// sel_all_fast's candidate set over a TopSub (as LdsCands over Cands)
struct TopCands {
  const TopSub* cd;
  int tid, nth;
  template <class Fn>
  KP_FI void each(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) fn((uint32_t)cd->r[i], cd->v[i]);
  }
  template <class Fn>
  KP_FI void each_set(Fn fn) const {
    for (int i = tid; i < cd->F; i += nth) cd->v[i] = fn((uint32_t)cd->r[i], cd->v[i]);
  }
  static constexpr bool kSettable = true;
  KP_FI uint64_t okey(const SelCtx& x, uint32_t rk, int32_t v0) const { return cand_order_key(x, rk, v0); }
  static constexpr bool kExact = false;
};

// Octave bucket of a vote (8 buckets per power of two), monotone in the vote: the
// histogram the no-class-order path (TopArgs::ord == nullptr) thresholds the votes by.
KP_HD inline int vote_octave(int32_t v) {
  if (v <= 0) return 0;
  const int e = 31 - __builtin_clz((uint32_t)v);
  const int m = e >= 3 ? (v >> (e - 3)) & 7 : (v << (3 - e)) & 7;
  return 1 + 8 * e + m;  // 1..248
}

template <class BLK>
KP_FI void top_fallback(const BLK& B, const KArgs& a, const TopArgs& t, int b, bool over_cap = false) {
  if (B.tid() != 0) return;
  if (over_cap && t.ofb) t.ofb[kp_atomic_add(t.ofb_n, 1u)] = b;
  else t.fb[kp_atomic_add(t.fb_n, 1u)] = b;
}

#ifndef KP_TOP_AHEAD
#define KP_TOP_AHEAD 8
#endif
#ifndef KP_TOP_GROUP
#define KP_TOP_GROUP 4
#endif
constexpr int kTopAhead = KP_TOP_AHEAD, kTopGroup = KP_TOP_GROUP;
constexpr int kTopRowRegs = 2;  // feasibility-row words preloaded per lane (C <= 8192 in full)
constexpr int kTopStream = 8;  // row chunks per step of the no-class-order passes
static_assert(kTopAhead % kTopGroup == 0, "the ring holds whole groups");

// Hand-off of a binding from wave 0's walk to its workgroup's selection (k_select_top_wg).
struct TopHand {
  int32_t go, n, complete, pad;
  int64_t F;
};

// The LDS slice of one binding: [red 64 B | mask W u64 | S votes cap | S ranks cap |
// SelScratch], carved the same way by every wave that reads it. The mask holds the
// feasibility row, then (after the scheduled clusters are taken) the feasible clusters
// that are not scheduled (the walk's candidates), then the feasible scheduled clusters
// (the division's target bits: it reads feasibility only for targets).
struct TopCarve {
  uint64_t* frow;
  TopSub cd;
  SelScratch ss;
};
KP_HD inline TopCarve top_carve(unsigned char* smem, const SnapView& s, int cap, unsigned long long* dbg) {
  TopCarve c;
  unsigned char* p = smem + 64;
  c.frow = (uint64_t*)p;
  p += 8 * (size_t)s.W;
  c.cd.v = (int32_t*)p;
  c.cd.r = (uint16_t*)(c.cd.v + cap);
  c.cd.F = 0;
  c.ss = carve_sel_scratch((unsigned char*)(c.cd.r + cap), 2 * cap);  // (cap % 64 == 0: 8-B aligned)
  c.ss.cap = top_ecap(cap);
  c.ss.dbg = dbg;
  return c;
}

// The scheduled replicas of a spec.Clusters entry by its rank (the target list, scanned:
// k_select_top keeps no target bits until its division)
KP_HD inline int32_t target_rep(const SelCtx& x, uint32_t rank) {
  const BindHdr& h = *x.h;
  for (int j = 0; j < h.tgt_cnt; j++)
    if ((uint32_t)x.bv->ipool[h.tgt_off + 2 * j] == rank) return x.bv->ipool[h.tgt_off + 2 * j + 1];
  return 0;
}

// hand: wave 0 of a k_select_top_wg workgroup stops after the walk and leaves the
// selection to the whole workgroup (the subset is in the slice, the counts in *hand).
template <class BLK>
KP_FI void body_select_top(const BLK& B, int blk, unsigned char* smem, const KArgs& a, const TopArgs& t,
                           TopHand* hand = nullptr) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const int32_t cls = a.lcls ? a.lcls[blk] : (a.bcls ? a.bcls[b] : 0);
  const SnapView& s = a.s;
  // the feasibility row's first kTopRowRegs words per lane, loaded with the header (the
  // row copy below is then not one more memory latency after the eligibility checks)
  uint64_t fw[kTopRowRegs];
#if defined(__clang__)
#pragma unroll
#endif
  for (int q = 0; q < kTopRowRegs; q++) {
    const int w = (int)(B.tid() % B.wwidth()) + q * B.wwidth();
    fw[q] = w < s.W ? a.fmask[(size_t)b * s.W + w] : 0ull;
  }
  // the header as a register copy: read through a.bv.hdr, its fields would be reloaded
  // (each reload waiting on every load in flight) after every store or wave barrier
  const BindHdr hloc = a.bv.hdr[b];
  const BindHdr* h = &hloc;
  // eligibility: SEL_ALL Dynamic/Aggregated workloads the subset argument covers
  const uint32_t fl = h->flags;
  const int st = h->strategy;
  // (header fields the loops test, held in registers: read through h, the compiler reloads
  // them after every LDS store it cannot tell from global memory, and each reload waits
  // for every load in flight, the walk's prefetch ring included)
  const bool has_tgt = kp_uniform(h->tgt_cnt) > 0;
  // the first chunks of the class order, loaded with the binding's header and row (the
  // walk is the first to read them; a binding that does not walk wastes a few L2 hits)
  // (no class orders: the votes are thresholded by a histogram instead of a walk)
  const uint64_t* ord = t.ord ? t.ord + (size_t)cls * s.Cp : nullptr;
  const int lane = B.tid() % B.wwidth();
  const int ww = B.wwidth();
  uint64_t ring[kTopAhead];
#if defined(__clang__)
#pragma unroll
#endif
  for (int q = 0; q < kTopAhead; q++) ring[q] = ord && lane + q * ww < s.C ? ord[lane + q * ww] : 0;
  bool elig = a.bcls != nullptr && h->sel == SEL_ALL && (st == ST_DYNAMIC || st == ST_AGGREGATED) &&
              (fl & BF_WORKLOAD_ASSIGN) && !(fl & (BF_EMPTY_PROP | BF_BAD | BF_DUP_TARGETS | BF_OVERFLOW)) &&
              h->ovf_mode == OVF_ZERO && h->replicas > 0 && (!ord || t.ok[cls] != 0);
  int64_t sch = 0;  // |scheduled replicas|
  if (elig) {  // no int32 wrap anywhere: every vote sum stays below the class total + |scheduled replicas|
    for (int j = 0; j < h->tgt_cnt; j++) {
      const int32_t r = kp_ldu(a.bv.ipool + h->tgt_off + 2 * j + 1);
      sch += r < 0 ? -(int64_t)r : (int64_t)r;
    }
    if (ord) elig = t.tot[cls] + sch < (int64_t)kInt32Max / 2;  // (else checked over the feasible votes below)
  }
  if (!elig) {
    if (a.bcls != nullptr && (h->sel == SEL_ERR_UNSUPPORTED || (fl & BF_BAD))) {
      // an error result needs only F (select_all_common's order: the bad request, the
      // FitError, then the unsupported spread constraint, select_clusters.go:54), so
      // it is written here instead of gathering every candidate in k_select_all
      SelCtx x = make_ctx(a, b, nullptr);
      x.h = h;
      int64_t F = 0;
      for (int w = B.tid(); w < s.W; w += B.nth()) F += popc64(x.frow[w]);
      F = B.sum64(F);
      if (pre_checks(B, x, (int)F)) return;
      if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_SPREAD_UNSUPPORTED, 0);
      return;
    }
    top_fallback(B, a, t, b);
    return;
  }
  KP_STAMPD(a.dbg, 62);  // (stamps build: [62] header and eligibility, [9] the row copy)
  TopCarve tc = top_carve(smem, s, t.cap, a.dbg);
  uint64_t* frow = tc.frow;
  TopSub cd = tc.cd;
  SelScratch ss = tc.ss;
  // (no target bits until the division: the walk's mask excludes the targets itself)
  SelCtx x = make_ctx(a, b, nullptr);
  x.h = h;
  if (a.bcls) {  // (the class from the list: make_ctx's reload of bcls[b] is dead)
    x.erow = a.est + (size_t)cls * s.Cp;
    x.mrep = cls ? h->replicas : kInt32Max;
  }
  int64_t F = 0;
  if (B.nth() == B.wwidth()) {  // (one wave: the preloaded words, then any past them)
#if defined(__clang__)
#pragma unroll
#endif
    for (int q = 0; q < kTopRowRegs; q++) {
      const int w = B.tid() + q * B.wwidth();
      if (w < s.W) {
        frow[w] = fw[q];
        F += popc64(fw[q]);
      }
    }
    for (int w = B.tid() + kTopRowRegs * B.wwidth(); w < s.W; w += B.nth()) {
      const uint64_t m = x.frow[w];
      frow[w] = m;
      F += popc64(m);
    }
  } else {
    for (int w = B.tid(); w < s.W; w += B.nth()) {
      const uint64_t m = x.frow[w];
      frow[w] = m;
      F += popc64(m);
    }
  }
  F = B.sum64(F);  // (also orders the frow copy before the walk)
  x.frow = frow;   // every later feasibility test reads the LDS copy
  KP_STAMP(x, 9);
  KP_COUNT(x, 15, 1);
  if (pre_checks(B, x, (int)F)) return;
#if defined(KP_TOP_EXIT) && KP_TOP_EXIT == 1  // timing experiments only: phases cut off (wrong results)
  if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, 0);
  return;
#endif
  // the scheduled clusters among the candidates (spec.Clusters ∩ feasible): always
  // in the subset, with the votes the division gives them
  const bool fresh = (fl & BF_FRESH) != 0;
  const bool agg = st == ST_AGGREGATED;
  uint32_t* ctr = (uint32_t*)smem;  // subset length
  int64_t asum = 0, apos = 0, tsum = 0;
  int64_t psum_t = 0;  // the votes of the scheduled clusters with replicas > 0 (the prior clusters)
  int32_t n = 0;
  if (h->tgt_cnt > 0) {  // (none: an empty subset and zero sums, no reductions)
    if (B.tid() == 0) *ctr = 0;
    B.sync();
    int32_t mine = 0;
    for (int j = B.tid(); j < h->tgt_cnt; j += B.nth())
      mine += mask_test(x.frow, (int)kp_ldu(a.bv.ipool + h->tgt_off + 2 * j)) ? 1 : 0;
    int32_t pos = B.wave_reserve(mine, ctr);
    for (int j = B.tid(); j < h->tgt_cnt; j += B.nth()) {
      const uint32_t r = (uint32_t)kp_ldu(a.bv.ipool + h->tgt_off + 2 * j);
      if (!mask_test(x.frow, (int)r)) continue;
      const int32_t sr = kp_ldu(a.bv.ipool + h->tgt_off + 2 * j + 1);
      const int32_t e = est_at(x, (int)r);  // the subset holds AllocatableReplicas (sel_all_fast adds
      if (pos < t.cap) {                     // the scheduled replicas to a fresh vote itself)
        cd.r[pos] = (uint16_t)r;
        cd.v[pos] = e;
      }
      pos++;
      asum += sr;
      apos += sr > 0 ? 1 : 0;
      tsum += fresh ? add32(e, sr) : e;
      psum_t += sr > 0 ? e : 0;
    }
    B.sum2(asum, apos);
    B.sum2(tsum, psum_t);
    n = (int32_t)*ctr;  // (the reductions ordered the reservation)
    // the mask drops the scheduled clusters: it is the walk's candidate set from here
    for (int j = B.tid(); j < h->tgt_cnt; j += B.nth()) {
      const uint32_t r = (uint32_t)kp_ldu(a.bv.ipool + h->tgt_off + 2 * j);
      kp_atomic_and((uint32_t*)frow + (r >> 5), ~(1u << (r & 31)));
    }
    B.sync();
  }
  const int32_t nsched = n;  // the subset's first nsched entries: the feasible scheduled clusters
  if (n > t.cap) {
    top_fallback(B, a, t, b, true);
    return;
  }
  const int32_t assigned = wrap32(asum);
  bool complete = false;
  KP_STAMP(x, 10);
  // No class order (about one binding per estimator class, so sorting a row per
  // binding costs more than walking it): one pass over the feasible row takes the
  // votes of the non-scheduled candidates, their total (the int32 wrap check the class
  // total makes otherwise) and, for a fresh / scale-up division, the subset: an octave
  // histogram of the votes (in the slice's SelScratch, free until sel_all_fast) finds
  // the deciding bucket, the highest one whose cumulative votes cover the walk's
  // condition, and every candidate in or above it joins the subset — the walk's
  // argument with vmin = that bucket's lower edge (a coarser vmin only adds candidates
  // with votes >= it, ties included). One quantity per bucket suffices: DynamicWeight
  // covers once the count reaches the seats (in buckets >= 1 every vote is >= 1, so the
  // sum then reaches them too, the scheduled votes being >= 0), Aggregated once
  // min(tsum, psum) plus the sum reaches the target. The bucket only rises as the pass
  // goes, so the list is compacted to it when it fills. The u32 sums only wrap when the
  // total does, and the binding falls back then.
  uint32_t* hq = ss.hist;
  int64_t rsum = 0, rcnt = 0;
  if (!ord) {
    const bool walk = fresh || assigned < h->replicas;
    const int32_t target = fresh ? h->replicas : sub32(h->replicas, assigned);
    // Aggregated scale up: the prior clusters lead the order
    const int64_t psum = walk && agg && !fresh && apos != 0 ? psum_t : 0;
    if (walk && tsum < 0) {  // (negative scheduled votes: the one-quantity argument needs >= 0)
      top_fallback(B, a, t, b);
      return;
    }
    const bool collect = walk && !(agg && tsum >= (int64_t)target && psum >= (int64_t)target);
    const int64_t base = agg ? (tsum < psum ? tsum : psum) : 0;
    // the list [n0, n) keeps the appended candidates whose bucket is >= lo
    const int32_t n0 = n;
    // The deciding bucket from the list: it holds every candidate seen so far whose
    // bucket is at or above the current one (and everything while none covers yet), so
    // its histogram answers exactly for those buckets; -1: none covers (every candidate).
    auto find_thr = [&]() -> int64_t {
      for (int i = B.tid(); i < 256; i += B.nth()) hq[i] = 0;
      B.sync();
      for (int i = n0 + B.tid(); i < n; i += B.nth()) {
        const int32_t v = cd.v[i];
        kp_atomic_add(&hq[vote_octave(v)], agg ? (uint32_t)v : 1u);
      }
      B.sync();  // (the histogram updates before the reads)
      int64_t thr = -1, run = 0;
      for (int j0 = 0; j0 < 256 && thr < 0; j0 += 4 * B.nth()) {
        const int j = j0 + 4 * B.tid();  // this thread's 4 buckets, descending: 255 - j - q
        int32_t q4 = 0;
        for (int q = 0; q < 4 && j + q < 256; q++) q4 += (int32_t)hq[255 - (j + q)];
        int32_t tq;
        int64_t pq = run + B.excl_scan(q4, &tq), mine = -1;
        for (int q = 0; q < 4 && j + q < 256 && mine < 0; q++) {
          const int bk = 255 - (j + q);
          pq += hq[bk];
          if (agg ? base + pq >= (int64_t)target : (bk >= 1 && pq >= (int64_t)target)) mine = bk;
        }
        thr = B.max64(mine);  // the first (highest) bucket that covers
        run += tq;
      }
      return thr;
    };
    auto compact = [&](int64_t lo) {
      int m = n0;
      for (int i0 = n0; i0 < n; i0 += B.nth()) {
        const int i = i0 + B.tid();
        uint32_t r = 0;
        int32_t v = 0;
        bool keep = false;
        if (i < n) {
          r = cd.r[i];
          v = cd.v[i];
          keep = vote_octave(v) >= lo;
        }
        int32_t tot;
        const int32_t pos = m + B.excl_scan(keep ? 1 : 0, &tot);  // (its barrier: reads before writes)
        if (keep) {
          cd.r[pos] = (uint16_t)r;
          cd.v[pos] = v;
        }
        m += tot;
      }
      B.sync();
      n = m;
    };
    int64_t neg = 0, thr = -1;
    bool over = false;
    KP_STAMP(x, 70);
    // kTopStream chunks per step: their row loads are issued together
    for (int c0 = 0; c0 < s.C; c0 += kTopStream * B.nth()) {
      int32_t vv[kTopStream];
      bool ff[kTopStream];
#if defined(__clang__)
#pragma unroll
#endif
      for (int u = 0; u < kTopStream; u++) {
        const int c = c0 + u * B.nth() + B.tid();
        ff[u] = c < s.C && ((frow[c >> 6] >> (c & 63)) & 1ull);  // (the mask: feasible, not scheduled)
        vv[u] = ff[u] ? x.erow[c] : 0;
      }
#if defined(__clang__)
#pragma unroll
#endif
      for (int u = 0; u < kTopStream; u++) {
        vv[u] = est_merge(x, vv[u]);
        if (!ff[u]) continue;
        if (vv[u] < 0) {
          neg = 1;
          ff[u] = false;
          continue;
        }
        rsum += vv[u];
        rcnt++;
      }
      if (!collect || over) continue;
#if defined(__clang__)
#pragma unroll
#endif
      for (int u = 0; u < kTopStream; u++) {
        bool in = ff[u] && vote_octave(vv[u]) >= thr;
        uint64_t m = B.wballot(in);
        if (n + popc64(m) > t.cap) {  // full: compact to the bucket as it stands now (it only rises)
          const int64_t th2 = find_thr();
          if (th2 > thr) thr = th2;
          compact(thr);
          KP_COUNT(x, 72, 1);
          in = in && vote_octave(vv[u]) >= thr;
          m = B.wballot(in);
          if (n + popc64(m) > t.cap) {
            over = true;
            break;
          }
        }
        if (in) {
          const int pos = n + popc64(m & B.wlt());
          cd.r[pos] = (uint16_t)(c0 + u * B.nth() + B.tid());
          cd.v[pos] = vv[u];
        }
        n += popc64(m);
      }
    }
    B.sum2(rsum, neg);
    rcnt = B.sum64(rcnt);  // (the reductions also order the histogram and the list before the reads)
    KP_STAMP(x, 71);
    KP_COUNT(x, 73, over ? 1 : 0);
    // negative votes / wrap risk (every vote sum the division takes is below this bound):
    // every candidate
    if (neg || rsum + (tsum < 0 ? -tsum : tsum) + sch >= (int64_t)kInt32Max / 2) {
      top_fallback(B, a, t, b);
      return;
    }
    if (collect) {
      if (over) {
        // past the capacity: the availability error needs only the votes' sum (below
        // 2^30); otherwise every candidate (the full-candidate kernel)
        if ((int64_t)(int32_t)(tsum + rsum) < (int64_t)target) {
          if (B.tid() == 0)
            sink_error(x, KP_STATUS_UNSCHEDULABLE, fresh ? KP_ERR_FRESH_NOT_ENOUGH : KP_ERR_SCALE_UP_NOT_ENOUGH,
                       (int32_t)(tsum + rsum));
          return;
        }
        top_fallback(B, a, t, b, true);
        return;
      }
      const int64_t th2 = find_thr();
      if (th2 > thr) thr = th2;
      compact(thr);  // exactly the candidates in or above the deciding bucket
      complete = (int64_t)(n - n0) == rcnt;
      KP_STAMP(x, 74);
      KP_COUNT(x, 75, n);
    }
  }
  if (fresh || assigned < h->replicas) {
    // fresh / scale up: walk the class order for the non-scheduled candidates
    const int32_t target = fresh ? h->replicas : sub32(h->replicas, assigned);
    // Aggregated scale up with prior clusters: they lead the order (resortAvailableClusters,
    // assignment.go:151-178); their votes count toward the cut before any walked one
    const int64_t psum = agg && !fresh && apos != 0 ? psum_t : 0;
    // The walk takes kTopGroup chunks of the class order per step: their feasibility
    // tests (LDS lookups of the binding's row) are issued together, their entries are
    // appended in order, and coverage is decided once per step over the group, with its
    // smallest walked vote as vmin. A coarser step only adds candidates with votes >= a
    // smaller vmin to the subset (plus the whole tie group at it), which the subset
    // argument allows; it divides the dependent reductions and decisions per entry by
    // kTopGroup. The loads run kTopAhead chunks ahead in a register ring (its first
    // loads were issued with the binding's own, above).
    int64_t walked = 0, wsum = 0;
    const int32_t n0 = n;  // the scheduled clusters lead the subset
    bool tie = false;
    int32_t tie_v = 0;
    // (Aggregated: the prior clusters alone may already reach the target; no walk)
    const bool cov0 = agg && tsum >= (int64_t)target && psum >= (int64_t)target;
    int i0_last = -B.wwidth();  // (the stamps build counts the walked chunks)
    (void)i0_last;
    // Hopeless: every unwalked candidate's vote is at most the last walked one (the
    // order is votes desc), so once the subset's votes plus vmin times the feasible
    // candidates not yet walked stay below the target, no candidate set covers it:
    // dynamicDivideReplicas' availability error (division_algorithm.go:75-78), whose
    // argument (the votes' sum) one parallel pass below takes instead of walking the
    // rest of the order. F - n0: the feasible candidates that are not scheduled.
    const int64_t unsched = F - (int64_t)n0;
    bool hopeless = false;
    for (int g0 = 0; ord && !cov0; g0 += kTopGroup * ww) {
      i0_last = g0 + (kTopGroup - 1) * ww;
      if (g0 >= s.C) {
        complete = true;
        break;
      }
      uint32_t rg[kTopGroup];
      int32_t vg[kTopGroup];
      uint64_t mg[kTopGroup];
      bool fg[kTopGroup];
      bool past = false;
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q < kTopGroup; q++) {
        const uint64_t e = ring[q];
        rg[q] = (uint32_t)e;
        vg[q] = (int32_t)(e >> 32);
        const bool valid = g0 + q * ww + lane < s.C;
        fg[q] = valid && ((frow[rg[q] >> 6] >> (rg[q] & 63)) & 1ull);  // (feasible, not scheduled)
        if (tie && valid) {
          past = past || vg[q] < tie_v;
          fg[q] = fg[q] && vg[q] == tie_v;
        }
      }
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q + kTopGroup < kTopAhead; q++) ring[q] = ring[q + kTopGroup];
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q < kTopGroup; q++) {
        const int i = g0 + (kTopAhead + q) * ww + lane;
        ring[kTopAhead - kTopGroup + q] = i < s.C ? ord[i] : 0;
      }
      int cnt = 0, last = -1;
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q < kTopGroup; q++) {
        mg[q] = B.wballot(fg[q]);
        cnt += popc64(mg[q]);
        if (mg[q]) last = q;
      }
      const bool any_past = B.wballot(past) != 0;
      if (n + cnt > t.cap) {
        n += cnt;
        break;
      }
      int base = n;
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q < kTopGroup; q++) {
        if (fg[q]) {
          const int pos = base + popc64(mg[q] & B.wlt());
          cd.r[pos] = (uint16_t)rg[q];
          cd.v[pos] = vg[q];
        }
        base += popc64(mg[q]);
      }
      n += cnt;
      if (tie) {
        if (any_past) break;
        continue;
      }
      // the group's sum (int32: the class row's total is below 2^30) and its smallest
      // walked vote: the last walked lane's of its last chunk with one, votes desc
      int32_t mine = 0;
#if defined(__clang__)
#pragma unroll
#endif
      for (int q = 0; q < kTopGroup; q++) mine += fg[q] ? vg[q] : 0;
      const int32_t add = B.wsum32(mine);
      int32_t vmin = 0;
      if (cnt > 0) {
        int32_t vl = vg[0];
#if defined(__clang__)
#pragma unroll
#endif
        for (int q = 1; q < kTopGroup; q++) vl = last == q ? vg[q] : vl;
        vmin = B.wread(vl, 63 - __builtin_clzll(mg[last]));
      }
      walked += cnt;
      wsum += add;
      // DynamicWeight: the subset (scheduled clusters + every walked party) holds at
      // least N seat priorities strictly above vmin, so the N-th largest priority t* is
      // above vmin, and every unwalked party (vote <= vmin) has all its priorities below
      // t*: no seat, no tie (#{k : v/(2k+1) > vmin} = ((v-1)/vmin + 1)/2 for v > vmin,
      // integers; float64 priorities order the same way for votes below 2^31). The rule
      // is pinned against the reference heap in tests/test_cpusim_units.py.
      // The count is bounded by (S / vmin + n) / 2 (S = the subset's vote sum), so the
      // exact pass runs only once the bound reaches the target; votes stay below 2^30
      // (eligibility), so it divides in 32 bits.
      if (!agg && cnt > 0 && vmin > 0 && tsum + wsum >= (int64_t)target &&
          (int64_t)((double)(tsum + wsum) / (double)vmin) / 2 + n / 2 + 2 >= (int64_t)target) {
        B.wsync();  // this group's subset entries, written by their lanes, before the reads
        const uint32_t vm = (uint32_t)vmin;
        int64_t above = 0;
        for (int j = lane; j < n; j += ww) {
          uint32_t vq = (uint32_t)cd.v[j];
          if (j < n0 && fresh) vq += (uint32_t)target_rep(x, cd.r[j]);
          above += vq > vm ? ((vq - 1) / vm + 1) / 2 : 0;
        }
        if (B.sum64(above) >= (int64_t)target) break;  // (wave-uniform)
      }
      // covered: the subset's votes reach the target (the availability check passes on
      // every candidate too) and the walked ones decide the division: the N-th largest
      // party vote (DynamicWeight) or the cut value (Aggregated) is >= vmin
      const bool cov = tsum + wsum >= (int64_t)target && (agg ? psum + wsum >= (int64_t)target : walked >= (int64_t)target);
      if (cov) {  // then the rest of the tie group at the last (smallest) vote
        tie = true;
        tie_v = vmin;
      } else if (cnt > 0 && (int64_t)target < kSeatWrap &&
                 tsum + wsum + (int64_t)vmin * (unsched - walked) < (int64_t)target) {
        hopeless = true;
        break;
      }
    }
    KP_COUNT(x, 13, (i0_last + B.wwidth()) / B.wwidth());
    if (n > t.cap || hopeless) {
      // Past capacity before covering the target: when every candidate's votes together
      // stay below it, the answer is dynamicDivideReplicas' availability error
      // (division_algorithm.go:75-78; the sum cannot wrap: the class total is below
      // 2^30), which needs only that sum; otherwise the full-candidate kernel decides.
      int64_t rest = 0;  // the votes of the feasible non-scheduled candidates
      for (int c = B.tid(); c < s.C; c += B.nth())
        if ((frow[c >> 6] >> (c & 63)) & 1ull) rest += est_at(x, c);
      rest = B.sum64(rest);
      if ((int64_t)(int32_t)(tsum + rest) < (int64_t)target) {
        if (B.tid() == 0)
          sink_error(x, KP_STATUS_UNSCHEDULABLE, fresh ? KP_ERR_FRESH_NOT_ENOUGH : KP_ERR_SCALE_UP_NOT_ENOUGH,
                     (int32_t)(tsum + rest));
        return;
      }
      top_fallback(B, a, t, b, !hopeless);
      return;
    }
  }
  KP_STAMP(x, 61);  // ([61] the walk or histogram pass, [11] the target mask)
  if (has_tgt) {
    // the mask becomes the feasible scheduled clusters (the subset's first nsched
    // entries): the division's target bits, and the only feasibility it reads
    for (int w = B.tid(); w < s.W; w += B.nth()) frow[w] = 0;
    B.sync();
    for (int i = B.tid(); i < nsched; i += B.nth())
      kp_atomic_or((uint32_t*)frow + (cd.r[i] >> 5), 1u << (cd.r[i] & 31));
    B.sync();
  }
  x.tgt_bits = (const uint32_t*)frow;
  KP_STAMP(x, 11);
#if defined(KP_TOP_EXIT) && KP_TOP_EXIT == 2
  if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, n);
  return;
#endif
  KP_COUNT(x, 14, n);
  KP_COUNT(x, 40 + (n <= 16 ? 0 : n <= 32 ? 1 : n <= 64 ? 2 : n <= 128 ? 3 : n <= 256 ? 4 : n <= 512 ? 5 : 6), 1);
  KP_COUNT(x, 47 + (agg ? 1 : 0), 1);
  cd.F = n;
  B.sync();
  if (hand) {
    if (B.tid() == 0) *hand = TopHand{1, n, complete ? 1 : 0, 0, F};
    return;
  }
  const TopInfo ti{F, complete};
  int why;
  if (n <= B.nth()) {  // (wave-uniform) at most one candidate per lane, in registers
    const bool has = B.tid() < n;
    why = sel_all_fast<true>(B, x, RegCands{has, has ? (uint32_t)cd.r[B.tid()] : 0u, has ? cd.v[B.tid()] : 0}, ss, &ti);
  } else {
    why = sel_all_fast<true>(B, x, TopCands{&cd, B.tid(), B.nth()}, ss, &ti);
  }
  KP_STAMP(x, 12);
  if (why == SLOW_TOP_FULL) top_fallback(B, a, t, b);
  else if (why != SLOW_NONE && B.tid() == 0) flag_slow(a, b, why);
}

// k_select_top_wg: one workgroup of kTopWgWaves waves per binding for the bindings that
// need a large subset (the second launch): wave 0 runs the walk exactly as the one-wave
// kernel does, then the whole workgroup runs the division over the subset, whose passes
// (Webster over hundreds of parties) dominate such a binding. LDS: [GpuBlk red |
// TopHand 64 B | the one-wave slice].
KP_HD inline size_t top_wg_lds_bytes(int Cp, int cap) { return kRedBytes + 64 + top_lds_bytes(Cp, cap); }
// W: wave 0's block policy over the slice (its red area = the slice's first 64 B).
KP_HD inline unsigned char* top_wg_slice(unsigned char* smem) { return smem + kRedBytes + 64; }
template <class GBLK, class WBLK>
KP_FI void body_select_top_wg(const GBLK& G, const WBLK& W, int blk, unsigned char* smem, const KArgs& a,
                              const TopArgs& t) {
  if (blk >= a.n) return;  // (block-uniform)
  TopHand* hand = (TopHand*)(smem + kRedBytes);
  unsigned char* slice = top_wg_slice(smem);
  if (G.tid() == 0) hand->go = 0;
  if (G.wid() == 0) body_select_top(W, blk, slice, a, t, hand);
  G.sync();
  const TopHand hh = *hand;
  if (!hh.go) return;  // wave 0 wrote the result or handed the binding on
  const int b = a.list[blk];
  TopCarve tc = top_carve(slice, a.s, t.cap, a.dbg);
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  SelCtx x = make_ctx(a, b, (const uint32_t*)tc.frow);  // (wave 0 left the target bits there)
  x.h = &hloc;
  x.frow = tc.frow;
  tc.cd.F = hh.n;
  const TopInfo ti{hh.F, hh.complete != 0};
  const int why = sel_all_fast<true>(G, x, TopCands{&tc.cd, G.tid(), G.nth()}, tc.ss, &ti);
  if (why == SLOW_TOP_FULL) top_fallback(G, a, t, b);
  else if (why != SLOW_NONE && G.tid() == 0) flag_slow(a, b, why);
}

}  // namespace kp
