// kp_kernels.h — bodies of the engine's kernels, written once against a block
// policy (kp_blk.h). kernels.hip instantiates them with GpuBlk as gfx950
// kernels (one 256-thread workgroup per binding); the test-only CPU build
// (dev_cpu.cpp -> libkp_cpusim.so) instantiates them with CpuBlk to check the
// same code paths on the host.
//
// Per-block LDS layouts (dynamic shared memory; sizes computed in engine.cpp):
//   pair      [512 red | tgt bits | evict bits | md table | predicate stage kPairStage | taint-set bits]
//   sel_all   [512 red | tgt bits | cand r [Cp] | cand v [Cp] | whist 2 KB | hist 1 KB | buf ecap*8]
//   sel_all_reg [512 red | tgt bits | whist 2 KB | hist 1 KB | buf ecap*8]  (candidates in registers)
//   sel_clus  [512 red | hist 1 KB | items 2*kSmallMax | keys 2*kSmallMax | tgt | cand/serial area]
//   region_a  [512 red | 8x8R + 4x4R region accumulators | tgt | cand]
//   region_b  [512 red | hist | items | keys | heads 8R | rsel 4R | tgt | cand/serial area]
//   slow      [512 red | tgt]   (candidates/keys/serial scratch in a global slot)
#pragma once
#include "kp_launch.h"
#include "kp_paths.h"
#include "kp_pdq.h"
#include "kp_filter.h"
#include "kp_nodes.h"

namespace kp {

KP_HD inline SelCtx make_ctx(const KArgs& a, int b, const uint32_t* tgt_bits) {
  SelCtx x;
  x.s = &a.s;
  x.bv = &a.bv;
  x.h = &a.bv.hdr[b];
  x.b = b;
  x.frow = a.fmask + (size_t)b * a.s.W;
  if (a.bcls) {
    const int32_t k = a.bcls[b];
    x.erow = a.est + (size_t)k * a.s.Cp;
    x.mrep = k ? x.h->replicas : kInt32Max;
    x.merge = true;
  } else {
    x.erow = a.est + (size_t)b * a.s.Cp;
    x.mrep = kInt32Max;
    x.merge = false;
  }
  x.tgt_bits = tgt_bits;
  x.sink = a.sink;
  x.dbg = a.dbg;
  return x;
}

// Bitset (LDS) of the binding's spec.Clusters ranks (TargetContains, locality).
// Empty lists leave the bitset untouched (no barrier): every reader tests the
// list's count first (tgt_cnt / evict_cnt > 0).
template <class BLK>
KP_FI void build_bits(const BLK& B, uint32_t* bits, int words, const int32_t* pool, int off, int cnt, int stride) {
  if (cnt == 0) return;  // block-uniform
  for (int i = B.tid(); i < words; i += B.nth()) bits[i] = 0;
  B.sync();
  for (int j = B.tid(); j < cnt; j += B.nth()) {
    int r = pool[off + stride * j];
    kp_atomic_or(&bits[r >> 5], 1u << (r & 31));
  }
  B.sync();
}

// p - bias as a flat (64-bit) address. Biasing the LDS pointer itself would be
// done in the 32-bit local address space, where a bias larger than the offset
// wraps; the wrapped offset, cast to flat and indexed again, then lands past
// the LDS aperture (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION). The integer
// round trip keeps the arithmetic in 64 bits.
template <class T>
KP_FI const T* rebase(const T* p, int64_t bias) {
  return (const T*)((uintptr_t)p - (uintptr_t)bias * sizeof(T));
}

// Region index of every gathered candidate into cd.g (one global load each, in
// parallel; the region kernels' passes then read LDS only).
template <class BLK>
KP_FI void region_of_cands(const BLK& B, const SnapView& s, const Cands& cd) {
  for (int i = B.tid(); i < cd.F; i += B.nth()) cd.g[i] = (int16_t)s.region_idx[c_rank(cd, i)];
  B.sync();
}

// Status of bindings that never reach selection.
template <class BLK>
KP_FI bool pre_checks(const BLK& B, const SelCtx& x, int F) {
  if (x.h->flags & BF_BAD) {
    const bool lim = (x.h->flags & BF_LIMIT_OVF) != 0;  // the engine's overflow-term limit
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, lim ? KP_ERR_OVERFLOW_TERMS : KP_ERR_NONE, lim ? x.h->ovf_cnt : 0);
    return true;
  }
  if (F == 0) {  // FitError (generic_scheduler.go:84-89)
    if (B.tid() == 0) sink_error(x, KP_STATUS_FIT_ERROR, KP_ERR_FIT, x.s->C);
    return true;
  }
  return false;
}

// ---------------------------------------------------------------------------
// Pair stage: each wave evaluates 64 consecutive clusters (coalesced SoA
// columns), stores their feasibility as one u64 word and calAvailableReplicas
// per cluster. est_mode 1: raw GeneralEstimator answers for every cluster.
// ---------------------------------------------------------------------------
// Per-binding LDS state of the pair stage: spec.Clusters and eviction bitsets,
// the per-template MaxDivided table, the binding's predicate data (programs,
// value lists, tolerations) and the per-taint-list TaintToleration answers.
struct PairLds {
  uint32_t* tgt;    // [words] TargetContains bits (also read by the select stage)
  uint32_t* evict;  // [words]
  int32_t* md;      // [md_cap]
  unsigned char* stage;  // kPairStage bytes
  uint32_t* tolb;   // kTsetMax bits
};
KP_HD inline PairLds pair_lds_carve(uint32_t* tgt, unsigned char* tail, int Cp, int md_cap) {
  const int words = (Cp + 31) >> 5;
  PairLds L;
  L.tgt = tgt;
  L.evict = (uint32_t*)tail;
  L.md = (int32_t*)(L.evict + ((words + 3) & ~3));
  L.stage = (unsigned char*)(L.md + ((md_cap + 3) & ~3));
  L.tolb = (uint32_t*)(L.stage + kPairStage);
  return L;
}

// Fills the pair stage's LDS state for binding h; returns the view of the batch
// whose predicate pools point into LDS when they fit the stage and `stage` is
// set (absolute pool indices keep working; the fast kernels read the programs
// with scalar loads from HBM instead). *use_md / *use_ts: whether the
// MaxDivided table and the taint-list answers were built.
template <class BLK>
KP_FI BatchView pair_setup(const BLK& B, const SnapView& s, const BatchView& bv, const BindHdr& h, const PairLds& L,
                           int est_mode, int md_cap, bool* use_md, bool* use_ts, bool stage = true) {
  const int words = (s.Cp + 31) >> 5;
  build_bits(B, L.tgt, words, bv.ipool, h.tgt_off, h.tgt_cnt, 2);
  build_bits(B, L.evict, words, bv.ipool, h.evict_off, h.evict_cnt, 1);
  *use_md = s.n_tmpl <= md_cap && (h.flags & BF_HAS_RR);
  if (*use_md) {
    for (int t = B.tid(); t < s.n_tmpl; t += B.nth()) L.md[t] = template_md(s, bv, h, t);
    for (int t = s.n_tmpl + B.tid(); t < kTmplDense; t += B.nth()) L.md[t] = 0;  // padded template rows
    B.sync();
  }
  // Stage this binding's predicate data (programs, value lists, tolerations) in
  // LDS: every lane reads it for every cluster, uniformly.
  BatchView lv = bv;
  {
    const int nin = h.in_end - h.in_beg, npr = h.pr_end - h.pr_beg, nip = h.ip_end - h.ip_beg, nto = h.tol_cnt;
    const size_t need = sizeof(Instr) * nin + sizeof(Prog) * npr + sizeof(Tol) * nto + 4 * (size_t)nip;
    if (stage && need <= (size_t)kPairStage) {
      Instr* si = (Instr*)L.stage;
      Prog* sp = (Prog*)(si + nin);
      Tol* so = (Tol*)(sp + npr);
      int32_t* sv = (int32_t*)(so + nto);
      for (int i = B.tid(); i < nin; i += B.nth()) si[i] = bv.instrs[h.in_beg + i];
      for (int i = B.tid(); i < npr; i += B.nth()) sp[i] = bv.progs[h.pr_beg + i];
      for (int i = B.tid(); i < nto; i += B.nth()) so[i] = bv.tols[h.tol_off + i];
      for (int i = B.tid(); i < nip; i += B.nth()) sv[i] = bv.ipool[h.ip_beg + i];
      B.sync();
      lv.instrs = rebase(si, h.in_beg);
      lv.progs = rebase(sp, h.pr_beg);
      lv.tols = rebase(so, h.tol_off);
      lv.ipool = rebase(sv, h.ip_beg);
    }
  }
  // TaintToleration once per distinct taint list of the snapshot, not per cluster
  *use_ts = est_mode == 0 && (h.enabled & 2) && s.n_tsets <= kTsetMax;
  if (*use_ts) {
    const int tw = (s.n_tsets + 31) >> 5;
    for (int i = B.tid(); i < tw; i += B.nth()) L.tolb[i] = 0;
    B.sync();
    for (int t = B.tid(); t < s.n_tsets; t += B.nth())
      if (taints_tolerated(s, lv, h, s.tset_rep[t])) kp_atomic_or(&L.tolb[t >> 5], 1u << (t & 31));
    B.sync();
  }
  return lv;
}

// The per-template MaxDivided table of the fast kernels in scalar registers
// (kTmplDense entries, zero past n_tmpl): built in LDS by pair_setup, one
// template per thread, then read once per binding.
struct MdTab {
  int32_t v[kTmplDense];
};
KP_FI MdTab md_regs(const int32_t* md) {
  MdTab t;
KP_UNROLL
  for (int i = 0; i < kTmplDense; i++) t.v[i] = kp_uniform(md[i]);
  return t;
}

// The fast instances' loop over the binding's clusters: kPairUnroll clusters
// per lane per step (c = base + u*nth + tid), fn(c, fit, value) for each c < Cp.
// Validity of a slot is wave-uniform (Cp and wave bases are multiples of 64).
#ifndef KP_PAIR_UNROLL
#define KP_PAIR_UNROLL 2
#endif
constexpr int kPairUnroll = KP_PAIR_UNROLL;
template <int Fast, class BLK, class Fn>
KP_FI void pair_loop_fast(const BLK& B, const SnapView& s, const BatchView& bv, const BindHdr& h, const PairLds& L,
                          const MdTab& mdt, Fn fn) {
  for (int base = 0; base < s.Cp; base += kPairUnroll * B.nth()) {
    int c[kPairUnroll];
    bool ok[kPairUnroll];
    int32_t v[kPairUnroll];
KP_UNROLL
    for (int u = 0; u < kPairUnroll; u++) {
      const int cu = base + u * B.nth() + B.tid();
      c[u] = cu < s.Cp ? cu : 0;  // (an out-of-range slot evaluates cluster 0 and is dropped)
    }
    pair_eval_fast<Fast, kPairUnroll>(s, bv, h, c, L.tgt, L.evict, L.tolb, mdt.v, ok, v);
KP_UNROLL
    for (int u = 0; u < kPairUnroll; u++)
      if (base + u * B.nth() + B.tid() < s.Cp) fn(base + u * B.nth() + B.tid(), ok[u], v[u]);
  }
}

// Fast: the estimator instance (EST_*, kp_algo.h); every instance but
// EST_GENERIC needs pair_fast_ok (engine.cpp): est_mode 0, the MaxDivided and
// taint-set tables in LDS, no cold fallbacks.
template <int Fast, class BLK>
KP_FI void pair_one(const BLK& B, int b, unsigned char* smem, const SnapView& s, const BatchView& bv, uint64_t* fmask,
                    int32_t* est, int64_t* score, int est_mode, int md_cap) {
  const BindHdr h = bv.hdr[b];
  const int words = (s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + kRedBytes);
  const PairLds L = pair_lds_carve(tgt, (unsigned char*)(tgt + ((words + 3) & ~3)), s.Cp, md_cap);
  bool use_md, use_ts;
  const BatchView lv = pair_setup(B, s, bv, h, L, est_mode, md_cap, &use_md, &use_ts, Fast == EST_GENERIC);
  MdTab mdt;
  if (Fast != EST_GENERIC) mdt = md_regs(L.md);
  uint64_t* frow = fmask + (size_t)b * s.W;
  int32_t* erow = est + (size_t)b * s.Cp;
  if constexpr (Fast != EST_GENERIC) {  // kPairUnroll clusters per lane per step
    pair_loop_fast<Fast>(B, s, bv, h, L, mdt, [&](int c, bool ok, int32_t v) {
      B.mask_store(frow, c, ok, s.W);
      erow[c] = v;
    });
    return;
  }
  for (int base = 0; base < s.Cp; base += B.nth()) {
    const int c = base + B.tid();
    if (c >= s.Cp) break;  // wave-uniform: Cp and the wave bases are multiples of 64
    bool fit = false;
    int32_t e = 0;
    if (Fast != EST_GENERIC) {
      e = pair_eval<Fast>(s, bv, h, c, tgt, L.evict, L.tolb, mdt.v, &fit);
    } else if (est_mode == 0) {
      e = pair_eval(s, lv, h, c, tgt, L.evict, use_ts ? L.tolb : nullptr, use_md ? L.md : nullptr, &fit);
    } else if (c < s.C) {
      e = general_estimate(s, lv, h, c, use_md ? L.md : nullptr);
      fit = true;
    }
    B.mask_store(frow, c, fit, s.W);
    erow[c] = e;
    if (score && c < s.C) {
      int64_t sc = 0;
      if ((h.enabled & KP_PLUGIN_CLUSTER_LOCALITY) && h.n_targets_all > 0 && h.tgt_cnt > 0 && bit_test(tgt, c)) sc = 100;
      score[(size_t)b * s.C + c] = sc;
    }
  }
}

// k_est_class: row k of the estimator classes' raw GeneralEstimator answers
// (est_compute_bf, the pair kernel's arithmetic) for every cluster, from the
// class's representative binding rep[k]; row 0 (non-workload bindings, whose
// calAvailableReplicas is MaxInt32, core/util.go:69-73) is MaxInt32.
// fmask set (a class serving one binding, in a batch without class orders): only the
// entries of that binding's feasible clusters, the only ones any select kernel reads
// (they gather feasible candidates; at config 10 the full rows were 2 GB of writes).
template <int Fast, class BLK>
KP_FI void body_est_class(const BLK& B, int k, unsigned char* smem, const SnapView& s, const BatchView& bv,
                          const int32_t* rep, int32_t* rows, const uint64_t* fmask = nullptr) {
  int32_t* row = rows + (size_t)k * s.Cp;
  if (k == 0) {
    for (int c = B.tid(); c < s.Cp; c += B.nth()) row[c] = kInt32Max;
    return;
  }
  if (rep[k] < 0) return;  // a component-set class (k_sets_rows writes it)
  const BindHdr h = bv.hdr[rep[k]];
  int32_t* md = (int32_t*)(smem + kRedBytes);  // MaxDivided per template, zero past n_tmpl
  const bool rr = (h.flags & BF_HAS_RR) != 0;
  for (int t = B.tid(); t < kTmplDense; t += B.nth()) md[t] = rr && t < s.n_tmpl ? template_md(s, bv, h, t) : 0;
  B.sync();
  const MdTab mdt = md_regs(md);
  if (fmask) {
    // the feasible clusters compacted into LDS first (one word per thread per pass, a
    // scan of the popcounts), so the lanes compute dense instead of idling on the
    // infeasible ~2/3 of a row
    const uint64_t* fr = fmask + (size_t)rep[k] * s.W;
    int32_t* list = md + kTmplDense;
    int F = 0;
    for (int w0 = 0; w0 < s.W; w0 += B.nth()) {
      const int w = w0 + B.tid();
      const uint64_t m = w < s.W ? fr[w] : 0ull;
      int32_t tot;
      int32_t pos = F + B.excl_scan(popc64(m), &tot);
      for (uint64_t q = m; q; q &= q - 1) list[pos++] = 64 * w + __builtin_ctzll(q);
      F += tot;
    }
    B.sync();
    for (int i = B.tid(); i < F; i += B.nth()) {
      const int c = list[i];
      row[c] = est_compute_bf<Fast>(s, bv, h, c, mdt.v, est_load<Fast>(s, bv, h, c, ldcol(s.flags, c), mdt.v));
    }
    return;
  }
  for (int c = B.tid(); c < s.Cp; c += B.nth())
    row[c] = est_compute_bf<Fast>(s, bv, h, c, mdt.v, est_load<Fast>(s, bv, h, c, ldcol(s.flags, c), mdt.v));
}

// Pair-row mode, BF_SETS binding list[blk]: its calAvailableReplicas row from its
// component-set class row (core/util.go:57-110 over MaxAvailableComponentSets), as
// pair_eval writes it: cal_merge_bf on feasible clusters, 0 elsewhere.
template <class BLK>
KP_FI void body_rows_from_class(const BLK& B, int blk, const SnapView& s, const BatchView& bv, const int32_t* list,
                                const int32_t* bcls, const int32_t* cls_rows, const uint64_t* fmask, int32_t* est) {
  const int b = list[blk];
  const int32_t rep = bv.hdr[b].replicas;
  const int32_t* cr = cls_rows + (size_t)bcls[b] * s.Cp;
  const uint64_t* fr = fmask + (size_t)b * s.W;
  int32_t* row = est + (size_t)b * s.Cp;
  for (int c = B.tid(); c < s.C; c += B.nth()) row[c] = mask_test(fr, c) ? cal_merge_bf(rep, cr[c]) : 0;
}

// Pair stage for binding list[b0 + blk] (b0 + blk without a list): each wave evaluates 64 consecutive clusters
// (coalesced SoA columns), stores their feasibility as one u64 word and
// calAvailableReplicas per cluster. est_mode 1: raw GeneralEstimator answers for
// every cluster.
template <int Fast, class BLK>
KP_FI void body_pair(const BLK& B, int blk, unsigned char* smem, const SnapView& s, const BatchView& bv,
                     const int32_t* list, int b0, uint64_t* fmask, int32_t* est, int64_t* score, int est_mode,
                     int md_cap) {
  pair_one<Fast>(B, list ? list[b0 + blk] : b0 + blk, smem, s, bv, fmask, est, score, est_mode, md_cap);
}

// ---------------------------------------------------------------------------
// Select stage: SEL_ALL (and spread-unsupported / FitError reporting)
// ---------------------------------------------------------------------------
// Hands binding b to k_slow for reason `why` (one thread).
KP_HD inline void flag_slow(const KArgs& a, int b, int why) {
  a.slow[b] = why;
  a.sink.count[b] = 0;
  const uint32_t i = kp_atomic_add(&a.stats[0], 1u);
  a.slow_ids[i] = b;
  kp_atomic_add(&a.stats[why], 1u);
}

template <class BLK, class CS>
KP_FI void select_all_common(const BLK& B, const KArgs& a, const SelCtx& x, const CS& cs, int F,
                             const SelScratch& ss) {
  const int b = x.b;
  if (pre_checks(B, x, F)) return;
  if (x.h->sel == SEL_ERR_UNSUPPORTED) {  // select_clusters.go:54
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_SPREAD_UNSUPPORTED, 0);
    return;
  }
  const int why = sel_all_fast(B, x, cs, ss);
  if (why != SLOW_NONE && B.tid() == 0) flag_slow(a, b, why);
}


// Candidates compacted in LDS (any block policy; the only form for CpuBlk).
template <class BLK>
KP_FI void body_select_all(const BLK& B, int blk, unsigned char* smem, const KArgs& a) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + kRedBytes);
  Cands cd;
  cd.r = tgt + ((words + 3) & ~3);
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  SelScratch ss = carve_sel_scratch((unsigned char*)(cd.v + a.s.Cp), a.s.Cp);
  ss.dbg = a.dbg;
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  const BindHdr* h = &hloc;
  SelCtx x = make_ctx(a, b, tgt);
  x.h = h;
  KP_STAMP(x, 0);
  const bool weights = h->strategy == ST_STATIC && h->sel == SEL_ALL;
  if (h->sel == SEL_ERR_UNSUPPORTED || (h->flags & BF_BAD)) {  // errors: only F (FitError first) is needed
    int64_t F = 0;
    for (int w = B.tid(); w < a.s.W; w += B.nth()) F += popc64(x.frow[w]);
    cd.F = (int)B.sum64(F);
    select_all_common(B, a, x, LdsCands{&cd, B.tid(), B.nth()}, cd.F, ss);
    return;
  }
  cd.F = gather(B, x, cd, weights, [&] { build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2); });
  KP_STAMP(x, 1);
  LdsCands cs{&cd, B.tid(), B.nth()};
  select_all_common(B, a, x, cs, cd.F, ss);
}

// ---------------------------------------------------------------------------
// SEL_ALL over streamed candidates (k_select_all_stream, the bits-mode path): no
// per-binding candidate arrays in LDS. Every pass walks the binding's feasibility
// row (fmask, k_filter) and reads each candidate's calAvailableReplicas from its
// estimator-class row (est_at; the class rows are shared by every binding of the
// class and stay in L2), or its StaticWeight vote from per-rule cluster bitsets
// built once in LDS (prog_word, kp_filter.h). The LDS left is the TargetContains
// bits and the selection scratch, so several times more workgroups share a CU.
// LDS: [red | tgt bits | rule bits kSwRules x W | SelScratch]
// ---------------------------------------------------------------------------
struct StreamCands {
  const SelCtx* x;
  int C, tid, nth;
  bool weights;
  const uint64_t* swb;  // weights && swb: [nsw][W] rule bitsets
  int nsw;
  KP_FI int32_t vote(int c) const {
    if (!weights) return est_at(*x, c);
    if (!swb) return static_vote(*x, c);
    const BindHdr& h = *x->h;
    if (!(h.flags & BF_HAS_WP)) return 1;
    int64_t wt = 0;
    for (int j = 0; j < nsw; j++)
      if ((swb[(size_t)j * x->s->W + (c >> 6)] >> (c & 63)) & 1ull) {
        const int64_t rw = kp_ldu(x->bv->lpool + h.sw_w_off + j);
        wt = rw > wt ? rw : wt;
      }
    return (int32_t)(wt > kInt32Max ? kInt32Max : wt);
  }
  template <class Fn>
  KP_FI void each(Fn fn) const {
    for (int c = tid; c < C; c += nth) {
      const uint64_t m = x->frow[c >> 6];  // wave-uniform word
      if ((m >> (c & 63)) & 1ull) fn((uint32_t)c, vote(c));
    }
  }
  static constexpr bool kSettable = false;
  KP_FI uint64_t okey(const SelCtx& xx, uint32_t rk, int32_t v0) const { return cand_order_key(xx, rk, v0); }
  static constexpr bool kExact = false;
};
// StaticWeight SEL_ALL at class level (k_select_static, one wave per binding):
// assignByStaticWeightStrategy (assignment.go:193-211) over getStaticWeightInfoList
// (division_algorithm.go:38-72) and AllocateWebsterSeats (webstermethod.go:112-161).
// A candidate's vote is the largest weight among the rules whose cluster bitset
// holds it, so the candidates fall into at most kSwRules + 1 vote classes (rules
// of equal weight form one), counted from the feasibility row by word popcounts.
// Parties of one class receive the same seats except at the tie priority t*, where
// the heap orders the tied parties by (seats asc, name): t* (the N-th largest
// priority, counted with class multiplicities) is found by a W-ary search over the
// double's bit pattern inside the divisor-method bracket, each class's seats above
// t* follow from w_count, the tied classes (distinct seat counts: two integer
// votes below 2^31 over one divisor never round to the same double) take their
// extra seat in seat order, and in the one class split by the remaining seats the
// first k members by name (the last k for a descending UID tie-breaker) take it.
// The host routes here only bindings this covers (select_static_ok); the rest keep
// the streamed kernel.
struct SwClass {
  int64_t v[kSwRules + 1];    // vote of class j (0: not a party)
  int64_t n[kSwRules + 1];    // members
  int64_t sgt[kSwRules + 1];  // seats above t*
  int32_t order[kSwRules];    // rules by weight desc
  int32_t lend[kSwRules];     // class j = rules order[lend[j-1] .. lend[j]) (equal weights: one class)
  int32_t bonus[kSwRules + 1];  // 1: every member takes a tie seat
  int32_t split, k, nc, nl;   // class split by the tie seats, members of it that take one; classes; rule classes
  int32_t ok, pad;
  uint64_t tbits;             // t*
};
// Per-binding LDS of k_select_static: [red 64 | SwClass | rule bits kSwRules x W |
// emitted W u64 | split members W u64 | split offsets W u32 | emit offsets W u32]
KP_HD inline size_t static_lds_bytes(int W) {
  return 64 + ((sizeof(SwClass) + 15) & ~(size_t)15) + 8 * (size_t)kSwRules * W + 16 * (size_t)W + 8 * (size_t)W;
}
template <class BLK>
KP_FI void body_select_static(const BLK& B, int blk, unsigned char* smem, const KArgs& a) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const SnapView& s = a.s;
  const int W = s.W;
  SwClass* sh = (SwClass*)(smem + 64);
  uint64_t* swb = (uint64_t*)(smem + 64 + ((sizeof(SwClass) + 15) & ~(size_t)15));
  uint64_t* em = swb + (size_t)kSwRules * W;
  uint64_t* cms = em + W;
  uint32_t* spo = (uint32_t*)(cms + W);
  uint32_t* eo = spo + W;
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  const BindHdr& h = hloc;
  SelCtx x = make_ctx(a, b, nullptr);
  x.h = &hloc;
  const bool wp = (h.flags & BF_HAS_WP) != 0;
  const int nr = wp ? h.sw_cnt : 0;
  // per-thread contiguous word runs (word order = rank order = name order)
  const int per = (W + B.nth() - 1) / B.nth();
  const int w0 = B.tid() * per < W ? B.tid() * per : W, w1 = w0 + per < W ? w0 + per : W;
  int64_t F = 0;
  for (int w = w0; w < w1; w++) F += popc64(x.frow[w]);
  for (int i = B.tid(); i < nr * W; i += B.nth())  // getStaticWeightInfoList's ClusterMatches per rule
    swb[i] = prog_word(s, a.bv, kp_ldu(a.bv.ipool + h.sw_off + i / W), i % W);
  if (B.tid() == 0) {
    // rules by weight desc: a candidate's vote is its first matching rule's
    // weight; rules of equal weight form one class
    int64_t wt[kSwRules];
    for (int j = 0; j < nr; j++) {
      wt[j] = kp_ldu(x.bv->lpool + h.sw_w_off + j);
      int m = j;
      while (m > 0 && wt[sh->order[m - 1]] < wt[j]) {
        sh->order[m] = sh->order[m - 1];
        m--;
      }
      sh->order[m] = j;
    }
    int nl = 0;
    for (int j = 0; j < nr; j++) {
      if (j > 0 && wt[sh->order[j]] == wt[sh->order[j - 1]]) {
        sh->lend[nl - 1] = j + 1;
        continue;
      }
      sh->v[nl] = wt[sh->order[j]];
      sh->lend[nl] = j + 1;
      nl++;
    }
    sh->nl = nl;
    sh->v[nl] = 0;
  }
  F = B.sum64(F);  // (its barrier also publishes swb and the rule order)
  if (pre_checks(B, x, (int)F)) return;
  const int nl = sh->nl;
  // members of rule class j in word w (j == nl: matching no rule)
  auto rule_mask = [&](int w, int j) {
    uint64_t rest = x.frow[w];
    int q = 0;
    for (int l = 0; l < nl; l++) {
      uint64_t u = 0;
      for (; q < sh->lend[l]; q++) u |= swb[(size_t)sh->order[q] * W + w];
      const uint64_t m = rest & u;
      if (l == j) return m;
      rest &= ~m;
    }
    return rest;
  };
  // class counts: 16-bit fields packed four to an int64 (C < 2^16), one reduction
  int64_t c03 = 0, c4 = 0;
  for (int w = w0; w < w1; w++) {
    uint64_t rest = x.frow[w];
    int q = 0;
    for (int l = 0; l < nl; l++) {
      uint64_t u = 0;
      for (; q < sh->lend[l]; q++) u |= swb[(size_t)sh->order[q] * W + w];
      const uint64_t m = rest & u;
      if (l < 4) c03 += (int64_t)popc64(m) << (16 * l);
      else c4 += popc64(m);
      rest &= ~m;
    }
    if (nl < 4) c03 += (int64_t)popc64(rest) << (16 * nl);
    else c4 += popc64(rest);
  }
  B.sum2(c03, c4);
  KP_STAMP(x, 2);
  if (B.tid() == 0) {
    SwClass& c = *sh;
    int64_t cnt[kSwRules + 1];
    for (int j = 0; j <= nl; j++) cnt[j] = j < 4 ? (c03 >> (16 * j)) & 0xffff : c4;
    int64_t wsum = 0;
    for (int j = 0; j < nl; j++) {
      c.n[j] = cnt[j];
      if (c.v[j] > 0 && c.n[j] > 0) wsum += c.v[j];
    }
    c.n[nl] = cnt[nl];
    if (!wp || wsum == 0) {  // every candidate weight 1 (getStaticWeightInfoList): one class
      c.nc = 1;
      c.v[0] = 1;
      c.n[0] = F;
    } else {
      c.nc = nl + 1;
    }
    for (int j = 0; j < c.nc; j++) {
      c.sgt[j] = 0;
      c.bonus[j] = 0;
    }
    c.split = -1;
    c.k = 0;
  }
  B.sync();
  const int32_t N = h.replicas;
  const int nc = sh->nc;
  const bool one = nc == 1;
  auto cls_mask = [&](int w, int j) { return one ? x.frow[w] : rule_mask(w, j); };
  if (N > 0) {
    // t* = the largest double t with #{priorities >= t} >= N, searched over the bit
    // patterns of positive doubles (they order as the values) inside the bracket
    // V/(2N+P) <= t* < V/(2N-P-1) (V: the votes' sum, P: the parties)
    auto cnt_ge = [&](double t) {
      int64_t tot = 0;
      for (int j = 0; j < nc; j++)
        if (sh->v[j] > 0 && sh->n[j] > 0) tot += sh->n[j] * w_count(sh->v[j], t, (int64_t)N + 1, true);
      return tot;
    };
    int64_t vmax = 0, V = 0, P = 0;
    for (int j = 0; j < nc; j++)
      if (sh->n[j] > 0 && sh->v[j] > 0) {
        vmax = sh->v[j] > vmax ? sh->v[j] : vmax;
        V += sh->v[j] * sh->n[j];
        P += sh->n[j];
      }
    uint64_t lo = kp_dbits((double)V / (double)(2 * (int64_t)N + P));
    lo = lo > 8 ? lo - 8 : 1;
    uint64_t hi = kp_dbits((double)vmax);
    if (2 * (int64_t)N - P - 1 > 0) {
      const uint64_t u = kp_dbits((double)V / (double)(2 * (int64_t)N - P - 1)) + 8;
      hi = u < hi ? u : hi;
    }
    if (hi < lo || !(cnt_ge(kp_bitsd(lo)) >= N)) {  // (rounding at the bracket's ends)
      lo = 1;
      hi = kp_dbits((double)vmax);
    }
    const int ww = B.wwidth();
    while (lo < hi) {
      const uint64_t step = (hi - lo) / (uint64_t)(ww + 1) + 1;
      const uint64_t probe = lo + step * (uint64_t)(B.lane() + 1);
      const bool good = probe <= hi && cnt_ge(kp_bitsd(probe)) >= N;
      const uint64_t bal = B.wballot(good);  // good probes form a prefix (cnt_ge is non-increasing)
      const int ng = bal ? 64 - __builtin_clzll(bal) : 0;
      const uint64_t nhi = lo + step * (uint64_t)(ng + 1) - 1;
      lo = lo + step * (uint64_t)ng;
      hi = nhi < hi ? nhi : hi;
    }
    if (B.tid() == 0) {
      const double t = kp_bitsd(lo);
      int64_t G = N;
      for (int j = 0; j < nc; j++) {
        if (sh->v[j] <= 0 || sh->n[j] <= 0) continue;
        sh->sgt[j] = w_count(sh->v[j], t, (int64_t)N + 1, false);
        G -= sh->n[j] * sh->sgt[j];
      }
      for (;;) {  // tied classes in seat order take the remaining G seats
        int best = -1;
        for (int j = 0; j < nc; j++) {
          if (sh->v[j] <= 0 || sh->n[j] <= 0 || sh->bonus[j] || j == sh->split) continue;
          if (w_prio(sh->v[j], sh->sgt[j]) != t) continue;
          if (best < 0 || sh->sgt[j] < sh->sgt[best]) best = j;
        }
        if (best < 0 || G <= 0) break;
        if (G >= sh->n[best]) {
          sh->bonus[best] = 1;
          G -= sh->n[best];
        } else {
          sh->split = best;
          sh->k = (int32_t)G;
          G = 0;
        }
      }
    }
    B.sync();
  }
  KP_STAMP(x, 3);
  // emit (removeZeroReplicasCluster unless EnableEmptyWorkloadPropagation), in rank
  // order: per-word emitted masks and offsets, then one thread per cluster
  const bool prop = (h.flags & BF_EMPTY_PROP) != 0;
  const bool desc = (h.flags & BF_UID_DESC) != 0;
  const int split = sh->split;
  auto seats = [&](int j) { return sh->v[j] > 0 ? (int32_t)(sh->sgt[j] + sh->bonus[j]) : (int32_t)0; };
  int32_t msplit = 0;
  for (int w = w0; w < w1; w++) {
    uint64_t e = 0, sp = 0;
    for (int j = 0; j < nc; j++) {
      const uint64_t m = cls_mask(w, j);
      if (j == split) sp = m;
      if (prop || seats(j) > 0) e |= m;
    }
    em[w] = e;
    cms[w] = sp;
    msplit += popc64(sp);
  }
  int32_t tsplit;
  int32_t run = B.excl_scan(msplit, &tsplit);
  // the split class's members with a tie seat: names [0, k) ascending, the last k descending
  const int64_t lo_i = desc ? (int64_t)tsplit - sh->k : 0, hi_i = desc ? (int64_t)tsplit : (int64_t)sh->k;
  int32_t mine = 0;
  for (int w = w0; w < w1; w++) {
    spo[w] = (uint32_t)run;
    uint64_t sp = cms[w];
    const int c = popc64(sp);
    if (split >= 0 && c > 0) {
      if (run >= lo_i && run + c <= hi_i) {
        em[w] |= sp;
      } else if (run < hi_i && run + c > lo_i) {
        int64_t idx = run;
        while (sp) {
          const uint64_t bit = sp & (~sp + 1);
          if (idx >= lo_i && idx < hi_i) em[w] |= bit;
          sp ^= bit;
          idx++;
        }
      }
    }
    run += c;
    mine += popc64(em[w]);
  }
  int32_t tot;
  int32_t off = B.excl_scan(mine, &tot);
  for (int w = w0; w < w1; w++) {
    eo[w] = (uint32_t)off;
    off += popc64(em[w]);
  }
  const uint64_t base = h.out_off;
  if (B.tid() == 0) {
    x.sink.status[x.b] = KP_STATUS_OK;
    x.sink.err[x.b] = KP_ERR_NONE;
    x.sink.arg[x.b] = 0;
    x.sink.start[x.b] = base;
    x.sink.count[x.b] = (uint32_t)tot;
  }
  B.sync();
  for (int c = B.tid(); c < s.C; c += B.nth()) {
    const int w = c >> 6;
    const uint64_t bit = 1ull << (c & 63), below = bit - 1;
    if (!(em[w] & bit)) continue;
    int j = 0;
    if (!one) {  // the first rule class (weight desc) whose bitset holds c
      int q = 0;
      for (; j < nl; j++) {
        bool in = false;
        for (; q < sh->lend[j]; q++) in = in || ((swb[(size_t)sh->order[q] * W + w] & bit) != 0);
        if (in) break;
      }
    }
    int32_t r = seats(j);
    if (j == split) {
      const int64_t idx = (int64_t)spo[w] + popc64(cms[w] & below);
      if (idx >= lo_i && idx < hi_i) r++;
    }
    const uint64_t o = base + eo[w] + (uint64_t)popc64(em[w] & below);
    x.sink.out_idx[o] = (uint32_t)c;  // (rank: k_compact maps it)
    x.sink.out_rep[o] = r;
  }
  KP_STAMP(x, 4);
}

template <class BLK>
KP_FI void body_select_all_stream(const BLK& B, int blk, unsigned char* smem, const KArgs& a) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const SnapView& s = a.s;
  const int words = (s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + kRedBytes);
  uint64_t* swb = (uint64_t*)(tgt + ((words + 3) & ~3));
  SelScratch ss = carve_sel_scratch((unsigned char*)(swb + (size_t)kSwRules * s.W), s.Cp);
  ss.dbg = a.dbg;
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  const bool weights = h->strategy == ST_STATIC && h->sel == SEL_ALL;
  const bool rules = weights && (h->flags & BF_HAS_WP) && h->sw_cnt <= kSwRules && s.n_bits > 0;
  if (rules) {  // getStaticWeightInfoList's ClusterMatches per rule, as cluster bitsets
    for (int i = B.tid(); i < h->sw_cnt * s.W; i += B.nth())
      swb[i] = prog_word(s, a.bv, kp_ldu(a.bv.ipool + h->sw_off + i / s.W), i % s.W);
  }
  int64_t F = 0;
  for (int w = B.tid(); w < s.W; w += B.nth()) F += popc64(x.frow[w]);
  F = B.sum64(F);  // (its barrier also publishes tgt and swb)
  KP_STAMP(x, 1);
  const StreamCands cs{&x, s.C, B.tid(), B.nth(), weights, rules ? swb : nullptr, rules ? h->sw_cnt : 0};
  select_all_common(B, a, x, cs, (int)F, ss);
}

// ---------------------------------------------------------------------------
// Select stage: SEL_CLUSTER
// ---------------------------------------------------------------------------
// Outcome of a class-order selection (cluster_order_select, region_order_select).
enum : int { ORD_NA = 0, ORD_DONE = 1, ORD_ITEMS = 2 };

// The class-order selections apply to a binding without overflow tiers (order 0)
// whose class row can be walked (k_class_order's ok: no MaxInt32, no negative
// estimate): a candidate outside spec.Clusters then has the sortClusters key
// (score 0, estimate desc, name asc), so those candidates are the class order
// filtered by the feasibility row. spec.Clusters (at most kOrdTargets distinct
// names, ClusterLocality on: `targets`) score 100, so the feasible ones sort ahead
// of all the others, among themselves by their keys (ord_targets). Returns the
// class, or -1.
constexpr int kOrdTargets = 16;
KP_HD inline bool ord_targets_ok(const BindHdr& h) {
  return h.tgt_cnt <= kOrdTargets && (h.flags & BF_SCORE_LOCALITY) && !(h.flags & BF_DUP_TARGETS);
}
KP_HD inline int32_t order_class(const KArgs& a, const SelCtx& x, bool targets = false) {
  const BindHdr& h = *x.h;
  if (!a.ord || !a.cok || !a.bcls) return -1;
  const int32_t cls = a.bcls[x.b];
  if (cls <= 0 || !a.cok[cls] || h.ovf_mode != OVF_ZERO || (h.flags & BF_BAD)) return -1;
  if (h.tgt_cnt != 0 && !(targets && ord_targets_ok(h))) return -1;
  return cls;
}
// The binding's feasible spec.Clusters entries as sortClusters keys (locality 100,
// AvailableReplicas = estimate + assigned), ascending, in tk[0, n); tmp: kOrdTargets
// entries of scratch. Returns n, or -1 when one has a negative AvailableReplicas (the
// callers' prefix arguments need every AvailableReplicas >= 0). Needs x.tgt_bits.
template <class BLK>
KP_FI int ord_targets(const BLK& B, const SelCtx& x, uint64_t* tk, uint64_t* tmp) {
  const BindHdr& h = *x.h;
  const int T = h.tgt_cnt;
  if (T == 0) return 0;  // block-uniform
  int64_t bad = 0;
  for (int j = B.tid(); j < T; j += B.nth()) {
    const uint32_t r = (uint32_t)x.bv->ipool[h.tgt_off + 2 * j];
    uint64_t k = ~0ull;
    if (mask_test(x.frow, (int)r)) {
      const int64_t av = (int64_t)est_at(x, (int)r) + (int64_t)x.bv->ipool[h.tgt_off + 2 * j + 1];
      if (av < 0) bad = 1;
      k = sort_key(0, 100, av, r);
    }
    tmp[j] = k;
  }
  if (B.sum64(bad) != 0) return -1;  // (its barrier also publishes tmp)
  int n = 0;
  for (int j = 0; j < T; j++) n += tmp[j] != ~0ull ? 1 : 0;
  for (int j = B.tid(); j < T; j += B.nth()) {
    const uint64_t k = tmp[j];
    if (k == ~0ull) continue;
    int p = 0;
    for (int q = 0; q < T; q++) p += tmp[q] < k ? 1 : 0;  // (distinct names: distinct keys)
    tk[p] = k;
  }
  B.sync();
  return n;
}
KP_HD inline Item order_item(uint64_t e) {
  Item it;
  it.rank = (uint32_t)e;
  it.alloc = (int32_t)(e >> 32);  // est_at: the class row holds no MaxInt32 (ok), so no merge
  it.avail = (int64_t)(int32_t)(e >> 32);
  it.ovf = 0;
  it.pad = 0;
  return it;
}

// selectBestClustersByCluster (select_clusters_by_cluster.go:25-102) over the
// binding's estimator-class order instead of a gather and a radix select: the
// first min(F, MaxGroups) feasible entries are the selection, and the swap step
// never fires (every rest cluster's AvailableReplicas is at most the last selected
// one's, and a swap needs a strictly larger one), so only the resource check
// remains. ORD_ITEMS: items[0, *n) in sortClusters order (at most max_items);
// ORD_DONE: the status is written; ORD_NA: nothing written.
// tk, tmp: kOrdTargets entries each (nullptr: bindings with spec.Clusters go ORD_NA);
// the feasible targets come first (ord_targets), then the filtered class order.
template <class BLK>
KP_FI int cluster_order_select(const BLK& B, const KArgs& a, const SelCtx& x, Item* items, int max_items, int* n_out,
                               uint64_t* tk = nullptr, uint64_t* tmp = nullptr) {
  const BindHdr& h = *x.h;
  const int32_t cls = order_class(a, x, tk != nullptr);
  if (cls < 0) return ORD_NA;
  KP_STAMP_INIT
  const SnapView& s = *x.s;
  int64_t F = 0;
  for (int w = B.tid(); w < s.W; w += B.nth()) F += popc64(x.frow[w]);
  F = B.sum64(F);
  KP_STAMP(x, 37);
  if (F == 0) {  // FitError (generic_scheduler.go:84-89)
    if (B.tid() == 0) sink_error(x, KP_STATUS_FIT_ERROR, KP_ERR_FIT, s.C);
    return ORD_DONE;
  }
  if (F < h.cluster_min) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_MIN_GROUPS, 0);
    return ORD_DONE;
  }
  int64_t needCnt = F < h.cluster_max ? F : h.cluster_max;
  if (needCnt < 0) needCnt = 0;
  const int32_t need = h.need_replicas;
  if (needCnt == 0) {
    if (B.tid() == 0) {
      if (need == -1) sink_error(x, KP_STATUS_ERROR, KP_ERR_NO_CLUSTERS, 0);
      else sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, 0);
    }
    return ORD_DONE;
  }
  if (needCnt > max_items) return ORD_NA;
  const int nt = h.tgt_cnt > 0 ? ord_targets(B, x, tk, tmp) : 0;
  if (nt < 0) return ORD_NA;
  const uint32_t* tb = h.tgt_cnt > 0 ? x.tgt_bits : nullptr;
  // the feasible targets first, then the class order (nth entries per step), keeping
  // the feasible non-targets in order
  const uint64_t* ord = a.ord + (size_t)cls * s.Cp;
  int n = nt < needCnt ? nt : (int)needCnt;
  int64_t tot = 0;
  for (int j = B.tid(); j < n; j += B.nth()) {
    items[j] = item_from_key(x, tk[j]);
    tot += key_avail(tk[j]);
  }
  for (int i0 = 0; i0 < s.C && n < needCnt; i0 += B.nth()) {
    const int i = i0 + B.tid();
    uint64_t e = 0;
    bool in = false;
    if (i < s.C) {
      e = ord[i];
      in = mask_test(x.frow, (int)(uint32_t)e) && !(tb && bit_test(tb, (int)(uint32_t)e));
    }
    int32_t cnt;
    const int32_t pos = n + B.excl_scan(in ? 1 : 0, &cnt);
    if (in && pos < needCnt) {
      items[pos] = order_item(e);
      tot += (int32_t)(e >> 32);
    }
    n += cnt;
  }
  B.sync();
  if (n > needCnt) n = (int)needCnt;
  tot = B.sum64(tot);
  KP_STAMP(x, 38);
  if (need != -1 && tot < (int64_t)need) {  // selectClustersByAvailableResource
    // a target in the list: a rest cluster may hold more than a selected target, so
    // the swap step may fire (the full kernel runs it); otherwise no swap can help
    if (nt > 0) return ORD_NA;
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, needCnt);
    return ORD_DONE;
  }
  *n_out = n;
  return ORD_ITEMS;
}

template <class BLK>
KP_FI void body_select_cluster(const BLK& B, int blk, unsigned char* smem, const KArgs& a, int scratch_cap) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* hist = (uint32_t*)(smem + kRedBytes);
  Item* items = (Item*)(smem + kRedBytes + 1024);
  uint64_t* keys = (uint64_t*)(items + 2 * kSmallMax);
  uint32_t* tgt = (uint32_t*)(keys + 2 * kSmallMax);
  unsigned char* area = (unsigned char*)(tgt + ((words + 3) & ~3));
  Cands cd;
  cd.r = (uint32_t*)area;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  KP_STAMP(x, 26);
  const size_t area_bytes = 8 * (size_t)a.s.Cp > serial_scratch_bytes(scratch_cap) ? 8 * (size_t)a.s.Cp
                                                                                    : serial_scratch_bytes(scratch_cap);
  {
    int n = 0;
    const int o = cluster_order_select(B, a, x, items, kSmallMax, &n, keys, keys + kOrdTargets);
    if (o == ORD_DONE) return;
    if (o == ORD_ITEMS) {
      if (B.tid() == 0 && a.n_order) kp_atomic_add(a.n_order, 1u);
      assign_small(B, x, items, n, area, scratch_cap, area_bytes);
      KP_STAMP(x, 39);
      return;
    }
  }
  cd.F = gather(B, x, cd, false);
  KP_STAMP(x, 27);
  if (pre_checks(B, x, cd.F)) return;
  if (!sel_cluster_fast(B, x, cd, hist, items, keys, area, scratch_cap, area_bytes)) {
    if (B.tid() == 0) flag_slow(a, b, SLOW_CLUSTER);
  }
}

// ---------------------------------------------------------------------------
// k_spread_order: the class-order selections of the spread kernels
// (cluster_order_select, region_order_select) and the assignment over the
// selected list, one wave per binding with a small LDS slice (no Cp-sized
// candidate arrays), so many bindings are resident per CU. A binding it does not
// finish (ORD_NA, a list past kOrderItems, or an assignment sel_all_fast refuses)
// is appended to a fallback list of list positions for the full kernel.
// ---------------------------------------------------------------------------
struct OrderArgs {
  const RegionOut* rout;  // region stage B: stage A's per-region counts [n][R]
  const int32_t* rsel;    // region stage B: selected region ids [n][R]
  const int32_t* rnsel;   // region stage B: their count (-1000 finalised by stage A, < 0 an error)
  int32_t* fb;            // list positions handed to the full kernel
  uint32_t* fb_n;
  int region;  // 0: cluster spread (k_select_cluster), 1: region stage B (k_region_b)
};
constexpr int kOrderItems = 64;  // selected-list capacity
constexpr int kOrderEcap = 128;  // sel_all_fast's party list (>= 64 + kOrderItems)
// slice: [red 64 | hpos 8R | rsel 4R | target heads 4R | items | target keys 16 B x
// kOrdTargets | spec.Clusters bits | selected bits 8W | whist 2 KB | hist 1 KB | buf]
KP_HD inline size_t order_lds_bytes(int W, int R) {
  return 64 + 8 * (size_t)R + 2 * 4 * (size_t)((R + 3) & ~3) + sizeof(Item) * kOrderItems + 16 * kOrdTargets +
         8 * (size_t)W + 8 * (size_t)W + 2048 + 1024 + 8 * (size_t)kOrderEcap;
}
template <class BLK>
KP_FI void body_spread_order(const BLK& B, int blk, unsigned char* smem, const KArgs& a, const OrderArgs& o) {
  if (blk >= a.n) return;
  const int b = a.list[blk];
  const int R = a.s.n_regions, W = a.s.W;
  unsigned char* p = smem + 64;
  unsigned long long* hpos = (unsigned long long*)p;
  p += 8 * (size_t)R;
  int32_t* rs = (int32_t*)p;
  p += 4 * (size_t)((R + 3) & ~3);
  int32_t* th = (int32_t*)p;
  p += 4 * (size_t)((R + 3) & ~3);
  Item* items = (Item*)p;
  p += sizeof(Item) * kOrderItems;
  uint64_t* tk = (uint64_t*)p;
  p += 16 * kOrdTargets;
  uint32_t* tgt = (uint32_t*)p;  // spec.Clusters bits (8W bytes: W u64 words)
  p += 8 * (size_t)W;
  uint64_t* selb = (uint64_t*)p;
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  const BindHdr& h0 = hloc;
  if (h0.tgt_cnt > 0 && ord_targets_ok(h0)) build_bits(B, tgt, 2 * W, a.bv.ipool, h0.tgt_off, h0.tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  x.h = &hloc;
  int n = 0, st = ORD_NA;
  if (o.region) {
    const int nsel = o.rnsel[blk];
    if (nsel == -1000) return;  // stage A wrote the status
    if (nsel >= 0)
      st = region_order_select(B, a, x, o.rout + (size_t)blk * R, o.rsel + (size_t)blk * R, nsel, hpos, rs, items,
                               kOrderItems, &n, tk, tk + kOrdTargets, th);
  } else {
    st = cluster_order_select(B, a, x, items, kOrderItems, &n, tk, tk + kOrdTargets);
  }
  if (st == ORD_DONE) return;
  int why = SLOW_NONE + 1;
  if (st == ORD_ITEMS) {  // assign_small's block-parallel assignment over the list
    for (int w = B.tid(); w < W; w += B.nth()) selb[w] = 0;
    B.sync();
    uint32_t* sel32 = (uint32_t*)selb;
    for (int i = B.tid(); i < n; i += B.nth()) kp_atomic_or(&sel32[items[i].rank >> 5], 1u << (items[i].rank & 31));
    B.sync();
    SelCtx y = x;
    y.frow = selb;
    SelScratch ss;
    ss.whist = (unsigned long long*)(selb + W);
    ss.hist = (uint32_t*)(ss.whist + 256);
    ss.buf = (uint64_t*)(ss.hist + 256);
    ss.cap = kOrderEcap;
    why = sel_all_fast(B, y, ItemCands{items, n, B.tid(), B.nth(), &y, x.h->strategy == ST_STATIC}, ss);
    B.sync();
  }
  if (why == SLOW_NONE) {
    if (B.tid() == 0 && a.n_order) kp_atomic_add(a.n_order, 1u);
    return;
  }
  if (B.tid() == 0) o.fb[kp_atomic_add(o.fb_n, 1u)] = blk;
}

// Region stage A for the order-eligible bindings (order_class), one wave per
// binding: their AvailableReplicas are the class row's estimates (all >= 0) and
// their cluster scores are 0, so every region's calcGroupScore walk is free
// (region_walk_free) and calcGroupScoreForDuplicate counts only the valid
// clusters; both need per-region sums over the feasible clusters, taken here
// straight from the feasibility row and the class row (no candidate arrays).
// spec.Clusters (ord_targets_ok): the feasible targets score 100 and lead their
// region's sortClusters order, so a region holding one is walked exactly
// (region_target_score) over its targets, then its class order.
// LDS slice: [red 64 B | cnt R | dvalid R | tcnt R | tdv R | sum 8R | tsum 8R |
// target keys 16 x kOrdTargets | spec.Clusters bits 8W]. The others go to fb.
KP_HD inline size_t region_a_order_lds_bytes(int R, int W) {
  return 64 + 4 * 4 * (size_t)((R + 3) & ~3) + 2 * 8 * (size_t)R + 16 * kOrdTargets + 8 * (size_t)W;
}
// calcGroupScore (group_clusters.go:238-351, divided) of a region with Tr >= 1
// feasible targets (keys tk[0, nt), ascending; their AvailableReplicas sum St) and
// cnt candidates summing sum: the walk breaks at the first n >= m with P(n) >=
// target, P the prefix over the region's sortClusters order (targets, then its
// class order: every AvailableReplicas >= 0, so P only grows and the break is at
// max(m, n_sum), n_sum the first n with P(n) >= target). Every lane returns it.
template <class BLK>
KP_FI int64_t region_target_score(const BLK& B, const KArgs& a, const SelCtx& x, int32_t cls, const uint64_t* tk,
                                  int nt, int r, int64_t Tr, int64_t St, int64_t cnt, int64_t sum, int64_t target,
                                  int64_t m) {
  const SnapView& s = a.s;
  int64_t n_sum = -1;
  {
    int64_t k = 0, p = 0;
    for (int j = 0; j < nt && n_sum < 0; j++) {
      if (s.region_idx[key_rank(tk[j])] != r) continue;
      k++;
      p += key_avail(tk[j]);
      if (p >= target) n_sum = k;
    }
  }
  if (n_sum < 0 && (m <= cnt)) {
    // the region's class-order entries (feasible, not targets) until Q(j) >= target - St
    const int64_t need = target - St;
    const uint64_t* ord = a.ord + (size_t)cls * s.Cp;
    int64_t run = 0, cj = 0;
    for (int i0 = 0; i0 < s.C && n_sum < 0; i0 += B.nth()) {
      const int i = i0 + B.tid();
      int64_t v = 0;
      bool in = false;
      if (i < s.C) {
        const uint64_t e = ord[i];
        const int c = (int)(uint32_t)e;
        if (mask_test(x.frow, c) && !bit_test(x.tgt_bits, c) && s.region_idx[c] == r) {
          in = true;
          v = (int64_t)(int32_t)(e >> 32);
        }
      }
      const int64_t tot = B.sum64(v);
      uint64_t mm = B.wballot(in);
      if (run + tot < need) {
        run += tot;
        cj += popc64(mm);
        continue;
      }
      while (mm) {  // the break is in this chunk: its members in order (uniform)
        const int l = (int)__builtin_ctzll(mm);
        mm &= mm - 1;
        cj++;
        run += B.wread(v, l);
        if (run >= need) {
          n_sum = Tr + cj;
          break;
        }
      }
    }
  }
  const int64_t valid = n_sum < 0 ? -1 : (m > n_sum ? m : n_sum);
  if (valid >= 1 && valid <= cnt)
    return add64(mul64(target, 1000), (100 * (valid < Tr ? valid : Tr)) / valid);
  if (sum < target) return add64(mul64(sum, 1000), (100 * Tr) / cnt);  // no break: the totals
  return add64(mul64(target, 1000), (100 * Tr) / cnt);
}
template <class BLK>
KP_FI void body_region_a_order(const BLK& B, int blk, unsigned char* smem, const KArgs& a, RegionOut* rout,
                               int32_t* rstat, int32_t* fb, uint32_t* fb_n) {
  if (blk >= a.n) return;
  const int b = a.list[blk];
  const SnapView& s = a.s;
  const int R = s.n_regions, R4 = (R + 3) & ~3;
  int32_t* cnt = (int32_t*)(smem + 64);
  int32_t* dvalid = cnt + R4;
  int32_t* tcnt = dvalid + R4;
  int32_t* tdv = tcnt + R4;
  unsigned long long* sum = (unsigned long long*)(tdv + R4);
  int64_t* tsum = (int64_t*)(sum + R);
  uint64_t* tk = (uint64_t*)(tsum + R);
  uint32_t* tgt = (uint32_t*)(tk + 2 * kOrdTargets);
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  const BindHdr& h0 = hloc;
  if (h0.tgt_cnt > 0 && ord_targets_ok(h0)) build_bits(B, tgt, 2 * s.W, a.bv.ipool, h0.tgt_off, h0.tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  x.h = &hloc;
  const int32_t cls = order_class(a, x, true);
  if (cls < 0) {
    if (B.tid() == 0) fb[kp_atomic_add(fb_n, 1u)] = blk;
#ifdef KP_STAMPS
    if (B.tid() == 0) {  // why: 55 no orders, 56 class 0, 57 row not walkable, 58 spec.Clusters, 59 other
      const BindHdr& h1 = *x.h;
      const int32_t c0 = a.bcls && a.ord ? a.bcls[b] : -1;
      KP_COUNT(x, !a.ord || !a.bcls ? 55 : c0 <= 0 ? 56 : !a.cok[c0] ? 57 : h1.tgt_cnt != 0 ? 58 : 59, 1);
    }
#endif
    return;
  }
  const BindHdr& h = *x.h;
  for (int r = B.tid(); r < R; r += B.nth()) {
    cnt[r] = 0;
    dvalid[r] = 0;
    tcnt[r] = 0;
    tdv[r] = 0;
    sum[r] = 0;
    tsum[r] = 0;
  }
  B.sync();
  const int nt = h.tgt_cnt > 0 ? ord_targets(B, x, tk, tk + kOrdTargets) : 0;
  if (nt < 0) {
    if (B.tid() == 0) fb[kp_atomic_add(fb_n, 1u)] = blk;
    return;
  }
  const uint32_t* tb = h.tgt_cnt > 0 ? tgt : nullptr;
  const bool dup = (h.flags & BF_GROUP_DUP) != 0;
  const int32_t* row = x.erow;
  int64_t F = 0;
  for (int w = 0; w < s.W; w++) {  // word by word (one wave-uniform load), a lane per cluster
    const uint64_t m = x.frow[w];
    if (!m) continue;
    for (int l = B.tid(); l < 64; l += B.nth()) {
      if (!((m >> l) & 1ull)) continue;
      const int c = w * 64 + l;
      F++;
      if (tb && bit_test(tb, c)) continue;  // (a target: below)
      const int r = s.region_idx[c];
      if (r >= 0) {
        const int32_t e = row[c];
        kp_atomic_add(&cnt[r], 1);
        kp_atomic_add(&sum[r], (unsigned long long)e);
        if (dup && e >= h.replicas) kp_atomic_add(&dvalid[r], 1);
      }
    }
  }
  for (int j = B.tid(); j < nt; j += B.nth()) {
    const int r = s.region_idx[key_rank(tk[j])];
    if (r < 0) continue;
    const int64_t av = key_avail(tk[j]);
    kp_atomic_add(&cnt[r], 1);
    kp_atomic_add(&sum[r], (unsigned long long)av);
    kp_atomic_add(&tcnt[r], 1);
    kp_atomic_add((unsigned long long*)&tsum[r], (unsigned long long)av);
    if (dup && av >= (int64_t)h.replicas) {
      kp_atomic_add(&dvalid[r], 1);
      kp_atomic_add(&tdv[r], 1);
    }
  }
  F = B.sum64(F);  // (its reduction also orders the LDS sums before the reads below)
  if (F == 0) {  // FitError (generic_scheduler.go:84-89), as pre_checks
    if (B.tid() == 0) {
      sink_error(x, KP_STATUS_FIT_ERROR, KP_ERR_FIT, s.C);
      rstat[blk] = -1;
    }
    return;
  }
  RegionOut* out = rout + (size_t)blk * R;
  const int64_t target = go_ceil_div_i64(h.replicas, h.region_min);
  int64_t mg = h.cluster_min;  // clusterMinGroups, at least the group's minGroups
  if (mg < h.region_min) mg = h.region_min;
  for (int r = B.tid(); r < R; r += B.nth()) {
    out[r].count = cnt[r];
    if (dup) out[r].score = dvalid[r] == 0 ? 0 : add64(mul64((int64_t)dvalid[r], 1000), (100 * (int64_t)tdv[r]) / dvalid[r]);
    else if (tcnt[r] == 0) out[r].score = region_score_totals(cnt[r], (int64_t)sum[r], 0, target);
  }
  if (!dup && nt > 0) {
    for (int r = 0; r < R; r++) {  // the regions holding a target: walked (wave-uniform loop)
      if (tcnt[r] == 0) continue;
      const int64_t sc = region_target_score(B, a, x, cls, tk, nt, r, tcnt[r], tsum[r], cnt[r], (int64_t)sum[r],
                                             target, mg);
      if (B.tid() == 0) out[r].score = sc;
    }
  }
  if (a.n_order && B.tid() == 0) kp_atomic_add(a.n_order, 1u);
  if (B.tid() == 0) rstat[blk] = 0;
}

// ---------------------------------------------------------------------------
// Region stage A: per-region count and group score for the host selectGroups.
// rout: [n][n_regions]; rstat[blk] = -1 when the final status is already written.
// ---------------------------------------------------------------------------
template <class BLK>
KP_FI void body_region_a(const BLK& B, int blk, unsigned char* smem, const KArgs& a, RegionOut* rout, int32_t* rstat) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const int words = (a.s.Cp + 31) >> 5;
  const int R = a.s.n_regions;
  unsigned char* p = smem + kRedBytes;
  RegionLds L;
  L.minkey = (unsigned long long*)p;
  p += 8 * R;
  L.last = (unsigned long long*)p;
  p += 8 * R;
  L.sumAvail = (int64_t*)p;
  p += 8 * R;
  L.sumScore = (int64_t*)p;
  p += 8 * R;
  L.dscore = (int64_t*)p;
  p += 8 * R;
  L.wsum = (int64_t*)p;
  p += 8 * R;
  L.wscore = (int64_t*)p;
  p += 8 * R;
  L.amin = (int64_t*)p;
  p += 8 * R;
  L.cnt = (int32_t*)p;
  p += 4 * R;
  L.dvalid = (int32_t*)p;
  p += 4 * R;
  L.wcnt = (int32_t*)p;
  p += 4 * R;
  L.done = (int32_t*)p;
  p += 4 * R;
  uint32_t* tgt = (uint32_t*)p;
  p += 4 * ((words + 3) & ~3);
  Cands cd;
  cd.r = (uint32_t*)p;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  cd.g = (int16_t*)(cd.v + a.s.Cp);
  const BindHdr hloc = a.bv.hdr[b];  // registers: no reload after LDS stores
  const BindHdr* h = &hloc;
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  x.h = h;
  KP_STAMP(x, 22);
  cd.F = gather(B, x, cd, false);
  region_of_cands(B, a.s, cd);
  KP_STAMP(x, 23);
  if (pre_checks(B, x, cd.F)) {
    if (B.tid() == 0) rstat[blk] = -1;
    return;
  }
  if (!region_a_fast(B, x, cd, L, rout + (size_t)blk * R)) region_a(B, x, cd, L, rout + (size_t)blk * R);
  KP_STAMP(x, 24);
  if (B.tid() == 0) rstat[blk] = 0;
}

// selectBestClustersByRegion (select_clusters_by_region.go:41-63) over the
// binding's estimator-class order (order_class): each selected region's head is
// its first entry in sortClusters order, the rest are the next restCnt entries of
// the selected regions that are not heads, and the candidate count comes from stage
// A's per-region counts, so the walk stops once the heads and the rest are found
// instead of gathering every candidate. With spec.Clusters (tk != nullptr; tk, tmp:
// kOrdTargets entries, th: [R]) the feasible targets precede every other candidate:
// a selected region holding one has its first target as head, and the other targets
// of the selected regions lead the rest. hpos, rsel: [R] LDS. ORD_ITEMS: items[0, *n)
// = the heads in path order, then the rest in sortClusters order.
template <class BLK>
KP_FI int region_order_select(const BLK& B, const KArgs& a, const SelCtx& x, const RegionOut* ro, const int32_t* sel,
                              int nsel, unsigned long long* hpos, int32_t* rsel, Item* items, int max_items,
                              int* n_out, uint64_t* tk = nullptr, uint64_t* tmp = nullptr, int32_t* th = nullptr) {
  const BindHdr& h = *x.h;
  const int32_t cls = order_class(a, x, tk != nullptr);
  if (cls < 0 || !ro) return ORD_NA;
  KP_STAMP_INIT
  const SnapView& s = *x.s;
  const int R = s.n_regions;
  int64_t total = 0;
  for (int j = 0; j < nsel; j++) total += ro[sel[j]].count;
  const int64_t needCnt = total < h.cluster_max ? total : h.cluster_max;
  const int64_t restCnt = needCnt - nsel;
  const int64_t want = restCnt > 0 ? restCnt : 0;
  if (nsel + want > max_items) return ORD_NA;  // the general path (and its engine limit)
  for (int r = B.tid(); r < R; r += B.nth()) {
    hpos[r] = ~0ull;
    rsel[r] = -1;
    if (th) th[r] = -1;
  }
  B.sync();
  for (int j = B.tid(); j < nsel; j += B.nth()) rsel[sel[j]] = j;
  B.sync();
  const int nt = h.tgt_cnt > 0 ? ord_targets(B, x, tk, tmp) : 0;
  if (nt < 0) return ORD_NA;
  const uint32_t* tb = h.tgt_cnt > 0 ? x.tgt_bits : nullptr;
  // target heads (a selected region's first target), then the other targets of the
  // selected regions, in key order, lead the rest (every thread walks the <= 16)
  int nth_ = 0, ntr = 0;
  if (nt > 0) {
    if (B.tid() == 0)
      for (int j = 0; j < nt; j++) {
        const int r = s.region_idx[key_rank(tk[j])];
        if (r >= 0 && rsel[r] >= 0 && th[r] < 0) th[r] = j;
      }
    B.sync();
    for (int j = 0; j < nt; j++) {
      const int r = s.region_idx[key_rank(tk[j])];
      if (r < 0 || rsel[r] < 0) continue;
      if (th[r] == j) {
        nth_++;
      } else {
        if (ntr < want && B.tid() == 0) items[nsel + ntr] = item_from_key(x, tk[j]);
        ntr++;
      }
    }
  }
  const int64_t tw = ntr < want ? ntr : want;  // rest entries the targets fill
  const int64_t want2 = want - tw;             // ... and the class order
  const int nh_need = nsel - nth_;
  const uint64_t* ord = a.ord + (size_t)cls * s.Cp;
  KP_STAMP(x, 32);
  int nh = 0, nr = 0;
  for (int i0 = 0; i0 < s.C && (nh < nh_need || nr < want2); i0 += B.nth()) {
    const int i = i0 + B.tid();
    uint64_t e = 0;
    int r = -1;
    if (i < s.C) {
      e = ord[i];
      const int c = (int)(uint32_t)e;
      if (mask_test(x.frow, c) && !(tb && bit_test(tb, c))) {
        r = s.region_idx[c];
        if (r >= 0 && rsel[r] < 0) r = -1;
      }
    }
    const bool thead = r >= 0 && th && th[r] >= 0;  // the region's head is a target
    // (a stale read is only larger: the minimum only falls)
    if (r >= 0 && !thead && hpos[r] > (unsigned long long)i) kp_atomic_min_u64(&hpos[r], (unsigned long long)i);
    B.sync();
    const bool head = r >= 0 && !thead && hpos[r] == (unsigned long long)i;
    const bool rest = r >= 0 && !head;
    int32_t cnt;
    const int32_t pk = B.excl_scan((rest ? 1 : 0) | (head ? 1 << 16 : 0), &cnt);
    const int32_t pos = nr + (pk & 0xffff);
    if (rest && pos < want2) items[nsel + tw + pos] = order_item(e);
    nr += cnt & 0xffff;
    nh += cnt >> 16;
    KP_COUNT(x, 36, 1);
  }
  B.sync();
  KP_STAMP(x, 33);
  if (nh < nh_need || nr < want2) return ORD_NA;  // a selected region without a feasible cluster
  for (int j = B.tid(); j < nsel; j += B.nth()) {
    const int r = sel[j];
    items[j] = th && th[r] >= 0 ? item_from_key(x, tk[th[r]]) : order_item(ord[hpos[r]]);
  }
  B.sync();
  KP_STAMP(x, 34);
  *n_out = nsel + (int)want;
  return ORD_ITEMS;
}

// Region stage B. rsel: [n][n_regions] selected region ids (path order); rnsel[n]:
// count, -1000 when stage A already finalized, or -KP_ERR_* from the host step.
template <class BLK>
KP_FI void body_region_b(const BLK& B, int blk, unsigned char* smem, const KArgs& a, const int32_t* rsel,
                         const int32_t* rnsel, const RegionOut* rout, int scratch_cap) {
  if (blk >= a.n) return;
  KP_STAMP_INIT
  const int b = a.list[blk];
  const int nsel = rnsel[blk];
  if (nsel == -1000) return;
  const int words = (a.s.Cp + 31) >> 5;
  const int R = a.s.n_regions;
  unsigned char* p = smem + kRedBytes;
  uint32_t* hist = (uint32_t*)p;
  p += 1024;
  Item* items = (Item*)p;
  p += sizeof(Item) * 2 * kSmallMax;
  uint64_t* keys = (uint64_t*)p;
  p += 8 * 2 * kSmallMax;
  unsigned long long* heads = (unsigned long long*)p;
  p += 8 * R;
  int32_t* rs = (int32_t*)p;
  p += 4 * ((R + 3) & ~3);
  uint32_t* tgt = (uint32_t*)p;
  p += 4 * ((words + 3) & ~3);
  Cands cd;
  cd.r = (uint32_t*)p;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  cd.g = (int16_t*)(cd.v + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  if (nsel < 0) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, -nsel, 0);
    return;
  }
  if ((h->flags & BF_DUP_TARGETS) && h->tgt_cnt > kTgtSmallMax) {  // engine limit (selected-list scratch)
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, -1);
    return;
  }
  KP_STAMP(x, 16);
  const size_t area_bytes = 8 * (size_t)a.s.Cp > serial_scratch_bytes(scratch_cap) ? 8 * (size_t)a.s.Cp
                                                                                    : serial_scratch_bytes(scratch_cap);
  {
    int n = 0;
    if (region_order_select(B, a, x, rout ? rout + (size_t)blk * R : nullptr, rsel + (size_t)blk * R, nsel, heads, rs,
                            items, kSmallMax, &n, keys, keys + kOrdTargets,
                            (int32_t*)(keys + 2 * kOrdTargets)) == ORD_ITEMS) {
      if (B.tid() == 0 && a.n_order) kp_atomic_add(a.n_order, 1u);
      assign_small(B, x, items, n, p, scratch_cap, area_bytes);
      KP_STAMP(x, 35);
      return;
    }
  }
  cd.F = gather(B, x, cd, false);
  region_of_cands(B, a.s, cd);
  KP_STAMP(x, 17);
  region_b(B, x, cd, rsel + (size_t)blk * R, nsel, hist, heads, rs, items, keys, p, scratch_cap, area_bytes);
}

// ---------------------------------------------------------------------------
// Exact serial path: candidates fully sorted by the sortClusters key in a
// global scratch slot, then the Go algorithm on thread 0 (Aggregated ties with
// the pdqsort emulation, scale-down, overflow tiers, duplicates, wrap-around).
// Persistent: block k handles list entries k, k+grid, ...
// ---------------------------------------------------------------------------
// The dynamic-strategy TargetClustersList of a fresh or scale-up binding
// (dynamicFreshScale / dynamicScaleUp, division_algorithm.go:121-166) built in
// LDS and sorted there by sort.Sort's wave emulation (kp_pdq.h), then handed
// to the serial assignment (SerialScratch::presorted). Returns false when the
// binding takes another route (the serial code then builds and sorts itself).
template <class BLK>
KP_FI bool presort_dynamic(const BLK& B, const SelCtx& x, const Item* items, int n, unsigned char* area,
                           int32_t* pos, SerialScratch& sc) {
  const BindHdr& h = *x.h;
  if (!(h.flags & BF_WORKLOAD_ASSIGN) || (h.flags & BF_OVERFLOW) || h.sel != SEL_ALL) return false;
  if (h.strategy != ST_DYNAMIC && h.strategy != ST_AGGREGATED) return false;
  PdqWave<BLK> pw = pdq_carve(B, area, n);
  for (int i = B.tid(); i < n; i += B.nth()) {
    pw.name[i] = items[i].rank;
    pw.rep[i] = items[i].alloc;
    pos[items[i].rank] = i;
  }
  B.sync();
  int go = 0;
  if (B.tid() == 0) {  // buildScheduledClusters over spec.Clusters order (assignment.go:125-142)
    const bool fresh = (h.flags & BF_FRESH) != 0;
    int32_t assigned = 0;
    for (int j = 0; j < h.tgt_cnt; j++) {
      const int32_t i = pos[x.bv->ipool[h.tgt_off + 2 * j]];
      if (i < 0) continue;
      const int32_t r = x.bv->ipool[h.tgt_off + 2 * j + 1];
      assigned = add32(assigned, r);
      if (fresh) pw.rep[i] = add32(pw.rep[i], r);  // first (only) occurrence of the name
    }
    go = fresh || assigned < h.replicas;
  }
  go = B.bcast(go);
  for (int i = B.tid(); i < n; i += B.nth()) pos[items[i].rank] = -1;
  if (!go) {
    B.sync();
    return false;
  }
  int ok = 1;
  if (B.wid() == 0) ok = pw.run(n) ? 1 : 0;
  ok = B.bcast(ok);
  if (!ok) return false;
  for (int i = B.tid(); i < n; i += B.nth()) {
    sc.an[i] = pw.name[i];
    sc.ar[i] = pw.rep[i];
  }
  B.sync();
  sc.presorted = 1;
  return true;
}

// The candidates in sortClusters order (items[0, F)) without sorting them: a
// non-target candidate's key is (overflow 0, score 0, estimate, rank), which ascends
// along its estimator class's order (k_class_order: estimate desc, rank asc), so the
// class order filtered by the binding's feasibility row is that part of the list,
// already sorted; the few feasible spec.Clusters entries (their locality score and
// scheduled replicas in the key) are merged in by binary search. O(C) per binding
// instead of the bitonic sort's O(C log^2 C). Returns false, with nothing written to
// items, when it does not apply (no class orders, overflow tiers, a class whose row
// the order cannot stand for, many or duplicate targets) or when the filtered order
// is not ascending in the keys; the caller then sorts.
constexpr int kSlowOrdTargets = 64;
template <class BLK>
KP_FI bool slow_items_from_order(const BLK& B, const KArgs& a, const SelCtx& x, int b, const uint32_t* tgt, int F,
                                 uint64_t* keys, Item* items) {
  const BindHdr& h = *x.h;
  if (!a.ord || !a.cok || !a.bcls || h.ovf_mode != OVF_ZERO || (h.flags & BF_DUP_TARGETS) ||
      h.tgt_cnt > kSlowOrdTargets)
    return false;
  const int32_t cls = a.bcls[b];
  if (cls <= 0 || !a.cok[cls]) return false;
  const uint64_t* ord = a.ord + (size_t)cls * a.s.Cp;
  const int C = a.s.C;
  int N = 0;
  for (int base = 0; base < C; base += B.nth()) {  // stream compaction of the class order
    const int i = base + B.tid();
    int32_t in = 0;
    uint32_t r = 0;
    int32_t e = 0;
    if (i < C) {
      const uint64_t o = ord[i];
      r = (uint32_t)o;
      e = (int32_t)(o >> 32);  // the class row's estimate: est_at's value (a walkable row: no merge)
      in = mask_test(x.frow, (int)r) && !(h.tgt_cnt > 0 && bit_test(tgt, (int)r)) ? 1 : 0;
    }
    int32_t tot;
    const int32_t off = B.excl_scan(in, &tot);
    if (in) keys[N + off] = sort_key(0, 0, (int64_t)e, r);
    N += tot;
  }
  int T = 0;  // the feasible targets, appended after the others (thread 0: at most kSlowOrdTargets)
  if (h.tgt_cnt > 0) {
    if (B.tid() == 0)
      for (int j = 0; j < h.tgt_cnt; j++) {
        const uint32_t r = (uint32_t)x.bv->ipool[h.tgt_off + 2 * j];
        if (!mask_test(x.frow, (int)r)) continue;
        const int64_t avail = (int64_t)est_at(x, (int)r) + (int64_t)assigned_of(*x.bv, h, x.tgt_bits, r);
        keys[N + T++] = sort_key(0, locality_score(h, x.tgt_bits, r), avail, r);
      }
    T = B.bcast(T);
  }
  B.sync();
  int64_t bad = N + T != F ? 1 : 0;
  for (int p = B.tid() + 1; p < N; p += B.nth()) bad |= keys[p - 1] >= keys[p] ? 1 : 0;
  if (B.sum64(bad) != 0) return false;  // (also orders every key write before the reads below)
  for (int p = B.tid(); p < N + T; p += B.nth()) {
    const uint64_t k = keys[p];
    int pos = 0;
    for (int q = 0; q < T; q++) pos += keys[N + q] < k ? 1 : 0;  // targets before it
    if (p < N) {
      pos += p;
    } else {
      int lo = 0, hi = N;  // non-targets before it
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < k) lo = mid + 1;
        else hi = mid;
      }
      pos += lo;
    }
    if (p < N) {  // (no scheduled replicas: allocatable = available = the estimate)
      Item it;
      it.rank = key_rank(k);
      it.alloc = (int32_t)key_avail(k);
      it.avail = key_avail(k);
      it.ovf = 0;
      it.pad = 0;
      items[pos] = it;
    } else {
      items[pos] = item_from_key(x, k);
    }
  }
  B.sync();
  if (B.tid() == 0) KP_COUNT(x, 54, 1);
  return true;
}

template <class BLK>
KP_HD void body_slow(const BLK& B, int blk, int grid, unsigned char* smem, const KArgs& a, unsigned char* scratch,
                     size_t slot_bytes, int scratch_cap, int lds_area, int lds_sort) {
  KP_STAMP_INIT
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + kRedBytes);
  unsigned char* larea = (unsigned char*)(tgt + ((words + 3) & ~3));  // lds_area bytes
  unsigned char* sarea = larea + lds_area;                             // lds_sort bytes
  unsigned char* mine = scratch + (size_t)blk * slot_bytes;
  // slot layout: cand r/v [Cp] | keys [P] | items [Cp] | pos [Cp] | serial scratch
  int P = 1;
  while (P < a.s.Cp) P <<= 1;
  Cands cd;
  cd.r = (uint32_t*)mine;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  // the candidates' sortClusters keys are sorted in LDS when they fit
  uint64_t* keys = (size_t)lds_sort >= 8 * (size_t)P ? (uint64_t*)sarea : (uint64_t*)(cd.v + a.s.Cp);
  const bool pdq_lds = (size_t)lds_sort >= pdq_wave_bytes(a.s.Cp);
  Item* items = (Item*)((uint64_t*)(cd.v + a.s.Cp) + P);
  int32_t* pos = (int32_t*)(items + a.s.Cp);
  unsigned char* ser = (unsigned char*)(pos + a.s.Cp);
  // the select kernels appended the flagged bindings to slow_ids (same stream: complete)
  const int nslow = (int)*(volatile uint32_t*)&a.stats[0];
  if (blk >= nslow || blk >= a.n) return;  // (block-uniform) a slot without a binding is never touched
  for (int i = B.tid(); i < a.s.Cp; i += B.nth()) pos[i] = -1;
  B.sync();
  const bool tie_lds = (size_t)lds_sort >= 3072 + 8 * (size_t)sel_all_ecap(a.s.Cp) + 64;
  for (int idx = blk; idx < nslow && idx < a.n; idx += grid) {
    const int b = a.list[idx];
    const int why = a.slow[b];
    const BindHdr* h = &a.bv.hdr[b];
    build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
    SelCtx x = make_ctx(a, b, tgt);
    int done = 0;
    if (B.tid() == 0 && ((lds_area > 0 && scale_down_targets(x, larea, (size_t)lds_area)) ||
                         scale_down_targets(x, ser, (size_t)serial_scratch_bytes(scratch_cap)))) {
      a.slow[b] = 0;
      done = 1;
    }
    if (B.bcast(done)) continue;
    KP_STAMP(x, 49);
    cd.F = gather(B, x, cd, false);
    const int F = cd.F;
    KP_STAMP(x, 50);
#ifdef KP_SLOW_CHECK
    // diagnostic build: the gathered candidates against the feasibility row (count,
    // rank sum and xor). dbg[0] += threads whose F differs, dbg[1] += bindings whose
    // list differs, dbg[8 + 4k ..] = (binding, F, F0, wave) of the first ones.
    {
      int F0 = 0;
      uint64_t s0 = 0, x0 = 0;
      for (int c = 0; c < a.s.C; c++)
        if (mask_test(x.frow, c)) F0++, s0 += (uint64_t)c, x0 ^= (uint64_t)c * 0x9E3779B97F4A7C15ull;
      if (F0 != F) {
        const unsigned long long k = kp_atomic_add(&a.dbg[0], 1ull);
        if (k < 8 && (B.tid() & 63) == 0) {
          a.dbg[8 + 4 * k] = (unsigned long long)b;
          a.dbg[9 + 4 * k] = (unsigned long long)(int64_t)F;
          a.dbg[10 + 4 * k] = (unsigned long long)F0;
          a.dbg[11 + 4 * k] = (unsigned long long)B.wid();
        }
      }
      if (B.tid() == 0) {
        uint64_t s1 = 0, x1 = 0;
        const int Fc = F < 0 ? 0 : (F > a.s.Cp ? a.s.Cp : F);
        for (int i = 0; i < Fc; i++) {
          const uint64_t c = c_rank(cd, i);
          s1 += c, x1 ^= c * 0x9E3779B97F4A7C15ull;
        }
        if (s1 != s0 || x1 != x0) kp_atomic_add(&a.dbg[1], 1ull);
      }
      B.sync();
    }
#endif
    if (!slow_items_from_order(B, a, x, b, tgt, F, keys, items)) {
      int PF = 1;
      while (PF < F) PF <<= 1;
      for (int i = B.tid(); i < PF; i += B.nth()) keys[i] = i < F ? cand_key(x, cd, i, cd.v[i]) : ~0ull;
      B.sync();
      for (int k = 2; k <= PF; k <<= 1)  // bitonic sort (ascending)
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = B.tid(); i < PF; i += B.nth()) {
            int l = i ^ j;
            if (l > i) {
              uint64_t ki = keys[i], kl = keys[l];
              bool up = (i & k) == 0;
              if ((ki > kl) == up) {
                keys[i] = kl;
                keys[l] = ki;
              }
            }
          }
          B.sync();
        }
      for (int i = B.tid(); i < F; i += B.nth()) items[i] = item_from_key(x, keys[i]);
      B.sync();
    }
#ifdef KP_SLOW_CHECK
    if (B.tid() == 0) {  // dbg[2] += bindings whose sorted items differ, dbg[3] += ... whose keys differ
      uint64_t s0 = 0, s1 = 0, k0 = 0;
      for (int c = 0; c < a.s.C; c++)
        if (mask_test(x.frow, c)) s0 += (uint64_t)c;
      const int Fc = F < 0 ? 0 : (F > a.s.Cp ? a.s.Cp : F);
      for (int i = 0; i < Fc; i++) s1 += items[i].rank, k0 += key_rank(keys[i]);
      if (s1 != s0) kp_atomic_add(&a.dbg[2], 1ull);
      if (k0 != s0) kp_atomic_add(&a.dbg[3], 1ull);
    }
    B.sync();
#endif
    KP_STAMP(x, 6);
    SerialScratch sc = serial_scratch_carve(ser, scratch_cap);
    const bool pre = pdq_lds && presort_dynamic(B, x, items, F, sarea, pos, sc);
    KP_STAMP(x, 51);
    if (pre && why == SLOW_TIE && tie_lds) {
      // The Aggregated tie group straddled the cut: with sort.Sort's output
      // order known, the block-parallel path decides it exactly.
      for (int i = B.tid(); i < F; i += B.nth()) pos[sc.an[i]] = i;
      B.sync();
      const SelScratch ss = carve_sel_scratch(sarea, a.s.Cp);
      const int w2 = sel_all_fast<true>(B, x, PosCands{&cd, pos, B.tid(), B.nth()}, ss);
      KP_STAMP(x, 52);
      KP_COUNT(x, 53, F);
      B.sync();  // every thread's last read of pos (emit) precedes the reset
      for (int i = B.tid(); i < F; i += B.nth()) pos[sc.an[i]] = -1;
      B.sync();
      if (w2 == SLOW_NONE) {
        if (B.tid() == 0) {
          a.slow[b] = 0;
          kp_atomic_add(&a.stats[7], 1u);  // resolved block-parallel
        }
        KP_STAMP(x, 7);
        continue;
      }
    }
    KP_STAMP(x, 7);
    if (B.tid() == 0) {
      sc.pos = pos;
      int n = F;
      bool err = false;
      if (h->sel == SEL_CLUSTER) {  // selectBestClustersByCluster on the sorted list
        if ((int64_t)F < h->cluster_min) {
          sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_MIN_GROUPS, 0);
          err = true;
        } else {
          int64_t needCnt = (int64_t)F < h->cluster_max ? (int64_t)F : h->cluster_max;
          if (needCnt < 0) needCnt = 0;
          if (h->need_replicas != -1) {
            auto check = [&]() {
              int64_t t = 0;
              for (int i = 0; i < needCnt; i++) t += items[i].avail;
              return t >= (int64_t)h->need_replicas;
            };
            int64_t upd = needCnt - 1;
            while (!check() && upd >= 0) {  // selectClustersByAvailableResource
              int64_t mv = items[upd].avail;
              int64_t id = -1;
              for (int64_t i = needCnt; i < F; i++)
                if (mv < items[i].avail) {
                  id = i;
                  mv = items[i].avail;
                }
              if (id < 0) {
                upd--;
                continue;
              }
              Item t = items[upd];
              items[upd] = items[id];
              items[id] = t;
              upd--;
            }
            if (!check() || needCnt == 0) {
              sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, needCnt);
              err = true;
            }
          } else if (needCnt == 0) {
            sink_error(x, KP_STATUS_ERROR, KP_ERR_NO_CLUSTERS, 0);
            err = true;
          }
          n = (int)needCnt;
        }
      }
      if (!err) {
        SerialAssign sa{x, sc, (h->flags & BF_UID_DESC) != 0};
        SerialOut o = sa.run(items, n);
        sink_serial(x, sc, o);
      }
      a.slow[b] = 0;
    }
    B.sync();
    KP_STAMP(x, 8);
  }
}

// kp_filter_reasons: one thread per (binding, cluster) pair, grid-strided;
// out[b * C + r] for cluster rank r < C.
// out[i] for pair i of bindings [b0, b0 + n / C): binding b0 + i / C, cluster rank i % C.
KP_HD inline void body_reasons(const SnapView& s, const BatchView& bv, int b0, uint64_t i, uint32_t* out) {
  const uint64_t C = (uint64_t)s.C;
  const int b = b0 + (int)(i / C), r = (int)(i % C);
  out[i] = pair_reason(s, bv, bv.hdr[b], r);
}

// CSR offsets of the per-binding results: offsets[b] = sum of the counts of the
// bindings before b whose status is OK (the others report no targets),
// offsets[n] = total. Two launches over chunks of kOffChunk bindings: pass A
// writes each chunk's local exclusive offsets and its total; pass B adds the
// totals of the chunks before it (and the last chunk writes offsets[n]).
template <class BLK>
KP_FI void body_offsets_a(const BLK& B, int blk, const int32_t* status, const uint32_t* count, int n,
                          uint64_t* offsets, uint64_t* part) {
  const int per = kOffChunk / B.nth();  // entries per thread (kOffPer on the GPU)
  const int lo = blk * kOffChunk + B.tid() * per;
  auto cnt = [&](int i) { return i < n && status[i] == KP_STATUS_OK ? count[i] : 0u; };
  int64_t mine = 0;
  for (int q = 0; q < per; q++) mine += cnt(lo + q);
  int32_t tlo, thi;  // 64-bit exclusive scan as two 32-bit ones (low 16 bits, the rest)
  const int32_t blo = B.excl_scan((int32_t)(mine & 0xffff), &tlo);
  const int32_t bhi = B.excl_scan((int32_t)(mine >> 16), &thi);
  uint64_t o = (uint64_t)(uint32_t)blo + ((uint64_t)(uint32_t)bhi << 16);
  for (int q = 0; q < per; q++) {
    if (lo + q < n) offsets[lo + q] = o;
    o += cnt(lo + q);
  }
  if (B.tid() == 0) part[blk] = (uint64_t)(uint32_t)tlo + ((uint64_t)(uint32_t)thi << 16);
}
template <class BLK>
KP_FI void body_offsets_b(const BLK& B, int blk, int nblk, int n, uint64_t* offsets, const uint64_t* part) {
  int64_t base = 0;
  for (int k = B.tid(); k < blk; k += B.nth()) base += (int64_t)part[k];
  base = B.sum64(base);
  const int lo = blk * kOffChunk, hi = lo + kOffChunk < n ? lo + kOffChunk : n;
  for (int i = lo + B.tid(); i < hi; i += B.nth()) offsets[i] += (uint64_t)base;
  if (blk == nblk - 1 && B.tid() == 0) offsets[n] = (uint64_t)base + part[blk];
}

// Gathers per-binding results into CSR order (offsets from body_offsets). The select
// kernels write snapshot ranks; the caller's cluster index is perm[rank], looked up
// here (a streaming pass) rather than at the end of each binding's dependency chain.
template <class BLK>
KP_FI void body_compact(const BLK& B, int blk, const uint64_t* start, const uint32_t* count, const uint64_t* offsets,
                        const uint32_t* in_idx, const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n,
                        const uint32_t* perm, uint32_t* h_idx = nullptr, int32_t* h_rep = nullptr,
                        uint64_t h_cap = 0) {
  if (blk >= n) return;
  uint64_t s = start[blk], o = offsets[blk];
  uint32_t c = (uint32_t)(offsets[blk + 1] - o);  // 0 unless the status is OK (body_offsets)
  for (uint32_t i = B.tid(); i < c; i += B.nth()) {
    const uint32_t ci = perm[in_idx[s + i]];
    const int32_t cr = in_rep[s + i];
    out_idx[o + i] = ci;
    out_rep[o + i] = cr;
    if (o + i < h_cap) {  // the page-locked host copy (coalesced stores over the bus)
      h_idx[o + i] = ci;
      h_rep[o + i] = cr;
    }
  }
}

}  // namespace kp
