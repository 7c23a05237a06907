// kp_filter.h — the filter stage as bitset algebra over cluster postings, and the
// GeneralEstimator evaluated once per estimator class.
//
// RunFilterPlugins (runtime/framework.go:93-122) is an AND of per-cluster
// predicates, and every predicate a binding can state is a union / intersection /
// complement of a few snapshot-wide cluster sets: the clusters carrying label k=v,
// provider p, region r or zone z, enabling GVK g, holding taint list t, not being
// deleted. upload_snapshot (engine.cpp) stores each of those sets once as a
// W-word bitset row (SnapView::bits); a binding's feasibility word w is then the
// same boolean expression over word w of the rows its selector names. One wave64
// per binding, one lane per word: a binding costs O(rows named x W / 64) word
// operations instead of C per-cluster evaluations, and the row it writes
// (fmask[b][W]) is the u64 feasibility layout the select kernels already read.
//
// The estimate (calAvailableReplicas' GeneralEstimator answer, general.go:57-108)
// depends on a binding only through its ReplicaRequirements (resource requests,
// in both the summary and the resource-model paths), so bindings with equal
// requests share one raw row per cluster; k_est_class computes each distinct
// class's row once, and the select kernels merge it with the binding's
// spec.Replicas as cal_merge_bf does (kp_select.h est_at).
#pragma once
#include "kp_algo.h"

namespace kp {

// Row of a hashed key (label, provider, region, zone value), -1 if no cluster has it.
// Uniform: every lane probes the same key.
KP_HD inline int32_t bits_find(const SnapView& s, uint64_t key) {
  uint32_t i = bits_hash(key) & s.bmask;
  for (;;) {
    const uint64_t k = kp_ldu(s.bkey + i);
    if (k == key) return kp_ldu(s.bval + i);
    if (k == kBitsEmpty) return -1;
    i = (i + 1) & s.bmask;
  }
}
KP_HD inline uint64_t bits_word(const SnapView& s, int row, int w) { return s.bits[(size_t)row * s.W + w]; }

// OR of the rows of the listed values (keys bits_key(kind, slot, value)).
KP_HD inline uint64_t bits_any(const SnapView& s, const int32_t* lst, int n, uint64_t kind, uint32_t slot, int w) {
  uint64_t m = 0;
  for (int k = 0; k < n; k++) {
    const int32_t row = bits_find(s, bits_key(kind, slot, kp_ldu(lst + k)));
    if (row >= 0) m |= bits_word(s, row, w);
  }
  return m;
}
// Bits of word w set for the listed cluster ranks.
KP_HD inline uint64_t rank_word(const int32_t* lst, int n, int w, int stride = 1) {
  uint64_t m = 0;
  for (int k = 0; k < n; k++) {
    const int32_t r = kp_ldu(lst + stride * k);
    if ((r >> 6) == w) m |= 1ull << (r & 63);
  }
  return m;
}

// Word w of one selector instruction (prog_eval_u's semantics, kp_algo.h; bits
// past C are cleared by BR_BASE).
KP_HD inline uint64_t instr_word(const SnapView& s, const BatchView& bv, const Instr& in, int w) {
  switch (in.op) {
    case OP_TRUE:
      return ~0ull;
    case OP_EXCLUDE:
      return ~rank_word(bv.ipool + in.a, in.b, w);
    case OP_NAMES:
      return rank_word(bv.ipool + in.a, in.b, w);
    case OP_LBL_IN:
      return bits_any(s, bv.ipool + in.b, in.c, BK_LABEL, (uint32_t)in.a, w);
    case OP_LBL_NOTIN:  // absent label, or a value outside the list
      return ~bits_any(s, bv.ipool + in.b, in.c, BK_LABEL, (uint32_t)in.a, w);
    case OP_LBL_EXISTS:
      return bits_word(s, s.br_lex + in.a, w);
    case OP_LBL_DNE:
      return ~bits_word(s, s.br_lex + in.a, w);
    case OP_FLD_IN:
      return bits_any(s, bv.ipool + in.b, in.c, in.a == 0 ? BK_PROVIDER : BK_REGION, 0, w);
    case OP_FLD_NOTIN:
      return ~bits_any(s, bv.ipool + in.b, in.c, in.a == 0 ? BK_PROVIDER : BK_REGION, 0, w);
    case OP_FLD_EXISTS:
      return bits_word(s, in.a == 0 ? BR_PROV_SET : BR_REG_SET, w);
    case OP_FLD_DNE:
      return ~bits_word(s, in.a == 0 ? BR_PROV_SET : BR_REG_SET, w);
    case OP_FLD_GT:
    case OP_FLD_LT: {  // integer compare: per cluster of the word
      uint64_t m = 0;
      for (int q = 0; q < 64; q++) {
        const int c = 64 * w + q;
        if (c >= s.C) break;
        const uint32_t f = s.flags[c];
        const bool has = (in.a == 0 ? (f & CF_PROVIDER_INT) : (f & CF_REGION_INT)) != 0;
        const int64_t x = in.a == 0 ? s.provider_int[c] : s.region_int[c];
        if (has && (in.op == OP_FLD_GT ? x > in.v : x < in.v)) m |= 1ull << q;
      }
      return m;
    }
    case OP_ZONE_IN:  // a listed zone implies a zone
      return bits_any(s, bv.ipool + in.b, in.c, BK_ZONE, 0, w);
    case OP_ZONE_NOTIN:
      return ~bits_any(s, bv.ipool + in.b, in.c, BK_ZONE, 0, w);
    case OP_ZONE_EXISTS:
      return bits_word(s, BR_ZONE_ANY, w);
    case OP_ZONE_DNE:
      return ~bits_word(s, BR_ZONE_ANY, w);
    default:  // OP_FALSE and unknown opcodes
      return 0;
  }
}
// A ClusterMatches program: the AND of its instructions.
KP_HD inline uint64_t prog_word(const SnapView& s, const BatchView& bv, int32_t prog_id, int w) {
  const Prog p = kp_ldu(bv.progs + prog_id);
  uint64_t m = ~0ull;
  for (int i = 0; i < p.ins_cnt; i++) m &= instr_word(s, bv, kp_ldu(bv.instrs + p.ins_off + i), w);
  return m;
}

// Feasibility word w of binding h: the same expression as pair_eval_fast's `ok`
// (kp_algo.h), over bitset rows. tolm: bit t = the binding tolerates taint list t.
KP_HD inline uint64_t filter_word(const SnapView& s, const BatchView& bv, const BindHdr& h, int w, uint64_t tolm) {
  const int en = h.enabled;
  uint64_t m = bits_word(s, BR_BASE, w);
  // spec.Clusters members pass APIEnablement and TaintToleration (TargetContains)
  const uint64_t in_t = h.tgt_cnt > 0 ? rank_word(bv.ipool + h.tgt_off, h.tgt_cnt, w, 2) : 0ull;
  if (en & 1) m &= in_t | (h.gvk >= 0 ? bits_word(s, s.br_api + h.gvk, w) : 0ull);
  if (en & 2) {
    uint64_t tl = 0;
    for (uint64_t t = tolm; t; t &= t - 1) tl |= bits_word(s, s.br_tset + ctz64(t), w);
    m &= in_t | tl;
  }
  if ((en & 4) && !(h.flags & BF_AFF_ALL)) {  // ClusterAffinity: any term matches
    uint64_t a = 0;
    for (int j = 0; j < h.filt_cnt; j++) a |= prog_word(s, bv, kp_ldu(bv.ipool + h.filt_off + j), w);
    m &= a;
  }
  if (en & 8) {  // SpreadConstraint presence checks
    if (h.flags & BF_NEED_PROVIDER) m &= bits_word(s, BR_HAS_PROVIDER, w);
    if (h.flags & BF_NEED_REGION) m &= bits_word(s, BR_HAS_REGION, w);
    if (h.flags & BF_NEED_ZONES) m &= bits_word(s, BR_HAS_ZONES, w);
  }
  if ((en & 32) && h.evict_cnt > 0) m &= ~rank_word(bv.ipool + h.evict_off, h.evict_cnt, w);  // ClusterEviction
  return m;
}

// k_filter: binding b's feasibility row fmask[b][0, W), by the calling wave (one
// lane per word; on the host build one "lane" walks every word).
template <class BLK>
KP_FI void body_filter(const BLK& B, int b, const SnapView& s, const BatchView& bv, uint64_t* fmask) {
  const BindHdr h = bv.hdr[b];
  const int ww = B.wwidth(), lane = B.lane() & (ww - 1);
  uint64_t tolm = 0;  // TaintToleration once per distinct taint list (n_tsets <= kTsetRowsMax)
  if (h.enabled & 2)
    for (int t0 = 0; t0 < s.n_tsets; t0 += ww) {
      const int t = t0 + lane;
      const bool ok = t < s.n_tsets && taints_tolerated(s, bv, h, s.tset_rep[t]);
      tolm |= B.wballot(ok) << t0;
    }
  uint64_t* row = fmask + (size_t)b * s.W;
  for (int w0 = 0; w0 < s.W; w0 += ww) {
    const int w = w0 + lane;
    if (w < s.W) row[w] = filter_word(s, bv, h, w, tolm);
  }
}

}  // namespace kp
