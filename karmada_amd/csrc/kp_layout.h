// kp_layout.h — packed HBM layout shared by the host packer and the HIP kernels.
//
// Snapshot (one per kp_snapshot): cluster-major SoA, clusters re-ordered by name
// (byte order), so a cluster's index ("rank") is also its name order. Every
// per-cluster column is padded to Cp = roundup(C, 64) so one wave64 reads 64
// consecutive clusters of one column with coalesced loads, and the feasibility
// of those 64 clusters is one u64 ballot word.
//
// Bindings (one per kp_batch): a fixed BindHdr per binding plus pools holding the
// compiled predicates (label/field/zone selector programs, tolerations, name
// lists) and the integer resource requests, all resolved to snapshot ids by the
// packer so kernels never see a string.
#pragma once
#include <stdint.h>

#include "../../include/kp/kp_api.h"
#include "kp_blk.h"

namespace kp {

constexpr int kWave = 64;
constexpr int kRankBits = 22;                  // cluster rank in packed candidate words
constexpr uint32_t kRankMask = (1u << kRankBits) - 1;
constexpr int kMaxClusters = 1 << 18;          // sort-key rank field (18 bits)
constexpr int32_t kInt32Max = 0x7fffffff;
constexpr int kMaxPodsPerNode = 110;           // general.go:41

// ---- cluster flag bits -------------------------------------------------------
enum : uint32_t {
  CF_DELETING = 1u << 0,
  CF_HAS_PROVIDER = 1u << 1,
  CF_HAS_REGION = 1u << 2,
  CF_HAS_ZONES = 1u << 3,
  CF_HAS_SUMMARY = 1u << 4,
  CF_MODEL_OK = 1u << 5,         // gate on, AllocatableModelings non-empty, buildModelNodes ok
  CF_PROVIDER_INT = 1u << 6,     // provider parses as int64 (field Gt/Lt)
  CF_REGION_INT = 1u << 7,
};

// ---- taint effects / tolerations --------------------------------------------
enum : int32_t { EFF_ANY = 0, EFF_NOSCHEDULE = 1, EFF_NOEXECUTE = 2, EFF_OTHER = 3 };
enum : int32_t { TOL_EQUAL = 0, TOL_EXISTS = 1 };
struct Tol {
  int32_t key;  // -1 = any key (empty toleration key)
  int32_t val;  // string id
  int32_t op;   // TOL_*
  int32_t eff;  // EFF_*
};

// ---- selector programs (pkg/util/selector.go:97-155) --------------------------
enum : int32_t {
  OP_FALSE = 0,
  OP_TRUE,
  OP_EXCLUDE,    // a=list off, b=count: cluster rank must NOT be listed
  OP_NAMES,      // cluster rank must be listed
  OP_LBL_IN,     // a=key slot, b=list off, c=count (values)
  OP_LBL_NOTIN,
  OP_LBL_EXISTS,
  OP_LBL_DNE,
  OP_FLD_IN,     // a=field (0 provider, 1 region), b,c=list
  OP_FLD_NOTIN,
  OP_FLD_EXISTS,
  OP_FLD_DNE,
  OP_FLD_GT,     // a=field, v=int
  OP_FLD_LT,
  OP_ZONE_IN,    // b,c=list
  OP_ZONE_NOTIN,
  OP_ZONE_EXISTS,
  OP_ZONE_DNE,
};
struct Instr {
  int32_t op, a, b, c;
  int64_t v;
};
struct Prog {
  int32_t ins_off, ins_cnt;
};

// ---- binding header -----------------------------------------------------------
enum : uint32_t {
  BF_HAS_RR = 1u << 0,          // ReplicaRequirements != nil
  BF_NONWORKLOAD_EST = 1u << 1, // Replicas==0 && no components: estimator skipped (util.go:69-73)
  BF_WORKLOAD_ASSIGN = 1u << 2, // (Replicas>0 || RR!=nil) && components<=1 (common.go:68)
  BF_SETS = 1u << 3,            // MultiplePodTemplatesScheduling gate + isMultiTemplateSchedulingApplicable:
                                // the estimator row is MaxAvailableComponentSets (core/util.go:113-118)
  BF_FRESH = 1u << 4,           // RescheduleRequired (assignment.go:118-120)
  BF_UID_DESC = 1u << 5,        // FNV-1a(uid) odd -> name-descending tie-break
  BF_OVERFLOW = 1u << 6,        // enableOverflow (common.go:156-170)
  BF_NEED_PROVIDER = 1u << 7,   // SpreadConstraint filter presence checks
  BF_NEED_REGION = 1u << 8,
  BF_NEED_ZONES = 1u << 9,
  BF_AFF_ALL = 1u << 10,        // ClusterAffinity filter passes every cluster
  BF_SCORE_LOCALITY = 1u << 11, // len(spec.Clusters) > 0 and ClusterLocality enabled
  BF_GROUP_DUP = 1u << 12,      // calcGroupScore uses the Duplicated formula
  BF_HAS_WP = 1u << 13,         // WeightPreference != nil
  BF_EMPTY_PROP = 1u << 14,     // EnableEmptyWorkloadPropagation
  BF_BAD = 1u << 15,            // packing error (unparsable quantity): status ERROR
  BF_DUP_TARGETS = 1u << 16,    // spec.Clusters names repeat: serial exact path
  BF_NEED_AVAIL = 1u << 17,     // selection reads AvailableReplicas
  BF_LIMIT_OVF = 1u << 18,      // with BF_BAD: an engine limit (more overflow terms than the
                                // sortClusters key orders), not a malformed request
};
enum : int32_t { ST_NONE = 0, ST_DUPLICATED, ST_AGGREGATED, ST_STATIC, ST_DYNAMIC };
enum : int32_t { SEL_ALL = 0, SEL_CLUSTER, SEL_REGION, SEL_ERR_UNSUPPORTED };
enum : int32_t { OVF_ZERO = 0, OVF_1000, OVF_PROGS };

struct alignas(16) BindHdr {
  int32_t replicas;
  uint32_t flags;
  int32_t strategy;
  int32_t sel;
  int32_t gvk;          // -1: no cluster enables it
  int32_t n_targets_all;
  int32_t tgt_off, tgt_cnt;      // i32 pool: (rank, replicas) pairs, spec.Clusters order
  int32_t evict_off, evict_cnt;  // i32 pool: ranks
  int32_t tol_off, tol_cnt;      // Tol pool
  int32_t filt_off, filt_cnt;    // i32 pool: program ids (filter affinities)
  int32_t ovf_mode, ovf_off, ovf_cnt;  // program ids for getClusterOverflowOrder
  int32_t sw_off, sw_cnt;        // i32 pool: program ids; weights in i64 pool at sw_w_off
  int32_t sw_w_off;
  int32_t sreq_off, sreq_cnt;    // i32 pool rids; divisors in i64 pool at sreq_q_off
  int32_t sreq_q_off;
  int32_t mreq_off, mreq_cnt;
  int32_t mreq_q_off;
  int32_t enabled;               // KP_PLUGIN_* mask
  int64_t cluster_min, cluster_max, region_min, region_max;
  int32_t need_replicas;         // SelectBestClusters needReplicas (-1 = ignore resources)
  int32_t spread_order;          // SpreadConstraint fields in first-appearance order, 2 bits each (1 provider, 2 region, 3 zone)
  uint64_t out_cap;               // result entries this binding can emit on the fast paths
  uint64_t out_off;               // its slot in the batch's result pool (prefix sum of out_cap)
  // this binding's slices of the pools (staged into LDS by the pair kernel)
  int32_t ip_beg, ip_end, pr_beg, pr_end, in_beg, in_end;
};

// ---- snapshot device view -----------------------------------------------------
constexpr int64_t kQaAbsent = INT64_MIN;
struct SnapView {
  int32_t C, Cp, W;              // clusters, padded clusters, ceil(C/64)
  int32_t n_label_keys, api_words, n_res, n_tmpl, n_regions;
  int32_t kmax;                  // model node groups per cluster (max over the snapshot)
  const uint32_t* flags;         // [Cp]
  const int32_t* provider;       // [Cp] string id or -1
  const int32_t* region;         // [Cp] string id or -1
  const int32_t* region_idx;     // [Cp] index in name-sorted region list, -1 if none
  const int64_t* provider_int;   // [Cp]
  const int64_t* region_int;     // [Cp]
  const int32_t* zone_off;       // [C+1]
  const int32_t* zone_ids;
  const int32_t* label_val;      // [n_label_keys][Cp] value string id or -1
  const int32_t* taint_off;      // [C+1]
  const int32_t* taint_key;
  const int32_t* taint_val;
  const int32_t* taint_eff;
  const int32_t* taint_set;      // [Cp] id of the cluster's taint list (identical lists share an id)
  const int32_t* tset_rep;       // [n_tsets] a cluster holding that list
  int32_t n_tsets;
  const uint64_t* api_bits;      // [api_words][Cp]
  const int64_t* allowed;        // [Cp] getAllowedPodNumber
  const int64_t* avail;          // [n_res][Cp] summary path available (milli for cpu), <=0 -> 0
  const int64_t* qa;             // [n_res][Cp] quantityAsInt64(allocatable - allocated - allocating)
                                 // (general.go:403-427), kQaAbsent where not allocatable
  const int32_t* mg_tid;         // [kmax][Cp] model node group: template id (grade ascending)
  const int32_t* mg_cnt;         // [kmax][Cp] node count, clamped to MaxInt32 (0 = no group)
  const int64_t* tmpl;           // [n_tmpl][n_res] model template values
  const int32_t* mt_cnt;         // [n_tmpl][Cp] model nodes per template, clamped to MaxInt32, or
                                 // nullptr (n_tmpl > kTmplDense or a negative template value)
  const uint32_t* perm;          // rank -> caller index
  // Cluster bitsets ("postings" of every filter predicate, bit c of word c >> 6;
  // kp_filter.h): fixed rows (BR_*), the API-enablement row of each GVK, the row of
  // each taint list, then one row per (label key, value), provider, region and zone
  // value, found through an open-addressed table keyed by bits_key(). n_bits == 0:
  // not built (over budget, or more than kTsetRowsMax taint lists).
  const uint64_t* bits;          // [n_bits][W]
  int32_t n_bits;
  int32_t br_api, br_tset, br_lex;  // first row of: GVK rows, taint-list rows, label-exists rows
  const uint64_t* bkey;          // [bmask + 1] table keys (kBitsEmpty = free)
  const int32_t* bval;           // [bmask + 1] row of the key
  uint32_t bmask;
};

// Fixed bitset rows.
enum : int32_t {
  BR_BASE = 0,      // c < C and not deleting (findClustersThatFit, generic_scheduler.go:140-143)
  BR_HAS_PROVIDER,  // CF_HAS_PROVIDER (SpreadConstraint filter)
  BR_HAS_REGION,
  BR_HAS_ZONES,
  BR_PROV_SET,      // provider string id >= 0 (field selector Exists)
  BR_REG_SET,
  BR_ZONE_ANY,      // at least one zone (matchZones Exists)
  BR_FIXED
};
enum : uint64_t { BK_LABEL = 1, BK_PROVIDER = 2, BK_REGION = 3, BK_ZONE = 4 };
constexpr uint64_t kBitsEmpty = ~0ull;
constexpr int kTsetRowsMax = 64;  // taint lists answered by one ballot word per binding
KP_HD inline uint64_t bits_key(uint64_t kind, uint32_t slot, int32_t vid) {
  return (kind << 60) | ((uint64_t)slot << 32) | (uint64_t)(uint32_t)vid;
}
KP_HD inline uint32_t bits_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k;
}

struct BatchView {
  int32_t B;
  const BindHdr* hdr;
  const int32_t* ipool;
  const int64_t* lpool;
  const Tol* tols;
  const Prog* progs;
  const Instr* instrs;
};

}  // namespace kp
