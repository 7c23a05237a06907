// engine.cpp — host side of the kp placement engine: the C-ABI of
// include/kp/kp_api.h, the snapshot/binding packer, kernel orchestration on one
// HIP stream, and the host-kept selectGroups step of region spreading.
#include "kp_dev.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <tuple>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kp/kp_api.h"
#include "k8s.h"
#include "kp_layout.h"
#include "kp_launch.h"
#include "kp_paths.h"
#include "kp_pdq.h"
#include "kp_sets.h"
#include "kp_nodes.h"
#include "kp_top.h"

using namespace kp;

namespace {

std::string S(const kp_str& s) { return (s.ptr && s.len) ? std::string(s.ptr, s.len) : std::string(); }
std::string_view SV(const kp_str& s) { return (s.ptr && s.len) ? std::string_view(s.ptr, s.len) : std::string_view(); }
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// String-keyed hash table with string_view lookups for the packing hot path (names,
// dictionary strings, memo keys): open addressing with linear probing over a
// power-of-two slot array kept at most half full, one multiply-xorshift hash over
// 8-byte words per lookup, entries in a deque (stable addresses). find() returns the
// entry or nullptr (== end()); it->first / it->second as with std::unordered_map.
inline uint64_t sv_hash(std::string_view v) {
  const unsigned char* p = (const unsigned char*)v.data();
  size_t n = v.size();
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  uint64_t w = 0;
  memcpy(&w, p, n);
  h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 29;
  return h | 1;  // 0 marks an empty slot
}
template <class V>
class SvMap {
 public:
  struct Entry {
    std::string first;
    V second;
  };
  Entry* find(std::string_view k) {
    if (slots_.empty()) return nullptr;
    const uint64_t h = sv_hash(k);
    for (size_t i = h & mask_;; i = (i + 1) & mask_) {
      const Slot& sl = slots_[i];
      if (sl.h == 0) return nullptr;
      if (sl.h == h && ent_[sl.i].first == k) return &ent_[sl.i];
    }
  }
  const Entry* find(std::string_view k) const { return const_cast<SvMap*>(this)->find(k); }
  Entry* end() const { return nullptr; }
  template <class K, class W>
  std::pair<Entry*, bool> emplace(K&& k, W&& v) {
    if (Entry* e = find(std::string_view(k))) return {e, false};
    if (2 * (ent_.size() + 1) > slots_.size()) grow();
    ent_.push_back(Entry{std::string(std::forward<K>(k)), V(std::forward<W>(v))});
    put(sv_hash(ent_.back().first), (uint32_t)(ent_.size() - 1));
    return {&ent_.back(), true};
  }
  V& operator[](std::string_view k) { return emplace(std::string(k), V()).first->second; }
  size_t size() const { return ent_.size(); }

 private:
  struct Slot {
    uint64_t h = 0;
    uint32_t i = 0;
  };
  std::vector<Slot> slots_;
  std::deque<Entry> ent_;
  size_t mask_ = 0;
  void put(uint64_t h, uint32_t i) {
    size_t j = h & mask_;
    while (slots_[j].h != 0) j = (j + 1) & mask_;
    slots_[j] = Slot{h, i};
  }
  void grow() {
    const size_t cap = std::max<size_t>(16, 2 * slots_.size());
    slots_.assign(cap, Slot{});
    mask_ = cap - 1;
    for (uint32_t i = 0; i < (uint32_t)ent_.size(); i++) put(sv_hash(ent_[i].first), i);
  }
};

struct Dict {
  SvMap<int32_t> m;
  std::vector<std::string> names;
  int32_t add(const std::string& s) {
    auto it = m.find(s);
    if (it != m.end()) return it->second;
    int32_t id = (int32_t)names.size();
    m.emplace(s, id);
    names.push_back(s);
    return id;
  }
  int32_t get(std::string_view s) const {
    auto it = m.find(s);
    return it == m.end() ? -1 : it->second;
  }
};

// Process-wide pools of freed batch buffers: a batch's device arena (per device)
// and its page-locked result buffers go back here on kp_batch_destroy and the next
// batch of a fitting size takes them, so a stream of batches pays hipMalloc /
// hipHostMalloc (and the frees) once. A block is reused for requests of at least
// half its size. Each pool (one per device, one for page-locked host memory) keeps
// at most kPoolKeep blocks and kPoolBytes (device) / kPoolHostBytes (host) bytes,
// oldest evicted first: several engines' batches in flight (bench lanes, kp_multi)
// each hold an arena and two host buffers.
struct BufPool {
  static constexpr size_t kPoolKeep = 32;
  static constexpr size_t kPoolBytes = (size_t)16 << 30;     // per device (288 GB of HBM)
  static constexpr size_t kPoolHostBytes = (size_t)4 << 30;  // page-locked host memory
  std::mutex mu;
  std::vector<std::tuple<int, void*, size_t>> free;  // (device or -1 for host, pointer, bytes), oldest first
  void* get(int dev_id, size_t bytes, size_t* got) {
    std::lock_guard<std::mutex> g(mu);
    size_t best = (size_t)-1;
    for (size_t i = 0; i < free.size(); i++) {
      auto& [d, p, n] = free[i];
      if (d == dev_id && n >= bytes && n <= 2 * bytes + (1u << 20) && (best == (size_t)-1 || n < std::get<2>(free[best])))
        best = i;
    }
    if (best == (size_t)-1) return nullptr;
    void* p = std::get<1>(free[best]);
    *got = std::get<2>(free[best]);
    free.erase(free.begin() + (long)best);
    return p;
  }
  void put(int dev_id, void* p, size_t bytes) {
    if (!p) return;
    std::vector<std::tuple<int, void*, size_t>> drop;
    {
      std::lock_guard<std::mutex> g(mu);
      free.emplace_back(dev_id, p, bytes);
      size_t cnt = 0, tot = 0;
      for (auto& f : free)
        if (std::get<0>(f) == dev_id) cnt++, tot += std::get<2>(f);
      const size_t cap = dev_id < 0 ? kPoolHostBytes : kPoolBytes;
      for (size_t i = 0; i < free.size() && (cnt > kPoolKeep || tot > cap);) {  // the oldest of this pool go
        if (std::get<0>(free[i]) != dev_id) {
          i++;
          continue;
        }
        cnt--, tot -= std::get<2>(free[i]);
        drop.push_back(free[i]);
        free.erase(free.begin() + (long)i);
      }
    }
    for (auto& d : drop) {
      if (std::get<0>(d) < 0) dev::host_release(std::get<1>(d));
      else dev::release(std::get<1>(d));
    }
  }
};
BufPool& buf_pool() {
  static BufPool* p = new BufPool();  // never destroyed: buffers may return during exit
  return *p;
}
void* pinned_get(size_t bytes, size_t* got) {
  if (void* p = buf_pool().get(-1, bytes, got)) return p;
  void* p = nullptr;
  if (dev::host_alloc(&p, bytes)) return nullptr;
  *got = bytes;
  return p;
}

// One device allocation carved into aligned sub-buffers. pool_dev >= 0: the
// allocation comes from (and returns to) the batch-buffer pool of that device.
struct Arena {
  std::vector<std::pair<void**, size_t>> req;
  void* base = nullptr;
  size_t total = 0;
  int pool_dev = -1;
  size_t got = 0;
  template <class T>
  void add(T** p, size_t count) {
    req.push_back({(void**)p, count * sizeof(T)});
  }
  int alloc() {
    total = 0;
    for (auto& r : req) total += (r.second + 255) & ~(size_t)255;
    if (total == 0) total = 256;
    if (pool_dev >= 0) base = buf_pool().get(pool_dev, total, &got);
    if (!base) {
      if (dev::alloc(&base, total)) return -1;
      got = total;
    }
    char* p = (char*)base;
    for (auto& r : req) {
      *r.first = p;
      p += (r.second + 255) & ~(size_t)255;
    }
    return 0;
  }
  // One block of `bytes` with no sub-buffers (a replica's copy of another arena).
  int alloc_raw(size_t bytes) {
    req.clear();
    total = bytes ? bytes : 256;
    got = total;
    return dev::alloc(&base, total);
  }
  void drop() {
    if (!base) return;
    if (pool_dev >= 0) buf_pool().put(pool_dev, base, got);
    else dev::release(base);
    base = nullptr;
  }
  void reset() {
    drop();
    req.clear();
    total = 0;
  }
  ~Arena() { drop(); }
};

#define HIPCHK(x)                                                            \
  do {                                                                       \
    if ((x) != 0) {                                                          \
      e->err = std::string(#x) + ": " + dev::last_error();                   \
      return KP_EDEVICE;                                                     \
    }                                                                        \
  } while (0)

}  // namespace

// std::allocator that leaves trivial elements uninitialized on resize: the packer
// writes every BindHdr itself (in parallel, so the pages are first touched there),
// and a value-initializing resize would zero 160 B per binding on one thread.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};

// ============================================================================
// Engine / snapshot / batch objects
// ============================================================================
struct kp_engine {
  int device = 0;
  dev::stream_t stream = nullptr;   // select kernels, copies (the batch's result order)
  dev::stream_t stream2 = nullptr;  // pair kernel, then the SEL_ALL select kernel
  dev::stream_t stream3 = nullptr;  // the cluster-spread select kernel, beside the other selects
  dev::event_t ev[16] = {};
  std::string err;
  kp_stage_times times{};
  struct {  // kp_schedule_affinities results
    std::vector<int32_t> status, err, idx, attempts;
    std::vector<int64_t> arg;
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> cidx;
    std::vector<int32_t> rep;
  } aff;
  int n_threads = 8;
  size_t max_lds = 65536;
  // k_select_top (kp_top.h): on, and its subset capacity per binding (LDS entries);
  // KP_TOP=0 / KP_TOP_CAP=<n> at engine creation (tests, tuning)
  bool top_on = true;
  int top_cap = 832;       // subset capacity of the large slice (LDS: 8 workgroups of two waves per CU)
  int top_cap_small = 256;  // ... and of the small one (bindings needing <= kTopSmallNeed)
  // the large-slice bindings run at this capacity first (more waves per CU); those whose
  // subset outgrows it run again at top_cap (0 / >= top_cap: one launch at top_cap)
  int top_cap_mid = 0;
  bool top_split = true;    // the two slices' launches on two streams (KP_TOP_SPLIT=0: one)
  bool slow_order = true;   // k_slow orders candidates from the class orders (KP_SLOW_ORDER=0: sorts)
  // with a region chain (whose host steps synchronise anyway) the fallback kernels over
  // device-appended lists are launched only after their counts are read back, so none runs
  // with an empty list (KP_GATE_FB=0: always launched, each workgroup reading the count;
  // 2: only the SEL_ALL and cluster-spread fallbacks, at k_slow's existing count read,
  // not the region fallbacks, whose reads add two host waits to the region chain)
  int gate_fb = 1;
  // KP_ZC=1: k_compact writes the result CSR into the page-locked buffers over the bus
  // (no copy, no size read-back); measured slower with batches in flight (its workgroups
  // hold CUs while their stores cross the bus: 51-53 vs 71-85 M/s), so off
  bool zc = false;
  // KP_SPEC_COPY=1: a batch scheduled again copies its previous CSR size ahead of the
  // total's read-back (one host round trip per call); measured no better with batches in
  // flight (59.7-81.5 vs 69.2-88.9 M/s, same box), so off
  bool spec_copy = false;
  bool top_wg = false;      // large-subset bindings on k_select_top_wg (KP_TOP_WG=1; measured slower)
  // per-kernel timing of kp_schedule_batch (kp_engine_set_profile): an event pair
  // around every launch on its own stream, folded by kernel name after the batch
  struct KProf {
    const char* name;
    uint64_t units;  // bindings (or rows) the launch covered
    int units_stat;  // >= 0: the count is device-side, h_stats[units_stat]
  };
  bool prof = false;
  uint64_t submit_seq = 0;  // schedule calls submitted on this engine (stage timing validity)
  std::vector<dev::event_t> pev;
  std::vector<KProf> pk;
  std::vector<kp_kernel_time> ktimes;
};

// Snapshot epochs: unique per snapshot object and renewed when kp_snapshot_update grows
// its dictionaries, so packed records (kp_pack_cache) know which ids they resolved against.
static uint64_t next_snap_epoch() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}
struct kp_snapshot {
  kp_engine* e = nullptr;
  uint64_t epoch = next_snap_epoch();
  kp_options opts{};
  int C = 0, Cp = 0, W = 0;
  Dict str, keys, gvk, res, regions;
  SvMap<int32_t> rank_of;  // cluster name -> rank
  std::vector<uint32_t> perm;                        // rank -> caller index
  std::vector<int32_t> inv;                          // caller index -> rank
  int32_t rid_cpu = -1, rid_mem = -1, rid_eph = -1;
  int n_tmpl = 0, kmax = 0;
  int est_kind = 0;  // EST_* pair-kernel instance the clusters allow (snapshot_est_kind)
  std::vector<std::string> names;  // cluster names in rank order
  std::vector<unsigned char> blob;  // kp_snapshot_export buffer
  // host copies
  std::vector<uint32_t> flags;
  std::vector<int32_t> provider, region, region_idx, zone_off, zone_ids, label_val, taint_off, taint_key, taint_val,
      taint_eff, mgrp_off, mgrp_tid, mg_tid, mg_cnt;
  std::vector<int64_t> provider_int, region_int, allowed, avail, mgrp_cnt, tmpl;
  std::vector<int64_t> qa;  // [R][Cp] quantityAsInt64 availability, kQaAbsent where not allocatable
  std::vector<uint64_t> api_bits;
  Arena dev;
  SnapView view{};
};

// diagnostic builds: phase stamps and counters, kDbgSlots x kDbgSpread (kp_select.h)
// The state schedule_submit leaves for schedule_finish (one submitted call per batch).
struct SchedPend {
  bool live = false, empty = false, zc = false, bits = false, top = false, spread_orders = false;
  int fast = 0;
  double t0 = 0, th0 = 0, th1 = 0;
  uint64_t spec = 0, seq = 0;
  dev::event_t ev = nullptr;  // recorded after the call's last read-back (kept across calls)
};

struct kp_batch {
  kp_snapshot* snap = nullptr;
  int B = 0;
  std::vector<BindHdr, NoInitAlloc<BindHdr>> hdr;
  std::vector<int32_t> ipool;
  std::vector<int64_t> lpool;
  std::vector<Tol> tols;
  std::vector<Prog> progs;
  std::vector<Instr> instrs;
  std::vector<int32_t> l_all, l_cluster, l_region, l_slow, l_cs;  // l_cs: cluster + region bindings
  int n_all_dyn = 0;  // l_all = [other strategies | StaticWeight]: the first n_all_dyn are not StaticWeight
  int n_top_small = 0;  // of those, the first n_top_small take k_select_top's small slice
  int n_static = 0;   // of the StaticWeight ones, the first n_static take k_select_static (static_ok)
  uint64_t out_cap = 0;
  std::vector<uint8_t> route;     // RT_* per binding (pack_parallel)
  int max_tgt = 0, max_tiers = 1;  // over the batch's headers (pack_parallel)
  Arena dev;
  BatchView view{};
  // device work buffers
  uint64_t* fmask = nullptr;
  int32_t* est = nullptr;  // [B][Cp] per-binding rows (allocated on first use: rows mode, diagnosis entries)
  // estimator classes (kp_filter.h): class of each binding (0 = non-workload) and
  // a representative binding per class; their raw GeneralEstimator rows [n][Cp]
  std::vector<int32_t> bcls, crep;
  int32_t *d_bcls = nullptr, *d_crep = nullptr, *cls_rows = nullptr;
  int32_t* d_all_cls = nullptr;  // the estimator class of each l_all entry (KArgs::lcls)
  std::vector<int32_t> l_all_cls;
  // Estimator classes serving one binding, in a batch without class orders (est_single):
  // their rows hold only that binding's feasible clusters, written after k_filter
  // (k_est_class over l_cls_single with the feasibility rows); l_cls_full: the others.
  bool est_single = false;
  std::vector<int32_t> l_cls_full, l_cls_single;
  int32_t *d_cls_full = nullptr, *d_cls_single = nullptr;
  // component-set classes (BF_SETS): class id and resolved component list of each;
  // their rows are MaxAvailableComponentSets per cluster (k_sets_rows), and in the
  // pair-row mode the BF_SETS bindings' rows are rebuilt from them (k_rows_from_class)
  // k_select_top: per-class candidate orders, row sums and walkability; its fallback list
  uint64_t* d_ord = nullptr;
  int64_t* d_ctot = nullptr;
  int32_t *d_cok = nullptr, *d_fb = nullptr, *d_ofb = nullptr;
  int32_t *d_fbc = nullptr, *d_fbr = nullptr;  // k_spread_order's fallback lists (cluster / region positions)
  int32_t* d_fba = nullptr;                     // k_region_a_order's fallback list
  std::vector<int32_t> sets_cls, l_sets;
  std::vector<SetsArgs> sets_args;
  SetsArgs* d_sets_args = nullptr;
  int64_t *d_sets_off = nullptr, *d_sets_scratch = nullptr;
  uint32_t* d_sets_ovf = nullptr;  // [sets_cls] per component-set class: overflowing rank + 1, or 0
  int32_t* d_sets_list = nullptr;
  std::string err;  // packing error text
  int32_t *d_all = nullptr, *d_cluster = nullptr, *d_region = nullptr, *d_slowlist = nullptr, *d_cs = nullptr;
  int32_t *status = nullptr, *errc = nullptr, *slow = nullptr;
  int64_t* arg = nullptr;
  uint64_t* start = nullptr;
  uint32_t* count = nullptr;
  unsigned long long* counter = nullptr;
  uint32_t* stats = nullptr;
  unsigned long long* dbg = nullptr;
  // launch arguments of the kernels that read them through a pointer (kp_launch.h
  // SelectExtra::dargs): kArgSlots device slots and their page-locked host staging
  KArgs* d_kargs = nullptr;
  KArgs* h_kargs = nullptr;
  size_t h_kargs_bytes = 0;
  uint32_t h_stats[20] = {};  // [0..7] slow-path counts, [8] component-set simulation overflow, [9] k_select_top
                              // fallbacks, [10] / [11] cluster- / region-spread bindings selected over the class order,
                              // [12] / [13] k_spread_order's fallback list lengths, [14] k_region_a_order's
                              // [16] k_select_top's capacity overflows (the top_cap_mid launch)
  uint32_t* out_idx = nullptr;
  int32_t* out_rep = nullptr;
  uint64_t* offsets_d = nullptr;
  uint64_t* off_part = nullptr;  // per-chunk totals of the offsets scan
  uint32_t* cidx_d = nullptr;
  int32_t* crep_d = nullptr;
  RegionOut* rout = nullptr;
  int32_t *rstat = nullptr, *rsel = nullptr, *rnsel = nullptr;
  uint32_t* nhost = nullptr;  // region bindings the device group search left to the host
  unsigned char* slow_scratch = nullptr;
  size_t slow_slot = 0;
  int slow_grid = 0, slow_cap = 0, slow_lds = 0, slow_sort = 0;
  bool fast_ok = false;  // the batch half of the fast pair-kernel condition (batch_fast_ok)
  int n_regions = 0;     // the snapshot's region count the region buffers were sized for
  // host results
  std::vector<int32_t> h_status, h_err, h_rstat, h_rsel, h_rnsel;
  std::vector<int64_t> h_arg;
  std::vector<uint64_t> h_start, h_offsets;
  std::vector<uint32_t> h_count;
  // result CSR in page-locked host memory (h_res_cap entries each)
  uint32_t* h_cidx = nullptr;
  int32_t* h_crep = nullptr;
  uint64_t h_res_cap = 0;
  uint64_t last_tot = 0;  // the previous call's CSR size (the speculative copy)
  SchedPend pend;         // a submitted call (schedule_submit) awaiting schedule_finish
  size_t h_cidx_bytes = 0, h_crep_bytes = 0;  // their pooled block sizes
  // The batch's device arena and page-locked buffers go back to the process-wide
  // pools on destruction, where another batch (of any engine) may take them at
  // once. An entry point that fails part-way leaves kernels queued that still
  // use them: it records these events on the engine's streams (batch_fence), and
  // destruction waits for them. kp_batch_create does the same through
  // create_stream while it runs.
  dev::event_t fence[3] = {};
  bool fenced = false;
  dev::stream_t create_stream = nullptr;
  void quiesce() {
    if (create_stream) (void)dev::sync(create_stream);
    create_stream = nullptr;
    for (auto& ev : fence)
      if (ev) {
        if (fenced) (void)dev::event_sync(ev);
        dev::event_destroy(ev);
        ev = nullptr;
      }
    fenced = false;
    if (pend.ev) {  // a submitted call never collected: its work uses the buffers
      if (pend.live) (void)dev::event_sync(pend.ev);
      dev::event_destroy(pend.ev);
      pend.ev = nullptr;
    }
    pend.live = false;
  }
  ~kp_batch() {
    quiesce();
    buf_pool().put(-1, h_cidx, h_cidx_bytes);
    buf_pool().put(-1, h_crep, h_crep_bytes);
    buf_pool().put(-1, h_kargs, h_kargs_bytes);
    if (est) dev::release(est);
  }
  std::vector<RegionOut> h_rout;
};

int build_sets_args(const kp_snapshot* s, const kp_component* comps, uint32_t K, SetsArgs* A, std::string* err);

// ============================================================================
// Snapshot packing (cache.Snapshot, cache.go:124-139, packed once)
// ============================================================================
namespace {

typedef std::map<std::string, k8s::Qty> QtyMap;
bool qmap(const kp_resource* r, uint32_t n, QtyMap* m) {
  bool ok = true;
  for (uint32_t i = 0; i < n; i++) {
    k8s::Qty q;
    if (!k8s::parse_quantity(S(r[i].quantity), &q)) ok = false;
    (*m)[S(r[i].name)] = q;
  }
  return ok;
}

int upload_snapshot(kp_engine* e, kp_snapshot* s);
int snapshot_est_kind(const kp_snapshot* s);

// One cluster's packed row before it is laid out in the snapshot columns
// (shared by kp_snapshot_create and kp_snapshot_update). Dictionary ids are
// taken with Dict::add: create has filled the dictionaries already (pass 1),
// an update may append to them.
struct ClusterRow {
  uint32_t flags = 0;
  int32_t provider = -1, region = -1;
  int64_t provider_int = 0, region_int = 0;
  std::vector<int32_t> zones;
  std::vector<std::pair<int32_t, int32_t>> labels;  // (key id, value id), later entries win
  std::vector<std::array<int32_t, 3>> taints;       // (key, value, effect), NoSchedule/NoExecute only
  std::vector<int32_t> gvks;
  int64_t allowed = 0;
  std::vector<std::pair<int32_t, int64_t>> avail;   // (resource id, available)
  std::vector<std::pair<int32_t, int64_t>> qa;      // (resource id, quantityAsInt64 availability)
  std::vector<std::pair<int32_t, int64_t>> groups;  // (template id, node count), grades ascending
};

int pack_row(kp_engine* e, kp_snapshot* s, const kp_cluster& c, std::map<std::vector<int64_t>, int32_t>& tmpl_ids,
             ClusterRow* out) {
  ClusterRow& w = *out;
  w = ClusterRow();
  uint32_t f = 0;
  if (c.deleting) f |= CF_DELETING;
  std::string prov = S(c.provider), reg = S(c.region);
  if (!prov.empty()) {
    f |= CF_HAS_PROVIDER;
    w.provider = s->str.add(prov);
    int64_t v;
    if (k8s::parse_int64(prov, &v)) {
      f |= CF_PROVIDER_INT;
      w.provider_int = v;
    }
  }
  if (!reg.empty()) {
    f |= CF_HAS_REGION;
    w.region = s->str.add(reg);
    int64_t v;
    if (k8s::parse_int64(reg, &v)) {
      f |= CF_REGION_INT;
      w.region_int = v;
    }
  }
  if (c.n_zones) f |= CF_HAS_ZONES;
  for (uint32_t i = 0; i < c.n_zones; i++) w.zones.push_back(s->str.add(S(c.zones[i])));
  for (uint32_t i = 0; i < c.n_labels; i++)
    w.labels.push_back({s->keys.add(S(c.labels[i].key)), s->str.add(S(c.labels[i].value))});
  for (uint32_t i = 0; i < c.n_taints; i++) {
    std::string eff = S(c.taints[i].effect);
    int32_t ef = eff == "NoSchedule" ? EFF_NOSCHEDULE : (eff == "NoExecute" ? EFF_NOEXECUTE : 0);
    if (!ef) continue;  // only NoSchedule/NoExecute are filtered (taint_toleration.go:65-67)
    w.taints.push_back({s->str.add(S(c.taints[i].key)), s->str.add(S(c.taints[i].value)), ef});
  }
  for (uint32_t i = 0; i < c.n_api_enablements; i++)
    w.gvks.push_back(s->gvk.add(S(c.api_enablements[i].group_version) + '\0' + S(c.api_enablements[i].kind)));
  if (c.has_resource_summary) {
    f |= CF_HAS_SUMMARY;
    QtyMap al, ad, ag;
    bool ok = qmap(c.allocatable, c.n_allocatable, &al) & qmap(c.allocated, c.n_allocated, &ad) &
              qmap(c.allocating, c.n_allocating, &ag);
    if (!ok) {
      e->err = "unparsable quantity in cluster " + S(c.name);
      return KP_EINVAL;
    }
    auto pods = [](const QtyMap& m) {
      auto it = m.find("pods");
      return it == m.end() ? 0 : k8s::value(it->second);
    };
    int64_t allowed = pods(al) - pods(ad) - pods(ag);  // getAllowedPodNumber (general.go:445-463)
    w.allowed = allowed > 0 ? allowed : 0;
    for (auto& kv : al) {  // getMaximumReplicasBasedOnClusterSummary operands (general.go:465-505)
      k8s::Qty q = kv.second;
      auto x = ad.find(kv.first);
      if (x != ad.end()) q.nano -= x->second.nano;
      x = ag.find(kv.first);
      if (x != ag.end()) q.nano -= x->second.nano;
      int64_t v = k8s::value(q);
      int64_t d = v <= 0 ? 0 : (kv.first == "cpu" ? k8s::milli(q) : v);
      w.avail.push_back({s->res.add(kv.first), d});
      // availableResourceMap (general.go:403-415): Sub keeps the allocatable's format
      k8s::Qty a = kv.second;
      if ((x = ad.find(kv.first)) != ad.end()) k8s::qsub(a, x->second);
      if ((x = ag.find(kv.first)) != ag.end()) k8s::qsub(a, x->second);
      w.qa.push_back({s->res.add(kv.first), k8s::as_int64(a)});
    }
    // buildModelNodes (general.go:296-361)
    if (s->opts.customized_cluster_resource_modeling && c.n_allocatable_modelings > 0 && c.n_resource_models > 0) {
      bool neg = false;
      std::map<uint32_t, int64_t> cnt;
      for (uint32_t i = 0; i < c.n_allocatable_modelings; i++) {
        if (c.allocatable_modelings[i].count < 0) neg = true;
        cnt[c.allocatable_modelings[i].grade] += c.allocatable_modelings[i].count;
      }
      if (!neg) {
        std::map<uint32_t, std::map<int32_t, int64_t>> caps;  // grade -> (resource id -> min)
        for (uint32_t m = 0; m < c.n_resource_models; m++) {
          QtyMap rl;
          for (uint32_t j = 0; j < c.resource_models[m].n_ranges; j++) {
            k8s::Qty q;
            if (!k8s::parse_quantity(S(c.resource_models[m].ranges[j].min), &q)) {
              e->err = "unparsable resource model quantity";
              return KP_EINVAL;
            }
            rl[S(c.resource_models[m].ranges[j].name)] = q;
          }
          std::map<int32_t, int64_t> t;
          for (auto& kv : rl) {  // util.NewResource (resource.go:46-75); pods forced to 110
            const std::string& nm = kv.first;
            int32_t rid = s->res.add(nm);
            if (nm == "cpu") t[rid] += k8s::milli(kv.second);
            else if (nm == "memory" || nm == "ephemeral-storage") t[rid] += k8s::value(kv.second);
            else if (nm == "pods") continue;
            else if (k8s::scalar_resource(nm)) t[rid] += k8s::value(kv.second);
          }
          caps[c.resource_models[m].grade] = t;
        }
        const int R = (int)s->res.names.size();
        for (auto& kv : caps) {  // grades ascending
          auto it = cnt.find(kv.first);
          int64_t k = it == cnt.end() ? 0 : it->second;
          if (k == 0) continue;
          std::vector<int64_t> t(R, 0);
          for (auto& rv : kv.second) t[rv.first] = rv.second;
          while (!t.empty() && t.back() == 0) t.pop_back();  // key independent of the resource count
          auto ti = tmpl_ids.find(t);
          int32_t tid;
          if (ti == tmpl_ids.end()) {
            tid = (int32_t)tmpl_ids.size();
            tmpl_ids.emplace(t, tid);
          } else {
            tid = ti->second;
          }
          w.groups.push_back({tid, k});
        }
        f |= CF_MODEL_OK;
      }
    }
  }
  w.flags = f;
  return KP_OK;
}

// Lays rows[0..C) (rank order) out in the snapshot's columns and derived arrays.
void apply_rows(kp_snapshot* s, const std::vector<ClusterRow>& rows,
                const std::map<std::vector<int64_t>, int32_t>& tmpl_ids) {
  const int C = s->C, Cp = s->Cp;
  const int K = (int)s->keys.names.size(), AW = ((int)s->gvk.names.size() + 63) / 64, R = (int)s->res.names.size();
  // regions in name order (region_idx); an update may have added names
  std::vector<std::string> regs;
  for (int r = 0; r < C; r++)
    if (rows[r].region >= 0) regs.push_back(s->str.names[rows[r].region]);
  std::sort(regs.begin(), regs.end());
  regs.erase(std::unique(regs.begin(), regs.end()), regs.end());
  s->regions = Dict();
  for (auto& r : regs) s->regions.add(r);
  s->flags.assign(Cp, 0);
  s->provider.assign(Cp, -1);
  s->region.assign(Cp, -1);
  s->region_idx.assign(Cp, -1);
  s->provider_int.assign(Cp, 0);
  s->region_int.assign(Cp, 0);
  s->label_val.assign((size_t)std::max(K, 1) * Cp, -1);
  s->api_bits.assign((size_t)std::max(AW, 1) * Cp, 0);
  s->allowed.assign(Cp, 0);
  s->avail.assign((size_t)std::max(R, 1) * Cp, 0);
  s->qa.assign((size_t)std::max(R, 1) * Cp, kQaAbsent);
  s->zone_off.assign(C + 1, 0);
  s->taint_off.assign(C + 1, 0);
  s->mgrp_off.assign(C + 1, 0);
  s->zone_ids.clear();
  s->taint_key.clear();
  s->taint_val.clear();
  s->taint_eff.clear();
  s->mgrp_tid.clear();
  s->mgrp_cnt.clear();
  for (int r = 0; r < C; r++) {
    const ClusterRow& w = rows[r];
    s->flags[r] = w.flags;
    s->provider[r] = w.provider;
    s->provider_int[r] = w.provider_int;
    s->region[r] = w.region;
    s->region_int[r] = w.region_int;
    if (w.region >= 0) s->region_idx[r] = s->regions.get(s->str.names[w.region]);
    for (int32_t z : w.zones) s->zone_ids.push_back(z);
    s->zone_off[r + 1] = (int32_t)s->zone_ids.size();
    for (auto& kv : w.labels) s->label_val[(size_t)kv.first * Cp + r] = kv.second;  // map semantics: later wins
    for (auto& t : w.taints) {
      s->taint_key.push_back(t[0]);
      s->taint_val.push_back(t[1]);
      s->taint_eff.push_back(t[2]);
    }
    s->taint_off[r + 1] = (int32_t)s->taint_key.size();
    for (int32_t g : w.gvks) s->api_bits[(size_t)(g >> 6) * Cp + r] |= 1ull << (g & 63);
    s->allowed[r] = w.allowed;
    for (auto& kv : w.avail) s->avail[(size_t)kv.first * Cp + r] = kv.second;
    for (auto& kv : w.qa) s->qa[(size_t)kv.first * Cp + r] = kv.second;
    for (auto& g : w.groups) {
      s->mgrp_tid.push_back(g.first);
      s->mgrp_cnt.push_back(g.second);
    }
    s->mgrp_off[r + 1] = (int32_t)s->mgrp_tid.size();
  }
  s->n_tmpl = (int)tmpl_ids.size();
  s->tmpl.assign((size_t)std::max(s->n_tmpl, 1) * std::max(R, 1), 0);
  for (auto& kv : tmpl_ids)  // (vectors of an earlier, shorter resource list read as zero-padded)
    for (int j = 0; j < R && j < (int)kv.first.size(); j++) s->tmpl[(size_t)kv.second * R + j] = kv.first[j];
  auto pad1 = [](auto& v) {
    if (v.empty()) v.resize(1);
  };
  pad1(s->zone_ids);
  pad1(s->taint_key);
  pad1(s->taint_val);
  pad1(s->taint_eff);
  // model groups transposed to [kmax][Cp] so a wave reads 64 clusters' k-th group coalesced
  int& kmax = s->kmax;
  kmax = 0;
  for (int r = 0; r < C; r++) kmax = std::max(kmax, s->mgrp_off[r + 1] - s->mgrp_off[r]);
  s->mg_tid.assign((size_t)std::max(kmax, 1) * Cp, 0);
  s->mg_cnt.assign((size_t)std::max(kmax, 1) * Cp, 0);
  for (int r = 0; r < C; r++)
    for (int g = s->mgrp_off[r]; g < s->mgrp_off[r + 1]; g++) {
      size_t k = (size_t)(g - s->mgrp_off[r]);
      s->mg_tid[k * Cp + r] = s->mgrp_tid[g];
      s->mg_cnt[k * Cp + r] = (int32_t)std::min<int64_t>(s->mgrp_cnt[g], kInt32Max);
    }
}

int build_snapshot(kp_engine* e, const kp_cluster* cl, uint64_t n, const kp_options* o, kp_snapshot* s) {
  s->opts = o ? *o : kp_options{0, 1, 0, KP_PLUGIN_ALL};
  if (n > (uint64_t)kMaxClusters) {
    e->err = "too many clusters";
    return KP_ENOTSUP;
  }
  const int C = (int)n;
  s->C = C;
  s->Cp = ((C + 63) / 64) * 64;
  if (s->Cp == 0) s->Cp = 64;
  s->W = s->Cp / 64;
  std::vector<uint32_t> order(C);
  std::vector<std::string> names(C);
  for (int i = 0; i < C; i++) {
    order[i] = i;
    names[i] = S(cl[i].name);
  }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return names[a] < names[b]; });
  s->perm = order;
  s->inv.assign(C, -1);
  for (int r = 0; r < C; r++) {
    s->inv[order[r]] = r;
    if (!s->rank_of.emplace(names[order[r]], r).second) {
      e->err = "duplicate cluster name " + names[order[r]];
      return KP_EINVAL;
    }
  }
  // pass 1: dictionaries
  for (int r = 0; r < C; r++) {
    const kp_cluster& c = cl[order[r]];
    for (uint32_t i = 0; i < c.n_labels; i++) {
      s->keys.add(S(c.labels[i].key));
      s->str.add(S(c.labels[i].value));
    }
    s->str.add(S(c.provider));
    s->str.add(S(c.region));
    for (uint32_t i = 0; i < c.n_zones; i++) s->str.add(S(c.zones[i]));
    for (uint32_t i = 0; i < c.n_taints; i++) {
      s->str.add(S(c.taints[i].key));
      s->str.add(S(c.taints[i].value));
    }
    for (uint32_t i = 0; i < c.n_api_enablements; i++)
      s->gvk.add(S(c.api_enablements[i].group_version) + '\0' + S(c.api_enablements[i].kind));
    for (uint32_t i = 0; i < c.n_allocatable; i++) s->res.add(S(c.allocatable[i].name));
    for (uint32_t m = 0; m < c.n_resource_models; m++)
      for (uint32_t j = 0; j < c.resource_models[m].n_ranges; j++) s->res.add(S(c.resource_models[m].ranges[j].name));
  }
  s->rid_cpu = s->res.add("cpu");
  s->rid_mem = s->res.add("memory");
  s->rid_eph = s->res.add("ephemeral-storage");
  std::map<std::vector<int64_t>, int32_t> tmpl_ids;
  std::vector<ClusterRow> rows(C);
  for (int r = 0; r < C; r++) {
    int rc = pack_row(e, s, cl[order[r]], tmpl_ids, &rows[r]);
    if (rc) return rc;
  }
  apply_rows(s, rows, tmpl_ids);
  s->names.resize(C);
  for (int r = 0; r < C; r++) s->names[r] = names[order[r]];
  return upload_snapshot(e, s);
}

// Device copy of a packed snapshot (kp_snapshot_create and kp_snapshot_import).
int upload_snapshot(kp_engine* e, kp_snapshot* s) {
  const int C = s->C, Cp = s->Cp, kmax = s->kmax;
  const int K = (int)s->keys.names.size(), AW = ((int)s->gvk.names.size() + 63) / 64,
            R = (int)s->res.names.size();
  SnapView& v = s->view;
  v.C = C;
  v.Cp = Cp;
  v.W = s->W;
  v.n_label_keys = K;
  v.api_words = AW;
  v.n_res = R;
  v.n_tmpl = s->n_tmpl;
  v.n_regions = (int)s->regions.names.size();
  Arena& a = s->dev;
  uint32_t *d_flags, *d_perm;
  int32_t *d_prov, *d_reg, *d_regidx, *d_zoff, *d_zid, *d_lbl, *d_toff, *d_tk, *d_tv, *d_te, *d_mtid, *d_mcnt;
  int64_t *d_pint, *d_rint, *d_allowed, *d_avail, *d_tmpl, *d_qa;
  uint64_t* d_api;
  // taint lists deduplicated: one TaintToleration answer per distinct list and binding
  std::vector<int32_t> tset(Cp, 0), trep;
  {
    std::map<std::vector<int32_t>, int32_t> ids;
    std::vector<int32_t> key;
    for (int r = 0; r < C; r++) {
      key.clear();
      for (int t = s->taint_off[r]; t < s->taint_off[r + 1]; t++) {
        key.push_back(s->taint_key[t]);
        key.push_back(s->taint_val[t]);
        key.push_back(s->taint_eff[t]);
      }
      auto it = ids.find(key);
      if (it == ids.end()) {
        it = ids.emplace(key, (int32_t)trep.size()).first;
        trep.push_back(r);
      }
      tset[r] = it->second;
    }
    if (trep.empty()) trep.push_back(0);
  }
  int32_t *d_tset, *d_trep, *d_mt = nullptr;
  // Cluster bitsets of the filter predicates (kp_filter.h; SnapView::bits).
  std::vector<uint64_t> bits, bkey;
  std::vector<int32_t> bval;
  int32_t n_bits = 0, br_api = 0, br_tset = 0, br_lex = 0;
  const int W = s->W;
  if (W > 0 && (int)trep.size() <= kTsetRowsMax) {
    const int G = (int)s->gvk.names.size();
    std::unordered_map<uint64_t, int32_t> row_of;
    std::vector<std::pair<uint64_t, int32_t>> order;  // (key, cluster) in row-assignment order
    br_api = BR_FIXED;
    br_tset = br_api + G;
    br_lex = br_tset + (int)trep.size();
    int32_t next = br_lex + K;
    auto key_row = [&](uint64_t key) {
      auto it = row_of.find(key);
      if (it != row_of.end()) return it->second;
      row_of.emplace(key, next);
      return next++;
    };
    std::vector<std::pair<int32_t, int>> sets;  // (row, cluster) of the hashed rows
    for (int k = 0; k < K; k++)
      for (int r = 0; r < C; r++) {
        const int32_t v = s->label_val[(size_t)k * Cp + r];
        if (v >= 0) sets.push_back({key_row(bits_key(BK_LABEL, (uint32_t)k, v)), r});
      }
    for (int r = 0; r < C; r++) {
      if (s->provider[r] >= 0) sets.push_back({key_row(bits_key(BK_PROVIDER, 0, s->provider[r])), r});
      if (s->region[r] >= 0) sets.push_back({key_row(bits_key(BK_REGION, 0, s->region[r])), r});
      for (int z = s->zone_off[r]; z < s->zone_off[r + 1]; z++)
        sets.push_back({key_row(bits_key(BK_ZONE, 0, s->zone_ids[z])), r});
    }
    // within budget: the rows stay a small fraction of HBM even at large C
    if ((uint64_t)next * (uint64_t)W * 8 <= ((uint64_t)256 << 20)) {
      n_bits = next;
      bits.assign((size_t)n_bits * W, 0);
      auto set = [&](int32_t row, int r) { bits[(size_t)row * W + (r >> 6)] |= 1ull << (r & 63); };
      for (int r = 0; r < C; r++) {
        const uint32_t f = s->flags[r];
        if (!(f & CF_DELETING)) set(BR_BASE, r);
        if (f & CF_HAS_PROVIDER) set(BR_HAS_PROVIDER, r);
        if (f & CF_HAS_REGION) set(BR_HAS_REGION, r);
        if (f & CF_HAS_ZONES) set(BR_HAS_ZONES, r);
        if (s->provider[r] >= 0) set(BR_PROV_SET, r);
        if (s->region[r] >= 0) set(BR_REG_SET, r);
        if (s->zone_off[r + 1] > s->zone_off[r]) set(BR_ZONE_ANY, r);
        for (int g = 0; g < G; g++)
          if ((s->api_bits[(size_t)(g >> 6) * Cp + r] >> (g & 63)) & 1ull) set(br_api + g, r);
        set(br_tset + tset[r], r);
        for (int k = 0; k < K; k++)
          if (s->label_val[(size_t)k * Cp + r] >= 0) set(br_lex + k, r);
      }
      for (auto& x : sets) set(x.first, x.second);
      size_t tsz = 16;
      while (tsz < 2 * row_of.size()) tsz <<= 1;
      bkey.assign(tsz, kBitsEmpty);
      bval.assign(tsz, -1);
      for (auto& kv : row_of) {
        uint32_t i = bits_hash(kv.first) & (uint32_t)(tsz - 1);
        while (bkey[i] != kBitsEmpty) i = (i + 1) & (uint32_t)(tsz - 1);
        bkey[i] = kv.first;
        bval[i] = kv.second;
      }
    }
  }
  uint64_t *d_bits = nullptr, *d_bkey = nullptr;
  int32_t* d_bval = nullptr;
  // model node counts per (template, cluster): the fast estimator's dense form
  std::vector<int32_t> mt;
  {
    bool dense = s->n_tmpl > 0 && s->n_tmpl <= kTmplDense;
    for (int64_t x : s->tmpl) dense = dense && x >= 0;
    if (dense) {
      std::vector<int64_t> acc((size_t)kTmplDense * Cp, 0);  // rows past n_tmpl stay zero
      for (int k = 0; k < kmax; k++)
        for (int r = 0; r < C; r++) {
          const int32_t cnt = s->mg_cnt[(size_t)k * Cp + r];
          if (cnt) acc[(size_t)s->mg_tid[(size_t)k * Cp + r] * Cp + r] += cnt;
        }
      mt.resize(acc.size());
      for (size_t i = 0; i < acc.size(); i++) mt[i] = (int32_t)std::min<int64_t>(acc[i], kInt32Max);
    }
  }
  a.add(&d_flags, Cp);
  a.add(&d_tset, Cp);
  a.add(&d_trep, trep.size());
  if (!mt.empty()) a.add(&d_mt, mt.size());
  a.add(&d_perm, Cp);
  a.add(&d_prov, Cp);
  a.add(&d_reg, Cp);
  a.add(&d_regidx, Cp);
  a.add(&d_zoff, C + 1);
  a.add(&d_zid, s->zone_ids.size());
  a.add(&d_lbl, s->label_val.size());
  a.add(&d_toff, C + 1);
  a.add(&d_tk, s->taint_key.size());
  a.add(&d_tv, s->taint_val.size());
  a.add(&d_te, s->taint_eff.size());
  a.add(&d_mtid, s->mg_tid.size());
  a.add(&d_mcnt, s->mg_cnt.size());
  a.add(&d_pint, Cp);
  a.add(&d_rint, Cp);
  a.add(&d_allowed, Cp);
  a.add(&d_avail, s->avail.size());
  a.add(&d_qa, s->qa.size());
  a.add(&d_tmpl, s->tmpl.size());
  a.add(&d_api, s->api_bits.size());
  if (n_bits) {
    a.add(&d_bits, bits.size());
    a.add(&d_bkey, bkey.size());
    a.add(&d_bval, bval.size());
  }
  HIPCHK(a.alloc());
  std::vector<uint32_t> permp(Cp, 0);
  for (int r = 0; r < C; r++) permp[r] = s->perm[r];
  auto up = [&](void* d, const void* h, size_t bytes) { return dev::h2d(d, h, bytes, e->stream); };
  HIPCHK(up(d_flags, s->flags.data(), 4 * Cp));
  HIPCHK(up(d_tset, tset.data(), 4 * Cp));
  HIPCHK(up(d_trep, trep.data(), 4 * trep.size()));
  if (!mt.empty()) HIPCHK(up(d_mt, mt.data(), 4 * mt.size()));
  HIPCHK(up(d_perm, permp.data(), 4 * Cp));
  HIPCHK(up(d_prov, s->provider.data(), 4 * Cp));
  HIPCHK(up(d_reg, s->region.data(), 4 * Cp));
  HIPCHK(up(d_regidx, s->region_idx.data(), 4 * Cp));
  HIPCHK(up(d_zoff, s->zone_off.data(), 4 * (C + 1)));
  HIPCHK(up(d_zid, s->zone_ids.data(), 4 * s->zone_ids.size()));
  HIPCHK(up(d_lbl, s->label_val.data(), 4 * s->label_val.size()));
  HIPCHK(up(d_toff, s->taint_off.data(), 4 * (C + 1)));
  HIPCHK(up(d_tk, s->taint_key.data(), 4 * s->taint_key.size()));
  HIPCHK(up(d_tv, s->taint_val.data(), 4 * s->taint_val.size()));
  HIPCHK(up(d_te, s->taint_eff.data(), 4 * s->taint_eff.size()));
  HIPCHK(up(d_mtid, s->mg_tid.data(), 4 * s->mg_tid.size()));
  HIPCHK(up(d_mcnt, s->mg_cnt.data(), 4 * s->mg_cnt.size()));
  HIPCHK(up(d_pint, s->provider_int.data(), 8 * Cp));
  HIPCHK(up(d_rint, s->region_int.data(), 8 * Cp));
  HIPCHK(up(d_allowed, s->allowed.data(), 8 * Cp));
  HIPCHK(up(d_avail, s->avail.data(), 8 * s->avail.size()));
  HIPCHK(up(d_qa, s->qa.data(), 8 * s->qa.size()));
  HIPCHK(up(d_tmpl, s->tmpl.data(), 8 * s->tmpl.size()));
  HIPCHK(up(d_api, s->api_bits.data(), 8 * s->api_bits.size()));
  if (n_bits) {
    HIPCHK(up(d_bits, bits.data(), 8 * bits.size()));
    HIPCHK(up(d_bkey, bkey.data(), 8 * bkey.size()));
    HIPCHK(up(d_bval, bval.data(), 4 * bval.size()));
  }
  HIPCHK(dev::sync(e->stream));
  v.flags = d_flags;
  v.perm = d_perm;
  v.provider = d_prov;
  v.region = d_reg;
  v.region_idx = d_regidx;
  v.provider_int = d_pint;
  v.region_int = d_rint;
  v.zone_off = d_zoff;
  v.zone_ids = d_zid;
  v.label_val = d_lbl;
  v.taint_off = d_toff;
  v.taint_key = d_tk;
  v.taint_val = d_tv;
  v.taint_eff = d_te;
  v.taint_set = d_tset;
  v.tset_rep = d_trep;
  v.n_tsets = (int32_t)trep.size();
  v.api_bits = d_api;
  v.allowed = d_allowed;
  v.avail = d_avail;
  v.qa = d_qa;
  v.kmax = kmax;
  v.mg_tid = d_mtid;
  v.mg_cnt = d_mcnt;
  v.tmpl = d_tmpl;
  v.mt_cnt = d_mt;
  v.bits = d_bits;
  v.n_bits = n_bits;
  v.br_api = br_api;
  v.br_tset = br_tset;
  v.br_lex = br_lex;
  v.bkey = d_bkey;
  v.bval = d_bval;
  v.bmask = n_bits ? (uint32_t)(bkey.size() - 1) : 0u;
  s->est_kind = snapshot_est_kind(s);
  return KP_OK;
}

// ============================================================================
// Binding packing
// ============================================================================
// Host-side pools of packed bindings (kp_batch's, or one packing thread's).
// (aligned to two cache lines: the packing threads fill adjacent chunks' pools at once, and
// every push_back writes its vector's end pointer; packed 120-B structs shared lines, and
// 16 threads packed at about a third of the single-thread rate per binding)
struct alignas(128) Pools {
  std::vector<int32_t> ipool;
  std::vector<int64_t> lpool;
  std::vector<Tol> tols;
  std::vector<Prog> progs;
  std::vector<Instr> instrs;
};

// Diagnostic build (-DKP_PACK_PROF): cycles per section of Packer::pack, summed over
// the process and printed by pack_parallel under KP_PACK_TIMING.
#ifdef KP_PACK_PROF
#include <x86intrin.h>
std::atomic<uint64_t> g_pack_cyc[8];
#define KP_PACK_MARK_INIT uint64_t kp_c0 = __rdtsc()
#define KP_PACK_MARK(i)                                                  \
  do {                                                                   \
    const uint64_t kp_c1 = __rdtsc();                                    \
    g_pack_cyc[i].fetch_add(kp_c1 - kp_c0, std::memory_order_relaxed); \
    kp_c0 = kp_c1;                                                       \
  } while (0)
#else
#define KP_PACK_MARK_INIT
#define KP_PACK_MARK(i)
#endif
struct Packer {
  kp_snapshot* s;
  Pools* bt;  // this packer's pools (one per packing thread, merged by kp_batch_create)
  // per-packer caches: the last (apiVersion, kind) and its GVK id, parsed quantity
  // strings, and scratch lists reused across bindings (no per-binding allocation)
  std::string gvkey;
  SvMap<std::pair<bool, k8s::Qty>> qcache;
  SvMap<int32_t> gvk_cache;  // apiVersion + '\0' + kind -> GVK id
  SvMap<bool> scalar_cache;  // resource name -> IsScalarResourceName
  std::vector<int32_t> tmp_t, tmp_rk, tmp_sr, tmp_mr;
  std::vector<int64_t> tmp_sq, tmp_mq;
  std::vector<std::pair<std::string_view, k8s::Qty>> tmp_rq;
  std::vector<Instr> tmp_out;
  std::vector<int32_t> tmp_vals;
  std::vector<std::pair<std::string_view, std::string_view>> tmp_ml;
  std::vector<int32_t> tmp_filt, tmp_ovf, tmp_ov, tmp_ids, tmp_ev;
  std::vector<int64_t> tmp_ws;
  // compiled programs by affinity content (a batch repeats a policy's placement across
  // its bindings): the instructions with their list references relative to the lists
  // they own, re-emitted into the pools on a hit
  struct CProg {
    std::vector<Instr> ins;
    std::vector<int32_t> lists;
  };
  SvMap<int32_t> cmemo;
  // ResourceRequest lists memoized by content (their names and quantity strings): a batch
  // repeats a few request specs, so most bindings skip the parse, sort and name lookups
  struct ReqMemo {
    bool bad;
    std::vector<int32_t> sr, mr;
    std::vector<int64_t> sq, mq;
  };
  SvMap<int32_t> rmemo;
  std::vector<ReqMemo> rlist;
  std::string rkey;
  std::vector<CProg> cprogs;
  std::string ckey;

  bool scalar(std::string_view nm) {
    auto it = scalar_cache.find(nm);
    if (it != scalar_cache.end()) return it->second;
    const bool v = k8s::scalar_resource(std::string(nm));
    if (scalar_cache.size() < 4096) scalar_cache.emplace(std::string(nm), v);
    return v;
  }

  bool qty(std::string_view str, k8s::Qty* q) {
    auto it = qcache.find(str);
    if (it != qcache.end()) {
      *q = it->second.second;
      return it->second.first;
    }
    k8s::Qty v;
    const bool ok = k8s::parse_quantity(str, &v);
    if (qcache.size() < 4096) qcache.emplace(std::string(str), std::make_pair(ok, v));
    *q = v;
    return ok;
  }

  int32_t list(const std::vector<int32_t>& v) {
    int32_t off = (int32_t)bt->ipool.size();
    bt->ipool.insert(bt->ipool.end(), v.begin(), v.end());
    return off;
  }
  std::vector<int32_t> ranks(const kp_str* names, uint32_t n) {
    std::vector<int32_t> r;
    for (uint32_t i = 0; i < n; i++) {
      auto it = s->rank_of.find(SV(names[i]));
      if (it != s->rank_of.end()) r.push_back(it->second);
    }
    return r;
  }
  // (the list lives until the next call: callers hand it to list() at once)
  const std::vector<int32_t>& vals(const kp_str* v, uint32_t n) {
    std::vector<int32_t>& r = tmp_vals;
    r.clear();
    for (uint32_t i = 0; i < n; i++) {
      int32_t id = s->str.get(SV(v[i]));
      if (id >= 0) r.push_back(id);
    }
    return r;
  }
  void ins(std::vector<Instr>& out, int32_t op, int32_t a = 0, int32_t b = 0, int32_t c = 0, int64_t v = 0) {
    Instr i;
    i.op = op;
    i.a = a;
    i.b = b;
    i.c = c;
    i.v = v;
    out.push_back(i);
  }
  // labels.NewRequirement validation (labels/selector.go:150-230)
  static bool valid_req(std::string_view key, std::string_view op, const kp_str* v, uint32_t n) {
    bool ok = k8s::label_key(key);
    if (op == "In" || op == "NotIn") ok = ok && n > 0;
    else if (op == "=") ok = ok && n == 1;
    else if (op == "Exists" || op == "DoesNotExist") ok = ok && n == 0;
    else if (op == "Gt" || op == "Lt") {
      ok = ok && n == 1;
      for (uint32_t i = 0; i < n; i++) {
        int64_t x;
        if (!k8s::parse_int64(SV(v[i]), &x)) ok = false;
      }
    } else {
      ok = false;
    }
    for (uint32_t i = 0; i < n; i++)
      if (!k8s::label_value(SV(v[i]))) ok = false;
    return ok;
  }
  static bool list_ref_a(int32_t op) { return op == OP_EXCLUDE || op == OP_NAMES; }
  static bool list_ref_b(int32_t op) {
    return op == OP_LBL_IN || op == OP_LBL_NOTIN || op == OP_FLD_IN || op == OP_FLD_NOTIN || op == OP_ZONE_IN ||
           op == OP_ZONE_NOTIN;
  }
  // The affinity's content as a key: every field, strings length-prefixed.
  void affinity_key(const kp_cluster_affinity& a) {
    std::string& k = ckey;
    k.clear();
    auto u32 = [&](uint32_t v) { k.append((const char*)&v, 4); };
    auto str = [&](const kp_str& x) {
      u32(x.len);
      if (x.len) k.append(x.ptr, x.len);
    };
    auto strs = [&](const kp_str* v, uint32_t n) {
      u32(n);
      for (uint32_t i = 0; i < n; i++) str(v[i]);
    };
    auto reqs = [&](const kp_requirement* r, uint32_t n) {
      u32(n);
      for (uint32_t i = 0; i < n; i++) {
        str(r[i].key);
        str(r[i].op);
        strs(r[i].values, r[i].n_values);
      }
    };
    u32(a.has_label_selector);
    u32(a.n_match_labels);
    for (uint32_t i = 0; i < a.n_match_labels; i++) {
      str(a.match_labels[i].key);
      str(a.match_labels[i].value);
    }
    reqs(a.match_expressions, a.n_match_expressions);
    u32(a.has_field_selector);
    reqs(a.field_expressions, a.n_field_expressions);
    strs(a.cluster_names, a.n_cluster_names);
    strs(a.exclude_clusters, a.n_exclude_clusters);
  }
  // util.ClusterMatches compiled to a conjunction program (selector.go:97-155),
  // memoized by content
  int32_t compile(const kp_cluster_affinity& a) {
    affinity_key(a);
    auto it = cmemo.find(std::string_view(ckey));
    if (it != cmemo.end()) {
      const CProg& c = cprogs[it->second];
      const int32_t base = (int32_t)bt->ipool.size();
      bt->ipool.insert(bt->ipool.end(), c.lists.begin(), c.lists.end());
      Prog p;
      p.ins_off = (int32_t)bt->instrs.size();
      p.ins_cnt = (int32_t)c.ins.size();
      for (Instr x : c.ins) {
        if (list_ref_a(x.op)) x.a += base;
        else if (list_ref_b(x.op)) x.b += base;
        bt->instrs.push_back(x);
      }
      bt->progs.push_back(p);
      return (int32_t)bt->progs.size() - 1;
    }
    const int32_t ip0 = (int32_t)bt->ipool.size();
    const int32_t id = compile_new(a);
    if (cprogs.size() < 4096) {
      CProg c;
      const Prog& p = bt->progs[id];
      c.lists.assign(bt->ipool.begin() + ip0, bt->ipool.end());
      c.ins.assign(bt->instrs.begin() + p.ins_off, bt->instrs.begin() + p.ins_off + p.ins_cnt);
      for (Instr& x : c.ins) {
        if (list_ref_a(x.op)) x.a -= ip0;
        else if (list_ref_b(x.op)) x.b -= ip0;
      }
      cmemo.emplace(ckey, (int32_t)cprogs.size());
      cprogs.push_back(std::move(c));
    }
    return id;
  }
  int32_t compile_new(const kp_cluster_affinity& a) {
    std::vector<Instr>& out = tmp_out;
    out.clear();
    bool never = false;
    if (a.n_exclude_clusters) {
      auto r = ranks(a.exclude_clusters, a.n_exclude_clusters);
      if (!r.empty()) ins(out, OP_EXCLUDE, list(r), (int32_t)r.size());
    }
    if (a.has_label_selector) {  // metav1.LabelSelectorAsSelector (helpers.go:36-74)
      // matchLabels as a map: key order, a repeated key's last value
      auto& ml = tmp_ml;
      ml.clear();
      for (uint32_t i = 0; i < a.n_match_labels; i++) {
        const std::string_view k = SV(a.match_labels[i].key), v = SV(a.match_labels[i].value);
        bool dup = false;
        for (auto& kv : ml)
          if (kv.first == k) {
            kv.second = v;
            dup = true;
          }
        if (!dup) ml.push_back({k, v});
      }
      std::sort(ml.begin(), ml.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      for (auto& kv : ml) {
        kp_str v{kv.second.data(), (uint32_t)kv.second.size()};
        if (!valid_req(kv.first, "=", &v, 1)) never = true;
        int32_t slot = s->keys.get(kv.first);
        int32_t id = s->str.get(kv.second);
        if (slot < 0 || id < 0) never = never || true;
        else {
          tmp_vals.assign(1, id);
          ins(out, OP_LBL_IN, slot, list(tmp_vals), 1);
        }
      }
      for (uint32_t i = 0; i < a.n_match_expressions; i++) {
        const kp_requirement& r = a.match_expressions[i];
        const std::string_view key = SV(r.key), op = SV(r.op);
        if (!(op == "In" || op == "NotIn" || op == "Exists" || op == "DoesNotExist") ||
            !valid_req(key, op, r.values, r.n_values)) {
          never = true;
          continue;
        }
        int32_t slot = s->keys.get(key);
        if (op == "In") {
          const auto& v = vals(r.values, r.n_values);
          if (slot < 0 || v.empty()) never = true;
          else ins(out, OP_LBL_IN, slot, list(v), (int32_t)v.size());
        } else if (op == "NotIn") {
          const auto& v = vals(r.values, r.n_values);
          if (slot >= 0) ins(out, OP_LBL_NOTIN, slot, list(v), (int32_t)v.size());
        } else if (op == "Exists") {
          if (slot < 0) never = true;
          else ins(out, OP_LBL_EXISTS, slot);
        } else if (slot >= 0) {
          ins(out, OP_LBL_DNE, slot);
        }
      }
    }
    if (a.has_field_selector) {
      bool any_other = false;
      bool others_ok = true;
      for (uint32_t i = 0; i < a.n_field_expressions; i++) {
        const kp_requirement& r = a.field_expressions[i];
        const std::string_view key = SV(r.key), op = SV(r.op);
        if (key == "zone") {  // matchZones (selector.go:208-235)
          const auto& v = vals(r.values, r.n_values);
          if (op == "In") ins(out, OP_ZONE_IN, 0, list(v), (int32_t)v.size());
          else if (op == "NotIn") ins(out, OP_ZONE_NOTIN, 0, list(v), (int32_t)v.size());
          else if (op == "Exists") ins(out, OP_ZONE_EXISTS);
          else if (op == "DoesNotExist") ins(out, OP_ZONE_DNE);
          else never = true;
          continue;
        }
        any_other = true;
        // lifted.NodeSelectorRequirementsAsSelector (nodeaffinity.go:36-71)
        if (!(op == "In" || op == "NotIn" || op == "Exists" || op == "DoesNotExist" || op == "Gt" || op == "Lt") ||
            !valid_req(key, op, r.values, r.n_values)) {
          others_ok = false;
          continue;
        }
        int field = key == "provider" ? 0 : (key == "region" ? 1 : 2);  // extractClusterFields
        if (op == "In") {
          const auto& v = vals(r.values, r.n_values);
          if (field == 2 || v.empty()) never = true;
          else ins(out, OP_FLD_IN, field, list(v), (int32_t)v.size());
        } else if (op == "NotIn") {
          const auto& v = vals(r.values, r.n_values);
          if (field != 2) ins(out, OP_FLD_NOTIN, field, list(v), (int32_t)v.size());
        } else if (op == "Exists") {
          if (field == 2) never = true;
          else ins(out, OP_FLD_EXISTS, field);
        } else if (op == "DoesNotExist") {
          if (field != 2) ins(out, OP_FLD_DNE, field);
        } else {
          int64_t x = 0;
          k8s::parse_int64(S(r.values[0]), &x);
          if (field == 2) never = true;
          else ins(out, op == "Gt" ? OP_FLD_GT : OP_FLD_LT, field, 0, 0, x);
        }
      }
      if (any_other && !others_ok) never = true;
    }
    if (a.n_cluster_names) {
      auto r = ranks(a.cluster_names, a.n_cluster_names);
      if (r.empty()) never = true;
      else ins(out, OP_NAMES, list(r), (int32_t)r.size());
    }
    if (never) {
      out.clear();
      ins(out, OP_FALSE);
    }
    Prog p;
    p.ins_off = (int32_t)bt->instrs.size();
    p.ins_cnt = (int32_t)out.size();
    bt->instrs.insert(bt->instrs.end(), out.begin(), out.end());
    bt->progs.push_back(p);
    return (int32_t)bt->progs.size() - 1;
  }

  void pack(const kp_binding& b, BindHdr& h) {
    KP_PACK_MARK_INIT;
    memset(&h, 0, sizeof(h));
    h.ip_beg = (int32_t)bt->ipool.size();
    h.pr_beg = (int32_t)bt->progs.size();
    h.in_beg = (int32_t)bt->instrs.size();
    const kp_options& o = s->opts;
    h.replicas = b.replicas;
    h.enabled = (int32_t)o.enabled_plugins;
    uint32_t f = 0;
    if (b.has_replica_requirements) f |= BF_HAS_RR;
    if (b.replicas == 0 && b.n_components == 0) f |= BF_NONWORKLOAD_EST;
    if ((b.replicas > 0 || b.has_replica_requirements) && b.n_components <= 1) f |= BF_WORKLOAD_ASSIGN;
    if (b.has_reschedule_triggered_at && b.has_last_scheduled_time &&
        b.reschedule_triggered_at_ns > b.last_scheduled_time_ns)
      f |= BF_FRESH;
    if (b.uid.len && (k8s::fnv32a(b.uid.ptr, b.uid.len) & 1)) f |= BF_UID_DESC;
    if (o.enable_empty_workload_propagation) f |= BF_EMPTY_PROP;
    if (b.has_weight_preference) f |= BF_HAS_WP;
    // APIEnablement GVK (group_version.go:211-226,300-305)
    {
      gvkey.assign(SV(b.api_version));
      gvkey.push_back('\0');
      gvkey.append(SV(b.kind));
      auto it = gvk_cache.find(std::string_view(gvkey));
      if (it != gvk_cache.end()) {
        h.gvk = it->second;  // (a batch repeats a few kinds)
      } else {
        std::string av = S(b.api_version), g, ver;
        size_t slashes = std::count(av.begin(), av.end(), '/');
        if (!(av.empty() || av == "/")) {
          if (slashes == 0) ver = av;
          else if (slashes == 1) {
            g = av.substr(0, av.find('/'));
            ver = av.substr(av.find('/') + 1);
          }
        }
        std::string gv = g.empty() ? ver : g + "/" + ver;
        h.gvk = s->gvk.get(gv + '\0' + S(b.kind));
        if (gvk_cache.size() < 4096) gvk_cache.emplace(gvkey, h.gvk);
      }
    }
    KP_PACK_MARK(0);
    // spec.Clusters
    h.n_targets_all = (int32_t)b.n_clusters;
    {
      std::vector<int32_t>& t = tmp_t;
      std::vector<int32_t>& rk = tmp_rk;
      t.clear();
      rk.clear();
      for (uint32_t i = 0; i < b.n_clusters; i++) {
        auto it = s->rank_of.find(SV(b.clusters[i].name));
        if (it == s->rank_of.end()) continue;
        rk.push_back(it->second);
        t.push_back(it->second);
        t.push_back(b.clusters[i].replicas);
      }
      std::sort(rk.begin(), rk.end());
      if (std::adjacent_find(rk.begin(), rk.end()) != rk.end()) f |= BF_DUP_TARGETS;
      h.tgt_off = list(t);
      h.tgt_cnt = (int32_t)t.size() / 2;
      if (b.n_clusters > 0 && (o.enabled_plugins & KP_PLUGIN_CLUSTER_LOCALITY)) f |= BF_SCORE_LOCALITY;
    }
    {
      auto& r = tmp_ev;
      r.clear();
      for (uint32_t i = 0; i < b.n_eviction_from; i++) {
        auto it = s->rank_of.find(SV(b.eviction_from[i]));
        if (it != s->rank_of.end()) r.push_back(it->second);
      }
      h.evict_off = list(r);
      h.evict_cnt = (int32_t)r.size();
    }
    KP_PACK_MARK(1);
    // tolerations
    h.tol_off = (int32_t)bt->tols.size();
    for (uint32_t i = 0; i < b.n_tolerations; i++) {
      const kp_toleration& t = b.tolerations[i];
      const std::string_view eff = SV(t.effect), key = SV(t.key), op = SV(t.op);
      Tol x;
      if (eff.empty()) x.eff = EFF_ANY;
      else if (eff == "NoSchedule") x.eff = EFF_NOSCHEDULE;
      else if (eff == "NoExecute") x.eff = EFF_NOEXECUTE;
      else continue;
      if (key.empty()) x.key = -1;
      else if ((x.key = s->str.get(key)) < 0) continue;
      if (op.empty() || op == "Equal") {
        x.op = TOL_EQUAL;
        if ((x.val = s->str.get(SV(t.value))) < 0) continue;
      } else if (op == "Exists") {
        x.op = TOL_EXISTS;
        x.val = -1;
      } else {
        continue;  // Lt/Gt disabled, unknown operators never tolerate
      }
      bt->tols.push_back(x);
    }
    h.tol_cnt = (int32_t)bt->tols.size() - h.tol_off;
    KP_PACK_MARK(2);
    // ClusterAffinity filter list + overflow order programs
    {
      auto &filt = tmp_filt, &ovf = tmp_ovf;
      filt.clear();
      ovf.clear();
      bool have = false;
      const kp_affinity_term* term = nullptr;
      if (b.has_cluster_affinity) {
        filt.push_back(compile(b.cluster_affinity));
        have = true;
      } else {
        const std::string_view obs = SV(b.observed_affinity_name);
        for (uint32_t i = 0; i < b.n_cluster_affinities; i++)
          if (SV(b.cluster_affinities[i].affinity_name) == obs) {
            term = &b.cluster_affinities[i];
            break;
          }
        if (term) {
          have = true;
          ovf.push_back(compile(term->affinity));
          filt.push_back(ovf[0]);
          auto& ov = tmp_ov;
          ov.clear();
          for (uint32_t j = 0; j < term->n_overflow; j++) ov.push_back(compile(term->overflow[j]));
          ovf.insert(ovf.end(), ov.begin(), ov.end());
          bool workload = b.replicas > 0 || b.has_replica_requirements || b.n_components >= 1;
          if (workload) filt.insert(filt.end(), ov.begin(), ov.end());
        }
      }
      if (!have) f |= BF_AFF_ALL;
      h.filt_off = list(filt);
      h.filt_cnt = (int32_t)filt.size();
      if (b.has_cluster_affinity || b.n_cluster_affinities == 0) h.ovf_mode = OVF_ZERO;
      else if (!term) h.ovf_mode = OVF_1000;
      else h.ovf_mode = OVF_PROGS;
      h.ovf_off = list(ovf);
      h.ovf_cnt = (int32_t)ovf.size();
      // engine limit: the sortClusters key orders kMaxOvfTerms overflow orders (kp_algo.h)
      // (reported as KP_ERR_OVERFLOW_TERMS, not as a malformed request)
      if (h.ovf_mode == OVF_PROGS && h.ovf_cnt > kMaxOvfTerms) f |= BF_BAD | BF_LIMIT_OVF;
      // enableOverflow (common.go:156-170)
      if (!b.has_cluster_affinity && b.n_cluster_affinities > 0 && b.observed_affinity_name.len > 0 && term &&
          term->n_overflow > 0)
        f |= BF_OVERFLOW;
    }
    KP_PACK_MARK(3);
    // static weights
    {
      auto& ids = tmp_ids;
      auto& ws = tmp_ws;
      ids.clear();
      ws.clear();
      for (uint32_t i = 0; i < b.n_static_weights; i++) {
        ids.push_back(compile(b.static_weights[i].target));
        ws.push_back(b.static_weights[i].weight);
      }
      h.sw_off = list(ids);
      h.sw_cnt = (int32_t)ids.size();
      h.sw_w_off = (int32_t)bt->lpool.size();
      bt->lpool.insert(bt->lpool.end(), ws.begin(), ws.end());
    }
    KP_PACK_MARK(4);
    // requests
    rkey.clear();
    for (uint32_t i = 0; i < b.n_resource_request; i++) {
      rkey.append(SV(b.resource_request[i].name));
      rkey.push_back('\0');
      rkey.append(SV(b.resource_request[i].quantity));
      rkey.push_back('\0');
    }
    if (auto* m = rmemo.find(std::string_view(rkey))) {
      const ReqMemo& q = rlist[m->second];
      if (q.bad) f |= BF_BAD;
      h.sreq_off = list(q.sr);
      h.sreq_cnt = (int32_t)q.sr.size();
      h.sreq_q_off = (int32_t)bt->lpool.size();
      bt->lpool.insert(bt->lpool.end(), q.sq.begin(), q.sq.end());
      h.mreq_off = list(q.mr);
      h.mreq_cnt = (int32_t)q.mr.size();
      h.mreq_q_off = (int32_t)bt->lpool.size();
      bt->lpool.insert(bt->lpool.end(), q.mq.begin(), q.mq.end());
    } else {
      bool bad = false;
      // the ResourceList as (name, quantity) in name order, a repeated name's last
      // entry winning (the map the reference decodes), without per-entry allocation
      auto& rq = tmp_rq;
      rq.clear();
      for (uint32_t i = 0; i < b.n_resource_request; i++) {
        k8s::Qty q;
        if (!qty(SV(b.resource_request[i].quantity), &q)) bad = true;
        const std::string_view nm = SV(b.resource_request[i].name);
        bool dup = false;
        for (auto& kv : rq)
          if (kv.first == nm) {
            kv.second = q;
            dup = true;
          }
        if (!dup) rq.push_back({nm, q});
      }
      std::sort(rq.begin(), rq.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      auto &sr = tmp_sr, &mr = tmp_mr;
      auto &sq = tmp_sq, &mq = tmp_mq;
      sr.clear(), mr.clear(), sq.clear(), mq.clear();
      for (auto& kv : rq) {
        const std::string_view nm = kv.first;
        const bool cpu = nm == "cpu", mem = nm == "memory";
        const int32_t rid = cpu ? s->rid_cpu : (mem ? s->rid_mem : s->res.get(nm));
        int64_t v = k8s::value(kv.second);
        if (v > 0) {  // summary path: every resource name (general.go:467-471)
          sr.push_back(rid);
          sq.push_back(cpu ? k8s::milli(kv.second) : v);
        }
        // model path: util.NewResource classes (resource.go:46-75)
        if (cpu) {
          int64_t m = k8s::milli(kv.second);
          if (m > 0) {
            mr.push_back(rid);
            mq.push_back(m);
          }
        } else if (mem || nm == "ephemeral-storage" || (nm != "pods" && scalar(nm))) {
          if (v > 0) {
            mr.push_back(rid);
            mq.push_back(v);
          }
        }
      }
      h.sreq_off = list(sr);
      h.sreq_cnt = (int32_t)sr.size();
      h.sreq_q_off = (int32_t)bt->lpool.size();
      bt->lpool.insert(bt->lpool.end(), sq.begin(), sq.end());
      h.mreq_off = list(mr);
      h.mreq_cnt = (int32_t)mr.size();
      h.mreq_q_off = (int32_t)bt->lpool.size();
      bt->lpool.insert(bt->lpool.end(), mq.begin(), mq.end());
      if (bad) f |= BF_BAD;
      if (rlist.size() < 4096) {
        rmemo.emplace(rkey, (int32_t)rlist.size());
        rlist.push_back(ReqMemo{bad, sr, mr, sq, mq});
      }
    }
    KP_PACK_MARK(5);
    // spread constraints: filter presence + selection kind (select_clusters.go:28-80)
    const std::string_view rst = b.has_replica_scheduling ? SV(b.replica_scheduling_type) : std::string_view("Duplicated");
    const std::string_view div = SV(b.replica_division_preference);
    bool hasRegion = false, hasCluster = false;
    int n_order = 0;
    for (uint32_t i = 0; i < b.n_spread_constraints; i++) {
      const kp_spread_constraint& sc = b.spread_constraints[i];
      const std::string_view fld = SV(sc.spread_by_field);
      const int code = fld == "provider" ? 1 : fld == "region" ? 2 : fld == "zone" ? 3 : 0;
      bool seen = false;
      for (int k = 0; k < n_order; k++) seen = seen || ((h.spread_order >> (2 * k)) & 3) == code;
      if (code && !seen) h.spread_order |= code << (2 * n_order++);
      if (fld == "provider") f |= BF_NEED_PROVIDER;
      if (fld == "region") {
        f |= BF_NEED_REGION;
        hasRegion = true;
        h.region_min = sc.min_groups;
        h.region_max = sc.max_groups;
      }
      if (fld == "zone") f |= BF_NEED_ZONES;
      if (fld == "cluster") {
        hasCluster = true;
        h.cluster_min = sc.min_groups;
        h.cluster_max = sc.max_groups;
      }
    }
    bool ignoreSpread = b.has_replica_scheduling && SV(b.replica_scheduling_type) == "Divided" && div == "Weighted" &&
                        (!b.has_weight_preference || (b.n_static_weights != 0 && b.dynamic_weight.len == 0));
    if (b.n_spread_constraints == 0 || ignoreSpread) h.sel = SEL_ALL;
    else if (hasRegion) h.sel = SEL_REGION;
    else if (hasCluster) h.sel = SEL_CLUSTER;
    else h.sel = SEL_ERR_UNSUPPORTED;
    h.need_replicas = (!b.has_replica_scheduling || SV(b.replica_scheduling_type) == "Duplicated") ? -1 : b.replicas;
    // runReplicaEstimator / SelectClusters with the MultiplePodTemplatesScheduling gate:
    // isMultiTemplateSchedulingApplicable (core/estimation.go:43-65) = components and a
    // cluster spread constraint with MinGroups == MaxGroups == 1. Such a binding's
    // estimator row is MaxAvailableComponentSets (core/util.go:113-118) and it needs one
    // available replica (one set) in SelectBestClusters (common.go:42-46).
    if (o.multiple_pod_templates_scheduling && b.n_components > 0) {
      bool one = false;
      for (uint32_t i = 0; i < b.n_spread_constraints; i++)
        one = one || (SV(b.spread_constraints[i].spread_by_field) == "cluster" &&
                      b.spread_constraints[i].min_groups == 1 && b.spread_constraints[i].max_groups == 1);
      if (one) {
        f |= BF_SETS;
        if (h.need_replicas != -1) h.need_replicas = 1;
      }
    }
    if (rst == "Duplicated") f |= BF_GROUP_DUP;
    // strategy (assignment.go:95-123)
    if (rst == "Duplicated") h.strategy = ST_DUPLICATED;
    else if (rst == "Divided") {
      if (div == "Aggregated") h.strategy = ST_AGGREGATED;
      else if (div == "Weighted")
        h.strategy = (b.has_weight_preference && b.dynamic_weight.len) ? ST_DYNAMIC : ST_STATIC;
      else h.strategy = ST_NONE;
    } else {
      h.strategy = ST_NONE;
    }
    h.flags = f;
    uint64_t C = (uint64_t)s->C;
    bool big = !(f & BF_WORKLOAD_ASSIGN) || h.strategy == ST_DUPLICATED || (f & BF_EMPTY_PROP);
    uint64_t rep = b.replicas > 0 ? (uint64_t)b.replicas : 0;
    h.out_cap = (big ? C : std::min<uint64_t>(C, rep)) + (uint64_t)h.tgt_cnt;
    h.ip_end = (int32_t)bt->ipool.size();
    h.pr_end = (int32_t)bt->progs.size();
    h.in_end = (int32_t)bt->instrs.size();
    KP_PACK_MARK(6);
  }
};

// ---------------------------------------------------------------------------
// selectGroups (select_groups.go:102-224): the host-kept group combination.
// groups: (region id == name order, value = #clusters, weight = group score).
// ---------------------------------------------------------------------------
struct G {
  int id;
  int64_t value, weight;
};
std::vector<int> select_groups(std::vector<G> groups, int64_t minC, int64_t maxC, int64_t target) {
  if (groups.empty()) return {};
  if (groups.size() > 1)
    std::sort(groups.begin(), groups.end(), [](const G& a, const G& b) {
      if (a.value != b.value) return a.value < b.value;
      if (a.weight != b.weight) return a.weight > b.weight;
      return a.id < b.id;
    });
  struct Path {
    int id;
    int64_t weight, value;
    std::vector<int> g;  // indices into groups, sorted by (weight desc, id asc)
  };
  std::vector<Path> paths;
  std::vector<int> root;
  int pid = 0;
  const int n = (int)groups.size();
  std::function<void(int64_t, int)> dfs = [&](int64_t sum, int begin) {
    int64_t len = (int64_t)root.size();
    if (sum >= target && len >= minC && len <= maxC) {
      Path p;
      p.id = ++pid;
      p.weight = 0;
      p.value = 0;
      p.g = root;
      for (int i : p.g) {
        p.weight += groups[i].weight;
        p.value += groups[i].value;
      }
      std::sort(p.g.begin(), p.g.end(), [&](int a, int b) {
        if (groups[a].weight != groups[b].weight) return groups[a].weight > groups[b].weight;
        return groups[a].id < groups[b].id;
      });
      paths.push_back(std::move(p));
      return;
    }
    if (len >= maxC) return;
    for (int i = begin; i < n; i++) {
      sum += groups[i].value;
      root.push_back(i);
      dfs(sum, i + 1);
      if ((int64_t)n == minC) break;  // select_groups.go:179-182 (no backtracking)
      sum -= groups[i].value;
      root.pop_back();
    }
  };
  dfs(0, 0);
  if (paths.empty()) return {};
  const Path* fin = &paths[0];
  if (paths.size() > 1) {
    std::sort(paths.begin(), paths.end(), [](const Path& a, const Path& b) {
      if (a.weight != b.weight) return a.weight > b.weight;
      if (a.value != b.value) return a.value > b.value;
      return a.id < b.id;
    });
    fin = &paths[0];
    for (size_t i = 1; i < paths.size(); i++) {
      const Path& sp = paths[i];
      bool m = sp.g.size() < fin->g.size();
      for (size_t k = 0; m && k < sp.g.size(); k++) m = groups[fin->g[k]].id == groups[sp.g[k]].id;
      if (m) fin = &paths[i];
    }
  }
  std::vector<int> out;
  for (int i : fin->g) out.push_back(groups[i].id);
  return out;
}

// Hardware threads, capped by the cgroup v2 CPU quota (cpu.max "quota period") when set.
int host_cpus() {
  int n = (int)std::max(1u, std::thread::hardware_concurrency());
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
      const long long quota = atoll(q);
      n = std::min<long long>(n, std::max<long long>(1, (quota + period - 1) / period));
    }
    fclose(f);
  }
  return n;
}

// Process-wide worker threads for the packer's per-thread phases (pack, merge, cache
// inserts): each phase of each batch used to start and join its own threads (three rounds
// of 16 per batch with kp_pack_cache), and two engines packing at once started 32 at a time.
// run(T, fn) calls fn(t) once for every t in [0, T), the caller taking tasks too; jobs of
// concurrent callers interleave task by task. Workers are started lazily, never joined.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();  // (never destroyed: workers may be blocked in wait)
    return *p;
  }
  void run(int T, const std::function<void(int)>& fn) {
    if (T <= 1) {
      if (T == 1) fn(0);
      return;
    }
    ensure(T - 1);
    Job j;
    j.fn = &fn;
    j.T = T;
    j.left = T;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(&j);
    }
    cv_.notify_all();
    for (;;) {  // the caller takes tasks of its own job until none is left to start
      int t;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (j.next >= j.T) break;
        t = j.next++;
        if (j.next >= j.T) q_.erase(std::find(q_.begin(), q_.end(), &j));
      }
      fn(t);
      std::lock_guard<std::mutex> g(mu_);
      j.left--;
    }
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return j.left == 0; });
  }

 private:
  struct Job {
    const std::function<void(int)>* fn = nullptr;
    int T = 0, next = 0, left = 0;
  };
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<Job*> q_;
  int n_workers_ = 0;
  void ensure(int n) {
    std::lock_guard<std::mutex> g(mu_);
    for (; n_workers_ < n; n_workers_++) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return !q_.empty(); });
      Job* j = q_.front();
      const int t = j->next++;
      if (j->next >= j->T) q_.erase(q_.begin());
      g.unlock();
      (*j->fn)(t);
      g.lock();
      if (--j->left == 0) done_.notify_all();
    }
  }
};

template <class F>
void parallel_for(int n, int threads, F fn) {
  if (n <= 0) return;
  if (threads <= 1 || n < 64) {
    for (int i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<int> next(0);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&]() {
      for (;;) {
        int i = next.fetch_add(16);
        if (i >= n) break;
        for (int k = i; k < std::min(n, i + 16); k++) fn(k);
      }
    });
  for (auto& t : th) t.join();
}

size_t smem_pair(const kp_snapshot* s, int md_cap) {
  int words = (s->Cp + 31) >> 5;
  return kRedBytes + 8 * (size_t)words + 4 * (size_t)((md_cap + 3) & ~3) + kPairStage + kTsetMax / 8 + 64;
}
size_t smem_all(const kp_snapshot* s) {
  int words = (s->Cp + 31) >> 5;
  return kRedBytes + 4 * (size_t)((words + 3) & ~3) + 8 * (size_t)s->Cp + 3072 + 8 * (size_t)sel_all_ecap(s->Cp) + 64;
}
size_t smem_cluster(const kp_snapshot* s, int cap) {
  int words = (s->Cp + 31) >> 5;
  size_t area = std::max(8 * (size_t)s->Cp, serial_scratch_bytes(cap));
  return kRedBytes + 1024 + sizeof(Item) * 2 * kSmallMax + 16 * kSmallMax + 4 * (size_t)((words + 3) & ~3) + area + 64;
}
size_t smem_region_a(const kp_snapshot* s) {
  int words = (s->Cp + 31) >> 5;
  size_t R = s->view.n_regions;
  return kRedBytes + 80 * R + 4 * (size_t)((words + 3) & ~3) + 10 * (size_t)s->Cp + 64;
}
size_t smem_region_b(const kp_snapshot* s, int cap) {
  int words = (s->Cp + 31) >> 5;
  size_t R = s->view.n_regions;
  size_t area = std::max(10 * (size_t)s->Cp, serial_scratch_bytes(cap));  // cand r/v/g, then the serial scratch
  return kRedBytes + 1024 + sizeof(Item) * 2 * kSmallMax + 16 * kSmallMax + 8 * R + 4 * ((R + 3) & ~3) +
         4 * (size_t)((words + 3) & ~3) + area + 64;
}
const int kMdCap = 4096;
// MaxDivided table entries staged per workgroup: the snapshot's template count.
int md_cap_of(const kp_snapshot* s) { return s->n_tmpl <= kMdCap ? std::max(kTmplDense, s->n_tmpl) : 0; }
// Whether the specialised pair kernel (est_compute<true>) covers every binding of
// the batch: MaxDivided and taint-set tables fit in LDS, the dense node-count
// matrix exists (or no cluster has models), at most kReqUnroll resource requests
// per binding, divisors <= 2^60.
// The snapshot half (its clusters' estimator paths and table sizes), kept in
// kp_snapshot::est_kind and refreshed by every upload; the batch half
// (request counts and divisors) in kp_batch::fast_ok. The launch takes
// est_kind when fast_ok, else EST_GENERIC.
bool batch_fast_ok(const kp_batch* bt) {
  for (const BindHdr& h : bt->hdr) {
    if (h.sreq_cnt > kReqUnroll) return false;
    for (int j = 0; j < h.sreq_cnt; j++)
      if (bt->lpool[h.sreq_q_off + j] > ((int64_t)1 << 60)) return false;
  }
  return true;
}
// The largest dynamic LDS any kernel of the batch takes must fit one workgroup.
// Checked at kp_batch_create and again at every kp_schedule_batch: an
// intervening kp_snapshot_update can change the region and template counts the
// sizes depend on.
int batch_lds_check(kp_engine* e, const kp_snapshot* s, const kp_batch* bt) {
  const int cap = kSmallMax + kTgtSmallMax + 16;
  size_t need = smem_pair(s, md_cap_of(s));
  if (!bt->l_all.empty()) need = std::max(need, smem_all(s));
  if (!bt->l_cluster.empty()) need = std::max(need, smem_cluster(s, cap));
  if (!bt->l_region.empty()) need = std::max({need, smem_region_a(s), smem_region_b(s, cap)});
  if (need > e->max_lds) {
    e->err = "snapshot too large for one workgroup's LDS (" + std::to_string(need) + " > " +
             std::to_string(e->max_lds) + " bytes)";
    return -1;
  }
  return 0;
}
int snapshot_est_kind(const kp_snapshot* s) {
  if (md_cap_of(s) == 0 || s->view.n_tsets > kTsetMax || (s->n_tmpl > 0 && !s->view.mt_cnt)) return EST_GENERIC;
  // which estimator paths the snapshot's clusters can take
  bool any_model = false, any_summary_only = false;
  for (int r = 0; r < s->C; r++) {
    const uint32_t f = s->flags[r];
    if (f & CF_MODEL_OK) any_model = true;
    else if (f & CF_HAS_SUMMARY) any_summary_only = true;
  }
  if (!any_model) return EST_SUMMARY;
  if (!any_summary_only) return s->n_tmpl <= 8 ? EST_MODEL8 : EST_MODEL16;
  return EST_MIXED;
}

}  // namespace

// Packed-snapshot bytes: pack once on one rank, broadcast the bytes, import on
// the others. Host-endian; same engine build on every rank.
namespace {
const char kSnapMagic[8] = {'K', 'P', 'S', 'N', 'A', 'P', '0', '4'};
struct Wr {
  std::vector<unsigned char>& b;
  void raw(const void* p, size_t n) { b.insert(b.end(), (const unsigned char*)p, (const unsigned char*)p + n); }
  void u64(uint64_t x) { raw(&x, 8); }
  void str(const std::string& x) {
    u64(x.size());
    raw(x.data(), x.size());
  }
  void strs(const std::vector<std::string>& v) {
    u64(v.size());
    for (auto& x : v) str(x);
  }
  template <class T>
  void vec(const std::vector<T>& v) {
    u64(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};
struct Rd {
  const unsigned char* p;
  const unsigned char* end;
  bool ok = true;
  bool raw(void* d, size_t n) {
    if ((size_t)(end - p) < n) return ok = false;
    memcpy(d, p, n);
    p += n;
    return true;
  }
  uint64_t u64() {
    uint64_t x = 0;
    raw(&x, 8);
    return x;
  }
  std::string str() {
    uint64_t n = u64();
    if (!ok || (size_t)(end - p) < n) {
      ok = false;
      return {};
    }
    std::string x((const char*)p, n);
    p += n;
    return x;
  }
  std::vector<std::string> strs() {
    uint64_t n = u64();
    std::vector<std::string> v;
    for (uint64_t i = 0; ok && i < n; i++) v.push_back(str());
    return v;
  }
  template <class T>
  std::vector<T> vec() {
    uint64_t n = u64();
    std::vector<T> v;
    if (!ok || n > (uint64_t)(end - p) / sizeof(T)) {
      ok = false;
      return v;
    }
    v.resize(n);
    raw(v.data(), n * sizeof(T));
    return v;
  }
};
void dict_from(Dict& d, const std::vector<std::string>& names) {
  for (auto& n : names) d.add(n);
}

// Every column of an imported snapshot against the sizes and id ranges the
// kernels and kp_snapshot_update index with (a foreign or corrupt image must
// fail here, not fault in a kernel).
bool snapshot_consistent(const kp_snapshot* s) {
  const int C = s->C;
  if (C < 0 || C > kMaxClusters) return false;
  const size_t Cp = (size_t)s->Cp, C1 = (size_t)C + 1;
  const int K = (int)s->keys.names.size(), AW = ((int)s->gvk.names.size() + 63) / 64, R = (int)s->res.names.size();
  const int NS = (int)s->str.names.size(), NR = (int)s->regions.names.size(), T = s->n_tmpl, km = s->kmax;
  if ((int)s->names.size() != C || s->perm.size() != (size_t)C || T < 0 || km < 0) return false;
  if (s->str.names.size() != s->str.m.size() || s->keys.names.size() != s->keys.m.size() ||
      s->gvk.names.size() != s->gvk.m.size() || s->res.names.size() != s->res.m.size() ||
      s->regions.names.size() != s->regions.m.size())
    return false;  // duplicate dictionary entries
  for (int r = 1; r < C; r++)
    if (!(s->names[r - 1] < s->names[r])) return false;  // ranks are name order, names unique
  std::vector<char> seen(C, 0);
  for (uint32_t p : s->perm) {
    if (p >= (uint32_t)C || seen[p]) return false;
    seen[p] = 1;
  }
  for (size_t n : {s->flags.size(), s->provider.size(), s->region.size(), s->region_idx.size(),
                   s->provider_int.size(), s->region_int.size(), s->allowed.size()})
    if (n != Cp) return false;
  if (s->label_val.size() != (size_t)std::max(K, 1) * Cp || s->api_bits.size() != (size_t)std::max(AW, 1) * Cp ||
      s->avail.size() != (size_t)std::max(R, 1) * Cp || s->qa.size() != (size_t)std::max(R, 1) * Cp || s->tmpl.size() != (size_t)std::max(T, 1) * std::max(R, 1) ||
      s->mg_tid.size() != (size_t)std::max(km, 1) * Cp || s->mg_cnt.size() != s->mg_tid.size())
    return false;
  if (s->taint_val.size() != s->taint_key.size() || s->taint_eff.size() != s->taint_key.size() ||
      s->mgrp_cnt.size() != s->mgrp_tid.size())
    return false;
  auto offsets_ok = [&](const std::vector<int32_t>& off, size_t pool) {
    if (off.size() != C1 || off[0] != 0 || (size_t)off[C] > pool) return false;
    for (int r = 0; r < C; r++)
      if (off[r + 1] < off[r]) return false;
    return true;
  };
  if (!offsets_ok(s->zone_off, s->zone_ids.size()) || !offsets_ok(s->taint_off, s->taint_key.size()) ||
      !offsets_ok(s->mgrp_off, s->mgrp_tid.size()))
    return false;
  int kmax = 0;
  for (int r = 0; r < C; r++) kmax = std::max(kmax, s->mgrp_off[r + 1] - s->mgrp_off[r]);
  if (kmax != km) return false;
  auto ids_ok = [](const std::vector<int32_t>& v, int lo, int hi) {
    for (int32_t x : v)
      if (x < lo || x >= hi) return false;
    return true;
  };
  if (!ids_ok(s->provider, -1, NS) || !ids_ok(s->region, -1, NS) || !ids_ok(s->region_idx, -1, std::max(NR, 1)) ||
      !ids_ok(s->label_val, -1, NS) || !ids_ok(s->zone_ids, 0, std::max(NS, 1)) ||
      !ids_ok(s->taint_key, 0, std::max(NS, 1)) || !ids_ok(s->taint_val, 0, std::max(NS, 1)) ||
      !ids_ok(s->taint_eff, 0, 4) || !ids_ok(s->mgrp_tid, 0, std::max(T, 1)) || !ids_ok(s->mg_tid, 0, std::max(T, 1)))
    return false;
  for (int32_t x : s->mg_cnt)
    if (x < 0) return false;
  for (int64_t x : s->mgrp_cnt)
    if (x < 0) return false;
  return s->rid_cpu >= 0 && s->rid_cpu < R && s->rid_mem >= 0 && s->rid_mem < R && s->rid_eph >= 0 && s->rid_eph < R;
}
}  // namespace


// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int kp_abi_version(void) { return KP_ABI_VERSION; }

int kp_engine_create(int device, kp_engine** out) {
  if (!out) return KP_EINVAL;
  if (device < 0 || dev::device_count() <= device) return KP_EDEVICE;
  auto* e = new kp_engine();
  e->device = device;
  // KP_STREAMS: distinct HIP streams per engine (default 3). HIP maps a process's streams
  // onto GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin, and streams that
  // share a queue run in order: several engines in one process (batches in flight) then
  // fit the default queues with fewer streams each. 2: the result/region stream and the
  // SEL_ALL stream are one (the class orders and the large select_top slice keep their
  // own); 1: every launch of the call in one stream.
  int n_streams = 3;
  if (const char* v = getenv("KP_STREAMS")) n_streams = std::max(1, std::min(3, atoi(v)));
  bool fail = dev::set_device(device) || dev::stream_create(&e->stream);
  if (!fail && n_streams >= 3) fail = dev::stream_create(&e->stream2) != 0;
  else e->stream2 = e->stream;
  if (!fail && n_streams >= 2) fail = dev::stream_create(&e->stream3) != 0;
  else e->stream3 = e->stream2;
  if (fail) {
    if (e->stream3 && e->stream3 != e->stream2 && e->stream3 != e->stream) dev::stream_destroy(e->stream3);
    if (e->stream2 && e->stream2 != e->stream) dev::stream_destroy(e->stream2);
    if (e->stream) dev::stream_destroy(e->stream);
    delete e;
    return KP_EDEVICE;
  }
  for (auto& ev : e->ev) (void)dev::event_create(&ev);
  e->max_lds = dev::max_lds_per_block(device);
  if (const char* v = getenv("KP_TOP")) e->top_on = atoi(v) != 0;
  if (const char* v = getenv("KP_TOP_SPLIT")) e->top_split = atoi(v) != 0;
  if (const char* v = getenv("KP_SLOW_ORDER")) e->slow_order = atoi(v) != 0;
  if (const char* v = getenv("KP_GATE_FB")) e->gate_fb = atoi(v);
  if (const char* v = getenv("KP_ZC")) e->zc = atoi(v) != 0;
  if (const char* v = getenv("KP_SPEC_COPY")) e->spec_copy = atoi(v) != 0;
  if (const char* v = getenv("KP_TOP_WG")) e->top_wg = atoi(v) != 0;
  if (const char* v = getenv("KP_TOP_CAP")) {  // (tests: one capacity for both slices)
    e->top_cap = std::max(64, std::min(1024, atoi(v) & ~63));
    e->top_cap_small = std::min(e->top_cap_small, e->top_cap);
  }
  if (const char* v = getenv("KP_TOP_CAP_MID")) e->top_cap_mid = std::max(0, std::min(1024, atoi(v) & ~63));
  unsigned hc = std::thread::hardware_concurrency();
  e->n_threads = (int)std::max(1u, std::min(16u, hc));
  *out = e;
  return KP_OK;
}

void kp_engine_destroy(kp_engine* e) {
  if (!e) return;
  (void)dev::set_device(e->device);
  for (auto& ev : e->ev)
    if (ev) dev::event_destroy(ev);
  for (auto& ev : e->pev) dev::event_destroy(ev);
  // (aliases: KP_STREAMS < 3)
  if (e->stream3 && e->stream3 != e->stream2 && e->stream3 != e->stream) dev::stream_destroy(e->stream3);
  if (e->stream2 && e->stream2 != e->stream) dev::stream_destroy(e->stream2);
  if (e->stream) dev::stream_destroy(e->stream);
  delete e;
}

const char* kp_last_error(const kp_engine* e) { return e ? e->err.c_str() : "null engine"; }

int kp_engine_set_profile(kp_engine* e, int on) {
  if (!e) return KP_EINVAL;
  e->prof = on != 0;
  e->ktimes.clear();
  return KP_OK;
}

int kp_last_kernel_times(const kp_engine* e, kp_kernel_time* out, uint32_t cap, uint32_t* n_out) {
  if (!e || !n_out || (cap && !out)) return KP_EINVAL;
  *n_out = (uint32_t)e->ktimes.size();
  for (uint32_t i = 0; i < cap && i < e->ktimes.size(); i++) out[i] = e->ktimes[i];
  return KP_OK;
}

int kp_engine_set_threads(kp_engine* e, int n_threads) {
  if (!e || n_threads < 1) return KP_EINVAL;
  e->n_threads = std::min(n_threads, 256);
  return KP_OK;
}

int kp_snapshot_create(kp_engine* e, const kp_cluster* clusters, uint64_t n, const kp_options* opts,
                       kp_snapshot** out) {
  if (!e || !out || (n && !clusters)) return KP_EINVAL;
  (void)dev::set_device(e->device);
  auto* s = new kp_snapshot();
  s->e = e;
  int rc = build_snapshot(e, clusters, n, opts, s);
  if (rc != KP_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return KP_OK;
}

void kp_snapshot_destroy(kp_snapshot* s) { delete s; }

namespace {
// Rank r's packed row read back from the snapshot's host columns (the inverse
// of apply_rows), for the clusters an update leaves as they are.
ClusterRow row_of(const kp_snapshot* s, int r) {
  ClusterRow w;
  const int Cp = s->Cp;
  const int K = (int)s->keys.names.size(), AW = ((int)s->gvk.names.size() + 63) / 64, R = (int)s->res.names.size();
  w.flags = s->flags[r];
  w.provider = s->provider[r];
  w.provider_int = s->provider_int[r];
  w.region = s->region[r];
  w.region_int = s->region_int[r];
  for (int z = s->zone_off[r]; z < s->zone_off[r + 1]; z++) w.zones.push_back(s->zone_ids[z]);
  for (int k = 0; k < K; k++) {
    const int32_t v = s->label_val[(size_t)k * Cp + r];
    if (v >= 0) w.labels.push_back({k, v});
  }
  for (int t = s->taint_off[r]; t < s->taint_off[r + 1]; t++)
    w.taints.push_back({s->taint_key[t], s->taint_val[t], s->taint_eff[t]});
  for (int wd = 0; wd < AW; wd++) {
    uint64_t bits = s->api_bits[(size_t)wd * Cp + r];
    while (bits) {
      const int b = __builtin_ctzll(bits);
      w.gvks.push_back(wd * 64 + b);
      bits &= bits - 1;
    }
  }
  w.allowed = s->allowed[r];
  for (int j = 0; j < R; j++) {
    const int64_t a = s->avail[(size_t)j * Cp + r];
    if (a != 0) w.avail.push_back({j, a});
    const int64_t q = s->qa[(size_t)j * Cp + r];
    if (q != kQaAbsent) w.qa.push_back({j, q});
  }
  for (int g = s->mgrp_off[r]; g < s->mgrp_off[r + 1]; g++) w.groups.push_back({s->mgrp_tid[g], s->mgrp_cnt[g]});
  return w;
}
}  // namespace

int kp_snapshot_update(kp_engine* e, kp_snapshot* s, const kp_cluster* clusters, uint64_t n, int* dict_grew) {
  if (!e || !s || (n && !clusters)) return KP_EINVAL;
  (void)dev::set_device(e->device);
  const int C = s->C;
  std::vector<int64_t> upd(C, -1);
  for (uint64_t i = 0; i < n; i++) {
    const std::string name = S(clusters[i].name);
    auto it = s->rank_of.find(name);
    if (it == s->rank_of.end()) {
      e->err = "kp_snapshot_update: no cluster named " + name + " in the snapshot (re-create it to add clusters)";
      return KP_EINVAL;
    }
    if (upd[it->second] >= 0) {
      e->err = "kp_snapshot_update: cluster " + name + " listed twice";
      return KP_EINVAL;
    }
    upd[it->second] = (int64_t)i;
  }
  const size_t n_str = s->str.names.size(), n_keys = s->keys.names.size(), n_gvk = s->gvk.names.size(),
               n_res = s->res.names.size();
  const std::vector<std::string> regions0 = s->regions.names;
  std::vector<ClusterRow> rows(C);
  for (int r = 0; r < C; r++)
    if (upd[r] < 0) rows[r] = row_of(s, r);
  // the snapshot's templates by value (trailing zeros dropped, as pack_row keys them)
  std::map<std::vector<int64_t>, int32_t> tmpl_ids;
  std::vector<std::vector<int64_t>> tv(s->n_tmpl);
  {
    const int R0 = (int)n_res;
    for (int t = 0; t < s->n_tmpl; t++) {
      std::vector<int64_t> v(s->tmpl.begin() + (size_t)t * R0, s->tmpl.begin() + (size_t)(t + 1) * R0);
      while (!v.empty() && v.back() == 0) v.pop_back();
      tmpl_ids.emplace(v, t);
      tv[t] = v;
    }
  }
  for (int r = 0; r < C; r++)
    if (upd[r] >= 0) {
      const int rc = pack_row(e, s, clusters[upd[r]], tmpl_ids, &rows[r]);
      if (rc) return rc;  // columns untouched (the dictionaries may hold unused entries)
    }
  // templates still in use, renumbered in first-use order
  tv.resize(tmpl_ids.size());
  for (auto& kv : tmpl_ids) tv[kv.second] = kv.first;
  std::vector<int32_t> remap(tv.size(), -1);
  std::map<std::vector<int64_t>, int32_t> used;
  for (auto& w : rows)
    for (auto& g : w.groups) {
      if (remap[g.first] < 0) {
        remap[g.first] = (int32_t)used.size();
        used.emplace(tv[g.first], remap[g.first]);
      }
      g.first = remap[g.first];
    }
  apply_rows(s, rows, used);
  s->blob.clear();
  // region ids index the batches' region buffers: a changed region set counts too
  const bool grew = s->str.names.size() != n_str || s->keys.names.size() != n_keys || s->gvk.names.size() != n_gvk ||
                    s->res.names.size() != n_res || s->regions.names != regions0;
  if (dict_grew) *dict_grew = grew ? 1 : 0;
  if (grew) s->epoch = next_snap_epoch();  // (packed records resolved against the old dictionaries)
  s->dev.reset();
  return upload_snapshot(e, s);
}

int kp_snapshot_export(const kp_snapshot* cs, const void** bytes, uint64_t* n_bytes) {
  if (!cs || !bytes || !n_bytes) return KP_EINVAL;
  kp_snapshot* s = const_cast<kp_snapshot*>(cs);
  s->blob.clear();
  Wr w{s->blob};
  w.raw(kSnapMagic, 8);
  w.u64((uint64_t)s->C);
  w.u64(s->opts.enable_empty_workload_propagation);
  w.u64(s->opts.customized_cluster_resource_modeling);
  w.u64(s->opts.enabled_plugins);
  w.u64(s->opts.multiple_pod_templates_scheduling);
  w.u64(s->opts.n_out_of_tree_plugins);
  w.u64((uint64_t)(int64_t)s->rid_cpu);
  w.u64((uint64_t)(int64_t)s->rid_mem);
  w.u64((uint64_t)(int64_t)s->rid_eph);
  w.u64((uint64_t)s->n_tmpl);
  w.u64((uint64_t)s->kmax);
  w.strs(s->str.names);
  w.strs(s->keys.names);
  w.strs(s->gvk.names);
  w.strs(s->res.names);
  w.strs(s->regions.names);
  w.strs(s->names);
  w.vec(s->perm);
  w.vec(s->flags);
  w.vec(s->provider);
  w.vec(s->region);
  w.vec(s->region_idx);
  w.vec(s->zone_off);
  w.vec(s->zone_ids);
  w.vec(s->label_val);
  w.vec(s->taint_off);
  w.vec(s->taint_key);
  w.vec(s->taint_val);
  w.vec(s->taint_eff);
  w.vec(s->mgrp_off);
  w.vec(s->mgrp_tid);
  w.vec(s->mgrp_cnt);
  w.vec(s->mg_tid);
  w.vec(s->mg_cnt);
  w.vec(s->provider_int);
  w.vec(s->region_int);
  w.vec(s->allowed);
  w.vec(s->avail);
  w.vec(s->qa);
  w.vec(s->tmpl);
  w.vec(s->api_bits);
  *bytes = s->blob.data();
  *n_bytes = s->blob.size();
  return KP_OK;
}

// The host half of kp_snapshot_import: every host column from the byte image
// (no device work).
static int import_host(kp_engine* e, const void* bytes, uint64_t n_bytes, kp_snapshot* s) {
  Rd r{(const unsigned char*)bytes, (const unsigned char*)bytes + n_bytes};
  char magic[8];
  if (!r.raw(magic, 8) || memcmp(magic, kSnapMagic, 8) != 0) {
    e->err = "not a kp snapshot";
    return KP_EINVAL;
  }
  s->e = e;
  s->C = (int)r.u64();
  s->Cp = s->C ? ((s->C + 63) / 64) * 64 : 64;
  s->W = s->Cp / 64;
  s->opts.enable_empty_workload_propagation = (uint8_t)r.u64();
  s->opts.customized_cluster_resource_modeling = (uint8_t)r.u64();
  s->opts.enabled_plugins = (uint32_t)r.u64();
  s->opts.multiple_pod_templates_scheduling = (uint8_t)r.u64();
  s->opts.n_out_of_tree_plugins = (uint32_t)r.u64();
  s->rid_cpu = (int32_t)(int64_t)r.u64();
  s->rid_mem = (int32_t)(int64_t)r.u64();
  s->rid_eph = (int32_t)(int64_t)r.u64();
  s->n_tmpl = (int)r.u64();
  s->kmax = (int)r.u64();
  dict_from(s->str, r.strs());
  dict_from(s->keys, r.strs());
  dict_from(s->gvk, r.strs());
  dict_from(s->res, r.strs());
  dict_from(s->regions, r.strs());
  s->names = r.strs();
  s->perm = r.vec<uint32_t>();
  s->flags = r.vec<uint32_t>();
  s->provider = r.vec<int32_t>();
  s->region = r.vec<int32_t>();
  s->region_idx = r.vec<int32_t>();
  s->zone_off = r.vec<int32_t>();
  s->zone_ids = r.vec<int32_t>();
  s->label_val = r.vec<int32_t>();
  s->taint_off = r.vec<int32_t>();
  s->taint_key = r.vec<int32_t>();
  s->taint_val = r.vec<int32_t>();
  s->taint_eff = r.vec<int32_t>();
  s->mgrp_off = r.vec<int32_t>();
  s->mgrp_tid = r.vec<int32_t>();
  s->mgrp_cnt = r.vec<int64_t>();
  s->mg_tid = r.vec<int32_t>();
  s->mg_cnt = r.vec<int32_t>();
  s->provider_int = r.vec<int64_t>();
  s->region_int = r.vec<int64_t>();
  s->allowed = r.vec<int64_t>();
  s->avail = r.vec<int64_t>();
  s->qa = r.vec<int64_t>();
  s->tmpl = r.vec<int64_t>();
  s->api_bits = r.vec<uint64_t>();
  if (!r.ok || r.p != r.end || !snapshot_consistent(s)) {
    e->err = "truncated or inconsistent snapshot bytes";
    return KP_EINVAL;
  }
  s->inv.assign(s->C, -1);
  for (int rk = 0; rk < s->C; rk++) {
    s->rank_of[s->names[rk]] = rk;
    if (s->perm[rk] < (uint32_t)s->C) s->inv[s->perm[rk]] = rk;
  }
  return KP_OK;
}

int kp_snapshot_import(kp_engine* e, const void* bytes, uint64_t n_bytes, kp_snapshot** out) {
  if (!e || !bytes || !out) return KP_EINVAL;
  (void)dev::set_device(e->device);
  auto* s = new kp_snapshot();
  std::unique_ptr<kp_snapshot> guard(s);
  int rc = import_host(e, bytes, n_bytes, s);
  if (rc != KP_OK) return rc;
  rc = upload_snapshot(e, s);
  if (rc != KP_OK) return rc;
  *out = guard.release();
  return KP_OK;
}

// A replica of `src` on engine e's device: the host columns from its byte image
// and the device arena copied device to device (hipMemcpyPeer: over xGMI between
// the GPUs of one node), its views rebased onto the copy. Nothing is re-derived.
int kp_snapshot_replicate(kp_engine* e, const kp_snapshot* src, kp_snapshot** out) {
  if (!e || !src || !out) return KP_EINVAL;
  const void* bytes = nullptr;
  uint64_t n_bytes = 0;
  int rc = kp_snapshot_export(src, &bytes, &n_bytes);
  if (rc != KP_OK) return rc;
  (void)dev::set_device(e->device);
  auto* s = new kp_snapshot();
  std::unique_ptr<kp_snapshot> guard(s);
  rc = import_host(e, bytes, n_bytes, s);
  if (rc != KP_OK) return rc;
  const size_t total = src->dev.total;
  HIPCHK(s->dev.alloc_raw(total));
  HIPCHK(dev::peer_copy(s->dev.base, e->device, src->dev.base, src->e->device, total, e->stream));
  HIPCHK(dev::sync(e->stream));
  s->view = src->view;
  const char* b0 = (const char*)src->dev.base;
  char* b1 = (char*)s->dev.base;
  auto rb = [&](auto& p) {
    if (p) p = (std::remove_reference_t<decltype(p)>)(b1 + ((const char*)p - b0));
  };
  SnapView& v = s->view;
  rb(v.flags), rb(v.perm), rb(v.provider), rb(v.region), rb(v.region_idx), rb(v.provider_int), rb(v.region_int);
  rb(v.zone_off), rb(v.zone_ids), rb(v.label_val), rb(v.taint_off), rb(v.taint_key), rb(v.taint_val);
  rb(v.taint_eff), rb(v.taint_set), rb(v.tset_rep), rb(v.api_bits), rb(v.allowed), rb(v.avail), rb(v.qa);
  rb(v.mg_tid), rb(v.mg_cnt), rb(v.tmpl), rb(v.mt_cnt), rb(v.bits), rb(v.bkey), rb(v.bval);
  s->est_kind = src->est_kind;
  *out = guard.release();
  return KP_OK;
}

// Packs bindings [0, n) into bt->hdr and bt's pools on T host threads: thread t
// packs a contiguous chunk into its own Pools (the Packer only reads the snapshot's
// dictionaries), then the chunks are concatenated and every pool reference is
// rebased: header offsets, program ids in the ipool lists, Prog::ins_off and the
// list offsets inside Instr. The result equals a sequential pack (test_abi).
// Threads: KP_PACK_THREADS, else the CPUs this process may use (hardware threads,
// capped by a cgroup CPU quota), one per 4096 bindings at most.
// Estimator class key of a packed binding: everything the GeneralEstimator reads
// from it (est_load / est_compute_bf / template_md, kp_algo.h): whether it has
// ReplicaRequirements and its summary and model requests (resource id, divisor).
void est_key(const BindHdr& h, const Pools& p, std::string* k) {
  k->clear();
  auto put = [&](const void* v, size_t n) { k->append((const char*)v, n); };
  const uint32_t rr = h.flags & BF_HAS_RR;
  put(&rr, 4);
  put(&h.sreq_cnt, 4);
  for (int j = 0; j < h.sreq_cnt; j++) {
    put(&p.ipool[h.sreq_off + j], 4);
    put(&p.lpool[h.sreq_q_off + j], 8);
  }
  put(&h.mreq_cnt, 4);
  for (int j = 0; j < h.mreq_cnt; j++) {
    put(&p.ipool[h.mreq_off + j], 4);
    put(&p.lpool[h.mreq_q_off + j], 8);
  }
}

// A binding's route through kp_schedule_batch, recorded while packing so that the
// batch's lists come from one pass over n bytes instead of passes over the headers.
enum : uint8_t { RT_CLUSTER = 1, RT_REGION = 2, RT_DYN = 4, RT_SMALL = 8, RT_STATIC_OK = 16 };
KP_HD inline bool route_static_ok(const SnapView& v, const BindHdr& h, const int64_t* lpool) {
  if (h.sel != SEL_ALL || h.strategy != ST_STATIC || h.replicas < 0 || (int64_t)h.replicas >= kSeatWrap) return false;
  if (!(h.flags & BF_WORKLOAD_ASSIGN) || (h.flags & (BF_OVERFLOW | BF_DUP_TARGETS | BF_BAD))) return false;
  if (v.C >= 65536) return false;  // packed class counts
  if (h.flags & BF_HAS_WP) {
    if (h.sw_cnt > kSwRules || v.n_bits <= 0) return false;
    for (int j = 0; j < h.sw_cnt; j++)
      if (lpool[h.sw_w_off + j] >= (int64_t)kInt32Max) return false;  // saturated votes: SLOW_WEIGHT
  }
  return true;
}
// Replicas + len(spec.Clusters) up to which a binding takes k_select_top's small slice
// (KP_TOP_SMALL_NEED overrides kTopSmallNeed, for measurement).
inline int64_t top_small_need() {
  static const int64_t v = [] {
    const char* e = getenv("KP_TOP_SMALL_NEED");
    return e ? std::max<int64_t>(0, atoll(e)) : kTopSmallNeed;
  }();
  return v;
}
inline uint8_t route_of(const SnapView& v, const BindHdr& h, const int64_t* lpool) {
  uint8_t r = h.sel == SEL_CLUSTER ? RT_CLUSTER : h.sel == SEL_REGION ? RT_REGION : 0;
  if (!r) {
    if (h.strategy != ST_STATIC) r |= RT_DYN;
    if ((int64_t)h.replicas + h.tgt_cnt <= top_small_need()) r |= RT_SMALL;
    if (route_static_ok(v, h, lpool)) r |= RT_STATIC_OK;
  }
  return r;
}

// Packing reads each binding's struct and the strings and arrays it points to once,
// scattered over the caller's memory: cache misses, not the parsing, bound it (about
// 3k cycles per config-3 binding, spread evenly over the struct's sections). So the
// loop prefetches three levels ahead of the binding it packs: the struct of i + 3,
// the arrays and strings i + 2 points to, the strings inside i + 1's arrays.
inline void pf(const void* p) {
  if (p) __builtin_prefetch(p, 0, 3);
}
inline void pf_struct(const kp_binding* b) {
  for (size_t o = 0; o < sizeof(kp_binding); o += 64) pf((const char*)b + o);
}
inline void pf_affinity(const kp_cluster_affinity& a) {
  pf(a.match_labels);
  pf(a.match_expressions);
  pf(a.field_expressions);
  pf(a.cluster_names);
  pf(a.exclude_clusters);
}
inline void pf_arrays(const kp_binding& b) {
  pf(b.uid.ptr);
  pf(b.api_version.ptr);
  pf(b.kind.ptr);
  pf(b.resource_request);
  pf(b.clusters);
  pf(b.eviction_from);
  pf(b.tolerations);
  pf(b.spread_constraints);
  pf(b.static_weights);
  pf(b.cluster_affinities);
  if (b.has_cluster_affinity) pf_affinity(b.cluster_affinity);
}
inline void pf_strings(const kp_binding& b) {
  for (uint32_t j = 0; j < b.n_resource_request && j < 4; j++) {
    pf(b.resource_request[j].name.ptr);
    pf(b.resource_request[j].quantity.ptr);
  }
  for (uint32_t j = 0; j < b.n_clusters && j < 4; j++) pf(b.clusters[j].name.ptr);
  for (uint32_t j = 0; j < b.n_tolerations && j < 2; j++) {
    pf(b.tolerations[j].key.ptr);
    pf(b.tolerations[j].value.ptr);
  }
  if (b.has_cluster_affinity)
    for (uint32_t j = 0; j < b.cluster_affinity.n_match_expressions && j < 2; j++) {
      pf(b.cluster_affinity.match_expressions[j].key.ptr);
      pf(b.cluster_affinity.match_expressions[j].values);
    }
}

// Shifts a packed binding's pool references by (di, dl, dt, dp, dn) (ipool, lpool, tols,
// progs, instrs): its header, the program ids in its ipool lists, its programs'
// instruction offsets and its instructions' list offsets. ip: the binding's ipool slice
// (index = header offset - h.ip_beg, taken before the shift); pr / in: its program and
// instruction slices. pack_parallel's chunk merge applies the same shifts.
static void shift_binding(BindHdr& h, int32_t* ip, Prog* pr, int n_pr, Instr* in, int n_in, int32_t di, int32_t dl,
                          int32_t dt, int32_t dp, int32_t dn) {
  for (int j = 0; j < h.filt_cnt; j++) ip[h.filt_off - h.ip_beg + j] += dp;
  for (int j = 0; j < h.ovf_cnt; j++) ip[h.ovf_off - h.ip_beg + j] += dp;
  for (int j = 0; j < h.sw_cnt; j++) ip[h.sw_off - h.ip_beg + j] += dp;
  h.tgt_off += di, h.evict_off += di, h.filt_off += di, h.ovf_off += di, h.sw_off += di;
  h.sreq_off += di, h.mreq_off += di, h.ip_beg += di, h.ip_end += di;
  h.sw_w_off += dl, h.sreq_q_off += dl, h.mreq_q_off += dl;
  h.tol_off += dt;
  h.pr_beg += dp, h.pr_end += dp;
  h.in_beg += dn, h.in_end += dn;
  for (int j = 0; j < n_pr; j++) pr[j].ins_off += dn;
  for (int j = 0; j < n_in; j++) {
    Instr& x = in[j];
    if (x.op == OP_EXCLUDE || x.op == OP_NAMES) x.a += di;
    else if (x.op == OP_LBL_IN || x.op == OP_LBL_NOTIN || x.op == OP_FLD_IN || x.op == OP_FLD_NOTIN ||
             x.op == OP_ZONE_IN || x.op == OP_ZONE_NOTIN)
      x.b += di;
  }
}

// One binding's packed record (kp_pack_cache), one allocation: this struct (the header
// with every pool reference relative to the record's own slices, the key and the status
// fields it was packed with), then its slices (lpool, instrs, tols, progs, ipool) and the
// uid, observed-affinity-name and estimator-class-key bytes.
struct PackRec {
  uint64_t key;
  int64_t gen, rt_ns, lst_ns;
  uint8_t has_rt, has_lst, nonworkload;  // nonworkload: bcls -1 (the estimator skipped)
  int32_t n_ip, n_lp, n_tol, n_pr, n_in;
  uint32_t uid_len, aff_len, cls_len;
  BindHdr h;
  unsigned char* tail() const { return (unsigned char*)(this + 1); }
  int64_t* lp() const { return (int64_t*)tail(); }
  Instr* in() const { return (Instr*)(lp() + n_lp); }
  Tol* tol() const { return (Tol*)(in() + n_in); }
  Prog* pr() const { return (Prog*)(tol() + n_tol); }
  int32_t* ip() const { return (int32_t*)(pr() + n_pr); }
  const char* uid() const { return (const char*)(ip() + n_ip); }
  const char* aff() const { return uid() + uid_len; }
  const char* cls() const { return aff() + aff_len; }
  static PackRec* make(int n_ip, int n_lp, int n_tol, int n_pr, int n_in, size_t n_str) {
    const size_t bytes = sizeof(PackRec) + 8 * (size_t)n_lp + sizeof(Instr) * (size_t)n_in +
                         sizeof(Tol) * (size_t)n_tol + sizeof(Prog) * (size_t)n_pr + 4 * (size_t)n_ip + n_str;
    auto* r = (PackRec*)::operator new(bytes, std::align_val_t(alignof(PackRec)));
    r->n_ip = n_ip, r->n_lp = n_lp, r->n_tol = n_tol, r->n_pr = n_pr, r->n_in = n_in;
    return r;
  }
  static void free(PackRec* r) { ::operator delete((void*)r, std::align_val_t(alignof(PackRec))); }
  bool same(const kp_binding_key& k, const kp_binding& b) const {
    return gen == k.generation && uid_len == k.uid.len && memcmp(uid(), k.uid.ptr, uid_len) == 0 &&
           has_rt == b.has_reschedule_triggered_at && has_lst == b.has_last_scheduled_time &&
           (!has_rt || rt_ns == b.reschedule_triggered_at_ns) && (!has_lst || lst_ns == b.last_scheduled_time_ns) &&
           std::string_view(aff(), aff_len) == SV(b.observed_affinity_name);
  }
};

// The records by key hash: kCacheShards open-addressed tables (linear probing, load <= 1/2;
// each slot holds the key beside the pointer, so a probe touches the table only), read-only
// while the packing threads look records up, filled shard by shard after.
constexpr int kCacheShards = 64;
struct PackTable {
  struct Slot {
    uint64_t key;  // 0: empty
    PackRec* r;
  };
  std::vector<Slot> slot;
  uint64_t n = 0;
  static size_t home(uint64_t key, size_t cap) { return (size_t)((key >> 6) * 0x9e3779b97f4a7c15ull >> 20) & (cap - 1); }
  const Slot* home_slot(uint64_t key) const { return slot.empty() ? nullptr : &slot[home(key, slot.size())]; }
  const PackRec* find(uint64_t key) const {
    if (slot.empty()) return nullptr;
    const size_t cap = slot.size();
    for (size_t i = home(key, cap);; i = (i + 1) & (cap - 1)) {
      if (slot[i].key == key) return slot[i].r;
      if (!slot[i].key) return nullptr;
    }
  }
  void put(PackRec* r) {  // (replaces a record of the same key)
    if (2 * (n + 1) > slot.size()) {
      std::vector<Slot> old(std::max<size_t>(64, 2 * slot.size()), Slot{0, nullptr});
      old.swap(slot);
      n = 0;
      for (const Slot& x : old)
        if (x.key) put(x.r);
    }
    const size_t cap = slot.size();
    for (size_t i = home(r->key, cap);; i = (i + 1) & (cap - 1)) {
      if (!slot[i].key) {
        slot[i] = Slot{r->key, r};
        n++;
        return;
      }
      if (slot[i].key == r->key) {
        PackRec::free(slot[i].r);
        slot[i].r = r;
        return;
      }
    }
  }
  void clear() {
    for (Slot& x : slot)
      if (x.key) PackRec::free(x.r), x = Slot{0, nullptr};
    n = 0;
  }
  ~PackTable() { clear(); }
};
}  // extern "C"

struct kp_pack_cache {
  uint64_t epoch = 0;  // the snapshot epoch the records resolved against (0: none yet)
  uint64_t max_entries = (uint64_t)4 << 20;
  uint64_t hits = 0, misses = 0, last_hits = 0;
  PackTable shard[kCacheShards];
  uint64_t entries() const {
    uint64_t e = 0;
    for (const auto& t : shard) e += t.n;
    return e;
  }
  void clear() {
    for (auto& t : shard) t.clear();
  }
};

extern "C" {
static inline uint64_t cache_key(const kp_binding_key& k) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the uid bytes, then the generation
  for (uint32_t i = 0; i < k.uid.len; i++) h = (h ^ (uint8_t)k.uid.ptr[i]) * 1099511628211ull;
  h ^= (uint64_t)k.generation * 0x9e3779b97f4a7c15ull;
  h ^= h >> 29;
  return h ? h : 1;
}

bool pack_parallel(kp_snapshot* s, const kp_binding* bindings, int n, kp_batch* bt, const kp_binding_key* keys = nullptr,
                   kp_pack_cache* cache = nullptr) {
  int T = host_cpus();
  if (const char* v = getenv("KP_PACK_THREADS")) T = atoi(v);
  T = std::max(1, std::min(T, n / 4096));
  // Chunks of kPackChunk bindings taken from a shared counter (a thread that meets heavy
  // bindings takes fewer chunks); each chunk packs into its own pools, concatenated in
  // chunk order below. Packer caches and class-id maps are per thread.
  constexpr int kPackChunk = 1024;
  const int K = std::max(1, (n + kPackChunk - 1) / kPackChunk);
  std::vector<Pools> pl(K);
  std::vector<int> lo(K + 1), owner(K, 0);
  for (int k = 0; k <= K; k++) lo[k] = std::min(n, k * kPackChunk);
  // estimator classes: thread-local ids (bt->bcls) and keys, unified below
  bt->bcls.resize(n);
  std::vector<std::vector<std::string>> tkeys(T);
  std::vector<std::string> terr(T);
  std::vector<double> tms(T, 0.0), tstart(T, 0.0);
  const auto tpack0 = std::chrono::steady_clock::now();
  std::atomic<int> next_chunk(0);
  bt->route.resize(n);
  std::vector<uint64_t> chunk_cap(K + 1, 0);  // result slots per chunk (out_off prefix sums)
  std::vector<int> tmax_tgt(T, 0), tmax_tiers(T, 1);
  // kp_pack_cache: records of another snapshot epoch, or past the size cap, are dropped
  // first; new records collect per (chunk, shard) and go into the shards after the pack
  if (cache && (cache->epoch != s->epoch || cache->entries() > cache->max_entries)) {
    cache->clear();
    cache->epoch = s->epoch;
  }
  std::vector<std::vector<PackRec*>> newrecs(cache ? (size_t)K * kCacheShards : 0);
  struct RecGuard {  // records not handed to the cache (a failed batch) are freed
    std::vector<std::vector<PackRec*>>* v;
    ~RecGuard() {
      for (auto& x : *v)
        for (PackRec* r : x)
          if (r) PackRec::free(r);
    }
  } rec_guard{&newrecs};
  std::vector<uint64_t> thits(T, 0);  // (added once per chunk: adjacent slots share a line)
  auto run = [&](int t) {
    const auto tt0 = std::chrono::steady_clock::now();
    struct Stamp {
      std::chrono::steady_clock::time_point t0;
      double* out;
      ~Stamp() { *out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } stamp{tt0, &tms[t]};
    tstart[t] = std::chrono::duration<double, std::milli>(tt0 - tpack0).count();
    Packer pk{s, nullptr};
    SvMap<int32_t> ids;
    std::string key;
    SetsArgs A;
    for (;;) {
      const int k = next_chunk.fetch_add(1);
      if (k >= K) break;
      owner[k] = t;
      pk.bt = &pl[k];
      uint64_t cap = 0, hits = 0;  // (chunk and thread totals kept in registers: the shared
      int max_tgt = 0, max_tiers = 1;  // arrays are written once per chunk, not once per binding)
      const int hi = lo[k + 1];
      // kp_pack_cache lookups run ahead of the packing in stages, each prefetching what the
      // next one reads: the uid bytes (8 ahead), the key hash and its table slot (4 ahead), the
      // record (2 ahead); bindings without a record get the packer's own prefetches instead
      constexpr int kRing = 16;
      uint64_t ck_ring[kRing];
      const PackRec* rec_ring[kRing];
      auto keyed_at = [&](int j) { return cache && j < hi && keys[j].uid.len > 0; };
      auto stage_hash = [&](int j) {
        if (!keyed_at(j)) return;
        const uint64_t c = cache_key(keys[j]);
        ck_ring[j % kRing] = c;
        pf(cache->shard[c % kCacheShards].home_slot(c));
      };
      auto stage_rec = [&](int j) {
        const PackRec* r = nullptr;
        if (keyed_at(j)) {
          const uint64_t c = ck_ring[j % kRing];
          r = cache->shard[c % kCacheShards].find(c);
          if (r)
            for (int o = 0; o < 8; o++) pf((const char*)r + 64 * o);
        }
        rec_ring[j % kRing] = r;
        if (!r && j < hi) pf_arrays(bindings[j]);
      };
      for (int q = lo[k]; q < std::min(hi, lo[k] + 3); q++) pf_struct(&bindings[q]);
      if (cache) {
        for (int q = lo[k]; q < std::min(hi, lo[k] + 8); q++)
          if (keyed_at(q)) pf(keys[q].uid.ptr);
        for (int q = lo[k]; q < lo[k] + 4; q++) stage_hash(q);
        for (int q = lo[k]; q < lo[k] + 2; q++) stage_rec(q);
      } else if (lo[k] + 1 < hi) {
        pf_arrays(bindings[lo[k] + 1]);
      }
      for (int i = lo[k]; i < hi; i++) {
        if (i + 3 < hi) pf_struct(&bindings[i + 3]);
        if (cache) {
          if (keyed_at(i + 8)) pf(keys[i + 8].uid.ptr);
          stage_hash(i + 4);
          stage_rec(i + 2);
          if (i + 1 < hi && !rec_ring[(i + 1) % kRing]) pf_strings(bindings[i + 1]);
        } else {
          if (i + 2 < hi) pf_arrays(bindings[i + 2]);
          if (i + 1 < hi) pf_strings(bindings[i + 1]);
        }
        // a cached record (kp_pack_cache): the same key, generation and status fields
        const bool keyed = keyed_at(i);
        const uint64_t ck = keyed ? ck_ring[i % kRing] : 0;
        const PackRec* hit = keyed ? rec_ring[i % kRing] : nullptr;
        if (hit && !hit->same(keys[i], bindings[i])) hit = nullptr;
        Pools& P = pl[k];
        const size_t ip0 = P.ipool.size(), lp0 = P.lpool.size(), to0 = P.tols.size(), pr0 = P.progs.size(),
                     in0 = P.instrs.size();
        if (hit) {  // the record's slices appended, its references shifted onto them
          BindHdr& h = bt->hdr[i];
          h = hit->h;
          P.ipool.insert(P.ipool.end(), hit->ip(), hit->ip() + hit->n_ip);
          P.lpool.insert(P.lpool.end(), hit->lp(), hit->lp() + hit->n_lp);
          P.tols.insert(P.tols.end(), hit->tol(), hit->tol() + hit->n_tol);
          P.progs.insert(P.progs.end(), hit->pr(), hit->pr() + hit->n_pr);
          P.instrs.insert(P.instrs.end(), hit->in(), hit->in() + hit->n_in);
          shift_binding(h, P.ipool.data() + ip0, P.progs.data() + pr0, hit->n_pr, P.instrs.data() + in0, hit->n_in,
                        (int32_t)ip0, (int32_t)lp0, (int32_t)to0, (int32_t)pr0, (int32_t)in0);
          hits++;
        } else {
          pk.pack(bindings[i], bt->hdr[i]);
        }
        {
          const BindHdr& h = bt->hdr[i];
          cap += h.out_cap;
          bt->route[i] = route_of(s->view, h, pl[k].lpool.data());  // (chunk-relative pool offsets)
          max_tgt = std::max(max_tgt, (int)h.tgt_cnt);
          max_tiers = std::max(max_tiers, (int)h.ovf_cnt + 2);  // primary, each overflow term, unmatched
        }
        bool nonworkload = false;
        if (hit) {
          nonworkload = hit->nonworkload;
          if (!nonworkload) key.assign(hit->cls(), hit->cls_len);
        } else if (bt->hdr[i].flags & BF_NONWORKLOAD_EST) {
          nonworkload = true;
        } else {
          if (bt->hdr[i].flags & BF_SETS) {
            // a component-set class: key 'S' + the resolved SetsArgs (est_key's keys
            // start with the 0/1 ReplicaRequirements word, never 'S')
            std::string err;
            const int rc = build_sets_args(s, bindings[i].components, bindings[i].n_components, &A, &err);
            if (rc == KP_EINVAL) {
              bt->hdr[i].flags = (bt->hdr[i].flags & ~(uint32_t)BF_SETS) | BF_BAD;  // status ERROR, as a bad request
            } else if (rc != KP_OK) {
              if (terr[t].empty()) terr[t] = err;
              bt->hdr[i].flags &= ~(uint32_t)BF_SETS;
            }
            bt->route[i] = route_of(s->view, bt->hdr[i], pl[k].lpool.data());  // (flags changed)
          }
          if (bt->hdr[i].flags & BF_SETS) {
            key.assign(1, 'S');
            key.append((const char*)&A, sizeof(A));
          } else {
            est_key(bt->hdr[i], pl[k], &key);
          }
        }
        if (keyed && !hit) {  // a new record: the binding's slices, references relative to them
          const kp_binding& bb = bindings[i];
          const uint32_t ul = keys[i].uid.len, al = bb.observed_affinity_name.len,
                         cl = nonworkload ? 0u : (uint32_t)key.size();
          PackRec* r = PackRec::make((int)(P.ipool.size() - ip0), (int)(P.lpool.size() - lp0),
                                     (int)(P.tols.size() - to0), (int)(P.progs.size() - pr0),
                                     (int)(P.instrs.size() - in0), (size_t)ul + al + cl);
          r->key = ck;
          r->gen = keys[i].generation;
          r->has_rt = bb.has_reschedule_triggered_at;
          r->has_lst = bb.has_last_scheduled_time;
          r->rt_ns = r->has_rt ? bb.reschedule_triggered_at_ns : 0;
          r->lst_ns = r->has_lst ? bb.last_scheduled_time_ns : 0;
          r->nonworkload = nonworkload ? 1 : 0;
          r->uid_len = ul, r->aff_len = al, r->cls_len = cl;
          r->h = bt->hdr[i];
          std::copy(P.ipool.begin() + (long)ip0, P.ipool.end(), r->ip());
          std::copy(P.lpool.begin() + (long)lp0, P.lpool.end(), r->lp());
          std::copy(P.tols.begin() + (long)to0, P.tols.end(), r->tol());
          std::copy(P.progs.begin() + (long)pr0, P.progs.end(), r->pr());
          std::copy(P.instrs.begin() + (long)in0, P.instrs.end(), r->in());
          if (ul) memcpy((char*)r->uid(), keys[i].uid.ptr, ul);
          if (al) memcpy((char*)r->aff(), bb.observed_affinity_name.ptr, al);
          if (cl) memcpy((char*)r->cls(), key.data(), cl);
          shift_binding(r->h, r->ip(), r->pr(), r->n_pr, r->in(), r->n_in, -(int32_t)ip0, -(int32_t)lp0,
                        -(int32_t)to0, -(int32_t)pr0, -(int32_t)in0);
          newrecs[(size_t)k * kCacheShards + ck % kCacheShards].push_back(r);
        }
        if (nonworkload) {
          bt->bcls[i] = -1;
          continue;
        }
        auto it = ids.find(key);
        if (it == ids.end()) {
          it = ids.emplace(key, (int32_t)tkeys[t].size()).first;
          tkeys[t].push_back(key);
        }
        bt->bcls[i] = it->second;
      }
      chunk_cap[k + 1] = cap;
      thits[t] += hits;
      tmax_tgt[t] = std::max(tmax_tgt[t], max_tgt);
      tmax_tiers[t] = std::max(tmax_tiers[t], max_tiers);
    }
  };
  auto on_threads = [&](auto fn) { HostPool::get().run(T, std::function<void(int)>(fn)); };
  const auto tq0 = std::chrono::steady_clock::now();
  on_threads(run);
  const auto tq1 = std::chrono::steady_clock::now();
  for (auto& x : terr)
    if (!x.empty()) {
      bt->err = x;
      return false;
    }
  // pools concatenated in chunk order: each chunk's bases are the prefix sums of the
  // pool sizes before it; the threads rebase the chunks' headers and instructions
  // and copy their pools into place, chunk by chunk from a shared counter
  std::vector<size_t> bi(K + 1, 0), bl(K + 1, 0), bo(K + 1, 0), bp(K + 1, 0), bn(K + 1, 0);
  for (int k = 0; k < K; k++) {
    bi[k + 1] = bi[k] + pl[k].ipool.size();
    bl[k + 1] = bl[k] + pl[k].lpool.size();
    bo[k + 1] = bo[k] + pl[k].tols.size();
    bp[k + 1] = bp[k] + pl[k].progs.size();
    bn[k + 1] = bn[k] + pl[k].instrs.size();
  }
  if (bi[K] > (size_t)INT32_MAX || bl[K] > (size_t)INT32_MAX || bo[K] > (size_t)INT32_MAX ||
      bp[K] > (size_t)INT32_MAX || bn[K] > (size_t)INT32_MAX)
    return false;  // pool offsets are int32
  bt->ipool.resize(bi[K]);
  bt->lpool.resize(bl[K]);
  bt->tols.resize(bo[K]);
  bt->progs.resize(bp[K]);
  bt->instrs.resize(bn[K]);
  // global class ids (1-based; 0 = non-workload): the threads' keys in thread order
  SvMap<int32_t> gid;
  bt->crep.assign(1, 0);
  std::vector<std::vector<int32_t>> remaps(T);
  for (int t = 0; t < T; t++) {
    std::vector<int32_t>& remap = remaps[t];
    remap.resize(tkeys[t].size());
    for (size_t j = 0; j < tkeys[t].size(); j++) {
      auto it = gid.emplace(tkeys[t][j], (int32_t)gid.size() + 1).first;
      remap[j] = it->second;
      if ((size_t)it->second == bt->crep.size()) {
        bt->crep.push_back(-1);
        const std::string& key = tkeys[t][j];
        if (!key.empty() && key[0] == 'S') {  // component-set class: its rows come from k_sets_rows
          SetsArgs A;
          memcpy(&A, key.data() + 1, sizeof(A));
          bt->sets_cls.push_back(it->second);
          bt->sets_args.push_back(A);
        }
      }
    }
  }
  for (int k = 0; k < K; k++) chunk_cap[k + 1] += chunk_cap[k];
  bt->out_cap = chunk_cap[K];
  bt->max_tgt = *std::max_element(tmax_tgt.begin(), tmax_tgt.end());
  bt->max_tiers = *std::max_element(tmax_tiers.begin(), tmax_tiers.end());
  std::atomic<int> next_merge(0);
  auto merge = [&](int) {
    for (;;) {
      const int k = next_merge.fetch_add(1);
      if (k >= K) break;
      Pools& q = pl[k];
      const int32_t oi = (int32_t)bi[k], ol = (int32_t)bl[k], oo = (int32_t)bo[k], op = (int32_t)bp[k],
                    on = (int32_t)bn[k];
      const std::vector<int32_t>& remap = remaps[owner[k]];
      uint64_t off = chunk_cap[k];
      for (int i = lo[k]; i < lo[k + 1]; i++) {
        BindHdr& h = bt->hdr[i];
        bt->bcls[i] = bt->bcls[i] < 0 ? 0 : remap[bt->bcls[i]];
        h.out_off = off;  // private result slots: no atomic on the emit path
        off += h.out_cap;
        if (k == 0) continue;
        for (int j = 0; j < h.filt_cnt; j++) q.ipool[h.filt_off + j] += op;
        for (int j = 0; j < h.ovf_cnt; j++) q.ipool[h.ovf_off + j] += op;
        for (int j = 0; j < h.sw_cnt; j++) q.ipool[h.sw_off + j] += op;
        h.tgt_off += oi, h.evict_off += oi, h.filt_off += oi, h.ovf_off += oi, h.sw_off += oi;
        h.sreq_off += oi, h.mreq_off += oi, h.ip_beg += oi, h.ip_end += oi;
        h.sw_w_off += ol, h.sreq_q_off += ol, h.mreq_q_off += ol;
        h.tol_off += oo;
        h.pr_beg += op, h.pr_end += op;
        h.in_beg += on, h.in_end += on;
      }
      if (k > 0) {
        for (Prog& p : q.progs) p.ins_off += on;
        for (Instr& x : q.instrs) {
          if (x.op == OP_EXCLUDE || x.op == OP_NAMES) x.a += oi;
          else if (x.op == OP_LBL_IN || x.op == OP_LBL_NOTIN || x.op == OP_FLD_IN || x.op == OP_FLD_NOTIN ||
                   x.op == OP_ZONE_IN || x.op == OP_ZONE_NOTIN)
            x.b += oi;
        }
      }
      std::copy(q.ipool.begin(), q.ipool.end(), bt->ipool.begin() + (long)bi[k]);
      std::copy(q.lpool.begin(), q.lpool.end(), bt->lpool.begin() + (long)bl[k]);
      std::copy(q.tols.begin(), q.tols.end(), bt->tols.begin() + (long)bo[k]);
      std::copy(q.progs.begin(), q.progs.end(), bt->progs.begin() + (long)bp[k]);
      std::copy(q.instrs.begin(), q.instrs.end(), bt->instrs.begin() + (long)bn[k]);
      q = Pools();
    }
  };
  on_threads(merge);
  if (cache) {  // the new records into the shards (thread t fills shards t, t + T, ...)
    on_threads([&](int t) {
      for (int sh = t; sh < kCacheShards; sh += T) {
        PackTable& tab = cache->shard[sh];
        for (int k = 0; k < K; k++)
          for (PackRec*& r : newrecs[(size_t)k * kCacheShards + sh]) {
            tab.put(r);
            r = nullptr;
          }
      }
    });
    uint64_t h = 0;
    for (uint64_t x : thits) h += x;
    cache->hits += h;
    cache->misses += (uint64_t)n - h;
    cache->last_hits = h;
  }
  // a class's representative: its first binding
  size_t left = bt->crep.size() - 1;
  for (int i = 0; i < n && left; i++) {
    const int32_t g = bt->bcls[i];
    if (g && bt->crep[g] < 0) {
      bt->crep[g] = i;
      left--;
    }
  }
  if (getenv("KP_PACK_TIMING")) {
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    fprintf(stderr, "pack_parallel: %d threads, %d chunks, pack %.1f ms, merge+classes %.1f ms; per thread", T, K,
            ms(tq0, tq1), ms(tq1, std::chrono::steady_clock::now()));
    for (double x : tms) fprintf(stderr, " %.1f", x);
    fprintf(stderr, "; started at");
    for (double x : tstart) fprintf(stderr, " %.1f", x);
    fprintf(stderr, "\n");
#ifdef KP_PACK_PROF
    fprintf(stderr, "pack sections (Mcycles, cumulative): gvk %.1f targets %.1f tolerations %.1f affinity %.1f "
            "static %.1f requests %.1f rest %.1f\n", g_pack_cyc[0] / 1e6, g_pack_cyc[1] / 1e6, g_pack_cyc[2] / 1e6,
            g_pack_cyc[3] / 1e6, g_pack_cyc[4] / 1e6, g_pack_cyc[5] / 1e6, g_pack_cyc[6] / 1e6);
#endif
  }
  return true;
}

// Bindings per estimator class below which a batch skips the class orders.
static int64_t order_amort() {  // (read per batch: tests switch it)
  const char* e = getenv("KP_ORDER_AMORT");
  return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)4;
}

static int batch_create_impl(kp_engine* e, const kp_snapshot* sc, const kp_binding* bindings, uint64_t n,
                             const kp_binding_key* keys, kp_pack_cache* cache, kp_batch** out);
int kp_batch_create(kp_engine* e, const kp_snapshot* sc, const kp_binding* bindings, uint64_t n, kp_batch** out) {
  return batch_create_impl(e, sc, bindings, n, nullptr, nullptr, out);
}
int kp_batch_create_keyed(kp_engine* e, const kp_snapshot* sc, const kp_binding* bindings, const kp_binding_key* keys,
                          uint64_t n, kp_pack_cache* cache, kp_batch** out) {
  if (!cache || (n && !keys)) return KP_EINVAL;
  return batch_create_impl(e, sc, bindings, n, keys, cache, out);
}
int kp_batch_digest(const kp_batch* b, uint64_t* out) {
  if (!b || !out) return KP_EINVAL;
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
  };
  mix(b->hdr.data(), sizeof(BindHdr) * b->hdr.size());
  mix(b->ipool.data(), 4 * b->ipool.size());
  mix(b->lpool.data(), 8 * b->lpool.size());
  mix(b->tols.data(), sizeof(Tol) * b->tols.size());
  mix(b->progs.data(), sizeof(Prog) * b->progs.size());
  mix(b->instrs.data(), sizeof(Instr) * b->instrs.size());
  mix(b->route.data(), b->route.size());
  for (size_t i = 0; i < b->bcls.size(); i++) {  // the class by its first binding (ids follow thread order)
    const int32_t g = b->bcls[i];
    const int32_t rep = g > 0 && (size_t)g < b->crep.size() ? b->crep[g] : -1;
    mix(&rep, 4);
  }
  *out = h;
  return KP_OK;
}
int kp_pack_cache_create(uint64_t max_entries, kp_pack_cache** out) {
  if (!out) return KP_EINVAL;
  auto* c = new kp_pack_cache();
  if (max_entries) c->max_entries = max_entries;
  *out = c;
  return KP_OK;
}
void kp_pack_cache_destroy(kp_pack_cache* c) { delete c; }
int kp_pack_cache_get_stats(const kp_pack_cache* c, kp_pack_cache_stats* out) {
  if (!c || !out) return KP_EINVAL;
  out->hits = c->hits;
  out->misses = c->misses;
  out->entries = c->entries();
  out->last_hits = c->last_hits;
  return KP_OK;
}
static int batch_create_impl(kp_engine* e, const kp_snapshot* sc, const kp_binding* bindings, uint64_t n,
                             const kp_binding_key* keys, kp_pack_cache* cache, kp_batch** out) {
  if (!e || !sc || !out || (n && !bindings)) return KP_EINVAL;
  if (n > (uint64_t)INT32_MAX) return KP_ENOTSUP;
  (void)dev::set_device(e->device);
  kp_snapshot* s = const_cast<kp_snapshot*>(sc);
  auto* bt = new kp_batch();
  std::unique_ptr<kp_batch> guard(bt);
  bt->snap = s;
  bt->B = (int)n;
  bt->hdr.resize(n);
  const auto tp0 = std::chrono::steady_clock::now();
  if (s->opts.multiple_pod_templates_scheduling)
    for (uint64_t i = 0; i < n; i++)
      if (bindings[i].n_components > 0 && !bindings[i].components) {
        e->err = "kp_batch_create: binding " + std::to_string(i) +
                 " has n_components > 0 but no components (the MultiplePodTemplatesScheduling gate reads them)";
        return KP_EINVAL;
      }
  if (!pack_parallel(s, bindings, (int)n, bt, keys, cache)) {
    e->err = bt->err.empty() ? "batch pools exceed 2^31 entries" : bt->err;
    return KP_ENOTSUP;
  }
  // the selection lists from the routes (binding order within each kind). SEL_ALL:
  // [non-StaticWeight | StaticWeight]; the non-StaticWeight ones split by the subset
  // they likely need (k_select_top's small LDS slice first: a DynamicWeight /
  // Aggregated subset holds the scheduled clusters and about as many walked parties
  // as the target replicas), each part grouped by estimator class (counting sort,
  // stable: the workgroups resident at any moment then cover a short run of the list,
  // i.e. few classes, whose orders and rows stay in every XCD's L2; k_select_top
  // 1.23 -> 1.10 ms at config 3, mapping each XCD to one contiguous run of the list
  // instead was slower, 1.33 ms); StaticWeight bindings the class-level kernel covers
  // (bits mode) before the others.
  {
    const std::vector<uint8_t>& rt = bt->route;
    const size_t ncls = std::max<size_t>(1, bt->crep.size());
    std::vector<int32_t> cnt(2 * ncls + 1, 0);
    int n_dyn = 0, n_small = 0, n_stat = 0, n_stat_ok = 0, n_cl = 0, n_rg = 0;
    for (uint64_t i = 0; i < n; i++) {
      const uint8_t r = rt[i];
      if (r & RT_CLUSTER) n_cl++;
      else if (r & RT_REGION) n_rg++;
      else if (r & RT_DYN) {
        n_dyn++;
        const bool sm = (r & RT_SMALL) != 0;
        n_small += sm;
        cnt[(sm ? 0 : ncls) + (size_t)std::max(0, bt->bcls[i]) + 1]++;
      } else {
        n_stat++;
        n_stat_ok += (r & RT_STATIC_OK) ? 1 : 0;
      }
    }
    for (size_t k = 1; k <= 2 * ncls; k++) cnt[k] += cnt[k - 1];
    bt->l_all.resize((size_t)n_dyn + n_stat);
    bt->l_cluster.resize(n_cl);
    bt->l_region.resize(n_rg);
    bt->l_cs.resize((size_t)n_cl + n_rg);
    int pc = 0, pr = 0, ps = n_dyn, pso = n_dyn + n_stat_ok, pcs = 0;
    for (uint64_t i = 0; i < n; i++) {
      const uint8_t r = rt[i];
      const int32_t b = (int32_t)i;
      if (r & (RT_CLUSTER | RT_REGION)) {
        bt->l_cs[pcs++] = b;
        if (r & RT_CLUSTER) bt->l_cluster[pc++] = b;
        else bt->l_region[pr++] = b;
      } else if (r & RT_DYN) {
        bt->l_all[cnt[((r & RT_SMALL) ? 0 : ncls) + (size_t)std::max(0, bt->bcls[i])]++] = b;
      } else if (r & RT_STATIC_OK) {
        bt->l_all[ps++] = b;
      } else {
        bt->l_all[pso++] = b;
      }
    }
    bt->n_all_dyn = n_dyn;
    bt->n_top_small = n_small;
    bt->n_static = n_stat_ok;
    // KP_SPREAD_GROUP=1: the spread lists grouped by estimator class too (stable), as the
    // SEL_ALL list is; measured no better (config 4 3.84 vs 3.74 ms), so binding order
    static const bool spread_group = [] {
      const char* v = getenv("KP_SPREAD_GROUP");
      return v && atoi(v) != 0;
    }();
    if (spread_group)
      for (std::vector<int32_t>* lst : {&bt->l_cluster, &bt->l_region}) {
        if (lst->size() < 2) continue;
        std::vector<int32_t> c2(ncls + 1, 0), o2(lst->size());
        for (int32_t b : *lst) c2[(size_t)std::max(0, bt->bcls[b]) + 1]++;
        for (size_t k = 1; k <= ncls; k++) c2[k] += c2[k - 1];
        for (int32_t b : *lst) o2[(size_t)c2[(size_t)std::max(0, bt->bcls[b])]++] = b;
        lst->swap(o2);
      }
    // KP_TOP_LPT=1: the large-subset part heaviest first (replicas desc) instead of by class
    static const bool lpt = [] {
      const char* v = getenv("KP_TOP_LPT");
      return v && atoi(v) != 0;
    }();
    if (lpt)
      std::stable_sort(bt->l_all.begin() + n_small, bt->l_all.begin() + n_dyn,
                       [&](int32_t x, int32_t y) { return bt->hdr[x].replicas > bt->hdr[y].replicas; });
  }
  bt->l_slow = bt->l_all;
  bt->l_slow.insert(bt->l_slow.end(), bt->l_cluster.begin(), bt->l_cluster.end());
  if (s->view.n_regions > kRegionMax && !bt->l_region.empty()) {
    e->err = "region spread over more than 256 regions is not supported";
    return KP_ENOTSUP;
  }
  if (batch_lds_check(e, s, bt)) return KP_ENOTSUP;
  bt->n_regions = s->view.n_regions;
  auto pad1 = [](auto& v) {
    if (v.empty()) v.resize(1);
  };
  pad1(bt->ipool);
  pad1(bt->lpool);
  pad1(bt->tols);
  pad1(bt->progs);
  pad1(bt->instrs);
  const int B = bt->B ? bt->B : 1;
  const int nr = (int)bt->l_region.size(), R = std::max(1, s->view.n_regions);
  const int max_tgt = bt->max_tgt, max_tiers = bt->max_tiers;
  // SerialAssign's result list: every candidate once, plus, per overflow tier, the
  // spec.Clusters entries MergeTargetClusters appends (common.go:97-139; util/binding.go:91-115).
  bt->slow_cap = s->Cp + max_tiers * max_tgt + 64;
  {  // LDS for the targets-only serial problems (scale-down), if small
    size_t b = sizeof(Item) * (size_t)max_tgt + serial_scratch_bytes(2 * max_tgt + 16) + 64;
    bt->slow_lds = b <= 32768 ? (int)((b + 15) & ~(size_t)15) : 0;
  }
  int P = 1;
  while (P < s->Cp) P <<= 1;
  {  // LDS for the candidate sorts (bitonic keys, then the sort.Sort emulation)
    const size_t base = kRedBytes + 512 + 4 * (size_t)(((s->Cp + 31) >> 5) + 4) + bt->slow_lds;
    const size_t sel = 3072 + 8 * (size_t)sel_all_ecap(s->Cp) + 64;  // SelScratch of the tie route
    const size_t pdq = (std::max(pdq_wave_bytes(s->Cp), sel) + 15) & ~(size_t)15;
    const size_t both = std::max(8 * (size_t)P, pdq);
    bt->slow_sort = base + both <= e->max_lds ? (int)both : (base + pdq <= e->max_lds ? (int)pdq : 0);
  }
  bt->slow_slot = (size_t)s->Cp * 8 + (size_t)P * 8 + sizeof(Item) * s->Cp + 4 * (size_t)s->Cp +
                  serial_scratch_bytes(bt->slow_cap) + 1024;
  bt->slow_slot = (bt->slow_slot + 255) & ~(size_t)255;
  // k_slow: one workgroup per CU pass over the flagged bindings (appended on device)
  bt->slow_grid = (int)std::max<size_t>(1, std::min<size_t>(256, bt->l_slow.size()));
  // diagnostics: KP_SLOW_GRID=<g> caps k_slow's grid, KP_SLOW_LDS=0 keeps its sort
  // keys and scale-down scratch in the global slot (no LDS sort, no wave sort.Sort)
  if (const char* g = getenv("KP_SLOW_GRID")) bt->slow_grid = std::max(1, std::min(bt->slow_grid, atoi(g)));
  if (const char* g = getenv("KP_SLOW_LDS"); g && g[0] == '0') bt->slow_sort = bt->slow_lds = 0;
  bt->fast_ok = batch_fast_ok(bt);
  Arena& a = bt->dev;
  a.pool_dev = e->device;
  BindHdr* d_hdr;
  int32_t* d_ipool;
  int64_t* d_lpool;
  Tol* d_tols;
  Prog* d_progs;
  Instr* d_instrs;
  a.add(&d_hdr, B);
  a.add(&d_ipool, bt->ipool.size());
  a.add(&d_lpool, bt->lpool.size());
  a.add(&d_tols, bt->tols.size());
  a.add(&d_progs, bt->progs.size());
  a.add(&d_instrs, bt->instrs.size());
  a.add(&bt->fmask, (size_t)B * s->W);
  a.add(&bt->d_bcls, B);
  a.add(&bt->d_crep, bt->crep.size());
  a.add(&bt->cls_rows, bt->crep.size() * (size_t)s->Cp);
  a.add(&bt->d_all, std::max<size_t>(1, bt->l_all.size()));
  a.add(&bt->d_all_cls, std::max<size_t>(1, bt->l_all.size()));
  a.add(&bt->d_cluster, std::max<size_t>(1, bt->l_cluster.size()));
  a.add(&bt->d_region, std::max<size_t>(1, bt->l_region.size()));
  a.add(&bt->d_slowlist, std::max<size_t>(1, bt->l_slow.size()));
  a.add(&bt->d_cs, std::max<size_t>(1, bt->l_cs.size()));
  a.add(&bt->status, B);
  a.add(&bt->errc, B);
  a.add(&bt->slow, B);
  a.add(&bt->arg, B);
  a.add(&bt->start, B);
  a.add(&bt->count, B);
  a.add(&bt->counter, 1);
  a.add(&bt->stats, 20);
  a.add(&bt->d_kargs, kArgSlots);
#if defined(KP_STAMPS) || defined(KP_SLOW_CHECK)
  a.add(&bt->dbg, kDbgSlots * kDbgSpread);
#endif
  // [0, out_cap): per-binding slots; [out_cap, 2 out_cap): serial results past their slot
  a.add(&bt->out_idx, std::max<uint64_t>(1, 2 * bt->out_cap));
  a.add(&bt->out_rep, std::max<uint64_t>(1, 2 * bt->out_cap));
  a.add(&bt->offsets_d, B + 1);
  a.add(&bt->off_part, (size_t)(B + kOffChunk - 1) / kOffChunk);
  a.add(&bt->cidx_d, std::max<uint64_t>(1, 2 * bt->out_cap));
  a.add(&bt->crep_d, std::max<uint64_t>(1, 2 * bt->out_cap));
  a.add(&bt->rout, (size_t)std::max(1, nr) * R);
  a.add(&bt->rstat, std::max(1, nr));
  a.add(&bt->rsel, (size_t)std::max(1, nr) * R);
  a.add(&bt->rnsel, std::max(1, nr));
  a.add(&bt->nhost, 1);
  a.add(&bt->slow_scratch, bt->slow_slot * bt->slow_grid);
  // k_select_top (bits mode): class orders, fallback list. k_class_order sorts a class
  // row in LDS (kRedBytes + 8 * nextpow2(C)): a device with less LDS per workgroup
  // keeps the full-candidate kernels instead of failing the launch.
  // Class orders pay off when each order serves several bindings: a batch of nearly
  // one class per binding (per-binding requests) sorts a Cp row per binding instead,
  // so it keeps the full-candidate kernels (KP_ORDER_AMORT: bindings per class needed)
  const bool orders_pay = (int64_t)bt->crep.size() * order_amort() <= (int64_t)B;
  // Without them k_select_top thresholds each binding's votes by a histogram instead of
  // walking an order (kp_top.h), so its fallback list exists either way.
  if (!bt->crep.empty()) {
    a.add(&bt->d_fb, std::max(1, bt->n_all_dyn));
    a.add(&bt->d_ofb, std::max(1, bt->n_all_dyn));
  }
  const bool with_orders = s->C <= 16384 && !bt->crep.empty() && orders_pay && kRedBytes + 8 * (size_t)P <= e->max_lds;
  // singleton classes: feasible entries only, when every reader gathers feasible candidates
  // (no class orders, which sort whole rows; no spread lists; no component-set classes)
  static const bool est_single_on = [] {
    const char* v = getenv("KP_EST_SINGLE");
    return !v || atoi(v) != 0;
  }();
  if (est_single_on && !with_orders && bt->crep.size() > 1 && bt->l_cluster.empty() && bt->l_region.empty() &&
      bt->sets_cls.empty()) {
    std::vector<int32_t> cnt(bt->crep.size(), 0);
    for (uint64_t i = 0; i < n; i++) cnt[(size_t)std::max(0, bt->bcls[i])]++;
    for (size_t g = 0; g < bt->crep.size(); g++) (g > 0 && cnt[g] == 1 ? bt->l_cls_single : bt->l_cls_full).push_back((int32_t)g);
    bt->est_single = !bt->l_cls_single.empty();
    if (bt->est_single) {
      a.add(&bt->d_cls_full, bt->l_cls_full.size());
      a.add(&bt->d_cls_single, bt->l_cls_single.size());
    }
  }
  if (with_orders) {
    a.add(&bt->d_ord, bt->crep.size() * (size_t)s->Cp);
    a.add(&bt->d_ctot, bt->crep.size());
    a.add(&bt->d_cok, bt->crep.size());
    a.add(&bt->d_fbc, std::max<size_t>(1, bt->l_cluster.size()));
    a.add(&bt->d_fbr, std::max(1, nr));
    a.add(&bt->d_fba, std::max(1, nr));
  }
  // component-set classes: per cluster rank its node-run scratch (one run per model
  // node at most, capped at kSetsRunsMax) for k_sets_rows, reused class after class
  std::vector<int64_t> sets_off;
  if (!bt->sets_cls.empty()) {
    for (uint64_t i = 0; i < n; i++)
      if (bt->hdr[i].flags & BF_SETS) bt->l_sets.push_back((int32_t)i);
    sets_off.assign((size_t)s->C + 1, 0);
    int64_t runs_cap = kSetsRunsMax;  // (KP_SETS_RUNS_CAP lowers it: tests of the overflow report)
    if (const char* v = getenv("KP_SETS_RUNS_CAP")) runs_cap = std::max<int64_t>(1, std::min<int64_t>(atoll(v), kSetsRunsMax));
    for (int r = 0; r < s->C; r++) {
      int64_t nodes = 0;
      for (int g = s->mgrp_off[r]; g < s->mgrp_off[r + 1]; g++) nodes += s->mgrp_cnt[g];
      sets_off[r + 1] = sets_off[r] + std::max<int64_t>(1, std::min<int64_t>(nodes, runs_cap));
    }
    a.add(&bt->d_sets_args, bt->sets_args.size());
    a.add(&bt->d_sets_off, sets_off.size());
    a.add(&bt->d_sets_scratch, (size_t)sets_off.back() * (1 + kSetsSlots));
    a.add(&bt->d_sets_ovf, bt->sets_cls.size());
    a.add(&bt->d_sets_list, bt->l_sets.size());
  }
  const auto tp1 = std::chrono::steady_clock::now();
  HIPCHK(a.alloc());
  bt->h_kargs = (KArgs*)pinned_get(sizeof(KArgs) * kArgSlots, &bt->h_kargs_bytes);
  if (!bt->h_kargs) {
    e->err = "kp_batch_create: page-locked launch-argument slots";
    return KP_EDEVICE;
  }
  bt->create_stream = e->stream;  // (an early return below waits for the uploads queued so far)
  const auto tp2 = std::chrono::steady_clock::now();
  auto up = [&](void* d, const void* h, size_t bytes) {
    return dev::h2d(d, h, bytes, e->stream);
  };
  HIPCHK(up(d_hdr, bt->hdr.data(), sizeof(BindHdr) * bt->hdr.size()));
  HIPCHK(up(d_ipool, bt->ipool.data(), 4 * bt->ipool.size()));
  HIPCHK(up(d_lpool, bt->lpool.data(), 8 * bt->lpool.size()));
  HIPCHK(up(d_tols, bt->tols.data(), sizeof(Tol) * bt->tols.size()));
  HIPCHK(up(d_progs, bt->progs.data(), sizeof(Prog) * bt->progs.size()));
  HIPCHK(up(d_instrs, bt->instrs.data(), sizeof(Instr) * bt->instrs.size()));
  HIPCHK(up(bt->d_bcls, bt->bcls.data(), 4 * bt->bcls.size()));
  {  // representatives of the k_est_class rows; -1 for the component-set classes (k_sets_rows)
    std::vector<int32_t> rep = bt->crep;
    for (int32_t g : bt->sets_cls) rep[g] = -1;
    HIPCHK(up(bt->d_crep, rep.data(), 4 * rep.size()));
  }
  if (!bt->sets_cls.empty()) {
    HIPCHK(up(bt->d_sets_args, bt->sets_args.data(), sizeof(SetsArgs) * bt->sets_args.size()));
    HIPCHK(up(bt->d_sets_off, sets_off.data(), 8 * sets_off.size()));
    HIPCHK(up(bt->d_sets_list, bt->l_sets.data(), 4 * bt->l_sets.size()));
  }
  if (bt->est_single) {
    HIPCHK(up(bt->d_cls_full, bt->l_cls_full.data(), 4 * bt->l_cls_full.size()));
    HIPCHK(up(bt->d_cls_single, bt->l_cls_single.data(), 4 * bt->l_cls_single.size()));
  }
  HIPCHK(up(bt->d_all, bt->l_all.data(), 4 * bt->l_all.size()));
  bt->l_all_cls.resize(bt->l_all.size());
  for (size_t i = 0; i < bt->l_all.size(); i++) bt->l_all_cls[i] = bt->bcls[bt->l_all[i]];
  HIPCHK(up(bt->d_all_cls, bt->l_all_cls.data(), 4 * bt->l_all_cls.size()));
  HIPCHK(up(bt->d_cluster, bt->l_cluster.data(), 4 * bt->l_cluster.size()));
  HIPCHK(up(bt->d_region, bt->l_region.data(), 4 * bt->l_region.size()));
  HIPCHK(up(bt->d_cs, bt->l_cs.data(), 4 * bt->l_cs.size()));
  HIPCHK(dev::fill(bt->slow, 0, 4 * (size_t)B, e->stream));
  HIPCHK(dev::sync(e->stream));
  if (getenv("KP_PACK_TIMING")) {
    const auto tp3 = std::chrono::steady_clock::now();
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    fprintf(stderr, "kp_batch_create: pack %.1f ms, alloc %.1f ms, upload %.1f ms\n", ms(tp0, tp1), ms(tp1, tp2),
            ms(tp2, tp3));
  }
  BatchView& v = bt->view;
  v.B = bt->B;
  v.hdr = d_hdr;
  v.ipool = d_ipool;
  v.lpool = d_lpool;
  v.tols = d_tols;
  v.progs = d_progs;
  v.instrs = d_instrs;
  bt->create_stream = nullptr;
  *out = guard.release();
  return KP_OK;
}

void kp_batch_destroy(kp_batch* b) { delete b; }

// After a failed entry point: the work it queued on the engine's streams may still
// use the batch's buffers, so destruction must wait for it (kp_batch::quiesce).
static int batch_fence(kp_engine* e, kp_batch* bt, int rc) {
  if (rc == KP_OK || !e || !bt) return rc;
  const dev::stream_t ss[3] = {e->stream, e->stream2, e->stream3};
  for (int i = 0; i < 3; i++) {
    if (!bt->fence[i] && dev::event_create(&bt->fence[i])) {
      bt->fence[i] = nullptr;
      (void)dev::sync(ss[i]);  // no event: wait here instead
      continue;
    }
    if (dev::event_record(bt->fence[i], ss[i])) (void)dev::sync(ss[i]);
  }
  bt->fenced = true;
  return rc;
}

// The per-binding [B][Cp] calAvailableReplicas rows, allocated on first use (the
// pair-row mode and the diagnosis entry points; the default path never needs them).
static int ensure_rows(kp_engine* e, kp_batch* bt) {
  if (bt->est) return 0;
  void* p = nullptr;
  if (dev::alloc(&p, 4 * (size_t)std::max(1, bt->B) * (size_t)bt->snap->Cp)) {
    e->err = std::string("per-binding estimate rows: ") + dev::last_error();
    return -1;
  }
  bt->est = (int32_t*)p;
  return 0;
}

// Per-kernel profiling (kp_engine_set_profile): prof_begin records the start event of
// launch i on its stream, prof_end its end event and what it covered.
static int prof_begin(kp_engine* e, dev::stream_t st) {
  if (!e->prof) return -1;
  const size_t i = e->pk.size();
  while (e->pev.size() < 2 * i + 2) {
    dev::event_t ev = nullptr;
    if (dev::event_create(&ev)) return -1;
    e->pev.push_back(ev);
  }
  if (dev::event_record(e->pev[2 * i], st)) return -1;
  e->pk.push_back({"", 0, -1});
  return (int)i;
}
static void prof_end(kp_engine* e, int i, dev::stream_t st, const char* name, uint64_t units, int units_stat = -1) {
  if (i < 0) return;
  (void)dev::event_record(e->pev[2 * (size_t)i + 1], st);
  e->pk[i] = {name, units, units_stat};
}
// After the batch's final sync: each kernel's launches folded by name.
static void prof_fold(kp_engine* e, const uint32_t* h_stats) {
  e->ktimes.clear();
  for (size_t i = 0; i < e->pk.size(); i++) {
    const auto& k = e->pk[i];
    const float ms = dev::event_ms(e->pev[2 * i], e->pev[2 * i + 1]);
    const uint64_t units = k.units_stat >= 0 ? h_stats[k.units_stat] : k.units;
    kp_kernel_time* t = nullptr;
    for (auto& x : e->ktimes)
      if (strncmp(x.name, k.name, sizeof(x.name)) == 0) t = &x;
    if (!t) {
      e->ktimes.push_back(kp_kernel_time{});
      t = &e->ktimes.back();
      snprintf(t->name, sizeof(t->name), "%s", k.name);
    }
    t->ms += ms > 0 ? ms : 0.f;
    t->launches++;
    t->units += units;
  }
  e->pk.clear();
}
#define KPROF(ST, NAME, UNITS, STAT, CALL)           \
  do {                                               \
    const int pi_ = prof_begin(e, ST);               \
    HIPCHK(CALL);                                    \
    prof_end(e, pi_, ST, NAME, (uint64_t)(UNITS), STAT); \
  } while (0)
// launch names of the select kernels (kernels.hip picks the wide instance past half
// the CU's LDS, as here)
static const char* sel_name(int which, size_t smem) {
  const bool wide = smem > 80 * 1024;
  switch (which) {
    case SEL_LAUNCH_ALL: return wide ? "k_select_all_wide" : "k_select_all";
    case SEL_LAUNCH_ALL_STREAM: return "k_select_all_stream";
    case SEL_LAUNCH_CLUSTER: return wide ? "k_select_cluster_wide" : "k_select_cluster";
    case SEL_LAUNCH_REGION_A: return wide ? "k_region_a_wide" : "k_region_a";
    case SEL_LAUNCH_REGION_B: return wide ? "k_region_b_wide" : "k_region_b";
    case SEL_LAUNCH_SLOW: return "k_slow";
  }
  return "k_select";
}
static const char* pair_name(int fast) {
  switch (fast) {
    case EST_MIXED: return "k_pair_fast";
    case EST_SUMMARY: return "k_pair_fast_summary";
    case EST_MODEL8: return "k_pair_fast_m8";
    case EST_MODEL16: return "k_pair_fast_m16";
  }
  return "k_pair";
}
static const char* est_class_feasible_name(int fast) {
  switch (fast) {
    case EST_SUMMARY: return "k_est_class_summary (feasible)";
    case EST_MODEL8: return "k_est_class_m8 (feasible)";
    case EST_MODEL16: return "k_est_class_m16 (feasible)";
    default: break;
  }
  return "k_est_class (feasible)";
}
static const char* est_class_name(int fast) {
  switch (fast) {
    case EST_SUMMARY: return "k_est_class_summary";
    case EST_MODEL8: return "k_est_class_m8";
    case EST_MODEL16: return "k_est_class_m16";
  }
  return "k_est_class";
}

// The batch path computes the in-tree plugin set only (kp_options.n_out_of_tree_plugins).
static int refuse_out_of_tree(kp_engine* e, const kp_snapshot* s) {
  if (s->opts.n_out_of_tree_plugins == 0) return KP_OK;
  e->err = "the scheduler registry holds " + std::to_string(s->opts.n_out_of_tree_plugins) +
           " filter/score plugin(s) outside the in-tree set: the batch path would ignore them "
           "(schedule through the framework with the per-pair entry points)";
  return KP_ENOTSUP;
}

// A schedule call in two halves: schedule_submit queues every launch and the per-binding
// read-backs of a batch (the region chain's host steps included) and records bt->pend.ev;
// schedule_finish waits for that event, copies the CSR back and fills the results.
// kp_schedule_batch runs both; kp_schedule_batch_submit / _collect let a caller keep the
// next batch's kernels queued on the engine's stream while it collects the previous one.
static int schedule_submit(kp_engine* e, kp_batch* bt) {
  if (!e || !bt) return KP_EINVAL;
  if (int rc = refuse_out_of_tree(e, bt->snap)) return rc;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  const int B = bt->B;
  double t0 = now_ms();
  kp_stage_times tm{};
  dev::stream_t st = e->stream;
  SchedPend& pd = bt->pend;
  {
    const dev::event_t ev = pd.ev;  // (the event is kept across calls)
    pd = SchedPend{};
    pd.ev = ev;
  }
  pd.t0 = t0;
  pd.seq = ++e->submit_seq;
  if (B == 0) {
    pd.empty = true;
    pd.live = true;
    return KP_OK;
  }
  if (!bt->l_region.empty() && s->view.n_regions != bt->n_regions) {
    e->err = "kp_schedule_batch: the snapshot's region set changed since the batch was packed (re-create it)";
    return KP_ESTATE;
  }
  if (batch_lds_check(e, s, bt)) return KP_ENOTSUP;
  e->pk.clear();
  HIPCHK(dev::h2d(bt->counter, &bt->out_cap, sizeof(unsigned long long), st));  // the shared area's start
  HIPCHK(dev::fill(bt->stats, 0, sizeof(bt->h_stats), st));
  if (!bt->sets_cls.empty()) HIPCHK(dev::fill(bt->d_sets_ovf, 0, 4 * bt->sets_cls.size(), st));
  KArgs ka;
  ka.s = s->view;
  ka.bv = bt->view;
  ka.fmask = bt->fmask;
  ka.est = bt->est;
  ka.sink.out_idx = bt->out_idx;
  ka.sink.out_rep = bt->out_rep;
  ka.sink.counter = bt->counter;
  ka.sink.status = bt->status;
  ka.sink.err = bt->errc;
  ka.sink.arg = bt->arg;
  ka.sink.start = bt->start;
  ka.sink.count = bt->count;
  ka.sink.cap_end = std::max<uint64_t>(1, 2 * bt->out_cap);
  ka.slow = bt->slow;
  ka.stats = bt->stats;
  ka.slow_ids = bt->d_slowlist;
  ka.dbg = bt->dbg;
#if defined(KP_STAMPS) || defined(KP_SLOW_CHECK)
  HIPCHK(dev::fill(bt->dbg, 0, kDbgSlots * kDbgSpread * 8, st));
#endif
  dev::stream_t sp = e->stream2;
  HIPCHK(dev::event_record(e->ev[0], st));
  HIPCHK(dev::stream_wait(sp, e->ev[0]));  // the fills above precede every kernel
  const int fast = getenv("KP_PAIR_GENERIC") || !bt->fast_ok ? EST_GENERIC : s->est_kind;
  const int md_cap = md_cap_of(s);
  // Feasibility and calAvailableReplicas: by default (fast estimator instance and
  // the snapshot's bitset rows built) the filter runs as bitset algebra (k_filter)
  // and the estimator once per estimator class (k_est_class), kp_filter.h; else
  // (or KP_PAIR_ROWS=1) the pair kernel writes every binding's rows.
  const bool bits = fast != EST_GENERIC && s->view.n_bits > 0 && !getenv("KP_PAIR_ROWS");
  if (!bits && ensure_rows(e, bt)) return KP_EDEVICE;
  ka.est = bits ? bt->cls_rows : bt->est;
  ka.bcls = bits ? bt->d_bcls : nullptr;
  SelectExtra sx;
  sx.rout = bt->rout;
  sx.rstat = bt->rstat;
  sx.rsel = bt->rsel;
  sx.rnsel = bt->rnsel;
  sx.scratch = bt->slow_scratch;
  sx.slot_bytes = bt->slow_slot;
  sx.grid = bt->slow_grid;
  sx.lds_area = bt->slow_lds;
  sx.lds_sort = bt->slow_sort;
  const int cap = kSmallMax + kTgtSmallMax + 16;
  // A launch's KArgs copied to its own device slot (ordered before the launch on its
  // stream): the select kernels that keep pointers into their arguments read them there
  // (kp_launch.h SelectExtra::dargs). One slot per launch within this call.
  int kslot = 0;
  auto with_args = [&](const KArgs& k, dev::stream_t sq) -> SelectExtra {
    SelectExtra r = sx;
    if (kslot >= kArgSlots) return r;  // (dargs stays null: the launch reports EINVAL)
    bt->h_kargs[kslot] = k;
    if (dev::h2d(bt->d_kargs + kslot, bt->h_kargs + kslot, sizeof(KArgs), sq) == 0) r.dargs = bt->d_kargs + kslot;
    kslot++;
    return r;
  };
  HIPCHK(dev::event_record(e->ev[3], sp));
  // component-set classes (BF_SETS bindings): their class rows (after the estimator
  // classes' rows, before k_class_order reads them all), and in the pair-row mode those
  // bindings' own rows rebuilt from them (feasible clusters only)
  auto sets_rows = [&]() -> int {
    for (size_t j = 0; j < bt->sets_cls.size(); j++)
      KPROF(sp, "k_sets_rows", 1, -1,
            dev::sets_rows(sp, s->view, bt->d_sets_args + j, bt->d_sets_off, bt->d_sets_scratch,
                           bt->cls_rows + (size_t)bt->sets_cls[j] * s->Cp, bt->d_sets_ovf + j));
    return KP_OK;
  };
  if (bits) {
    const bool single = bt->est_single;
    const int n_full = single ? (int)bt->l_cls_full.size() : (int)bt->crep.size();
    KPROF(sp, est_class_name(fast), n_full, -1,
          dev::est_class(sp, s->view, bt->view, bt->d_crep, n_full, bt->cls_rows, fast, single ? bt->d_cls_full : nullptr));
    if (int rc = sets_rows()) return rc;
    HIPCHK(dev::event_record(e->ev[5], sp));  // every class row is written (k_class_order's input)
    KPROF(sp, "k_filter", B, -1, dev::filter(sp, s->view, bt->view, bt->fmask));
    if (single)  // the singleton classes' feasible entries, from the feasibility rows
      KPROF(sp, est_class_feasible_name(fast), bt->l_cls_single.size(), -1,
            dev::est_class(sp, s->view, bt->view, bt->d_crep, (int)bt->l_cls_single.size(), bt->cls_rows, fast,
                           bt->d_cls_single, bt->fmask));
  } else {
    KPROF(sp, pair_name(fast), B, -1,
          dev::pair(sp, s->view, bt->view, nullptr, 0, B, bt->fmask, bt->est, nullptr, 0, md_cap, smem_pair(s, md_cap),
                    fast));
    if (int rc = sets_rows()) return rc;
  }
  if (!bits && !bt->l_sets.empty())
    KPROF(sp, "k_rows_from_class", bt->l_sets.size(), -1,
          dev::rows_from_class(sp, s->view, bt->view, bt->d_sets_list, (int)bt->l_sets.size(), bt->d_bcls,
                               bt->cls_rows, bt->fmask, bt->est));
  // SEL_ALL DynamicWeight / Aggregated over the deciding candidates (kp_top.h): the
  // class rows' orders first
  // the large slice's capacity, lowered until the slices fit the device's LDS
  int top_cap = e->top_cap;
  while (top_cap > 64 && kTopWaves * ((top_lds_bytes(s->Cp, top_cap) + 15) & ~(size_t)15) > e->max_lds) top_cap /= 2;
  const int top_cap_small = std::min(e->top_cap_small, top_cap);
  // (without class orders, k_select_top thresholds the votes by a histogram: KP_TOPK=0 keeps
  // the full-candidate kernel there instead)
  static const bool topk_on = [] {
    const char* v = getenv("KP_TOPK");
    return !v || atoi(v) != 0;
  }();
  const bool top = bits && e->top_on && s->Cp <= kTopMaxCp && (bt->d_ord != nullptr || (topk_on && bt->d_fb != nullptr)) &&
                   bt->n_all_dyn > 0 && kTopWaves * ((top_lds_bytes(s->Cp, top_cap) + 15) & ~(size_t)15) <= e->max_lds;
  // class orders: k_select_top's walk, and the spread selections over them
  // (k_spread_order, k_region_a_order), each where its LDS slices fit the device
  const bool spread_orders = bits && e->top_on && bt->d_ord != nullptr &&
                             (!bt->l_cluster.empty() || !bt->l_region.empty()) &&
                             kOrderWaves * ((order_lds_bytes(s->view.W, s->view.n_regions) + 15) & ~(size_t)15) <=
                                 e->max_lds &&
                             kOrderWaves * ((region_a_order_lds_bytes(s->view.n_regions, s->view.W) + 15) & ~(size_t)15) <=
                                 e->max_lds;
  const bool orders = (top && bt->d_ord != nullptr) || spread_orders;
  if (orders) {
    // k_class_order reads only the class rows (k_est_class), so it runs on stream3 beside
    // k_filter and stream2 waits for it (profiled runs keep it on stream2: each kernel's
    // event time is then its own)
    dev::stream_t so = e->prof ? sp : e->stream3;
    if (so != sp) HIPCHK(dev::stream_wait(so, e->ev[5]));
    KPROF(so, "k_class_order", bt->crep.size(), -1,
          dev::class_order(so, s->view, bt->cls_rows, (int)bt->crep.size(), bt->d_ord, bt->d_ctot, bt->d_cok));
    if (so != sp) {
      HIPCHK(dev::event_record(e->ev[6], so));
      HIPCHK(dev::stream_wait(sp, e->ev[6]));
    }
  }
  HIPCHK(dev::event_record(e->ev[4], sp));
  HIPCHK(dev::stream_wait(st, e->ev[4]));  // every pair row precedes the rest
  HIPCHK(dev::event_record(e->ev[1], st));
  // The three selection kinds touch disjoint bindings: SEL_ALL on stream2 (after the
  // pair kernel there), cluster spread on stream3, the region chain on stream, so a
  // latency-bound kernel shares the CUs with the others instead of running alone.
  HIPCHK(dev::event_record(e->ev[7], sp));
  // Fallback launches over device-appended lists, with a region chain (e->gate_fb): their
  // counts are read back where the host synchronises anyway (the region chain, k_slow's
  // count), so a list left empty launches nothing; the SEL_ALL and cluster-spread
  // fallbacks move to stream3 after that read, before k_slow.
  const bool gate = e->gate_fb != 0 && !bt->l_region.empty();
  const bool gate_region = gate && e->gate_fb == 1;
  bool defer_all = false, defer_all_stream = false, defer_cl = false;
  KArgs f_def{}, cl_def{};
  if (!bt->l_all.empty()) {
    KArgs k = ka;
    k.list = bt->d_all;
    k.n = (int)bt->l_all.size();
    // Candidates gathered into LDS (k_select_all), or, in bits mode, streamed from
    // the feasibility and class rows (k_select_all_stream): for the StaticWeight
    // bindings (votes from per-rule bitsets), and for all when the gathered
    // candidates would leave one workgroup per CU (C ~ 8.6k+).
    const bool stream_all = bits && smem_all(s) > 80 * 1024;
    const bool stream_w = bits;
    const int na = stream_all ? 0 : (stream_w ? bt->n_all_dyn : k.n);
    if (top) {
      // k_select_top over [0, n_all_dyn), small slices for [0, n_top_small); the
      // bindings it hands back (other strategies, subsets past capacity, ...) run with
      // every candidate from its fallback list
      HIPCHK(dev::event_record(e->ev[12], sp));
      // the two slices' launches run concurrently, the large one on stream3 (which the
      // cluster-spread kernels use after it), so neither drains the CUs alone
      // (profiled steps keep both on one stream: each launch's HIP-event time is then its own)
      const bool split = e->top_split && !e->prof && bt->n_top_small > 0 && bt->n_all_dyn > bt->n_top_small;
      // the large slice in two capacities: top_cap_mid first (its smaller LDS slices
      // keep more waves per CU), then top_cap over the bindings whose subset outgrew it
      // (a device-appended list, grid-stride waves; the capacity only bounds the subset,
      // so both runs give the same answer)
      const bool mid = e->top_cap_mid >= 64 && e->top_cap_mid < top_cap && !e->top_wg;
      for (int part = 0; part < 2; part++) {
        KArgs g = k;
        const int cap_p = part == 0 ? top_cap_small : (mid ? e->top_cap_mid : top_cap);
        g.list = bt->d_all + (part == 0 ? 0 : bt->n_top_small);
        g.lcls = bt->d_all_cls + (part == 0 ? 0 : bt->n_top_small);
        g.n = part == 0 ? bt->n_top_small : bt->n_all_dyn - bt->n_top_small;
        if (g.n <= 0) continue;
        TopArgs ta{bt->d_ord, bt->d_ctot, bt->d_cok, bt->d_fb, bt->stats + 9, cap_p};
        if (part == 1 && mid) {
          ta.ofb = bt->d_ofb;
          ta.ofb_n = bt->stats + 16;
        }
        const size_t slice = (top_lds_bytes(s->Cp, cap_p) + 15) & ~(size_t)15;
        dev::stream_t sx_ = split && part == 1 ? e->stream3 : sp;
        if (split && part == 1) HIPCHK(dev::stream_wait(sx_, e->ev[4]));
        // the large-subset bindings: a workgroup each (wave 0 walks, the workgroup divides)
        const size_t wg_lds = (top_wg_lds_bytes(s->Cp, cap_p) + 15) & ~(size_t)15;
        if (part == 1 && e->top_wg && wg_lds <= e->max_lds)
          KPROF(sx_, "k_select_top_wg", g.n, -1, dev::select_top_wg(sx_, g, ta, wg_lds));
        else
          KPROF(sx_, "k_select_top", g.n, -1, dev::select_top(sx_, g, ta, slice));
        if (part == 1 && mid) {
          KArgs o = k;
          o.list = bt->d_ofb;
          o.n = g.n;  // (the list's capacity; its length is stats[16])
          o.n_dev = bt->stats + 16;
          TopArgs tb{bt->d_ord, bt->d_ctot, bt->d_cok, bt->d_fb, bt->stats + 9, top_cap};
          const size_t slice_l = (top_lds_bytes(s->Cp, top_cap) + 15) & ~(size_t)15;
          // (units 0: the launch re-runs bindings the kernel's units already count)
          KPROF(sx_, "k_select_top", 0, -1, dev::select_top(sx_, o, tb, slice_l, kTopOverGrid));
        }
        if (split && part == 1) {
          HIPCHK(dev::event_record(e->ev[10], sx_));
          HIPCHK(dev::stream_wait(sp, e->ev[10]));  // both slices' fallbacks precede k_select_all
        }
      }
      HIPCHK(dev::event_record(e->ev[13], sp));
      KArgs f = k;
      f.list = bt->d_fb;
      f.n = bt->n_all_dyn;
      f.n_dev = bt->stats + 9;
      if (gate) {
        f_def = f;
        defer_all = true;
        defer_all_stream = stream_all;
      } else if (stream_all) {
        const SelectExtra sxa1 = with_args(f, sp);  // (the slot is copied before the launch is timed)
        KPROF(sp, "k_select_all_stream", 0, 9,
              dev::select(sp, SEL_LAUNCH_ALL_STREAM, f, sel_stream_lds_bytes(s->Cp), cap, sxa1));
      } else {
        KPROF(sp, sel_name(SEL_LAUNCH_ALL, smem_all(s)), 0, 9, dev::select(sp, SEL_LAUNCH_ALL, f, smem_all(s), cap, sx));
      }
    } else if (na > 0) {
      KArgs g = k;
      g.n = na;
      KPROF(sp, sel_name(SEL_LAUNCH_ALL, smem_all(s)), g.n, -1, dev::select(sp, SEL_LAUNCH_ALL, g, smem_all(s), cap, sx));
    }
    // the rest: StaticWeight at class level (k_select_static) where it applies, then
    // the streamed kernel
    int rest0 = top ? bt->n_all_dyn : na;
    if (bits && rest0 == bt->n_all_dyn && bt->n_static > 0 &&
        kStaticWaves * ((static_lds_bytes(s->view.W) + 15) & ~(size_t)15) <= e->max_lds) {
      KArgs g = k;
      g.list = bt->d_all + rest0;
      g.n = bt->n_static;
      KPROF(sp, "k_select_static", g.n, -1, dev::select_static(sp, g, (static_lds_bytes(s->view.W) + 15) & ~(size_t)15));
      rest0 += bt->n_static;
    }
    if (k.n - rest0 > 0) {
      KArgs g = k;
      g.list = bt->d_all + rest0;
      g.n = k.n - rest0;
      {  // (the argument slot is copied before the launch is timed)
        const SelectExtra sxa2 = with_args(g, sp);
        KPROF(sp, "k_select_all_stream", g.n, -1,
              dev::select(sp, SEL_LAUNCH_ALL_STREAM, g, sel_stream_lds_bytes(s->Cp), cap, sxa2));
      }
    }
  }
  HIPCHK(dev::event_record(e->ev[8], sp));  // k_select_all alone: ev[7] -> ev[8]
  dev::stream_t s3 = e->stream3;
  HIPCHK(dev::stream_wait(s3, e->ev[4]));
  if (!bt->l_cluster.empty()) {
    KArgs k = ka;
    k.list = bt->d_cluster;
    k.n = (int)bt->l_cluster.size();
    HIPCHK(dev::event_record(e->ev[14], s3));
    if (spread_orders) {
      // the class-order selection, one wave per binding; what it hands back runs below
      k.ord = bt->d_ord;
      k.cok = bt->d_cok;
      k.n_order = bt->stats + 10;
      OrderArgs oa{nullptr, nullptr, nullptr, bt->d_fbc, bt->stats + 12, 0};
      KPROF(s3, "k_spread_order", k.n, -1,
            dev::spread_order(s3, k, oa, (order_lds_bytes(s->view.W, s->view.n_regions) + 15) & ~(size_t)15));
      k.sub = bt->d_fbc;
      k.n_dev = bt->stats + 12;
    }
    if (gate && k.n_dev) {
      cl_def = k;
      defer_cl = true;
    } else {  // (the argument slot is copied before the launch is timed)
      const SelectExtra sxa3 = with_args(k, s3);
      KPROF(s3, sel_name(SEL_LAUNCH_CLUSTER, smem_cluster(s, cap)), k.n_dev ? 0 : k.n, k.n_dev ? 12 : -1,
            dev::select(s3, SEL_LAUNCH_CLUSTER, k, smem_cluster(s, cap), cap, sxa3));
    }
    HIPCHK(dev::event_record(e->ev[15], s3));
  }
  // k_slow after every kernel that flags bindings (SEL_ALL on stream2, cluster spread
  // here; the region chain flags none), so it runs beside the region chain
  double th0 = 0, th1 = 0;
  if (!bt->l_region.empty()) {
    const int nr = (int)bt->l_region.size(), R = s->view.n_regions;
    KArgs k = ka;
    k.list = bt->d_region;
    k.n = nr;
    if (spread_orders) {  // region_b_by_order
      k.ord = bt->d_ord;
      k.cok = bt->d_cok;
      k.n_order = bt->stats + 11;
    }
    if (spread_orders) {  // stage A of the order-eligible bindings, one wave each; the rest below
      KArgs ko = k;
      ko.n_order = nullptr;
      KPROF(st, "k_region_a_order", ko.n, -1, dev::region_a_order(st, ko, bt->rout, bt->rstat, bt->d_fba, bt->stats + 14,
                                 (region_a_order_lds_bytes(R, s->view.W) + 15) & ~(size_t)15));
      KArgs kf = k;
      kf.sub = bt->d_fba;
      kf.n_dev = bt->stats + 14;
      uint32_t nfa = 1;
      if (gate_region) {  // (the grid is then sized by the count: spread_grid)
        HIPCHK(dev::d2h(&nfa, bt->stats + 14, 4, st));
        HIPCHK(dev::sync(st));
      }
      if (nfa > 0) {  // (the argument slot is copied before the launch is timed)
        SelectExtra sxa4 = with_args(kf, st);
        if (gate_region) sxa4.list_grid = (int)nfa;
        KPROF(st, sel_name(SEL_LAUNCH_REGION_A, smem_region_a(s)), 0, 14,
              dev::select(st, SEL_LAUNCH_REGION_A, kf, smem_region_a(s), cap, sxa4));
      }
    } else {
      {  // (the argument slot is copied before the launch is timed)
        const SelectExtra sxa5 = with_args(k, st);
        KPROF(st, sel_name(SEL_LAUNCH_REGION_A, smem_region_a(s)), k.n, -1,
              dev::select(st, SEL_LAUNCH_REGION_A, k, smem_region_a(s), cap, sxa5));
      }
    }
    // selectGroups: on the device (one thread per binding) unless the snapshot
    // has more regions than its arrays hold; bindings whose DFS exceeds the node
    // budget, and every binding on the other route, take the host DFS.
    const bool dev_groups = R <= kGroupMax && !getenv("KP_REGION_HOST");
    uint32_t nh = 0;
    if (dev_groups) {
      HIPCHK(dev::fill(bt->nhost, 0, 4, st));
      KPROF(st, "k_region_groups", nr, -1, dev::region_groups(st, bt->rout, bt->rstat, bt->view.hdr, bt->d_region, nr, R, bt->rsel, bt->rnsel,
                                bt->nhost));
      HIPCHK(dev::d2h(&nh, bt->nhost, 4, st));
      HIPCHK(dev::sync(st));
    }
    if (!dev_groups || nh > 0) {
      bt->h_rout.resize((size_t)nr * std::max(R, 1));
      bt->h_rstat.resize(nr);
      HIPCHK(dev::d2h(bt->h_rout.data(), bt->rout, sizeof(RegionOut) * bt->h_rout.size(), st));
      HIPCHK(dev::d2h(bt->h_rstat.data(), bt->rstat, 4 * nr, st));
      bt->h_rsel.assign((size_t)nr * std::max(R, 1), -1);
      bt->h_rnsel.assign(nr, 0);
      if (dev_groups) {
        HIPCHK(dev::d2h(bt->h_rsel.data(), bt->rsel, 4 * bt->h_rsel.size(), st));
        HIPCHK(dev::d2h(bt->h_rnsel.data(), bt->rnsel, 4 * nr, st));
      }
      HIPCHK(dev::sync(st));
      th0 = now_ms();
      parallel_for(nr, e->n_threads, [&](int j) {
        if (dev_groups && bt->h_rnsel[j] != kGroupsHost) return;
        if (bt->h_rstat[j] != 0) {
          bt->h_rnsel[j] = -1000;
          return;
        }
        const BindHdr& h = bt->hdr[bt->l_region[j]];
        std::vector<G> groups;
        for (int r = 0; r < R; r++) {
          const RegionOut& ro = bt->h_rout[(size_t)j * R + r];
          if (ro.count > 0) groups.push_back({r, ro.count, ro.score});
        }
        // selectBestClustersByRegion (select_clusters_by_region.go:25-40)
        if ((int64_t)groups.size() < h.region_min) {
          bt->h_rnsel[j] = -KP_ERR_REGION_MIN_GROUPS;
          return;
        }
        auto sel = select_groups(groups, h.region_min, h.region_max, h.cluster_min);
        if (sel.empty()) {
          bt->h_rnsel[j] = -KP_ERR_REGION_CLUSTER_MIN;
          return;
        }
        for (int r = 0; r < R; r++) bt->h_rsel[(size_t)j * R + r] = -1;
        for (size_t q = 0; q < sel.size(); q++) bt->h_rsel[(size_t)j * R + q] = sel[q];
        bt->h_rnsel[j] = (int32_t)sel.size();
      });
      th1 = now_ms();
      HIPCHK(dev::h2d(bt->rsel, bt->h_rsel.data(), 4 * bt->h_rsel.size(), st));
      HIPCHK(dev::h2d(bt->rnsel, bt->h_rnsel.data(), 4 * nr, st));
    }
    if (spread_orders) {
      OrderArgs oa{bt->rout, bt->rsel, bt->rnsel, bt->d_fbr, bt->stats + 13, 1};
      KPROF(st, "k_spread_order", k.n, -1, dev::spread_order(st, k, oa, (order_lds_bytes(s->view.W, R) + 15) & ~(size_t)15));
      k.sub = bt->d_fbr;
      k.n_dev = bt->stats + 13;
    }
    uint32_t nfb = 1;
    if (gate_region && k.n_dev) {
      HIPCHK(dev::d2h(&nfb, bt->stats + 13, 4, st));
      HIPCHK(dev::sync(st));
    }
    if (nfb > 0) {  // (the argument slot is copied before the launch is timed)
      SelectExtra sxa6 = with_args(k, st);
      if (gate_region && k.n_dev) sxa6.list_grid = (int)nfb;
      KPROF(st, sel_name(SEL_LAUNCH_REGION_B, smem_region_b(s, cap)), k.n_dev ? 0 : k.n, k.n_dev ? 13 : -1,
            dev::select(st, SEL_LAUNCH_REGION_B, k, smem_region_b(s, cap), cap, sxa6));
    }
  }
  // k_slow after every kernel that flags bindings (SEL_ALL on stream2, cluster spread on
  // stream3; the region chain, queued above, flags none), beside the region chain. With a
  // region chain the flagged count is read back first (the host waits for the flagging
  // kernels only): a batch that flags none launches nothing, and a few flagged take a
  // small grid, instead of up to 256 workgroups whose LDS slices wait for CUs behind the
  // region kernels (config 4: 3.87 -> 3.74 ms). Without one the wait costs more than it
  // saves (config 3: 2.00 -> 2.20 ms with four batches in flight), so k_slow is queued.
  HIPCHK(dev::stream_wait(s3, e->ev[8]));
  uint32_t nslow = (uint32_t)bt->slow_grid;
  if (!bt->l_region.empty() && (gate || !bt->l_slow.empty())) {
    uint32_t hs[16];  // (stats [0] flagged, [9] SEL_ALL fallbacks, [12] cluster-spread fallbacks)
    HIPCHK(dev::d2h(hs, bt->stats, sizeof(hs), s3));
    HIPCHK(dev::sync(s3));
    nslow = hs[0];
    bool more = false;  // a deferred fallback runs: it may flag bindings for k_slow
    if (defer_all && hs[9] > 0) {
      const KArgs& f = f_def;
      if (defer_all_stream) {
        SelectExtra sxa1 = with_args(f, s3);
        sxa1.list_grid = (int)hs[9];
        KPROF(s3, "k_select_all_stream", hs[9], -1,
              dev::select(s3, SEL_LAUNCH_ALL_STREAM, f, sel_stream_lds_bytes(s->Cp), cap, sxa1));
      } else {
        SelectExtra sxg = sx;
        sxg.list_grid = (int)hs[9];
        KPROF(s3, sel_name(SEL_LAUNCH_ALL, smem_all(s)), hs[9], -1,
              dev::select(s3, SEL_LAUNCH_ALL, f, smem_all(s), cap, sxg));
      }
      more = true;
    }
    if (defer_cl && hs[12] > 0) {
      const KArgs& k = cl_def;
      SelectExtra sxa3 = with_args(k, s3);
      sxa3.list_grid = (int)hs[12];
      KPROF(s3, sel_name(SEL_LAUNCH_CLUSTER, smem_cluster(s, cap)), hs[12], -1,
            dev::select(s3, SEL_LAUNCH_CLUSTER, k, smem_cluster(s, cap), cap, sxa3));
      more = true;
    }
    if (more) nslow = (uint32_t)bt->slow_grid;  // (the kernel reads the final count itself)
  }
  if (!bt->l_slow.empty() && nslow > 0) {
    KArgs k = ka;
    k.list = bt->d_slowlist;
    k.n = (int)bt->l_slow.size();
    k.ord = orders ? bt->d_ord : nullptr;  // sortClusters order from the class orders (kp_kernels.h)
    k.cok = orders ? bt->d_cok : nullptr;
    if (!e->slow_order) k.ord = nullptr;
    SelectExtra sxs = with_args(k, s3);
    sxs.grid = (int)std::min<uint32_t>((uint32_t)bt->slow_grid, nslow);
    KPROF(s3, "k_slow", 0, 0,
          dev::select(s3, SEL_LAUNCH_SLOW, k,
                      kRedBytes + 512 + 4 * (size_t)(((s->Cp + 31) >> 5) + 4) + sx.lds_area + sx.lds_sort,
                      bt->slow_cap, sxs));
  }
  HIPCHK(dev::event_record(e->ev[9], s3));
  HIPCHK(dev::stream_wait(st, e->ev[8]));
  HIPCHK(dev::stream_wait(st, e->ev[9]));  // k_slow (stream3) and every select kernel precede the results
  HIPCHK(dev::event_record(e->ev[2], st));
  // results -> host, compacted to CSR: offsets scanned and results compacted on
  // the device, then the per-binding arrays and the CSR copied back
  KPROF(st, "k_offsets", B, -1, dev::offsets(st, bt->status, bt->count, B, bt->offsets_d, bt->off_part));
  // With page-locked result buffers from an earlier call (their capacity known before the
  // launch), k_compact also writes the CSR straight into them over the bus (e->zc): the
  // call then needs no host round trip for the CSR's size and no copy after it, so an
  // engine's stream stays queued to its end (several engines in flight no longer idle the
  // GPU while each one reads its total back). A total past the capacity takes the copy.
  uint32_t* zc_idx = nullptr;
  int32_t* zc_rep = nullptr;
  if (e->zc && bt->h_cidx && bt->h_crep && bt->h_res_cap > 0) {
    void *di = nullptr, *dr = nullptr;
    if (dev::host_device_ptr(bt->h_cidx, &di) == 0 && dev::host_device_ptr(bt->h_crep, &dr) == 0) {
      zc_idx = (uint32_t*)di;
      zc_rep = (int32_t*)dr;
    }
  }
  KPROF(st, "k_compact", B, -1,
        dev::compact(st, bt->start, bt->count, bt->offsets_d, bt->out_idx, bt->out_rep, bt->cidx_d, bt->crep_d, B,
                     s->view.perm, zc_idx, zc_rep, zc_idx ? bt->h_res_cap : 0));
  bt->h_status.resize(B);
  bt->h_err.resize(B);
  bt->h_arg.resize(B);
  bt->h_offsets.resize(B + 1);
  HIPCHK(dev::d2h(bt->h_status.data(), bt->status, 4 * (size_t)B, st));
  HIPCHK(dev::d2h(bt->h_err.data(), bt->errc, 4 * (size_t)B, st));
  HIPCHK(dev::d2h(bt->h_arg.data(), bt->arg, 8 * (size_t)B, st));
  HIPCHK(dev::d2h(bt->h_offsets.data(), bt->offsets_d, 8 * (size_t)(B + 1), st));
  HIPCHK(dev::d2h(bt->h_stats, bt->stats, sizeof(bt->h_stats), st));
  pd.zc = zc_idx != nullptr;
  pd.bits = bits;
  pd.fast = fast;
  pd.top = top;
  pd.spread_orders = spread_orders;
  pd.th0 = th0;
  pd.th1 = th1;
  // A batch scheduled again copies its previous call's CSR size ahead of the read-back of
  // this call's total (the rest, if this total is larger, after it): one host round trip
  // per call instead of two, so the stream has the copy queued behind the kernels.
  uint64_t spec = 0;
  if (!zc_idx && bt->h_cidx && bt->h_crep && e->spec_copy) {
    spec = std::min<uint64_t>(bt->last_tot, bt->h_res_cap);
    if (spec) {
      HIPCHK(dev::d2h(bt->h_cidx, bt->cidx_d, 4 * spec, st));
      HIPCHK(dev::d2h(bt->h_crep, bt->crep_d, 4 * spec, st));
    }
  }
  pd.spec = spec;
  if (!pd.ev && dev::event_create(&pd.ev)) {
    pd.ev = nullptr;
    e->err = "kp_schedule_batch: event";
    return KP_EDEVICE;
  }
  HIPCHK(dev::event_record(pd.ev, st));
  pd.live = true;
  return KP_OK;
}

static int schedule_finish(kp_engine* e, kp_batch* bt, kp_results* out) {
  if (!e || !bt || !out) return KP_EINVAL;
  SchedPend& pd = bt->pend;
  if (!pd.live) {
    e->err = "kp_schedule_batch_collect: the batch has no submitted call";
    return KP_ESTATE;
  }
  pd.live = false;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  const int B = bt->B;
  if (pd.empty) {
    memset(out, 0, sizeof(*out));
    bt->h_offsets.assign(1, 0);
    out->offsets = bt->h_offsets.data();
    return KP_OK;
  }
  dev::stream_t st = e->stream;
  const double t0 = pd.t0, th0 = pd.th0, th1 = pd.th1;
  const bool bits = pd.bits, top = pd.top, spread_orders = pd.spread_orders;
  const int fast = pd.fast;
  const uint64_t spec = pd.spec;
  const bool zc = pd.zc;
  kp_stage_times tm{};
  HIPCHK(dev::event_sync(pd.ev));
  std::vector<uint32_t> sets_ovf(bt->sets_cls.size(), 0);
  if (!sets_ovf.empty()) {
    HIPCHK(dev::d2h(sets_ovf.data(), bt->d_sets_ovf, 4 * sets_ovf.size(), st));
    HIPCHK(dev::sync(st));
  }
  double tc0 = now_ms();
  const uint64_t tot = bt->h_offsets[B];
  bool copy = !zc;  // (written by k_compact unless the total outgrew the buffers)
  uint64_t have = zc ? tot : spec;  // entries already in the page-locked buffers
  bt->last_tot = tot;
  if (tot > bt->h_res_cap || !bt->h_cidx) {
    copy = true;
    have = 0;
    buf_pool().put(-1, bt->h_cidx, bt->h_cidx_bytes);
    buf_pool().put(-1, bt->h_crep, bt->h_crep_bytes);
    bt->h_cidx = nullptr;
    bt->h_crep = nullptr;
    bt->h_res_cap = 0;
    const uint64_t cap = std::max<uint64_t>(1, tot + tot / 4);  // headroom for repeated calls
    bt->h_cidx = (uint32_t*)pinned_get(4 * cap, &bt->h_cidx_bytes);
    bt->h_crep = (int32_t*)pinned_get(4 * cap, &bt->h_crep_bytes);
    if (!bt->h_cidx || !bt->h_crep) {
      e->err = "kp_schedule_batch: page-locked result buffers";
      return KP_ENOMEM;
    }
    bt->h_res_cap = std::min(bt->h_cidx_bytes, bt->h_crep_bytes) / 4;
  }
  if (copy && tot > have) {
    HIPCHK(dev::d2h(bt->h_cidx + have, bt->cidx_d + have, 4 * (tot - have), st));
    HIPCHK(dev::d2h(bt->h_crep + have, bt->crep_d + have, 4 * (tot - have), st));
    HIPCHK(dev::sync(st));
  }
  // A component-set class whose simulation outgrew the device's node runs in some
  // cluster (kSetsRunsMax): its bindings report KP_ERR_SETS_CAPACITY, every other
  // binding keeps its result (the CSR is re-packed without their targets).
  for (size_t j = 0; j < sets_ovf.size(); j++) {
    if (!sets_ovf[j]) continue;
    const int32_t cls = bt->sets_cls[j];
    for (int32_t b : bt->l_sets)
      if (bt->bcls[b] == cls) {
        bt->h_status[b] = KP_STATUS_ERROR;
        bt->h_err[b] = KP_ERR_SETS_CAPACITY;
        bt->h_arg[b] = (int64_t)s->perm[sets_ovf[j] - 1];
      }
  }
  if (std::any_of(sets_ovf.begin(), sets_ovf.end(), [](uint32_t v) { return v != 0; })) {
    uint64_t w = 0;
    for (int b = 0; b < B; b++) {
      const uint64_t lo = bt->h_offsets[b], hi = bt->h_offsets[b + 1];
      bt->h_offsets[b] = w;
      if (bt->h_status[b] != KP_STATUS_OK) continue;
      for (uint64_t k = lo; k < hi; k++, w++) {
        bt->h_cidx[w] = bt->h_cidx[k];
        bt->h_crep[w] = bt->h_crep[k];
      }
    }
    bt->h_offsets[B] = w;
  }
  const uint64_t tot_out = bt->h_offsets[B];
  double t1 = now_ms();
  if (e->prof) prof_fold(e, bt->h_stats);
  // pair: the pair launch, or k_est_class + k_filter (stream2; filter: k_filter
  // alone); select: from the point where they are complete to the end of the last
  // select kernel.
  // (the engine's events time this call unless a later submit has re-recorded them)
  const bool timed = pd.seq == e->submit_seq;
  auto ems = [&](int a, int b) { return timed ? dev::event_ms(e->ev[a], e->ev[b]) : 0.f; };
  const float ms_pair = ems(3, 4);
  const float ms_filter = bits ? ems(5, 4) : 0.f;
  const float ms_sel = ems(1, 2);
  tm.pair_launches = bits ? 2 : 1;
  tm.pair_kind = (uint32_t)fast;
  tm.pair_kernel_ms = ms_pair;
  tm.select_kernel_ms = ms_sel;
  tm.filter_kernel_ms = ms_filter;
  tm.sel_all_kernel_ms = ems(7, 8);
  tm.n_sel_all = (uint32_t)bt->l_all.size();
  tm.bits = bits ? 1u : 0u;
  tm.n_classes = bits ? (uint32_t)bt->crep.size() : 0u;
  tm.n_slow = bt->h_stats[0];
  tm.n_top = top ? (uint32_t)bt->n_all_dyn : 0u;
  tm.n_top_fallback = top ? bt->h_stats[9] : 0u;
  tm.top_kernel_ms = top ? ems(12, 13) : 0.f;
  tm.n_cluster = (uint32_t)bt->l_cluster.size();
  tm.n_cluster_order = spread_orders ? bt->h_stats[10] : 0u;
  tm.cluster_kernel_ms = bt->l_cluster.empty() ? 0.f : ems(14, 15);
  tm.n_region = (uint32_t)bt->l_region.size();
  tm.n_region_order = spread_orders ? bt->h_stats[11] : 0u;
#if defined(KP_STAMPS) || defined(KP_SLOW_CHECK)
  {
    std::vector<unsigned long long> hv((size_t)kDbgSlots * kDbgSpread);
    HIPCHK(dev::d2h(hv.data(), bt->dbg, 8 * hv.size(), st));
    HIPCHK(dev::sync(st));
    unsigned long long h[kDbgSlots] = {};
    for (size_t q = 0; q < hv.size(); q++) h[q % kDbgSlots] += hv[q];
    fprintf(stderr, "kp stamps (s_memtime ticks, summed over workgroups):");
    for (int i = 0; i < kDbgSlots; i++)
      if (h[i]) fprintf(stderr, " [%d]=%llu", i, h[i]);
    fprintf(stderr, "\n");
  }
#endif
  if (getenv("KP_DEBUG_SLOW"))
    fprintf(stderr,
            "kp slow: total %u overflow/dup %u scale-down %u wrap %u tie %u weight %u cluster %u "
            "(ties resolved block-parallel %u); class-order spread fallbacks: cluster %u region %u (stage A %u)"
            " check %u\n",
            bt->h_stats[0], bt->h_stats[1], bt->h_stats[2], bt->h_stats[3], bt->h_stats[4], bt->h_stats[5],
            bt->h_stats[6], bt->h_stats[7], bt->h_stats[12], bt->h_stats[13], bt->h_stats[14], bt->h_stats[15]);
  tm.pair_ms = ms_pair;
  tm.select_ms = ms_sel;
  tm.host_ms = th1 - th0;
  tm.copy_ms = t1 - tc0;
  tm.total_ms = t1 - t0;
  e->times = tm;
  out->n_bindings = (uint64_t)B;
  out->status = bt->h_status.data();
  out->err_code = bt->h_err.data();
  out->err_arg = bt->h_arg.data();
  out->offsets = bt->h_offsets.data();
  out->cluster_idx = bt->h_cidx;
  out->replicas = bt->h_crep;
  out->n_targets = tot_out;
  return KP_OK;
}
static int schedule_batch_impl(kp_engine* e, kp_batch* bt, kp_results* out) {
  if (!out) return KP_EINVAL;
  if (int rc = schedule_submit(e, bt)) return rc;
  return schedule_finish(e, bt, out);
}
int kp_schedule_batch(kp_engine* e, kp_batch* bt, kp_results* out) { return batch_fence(e, bt, schedule_batch_impl(e, bt, out)); }
int kp_schedule_batch_submit(kp_engine* e, kp_batch* bt) {
  if (e && e->prof) {
    e->err = "kp_schedule_batch_submit: per-kernel profiling covers kp_schedule_batch only";
    return KP_EINVAL;
  }
  if (bt && bt->pend.live) {
    e->err = "kp_schedule_batch_submit: the batch's previous call is not collected";
    return KP_ESTATE;
  }
  return batch_fence(e, bt, schedule_submit(e, bt));
}
int kp_schedule_batch_collect(kp_engine* e, kp_batch* bt, kp_results* out) {
  return batch_fence(e, bt, schedule_finish(e, bt, out));
}

// Runs the pair kernel and returns the rank-ordered device row pointers.
static int run_pair(kp_engine* e, kp_batch* bt, int64_t* score, int est_mode, int b0, int nb) {
  if (ensure_rows(e, bt)) return KP_EDEVICE;
  kp_snapshot* s = bt->snap;
  HIPCHK(dev::pair(e->stream, s->view, bt->view, nullptr, b0, nb, bt->fmask, bt->est, score, est_mode, md_cap_of(s),
                     smem_pair(s, md_cap_of(s))));
  HIPCHK(dev::sync(e->stream));
  return KP_OK;
}

static int filter_batch_impl(kp_engine* e, kp_batch* bt, uint64_t* out_mask) {
  if (!e || !bt || !out_mask) return KP_EINVAL;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  if (bt->B == 0) return KP_OK;
  if (s->view.n_bits > 0 && !getenv("KP_PAIR_ROWS")) {  // the schedule path's bitset filter
    HIPCHK(dev::filter(e->stream, s->view, bt->view, bt->fmask));
  } else {
    int rc = run_pair(e, bt, nullptr, 0, 0, bt->B);
    if (rc) return rc;
  }
  std::vector<uint64_t> m((size_t)bt->B * s->W);
  HIPCHK(dev::d2h(m.data(), bt->fmask, 8 * m.size(), e->stream));
  HIPCHK(dev::sync(e->stream));
  const int Wc = (s->C + 63) / 64;
  memset(out_mask, 0, 8 * (size_t)bt->B * Wc);
  for (int b = 0; b < bt->B; b++)
    for (int r = 0; r < s->C; r++)
      if ((m[(size_t)b * s->W + (r >> 6)] >> (r & 63)) & 1) {
        uint32_t c = s->perm[r];
        out_mask[(size_t)b * Wc + (c >> 6)] |= 1ull << (c & 63);
      }
  return KP_OK;
}
int kp_filter_batch(kp_engine* e, kp_batch* bt, uint64_t* out_mask) { return batch_fence(e, bt, filter_batch_impl(e, bt, out_mask)); }

static int filter_reasons_impl(kp_engine* e, kp_batch* bt, uint32_t* out_reasons) {
  if (!e || !bt || !out_reasons) return KP_EINVAL;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  if (bt->B == 0 || s->C == 0) return KP_OK;
  // bindings in chunks of at most kChunkPairs pairs through one reused device
  // buffer (a 100k x 5k batch would otherwise take 2 GB on each side)
  size_t chunk = (size_t)1 << 24;
  if (const char* v = getenv("KP_REASONS_CHUNK")) chunk = std::max<size_t>(1, (size_t)atoll(v));  // (tests)
  const int nb = (int)std::max<size_t>(1, std::min<size_t>((size_t)bt->B, chunk / (size_t)s->C));
  const size_t pairs = (size_t)nb * s->C;
  uint32_t* d = nullptr;
  HIPCHK(dev::alloc((void**)&d, 4 * pairs));
  std::vector<uint32_t> h(pairs);
  int rc = KP_OK;
  for (int b0 = 0; b0 < bt->B && rc == KP_OK; b0 += nb) {
    const int m = std::min(nb, bt->B - b0);
    if (dev::reasons(e->stream, s->view, bt->view, b0, m, d) || dev::d2h(h.data(), d, 4 * (size_t)m * s->C, e->stream) ||
        dev::sync(e->stream)) {
      e->err = std::string("kp_filter_reasons: ") + dev::last_error();
      rc = KP_EDEVICE;
      break;
    }
    for (int b = 0; b < m; b++)
      for (int r = 0; r < s->C; r++) out_reasons[(size_t)(b0 + b) * s->C + s->perm[r]] = h[(size_t)b * s->C + r];
  }
  dev::release(d);
  if (rc) return rc;
  return KP_OK;
}
int kp_filter_reasons(kp_engine* e, kp_batch* bt, uint32_t* out_reasons) { return batch_fence(e, bt, filter_reasons_impl(e, bt, out_reasons)); }

}  // extern "C"

// One component list resolved against the snapshot's resource dictionary (SetsArgs,
// kp_sets.h): podsInSet, perSetRequirement (general.go:371-401, wrapping int64) and
// each component's util.NewResource request (resource.go:46-75). KP_EINVAL for an
// unparsable quantity, KP_ENOTSUP beyond the device limits.
int build_sets_args(const kp_snapshot* s, const kp_component* comps, uint32_t K, SetsArgs* A, std::string* err) {
  if (K > (uint32_t)kSetsComp) {
    *err = "MaxAvailableComponentSets: more than 16 components";
    return KP_ENOTSUP;
  }
  memset(A, 0, sizeof(*A));
  A->K = (int32_t)K;
  std::map<std::string, int64_t> per;       // perSetRequirement (general.go:389-401), wrapping int64
  std::vector<std::map<std::string, int64_t>> nr(K);  // util.NewResource of each request
  std::vector<std::string> slots;
  int64_t pps = 0;
  for (uint32_t k = 0; k < K; k++) {
    A->replicas[k] = comps[k].replicas;
    pps += comps[k].replicas;  // podsInSet
    if (!comps[k].has_replica_requirements) continue;
    QtyMap rq;
    if (!qmap(comps[k].resource_request, comps[k].n_resource_request, &rq)) {
      *err = "MaxAvailableComponentSets: unparsable quantity";
      return KP_EINVAL;
    }
    for (auto& kv : rq) {
      const std::string& nm = kv.first;
      per[nm] = (int64_t)((uint64_t)per[nm] + (uint64_t)k8s::as_int64(kv.second) * (uint64_t)(int64_t)comps[k].replicas);
      int64_t v;
      if (nm == "cpu") v = k8s::milli(kv.second);
      else if (nm == "memory" || nm == "ephemeral-storage" || (nm != "pods" && k8s::scalar_resource(nm)))
        v = k8s::value(kv.second);
      else continue;  // pods: requiredPerReplica.AllowedPodNumber = 1
      nr[k][nm] += v;
      if (std::find(slots.begin(), slots.end(), nm) == slots.end()) slots.push_back(nm);
    }
  }
  if (slots.size() + 1 > (size_t)kSetsSlots || per.size() > (size_t)kSetsPer) {
    *err = "MaxAvailableComponentSets: too many distinct resources";
    return KP_ENOTSUP;
  }
  A->NS = (int32_t)slots.size() + 1;
  for (size_t j = 0; j < slots.size(); j++) A->slot_rid[j] = s->res.get(slots[j]);
  A->slot_rid[slots.size()] = -2;  // pods
  for (uint32_t k = 0; k < K; k++) {
    for (size_t j = 0; j < slots.size(); j++) {
      auto it = nr[k].find(slots[j]);
      const int64_t v = it == nr[k].end() ? 0 : it->second;
      A->req[k][j] = v;
      A->pos[k][j] = v > 0 ? v : 0;
    }
    A->req[k][slots.size()] = 1;
    A->pos[k][slots.size()] = 1;
  }
  A->pods_per_set = pps;
  for (auto& kv : per) {
    A->per_rid[A->nper] = s->res.get(kv.first);
    A->per_req[A->nper] = kv.second;
    A->per_nonzero |= kv.second != 0 ? 1 : 0;
    A->nper++;
  }
  return KP_OK;
}

extern "C" {

int kp_max_available_component_sets(kp_engine* e, const kp_snapshot* sc, const kp_component* comps, uint32_t K,
                                    const uint32_t* cluster_idx, uint64_t n, int32_t* out) {
  if (!e || !sc || (K && !comps) || (n && (!cluster_idx || !out))) return KP_EINVAL;
  (void)dev::set_device(e->device);
  kp_snapshot* s = const_cast<kp_snapshot*>(sc);
  if (!s->opts.multiple_pod_templates_scheduling) {
    e->err = "MaxAvailableComponentSets: the MultiplePodTemplatesScheduling gate is off";
    return KP_ENOTSUP;
  }
  SetsArgs A;
  if (int rc = build_sets_args(s, comps, K, &A, &e->err)) return rc;
  std::vector<int32_t> ranks(n);
  std::vector<int64_t> off(n + 1, 0);  // runs per cluster: its model node count (a run holds >= 1 node)
  for (uint64_t i = 0; i < n; i++) {
    if (cluster_idx[i] >= (uint32_t)s->C) return KP_EINVAL;
    const int r = s->inv[cluster_idx[i]];
    ranks[i] = r;
    int64_t nodes = 0;
    for (int g = s->mgrp_off[r]; g < s->mgrp_off[r + 1]; g++) nodes += s->mgrp_cnt[g];
    off[i + 1] = off[i] + std::max<int64_t>(1, std::min<int64_t>(nodes, kSetsRunsMax));
  }
  if (n == 0) return KP_OK;
  Arena a;
  SetsArgs* dA;
  int32_t *dr, *dout;
  int64_t *doff, *scratch;
  a.add(&dA, 1);
  a.add(&dr, n);
  a.add(&doff, n + 1);
  a.add(&dout, n);
  a.add(&scratch, (size_t)off[n] * (1 + kSetsSlots));
  HIPCHK(a.alloc());
  HIPCHK(dev::h2d(dA, &A, sizeof(A), e->stream));
  HIPCHK(dev::h2d(dr, ranks.data(), 4 * n, e->stream));
  HIPCHK(dev::h2d(doff, off.data(), 8 * (n + 1), e->stream));
  HIPCHK(dev::component_sets(e->stream, s->view, dA, dr, doff, n, scratch, dout));
  HIPCHK(dev::d2h(out, dout, 4 * n, e->stream));
  HIPCHK(dev::sync(e->stream));
  for (uint64_t i = 0; i < n; i++)
    if (out[i] == kSetsOverflow) {
      e->err = "MaxAvailableComponentSets: cluster " + s->names[ranks[i]] + " needs more than " +
               std::to_string(kSetsRunsMax) + " node runs";
      return KP_ENOTSUP;
    }
  return KP_OK;
}

static int score_batch_impl(kp_engine* e, kp_batch* bt, int64_t* out_scores) {
  if (!e || !bt || !out_scores) return KP_EINVAL;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  if (bt->B == 0) return KP_OK;
  int64_t* d = nullptr;
  size_t n = (size_t)bt->B * std::max(1, s->C);
  HIPCHK(dev::alloc((void**)&d, 8 * n));
  int rc = run_pair(e, bt, d, 0, 0, bt->B);
  std::vector<int64_t> h(n);
  if (rc == KP_OK) rc = (dev::d2h(h.data(), d, 8 * n, e->stream) || dev::sync(e->stream)) ? KP_EDEVICE : KP_OK;
  dev::release(d);
  if (rc) return rc;
  for (int b = 0; b < bt->B; b++)
    for (int r = 0; r < s->C; r++) out_scores[(size_t)b * s->C + s->perm[r]] = h[(size_t)b * s->C + r];
  return KP_OK;
}
int kp_score_batch(kp_engine* e, kp_batch* bt, int64_t* out_scores) { return batch_fence(e, bt, score_batch_impl(e, bt, out_scores)); }

static int max_available_replicas_impl(kp_engine* e, kp_batch* bt, uint64_t binding, const uint32_t* cluster_idx, uint64_t n,
                                       int32_t* out) {
  if (!e || !bt || (n && (!cluster_idx || !out)) || binding >= (uint64_t)bt->B) return KP_EINVAL;
  (void)dev::set_device(e->device);
  kp_snapshot* s = bt->snap;
  int rc = run_pair(e, bt, nullptr, 1, (int)binding, 1);
  if (rc) return rc;
  std::vector<int32_t> row(s->Cp);
  HIPCHK(dev::d2h(row.data(), bt->est + (size_t)binding * s->Cp, 4 * (size_t)s->Cp, e->stream));
  HIPCHK(dev::sync(e->stream));
  for (uint64_t i = 0; i < n; i++) {
    if (cluster_idx[i] >= (uint32_t)s->C) return KP_EINVAL;
    out[i] = row[s->inv[cluster_idx[i]]];
  }
  return KP_OK;
}
int kp_max_available_replicas(kp_engine* e, kp_batch* bt, uint64_t binding, const uint32_t* cluster_idx, uint64_t n,
                              int32_t* out) {
  return batch_fence(e, bt, max_available_replicas_impl(e, bt, binding, cluster_idx, n, out));
}

// ---------------------------------------------------------------------------
// Member-cluster nodes
// ---------------------------------------------------------------------------
namespace {
// util.Resource (util/resource.go:28-93): cpu in milli, the rest in units; scalar
// resources only under IsScalarResourceName.
struct NodeRes {
  int64_t cpu = 0, mem = 0, eph = 0, pods = 0;
  std::map<std::string, int64_t> sc;
};
void res_add(NodeRes& r, const QtyMap& rl) {
  for (auto& kv : rl) {
    const std::string& n = kv.first;
    if (n == "cpu") r.cpu += k8s::milli(kv.second);
    else if (n == "memory") r.mem += k8s::value(kv.second);
    else if (n == "pods") r.pods += k8s::value(kv.second);
    else if (n == "ephemeral-storage") r.eph += k8s::value(kv.second);
    else if (k8s::scalar_resource(n)) r.sc[n] += k8s::value(kv.second);
  }
}
k8s::Qty qty_of(int64_t v, int64_t unit_nano, int fmt) {
  k8s::Qty q;
  q.nano = (k8s::i128)v * unit_nano;
  q.fmt = fmt;
  return q;
}
// getNodeAvailable (cluster_status_controller.go:613-639); false: no pod room
// (the caller's walk stops there).
bool node_available(const kp_node& nd, QtyMap* out) {
  QtyMap alloc;
  if (!qmap(nd.allocatable, nd.n_allocatable, &alloc)) return false;
  if (nd.n_pods == 0) {  // no pods on the node: nodePodResourcesMap has no entry
    *out = alloc;
    return true;
  }
  QtyMap req;
  qmap(nd.requested, nd.n_requested, &req);
  NodeRes pr;
  res_add(pr, req);
  pr.pods += nd.n_pods;  // AddResourcePods
  QtyMap al;  // Resource.ResourceList(): the positive fields
  if (pr.cpu > 0) al["cpu"] = qty_of(pr.cpu, 1000000, 0);
  if (pr.mem > 0) al["memory"] = qty_of(pr.mem, 1000000000, 1);
  if (pr.eph > 0) al["ephemeral-storage"] = qty_of(pr.eph, 1000000000, 1);
  if (pr.pods > 0) al["pods"] = qty_of(pr.pods, 1000000000, 0);
  for (auto& kv : pr.sc)
    if (kv.second > 0) al[kv.first] = qty_of(kv.second, 1000000000, kv.first.rfind("hugepages-", 0) == 0 ? 1 : 0);
  auto pods_of = [](const QtyMap& m) {
    auto it = m.find("pods");
    return it == m.end() ? (int64_t)0 : k8s::value(it->second);
  };
  if (pods_of(alloc) - pods_of(al) <= 0) return false;
  for (auto& kv : al) {
    auto it = alloc.find(kv.first);
    if (it != alloc.end()) k8s::qsub(it->second, kv.second);
  }
  *out = alloc;
  return true;
}
// A member cluster's nodes in one call's dictionary (NodeView's host arrays).
struct HostNodes {
  std::vector<uint32_t> flags;
  std::vector<int32_t> name, lbl_off{0}, tnt_off{0}, tnt;
  std::vector<int64_t> lbl, lbl_int;
  std::vector<uint8_t> lbl_int_ok;
};
void pack_nodes(const kp_node* nodes, uint64_t n, Dict& d, HostNodes& h) {
  for (uint64_t i = 0; i < n; i++) {
    const kp_node& nd = nodes[i];
    h.flags.push_back(nd.unschedulable ? 1u : 0u);
    const std::string nm = S(nd.name);
    h.name.push_back(nm.empty() ? -1 : d.add(nm));
    std::map<std::string, std::string> lm;  // node.Labels is a map
    for (uint32_t j = 0; j < nd.n_labels; j++) lm[S(nd.labels[j].key)] = S(nd.labels[j].value);
    for (auto& kv : lm) {
      h.lbl.push_back(((int64_t)d.add(kv.first) << 32) | (int64_t)(uint32_t)d.add(kv.second));
      int64_t x = 0;
      const bool ok = k8s::parse_int64(kv.second, &x);
      h.lbl_int.push_back(ok ? x : 0);
      h.lbl_int_ok.push_back(ok ? 1 : 0);
    }
    h.lbl_off.push_back((int32_t)h.lbl.size());
    for (uint32_t j = 0; j < nd.n_taints; j++) {
      const std::string ef = S(nd.taints[j].effect);
      if (ef != "NoSchedule" && ef != "NoExecute") continue;  // DoNotScheduleTaintsFilterFunc
      h.tnt.push_back(d.add(S(nd.taints[j].key)));
      h.tnt.push_back(d.add(S(nd.taints[j].value)));
      h.tnt.push_back(ef == "NoSchedule" ? EFF_NOSCHEDULE : EFF_NOEXECUTE);
    }
    h.tnt_off.push_back((int32_t)(h.tnt.size() / 3));
  }
}
// pb.NodeClaim -> ClaimProg's host arrays (offsets relative to this claim).
struct HostClaim {
  std::vector<int64_t> sel;
  std::vector<Tol> tols;
  int32_t tol_unsched = 0, has_aff = 0;
  std::vector<int32_t> term_off{0};
  std::vector<NodeReq> reqs;
  std::vector<int32_t> vals;
};
void compile_claim(const kp_node_claim* c, Dict& d, HostClaim& h) {
  if (!c) return;
  std::map<std::string, std::string> sm;  // labels.SelectorFromSet: one requirement per key
  for (uint32_t j = 0; j < c->n_node_selector; j++) sm[S(c->node_selector[j].key)] = S(c->node_selector[j].value);
  for (auto& kv : sm) h.sel.push_back(((int64_t)d.add(kv.first) << 32) | (int64_t)(uint32_t)d.add(kv.second));
  for (uint32_t j = 0; j < c->n_tolerations; j++) {
    const kp_toleration& t = c->tolerations[j];
    const std::string ef = S(t.effect), key = S(t.key), op = S(t.op), val = S(t.value);
    // TolerationsTolerateTaint for {node.kubernetes.io/unschedulable, NoSchedule}
    if ((ef.empty() || ef == "NoSchedule") && (key.empty() || key == "node.kubernetes.io/unschedulable") &&
        (op == "Exists" || ((op.empty() || op == "Equal") && val.empty())))
      h.tol_unsched = 1;
    Tol x;
    if (ef.empty()) x.eff = EFF_ANY;
    else if (ef == "NoSchedule") x.eff = EFF_NOSCHEDULE;
    else if (ef == "NoExecute") x.eff = EFF_NOEXECUTE;
    else continue;
    x.key = key.empty() ? -1 : d.add(key);
    if (op.empty() || op == "Equal") {
      x.op = TOL_EQUAL;
      x.val = d.add(val);
    } else if (op == "Exists") {
      x.op = TOL_EXISTS;
      x.val = -1;
    } else {
      continue;  // Lt/Gt disabled, unknown operators never tolerate
    }
    h.tols.push_back(x);
  }
  // nodeaffinity.NewLazyErrorNodeSelector (nodeaffinity.go:50-67, 155-263): empty
  // terms select nothing and are dropped; a term with a parse error never matches.
  h.has_aff = c->has_node_affinity ? 1 : 0;
  if (!h.has_aff) return;
  for (uint32_t t = 0; t < c->n_node_affinity_terms; t++) {
    const kp_node_selector_term& term = c->node_affinity_terms[t];
    if (term.n_match_expressions == 0 && term.n_match_fields == 0) continue;
    std::vector<NodeReq> rq;
    std::vector<int32_t> vl;
    bool ok = true;
    for (uint32_t q = 0; q < term.n_match_expressions && ok; q++) {  // nodeSelectorRequirementsAsSelector
      const kp_requirement& r = term.match_expressions[q];
      const std::string key = S(r.key), op = S(r.op);
      if (!(op == "In" || op == "NotIn" || op == "Exists" || op == "DoesNotExist" || op == "Gt" || op == "Lt") ||
          !Packer::valid_req(key, op, r.values, r.n_values)) {
        ok = false;
        break;
      }
      NodeReq x{};
      x.key = d.add(key);
      if (op == "In" || op == "NotIn") {
        x.op = op == "In" ? NA_IN : NA_NOTIN;
        x.voff = (int32_t)(h.vals.size() + vl.size());
        for (uint32_t j = 0; j < r.n_values; j++) vl.push_back(d.add(S(r.values[j])));
        x.nv = (int32_t)r.n_values;
      } else if (op == "Exists" || op == "DoesNotExist") {
        x.op = op == "Exists" ? NA_EXISTS : NA_DNE;
      } else {
        x.op = op == "Gt" ? NA_GT : NA_LT;
        k8s::parse_int64(S(r.values[0]), &x.x);
      }
      rq.push_back(x);
    }
    for (uint32_t q = 0; q < term.n_match_fields && ok; q++) {  // nodeSelectorRequirementsAsFieldSelector
      const kp_requirement& r = term.match_fields[q];
      const std::string key = S(r.key), op = S(r.op);
      if (!(op == "In" || op == "NotIn") || r.n_values != 1) {
        ok = false;
        break;
      }
      const std::string v = S(r.values[0]);
      NodeReq x{};
      if (key == "metadata.name") {  // extractNodeFields: the only field a node carries
        x.op = op == "In" ? NA_NAME_IN : NA_NAME_NOTIN;
        x.voff = d.add(v);
      } else {  // fields.Set.Get of an absent field is ""
        x.op = ((op == "In") == v.empty()) ? NA_FIELD_TRUE : NA_FIELD_FALSE;
      }
      rq.push_back(x);
    }
    if (!ok) continue;
    h.reqs.insert(h.reqs.end(), rq.begin(), rq.end());
    h.vals.insert(h.vals.end(), vl.begin(), vl.end());
    h.term_off.push_back((int32_t)h.reqs.size());
  }
}
// Device copies of HostNodes and of several claims (one ClaimProg each).
struct DevNodes {
  NodeView v{};
  std::vector<ClaimProg> progs;
  uint32_t *d_flags = nullptr;
  int32_t *d_name = nullptr, *d_loff = nullptr, *d_toff = nullptr, *d_tnt = nullptr, *d_toffs = nullptr,
          *d_vals = nullptr;
  int64_t *d_lbl = nullptr, *d_lint = nullptr, *d_sel = nullptr;
  uint8_t* d_lok = nullptr;
  Tol* d_tols = nullptr;
  NodeReq* d_reqs = nullptr;
  std::vector<int64_t> sel;
  std::vector<Tol> tols;
  std::vector<int32_t> toffs, vals;
  std::vector<NodeReq> reqs;
  std::vector<size_t> o_sel, o_tol, o_toff, o_req, o_val;
  void plan(Arena& ar, const HostNodes& h, const std::vector<HostClaim>& cl) {
    for (auto& c : cl) {
      o_sel.push_back(sel.size());
      o_tol.push_back(tols.size());
      o_toff.push_back(toffs.size());
      o_req.push_back(reqs.size());
      o_val.push_back(vals.size());
      sel.insert(sel.end(), c.sel.begin(), c.sel.end());
      tols.insert(tols.end(), c.tols.begin(), c.tols.end());
      toffs.insert(toffs.end(), c.term_off.begin(), c.term_off.end());
      reqs.insert(reqs.end(), c.reqs.begin(), c.reqs.end());
      vals.insert(vals.end(), c.vals.begin(), c.vals.end());
    }
    ar.add(&d_flags, std::max<size_t>(1, h.flags.size()));
    ar.add(&d_name, std::max<size_t>(1, h.name.size()));
    ar.add(&d_loff, h.lbl_off.size());
    ar.add(&d_lbl, std::max<size_t>(1, h.lbl.size()));
    ar.add(&d_lint, std::max<size_t>(1, h.lbl_int.size()));
    ar.add(&d_lok, std::max<size_t>(1, h.lbl_int_ok.size()));
    ar.add(&d_toff, h.tnt_off.size());
    ar.add(&d_tnt, std::max<size_t>(1, h.tnt.size()));
    ar.add(&d_sel, std::max<size_t>(1, sel.size()));
    ar.add(&d_tols, std::max<size_t>(1, tols.size()));
    ar.add(&d_toffs, std::max<size_t>(1, toffs.size()));
    ar.add(&d_reqs, std::max<size_t>(1, reqs.size()));
    ar.add(&d_vals, std::max<size_t>(1, vals.size()));
  }
  int upload(dev::stream_t st, const HostNodes& h, const std::vector<HostClaim>& cl, uint64_t n) {
    auto up = [&](void* dd, const void* hp, size_t bytes) { return bytes ? dev::h2d(dd, hp, bytes, st) : 0; };
    if (up(d_flags, h.flags.data(), 4 * h.flags.size()) || up(d_name, h.name.data(), 4 * h.name.size()) ||
        up(d_loff, h.lbl_off.data(), 4 * h.lbl_off.size()) || up(d_lbl, h.lbl.data(), 8 * h.lbl.size()) ||
        up(d_lint, h.lbl_int.data(), 8 * h.lbl_int.size()) || up(d_lok, h.lbl_int_ok.data(), h.lbl_int_ok.size()) ||
        up(d_toff, h.tnt_off.data(), 4 * h.tnt_off.size()) || up(d_tnt, h.tnt.data(), 4 * h.tnt.size()) ||
        up(d_sel, sel.data(), 8 * sel.size()) || up(d_tols, tols.data(), sizeof(Tol) * tols.size()) ||
        up(d_toffs, toffs.data(), 4 * toffs.size()) || up(d_reqs, reqs.data(), sizeof(NodeReq) * reqs.size()) ||
        up(d_vals, vals.data(), 4 * vals.size()))
      return -1;
    v = NodeView{n, d_flags, d_name, d_loff, d_lbl, d_lint, d_lok, d_toff, d_tnt};
    for (size_t k = 0; k < cl.size(); k++) {
      ClaimProg p{};
      p.sel = d_sel + o_sel[k];
      p.n_sel = (int32_t)cl[k].sel.size();
      p.tols = d_tols + o_tol[k];
      p.n_tols = (int32_t)cl[k].tols.size();
      p.tol_unsched = cl[k].tol_unsched;
      p.has_aff = cl[k].has_aff;
      p.n_terms = (int32_t)cl[k].term_off.size() - 1;
      p.term_off = d_toffs + o_toff[k];
      p.reqs = d_reqs + o_req[k];
      p.vals = d_vals + o_val[k];
      progs.push_back(p);
    }
    return 0;
  }
};
void split128(k8s::i128 v, int64_t* hi, uint64_t* lo) {
  *hi = (int64_t)(v >> 64);
  *lo = (uint64_t)v;
}
}  // namespace

int kp_model_grades(kp_engine* e, const kp_resource_model* models, uint32_t n_models, const kp_node* nodes,
                    uint64_t n_nodes, int64_t* out_counts) {
  if (!e || (n_models && !models) || (n_nodes && !nodes) || (n_models && !out_counts)) return KP_EINVAL;
  (void)dev::set_device(e->device);
  if (n_models == 0) return KP_OK;  // getAllocatableModelings returns nil
  // modeling.InitSummary (modeling.go:75-102)
  std::vector<std::string> rs_name;
  std::vector<QtyMap> rs_list;
  for (uint32_t g = 0; g < n_models; g++) {
    QtyMap tmp;
    for (uint32_t j = 0; j < models[g].n_ranges; j++) {
      const kp_model_range& it = models[g].ranges[j];
      if (rs_name.size() != models[g].n_ranges) rs_name.push_back(S(it.name));
      k8s::Qty q;
      if (!k8s::parse_quantity(S(it.min), &q)) {
        e->err = "kp_model_grades: unparsable range minimum";
        return KP_EINVAL;
      }
      tmp[S(it.name)] = q;
    }
    rs_list.push_back(tmp);
  }
  if (!rs_name.empty() && rs_name.size() != rs_list[0].size()) {
    e->err = "the number of resourceName is not equal the number of resourceList";
    return KP_EINVAL;
  }
  if (rs_name.empty()) {  // getIndex would index RMs[MaxInt]
    e->err = "kp_model_grades: resource models without ranges";
    return KP_EINVAL;
  }
  const int K = (int)n_models, NR = (int)rs_name.size();
  std::vector<int64_t> mh((size_t)NR * K), vh;
  std::vector<uint64_t> ml((size_t)NR * K), vl;
  for (int r = 0; r < NR; r++)
    for (int g = 0; g < K; g++) {
      auto it = rs_list[g].find(rs_name[r]);
      split128(it == rs_list[g].end() ? (k8s::i128)0 : it->second.nano, &mh[(size_t)r * K + g], &ml[(size_t)r * K + g]);
    }
  // the nodes' available resources, up to the first without pod room
  uint64_t n = 0;
  vh.reserve((size_t)n_nodes * NR);
  vl.reserve((size_t)n_nodes * NR);
  for (; n < n_nodes; n++) {
    QtyMap av;
    if (!node_available(nodes[n], &av)) break;
    for (int r = 0; r < NR; r++) {
      auto it = av.find(rs_name[r]);
      int64_t h;
      uint64_t l;
      split128(it == av.end() ? (k8s::i128)0 : it->second.nano, &h, &l);
      vh.push_back(h);
      vl.push_back(l);
    }
  }
  Arena a;
  int64_t *d_mh, *d_vh;
  uint64_t *d_ml, *d_vl;
  unsigned long long* d_cnt;
  a.add(&d_mh, mh.size());
  a.add(&d_ml, ml.size());
  a.add(&d_vh, std::max<size_t>(1, vh.size()));
  a.add(&d_vl, std::max<size_t>(1, vl.size()));
  a.add(&d_cnt, K);
  HIPCHK(a.alloc());
  dev::stream_t st = e->stream;
  HIPCHK(dev::h2d(d_mh, mh.data(), 8 * mh.size(), st));
  HIPCHK(dev::h2d(d_ml, ml.data(), 8 * ml.size(), st));
  HIPCHK(dev::h2d(d_vh, vh.data(), 8 * vh.size(), st));
  HIPCHK(dev::h2d(d_vl, vl.data(), 8 * vl.size(), st));
  HIPCHK(dev::fill(d_cnt, 0, 8 * (size_t)K, st));
  GradesArgs A{K, NR, d_mh, d_ml, d_vh, d_vl, n, d_cnt};
  HIPCHK(dev::grades(st, A));
  std::vector<unsigned long long> c(K);
  HIPCHK(dev::d2h(c.data(), d_cnt, 8 * (size_t)K, st));
  HIPCHK(dev::sync(st));
  for (int g = 0; g < K; g++) out_counts[g] = (int64_t)c[g];
  return KP_OK;
}

}  // extern "C"

namespace {
// One estimator-server call over a member cluster's nodes: the slots of every
// resource the components (and the Estimate request) name, the nodes' available
// resources in those slots, and a ClaimProg per component (+ the request's claim).
struct NodeJob {
  std::vector<std::string> slot{"pods"};
  NodeSetsArgs A{};
  std::vector<int64_t> avail;
  std::vector<uint32_t> present;
  Dict d;
  HostNodes hn;
  std::vector<HostClaim> cl;
  std::string err;
  int rc = KP_OK;
  static bool divides(const std::string& nm) {
    return nm == "cpu" || nm == "memory" || nm == "ephemeral-storage" || k8s::scalar_resource(nm);
  }
  static int64_t field(const NodeRes& r, const std::string& nm, bool* present) {
    *present = true;
    if (nm == "pods") return r.pods;
    if (nm == "cpu") return r.cpu;
    if (nm == "memory") return r.mem;
    if (nm == "ephemeral-storage") return r.eph;
    auto it = r.sc.find(nm);
    *present = it != r.sc.end();
    return *present ? it->second : 0;
  }
  int fail(int code, const char* m) {
    rc = code;
    err = m;
    return code;
  }
  // phases: the assumed workloads (empty ones skipped), then `main` (may be empty).
  int build(const kp_node* nodes, uint64_t n, const kp_assumed_workload* assumed, uint32_t n_assumed,
            const kp_node_component* main, uint32_t K, const QtyMap* extra) {
    std::vector<const kp_node_component*> comps;
    A.n = n;
    A.mono = 1;
    A.n_phase = 0;
    for (uint32_t w = 0; w < n_assumed; w++) {
      if (assumed[w].n_components == 0) continue;  // noderesource.go:168-170
      if (assumed[w].n_components > (uint32_t)kNodeComp || A.n_phase + 1 >= kNodePhase)
        return fail(KP_ENOTSUP, "more than 16 assumed workloads or 16 components in one");
      A.ph_k0[A.n_phase++] = (int32_t)comps.size();
      for (uint32_t k = 0; k < assumed[w].n_components; k++) comps.push_back(&assumed[w].components[k]);
    }
    if (K) {
      A.ph_k0[A.n_phase++] = (int32_t)comps.size();
      for (uint32_t k = 0; k < K; k++) comps.push_back(&main[k]);
    }
    A.ph_k0[A.n_phase] = (int32_t)comps.size();
    A.last_upper = K ? INT32_MAX : 1;
    if (comps.size() > (size_t)kNodeCompAll) return fail(KP_ENOTSUP, "more than 64 components in all");
    std::vector<NodeRes> creq(comps.size());
    for (size_t k = 0; k < comps.size(); k++) {
      const kp_node_component& c = *comps[k];
      if (!c.has_replica_requirements) continue;
      QtyMap q;
      if (!qmap(c.resource_request, c.n_resource_request, &q)) return fail(KP_EINVAL, "unparsable resource request");
      res_add(creq[k], q);
      for (auto& kv : q)
        if (divides(kv.first) && std::find(slot.begin(), slot.end(), kv.first) == slot.end()) slot.push_back(kv.first);
    }
    if (extra)
      for (auto& kv : *extra)
        if (divides(kv.first) && std::find(slot.begin(), slot.end(), kv.first) == slot.end()) slot.push_back(kv.first);
    if (slot.size() > (size_t)kNodeRes) return fail(KP_ENOTSUP, "more than 7 distinct requested resources");
    A.NU = (int32_t)slot.size();
    for (size_t k = 0; k < comps.size(); k++) {
      A.replicas[k] = comps[k]->replicas;
      if (comps[k]->replicas < 0) A.mono = 0;
      for (int u = 0; u < A.NU; u++) {
        bool pr;
        const int64_t v = u == 0 ? 1 : field(creq[k], slot[u], &pr);
        A.req[k][u] = v;
        A.pos[k][u] = v > 0 ? v : 0;
        if (v < 0) A.mono = 0;
      }
    }
    // getNodesAvailableResources / getNodeAvailableResource (noderesource.go:135-144,205-220)
    avail.assign((size_t)n * A.NU, 0);
    present.assign(n, 0);
    for (uint64_t i = 0; i < n; i++) {
      const kp_node& nd = nodes[i];
      QtyMap al, rqd;
      if (!qmap(nd.allocatable, nd.n_allocatable, &al) || !qmap(nd.requested, nd.n_requested, &rqd))
        return fail(KP_EINVAL, "unparsable node quantity");
      NodeRes a, r;
      res_add(a, al);
      res_add(r, rqd);
      uint32_t pm = 0;
      for (int u = 0; u < A.NU; u++) {
        bool pa, prq;
        const int64_t va = field(a, slot[u], &pa), vr = field(r, slot[u], &prq);
        int64_t x = 0;
        if (u == 0) x = std::max<int64_t>(std::max<int64_t>(va - vr, 0) - (int64_t)nd.n_pods, 0);
        else if (pa) x = prq ? std::max<int64_t>(va - vr, 0) : va;  // SubResource: absent scalars stay absent
        avail[(size_t)i * A.NU + u] = x;
        if (pa) pm |= 1u << u;
      }
      present[i] = pm;
    }
    A.max_steps = A.mono ? 4 * (int64_t)comps.size() * ((int64_t)n + 2) + 64 : (int64_t)1 << 20;
    pack_nodes(nodes, n, d, hn);
    cl.resize(comps.size());
    for (size_t k = 0; k < comps.size(); k++)
      if (comps[k]->has_replica_requirements) compile_claim(comps[k]->node_claim, d, cl[k]);
    return KP_OK;
  }
};
}  // namespace

extern "C" {

// Runs the job's set phases on the device; *sets = the last phase's count. On
// return the job's node state (d_avail) holds the deducted resources.
static int node_job_run(kp_engine* e, NodeJob& J, const kp_node_claim* est_claim, NodeEstArgs* est, int32_t* sets) {
  Arena ar;
  DevNodes dn;
  if (est) J.cl.emplace_back(), compile_claim(est_claim, J.d, J.cl.back());
  dn.plan(ar, J.hn, J.cl);
  const size_t NP = J.cl.size();
  const int KS = J.A.ph_k0[J.A.n_phase];
  ClaimProg* d_progs;
  NodeSetsArgs* d_args;
  int64_t* d_avail;
  uint32_t *d_present, *d_ovf, *d_sum;
  uint8_t* d_match;
  int32_t* d_out;
  ar.add(&d_progs, std::max<size_t>(1, NP));
  ar.add(&d_args, 1);
  ar.add(&d_avail, std::max<size_t>(1, J.avail.size()));
  ar.add(&d_present, std::max<size_t>(1, J.present.size()));
  ar.add(&d_match, std::max<size_t>(1, (size_t)KS * J.A.n));
  ar.add(&d_out, 1);
  ar.add(&d_ovf, 1);
  ar.add(&d_sum, 1);
  HIPCHK(ar.alloc());
  dev::stream_t st = e->stream;
  HIPCHK(dn.upload(st, J.hn, J.cl, J.A.n));
  J.A.avail = d_avail;
  J.A.present = d_present;
  J.A.match = d_match;
  J.A.out = d_out;
  J.A.ovf = d_ovf;
  if (NP) HIPCHK(dev::h2d(d_progs, dn.progs.data(), sizeof(ClaimProg) * NP, st));
  HIPCHK(dev::h2d(d_args, &J.A, sizeof(J.A), st));
  if (!J.avail.empty()) HIPCHK(dev::h2d(d_avail, J.avail.data(), 8 * J.avail.size(), st));
  if (!J.present.empty()) HIPCHK(dev::h2d(d_present, J.present.data(), 4 * J.present.size(), st));
  HIPCHK(dev::fill(d_out, 0, 4, st));
  HIPCHK(dev::fill(d_ovf, 0, 4, st));
  if (KS > 0 && J.A.n > 0) {
    HIPCHK(dev::node_match(st, dn.v, d_progs, KS, d_match));
    HIPCHK(dev::node_sets(st, d_args));
  }
  if (est) {
    HIPCHK(dev::fill(d_sum, 0, 4, st));
    est->v = dn.v;
    est->p = dn.progs.back();
    est->NU = J.A.NU;
    est->avail = d_avail;
    est->sum = d_sum;
    HIPCHK(dev::node_est(st, *est));
  }
  int32_t res = 0;
  uint32_t ovf = 0, sum = 0;
  HIPCHK(dev::d2h(&res, d_out, 4, st));
  HIPCHK(dev::d2h(&ovf, d_ovf, 4, st));
  if (est) HIPCHK(dev::d2h(&sum, d_sum, 4, st));
  HIPCHK(dev::sync(st));
  if (ovf) {
    e->err = "the first-fit simulation exceeded its step bound";
    return KP_ENOTSUP;
  }
  *sets = est ? (int32_t)sum : res;
  return KP_OK;
}

int kp_node_max_replicas(kp_engine* e, const kp_node* nodes, uint64_t n_nodes, const kp_resource* request,
                         uint32_t n_request, const kp_node_claim* claim, const kp_assumed_workload* assumed,
                         uint32_t n_assumed, int32_t* out) {
  if (!e || !out || (n_nodes && !nodes) || (n_request && !request) || (n_assumed && !assumed)) return KP_EINVAL;
  (void)dev::set_device(e->device);
  *out = 0;
  QtyMap rq;
  if (!qmap(request, n_request, &rq)) {
    e->err = "kp_node_max_replicas: unparsable resource request";
    return KP_EINVAL;
  }
  if (n_nodes == 0) return KP_OK;  // estimate.go:43-45
  NodeJob J;
  if (J.build(nodes, n_nodes, assumed, n_assumed, nullptr, 0, &rq) != KP_OK) {
    e->err = "kp_node_max_replicas: " + J.err;
    return J.rc;
  }
  // MaxDivided's dividing entries (resource.go:221-248): cpu milli, memory,
  // ephemeral-storage, scalar resources, each > 0
  NodeEstArgs E{};
  for (auto& kv : rq) {
    const std::string& nm = kv.first;
    if (!NodeJob::divides(nm)) continue;
    const int64_t v = nm == "cpu" ? k8s::milli(kv.second) : k8s::value(kv.second);
    const int u = (int)(std::find(J.slot.begin(), J.slot.end(), nm) - J.slot.begin());
    if (v > 0) E.q[u] = v;
  }
  int32_t sum = 0;
  const int rc = node_job_run(e, J, claim, &E, &sum);
  if (rc != KP_OK) return rc;
  *out = sum;
  return KP_OK;
}

int kp_node_max_component_sets(kp_engine* e, const kp_node* nodes, uint64_t n_nodes,
                               const kp_node_component* comps, uint32_t K, const kp_assumed_workload* assumed,
                               uint32_t n_assumed, int32_t* out) {
  if (!e || !out || (n_nodes && !nodes) || (K && !comps) || (n_assumed && !assumed)) return KP_EINVAL;
  (void)dev::set_device(e->device);
  *out = 0;
  if (K == 0) {  // noNodeConstraint (noderesource.go:155-158)
    *out = INT32_MAX;
    return KP_OK;
  }
  if (K > (uint32_t)kNodeComp) {
    e->err = "kp_node_max_component_sets: more than 16 components";
    return KP_ENOTSUP;
  }
  NodeJob J;
  if (J.build(nodes, n_nodes, assumed, n_assumed, comps, K, nullptr) != KP_OK) {
    e->err = "kp_node_max_component_sets: " + J.err;
    return J.rc;
  }
  if (n_nodes == 0) return KP_OK;  // no node holds a set
  int32_t sets = 0;
  const int rc = node_job_run(e, J, nullptr, nullptr, &sets);
  if (rc != KP_OK) return rc;
  *out = sets;
  return KP_OK;
}

int kp_last_stage_times(const kp_engine* e, kp_stage_times* out) {
  if (!e || !out) return KP_EINVAL;
  *out = e->times;
  return KP_OK;
}

}  // extern "C"

// getAffinityIndex (pkg/scheduler/helper.go:99-110).
static uint32_t affinity_index_of(const kp_binding& b) {
  if (!b.observed_affinity_name.ptr || b.observed_affinity_name.len == 0) return 0;
  const std::string obs(b.observed_affinity_name.ptr, b.observed_affinity_name.len);
  for (uint32_t i = 0; i < b.n_cluster_affinities; i++) {
    const kp_str& nm = b.cluster_affinities[i].affinity_name;
    if (nm.len == obs.size() && (nm.len == 0 || memcmp(nm.ptr, obs.data(), nm.len) == 0)) return i;
  }
  return 0;
}

int kp_schedule_affinities(kp_engine* e, const kp_snapshot* s, const kp_binding* bs, uint64_t n,
                           kp_affinity_results* out) {
  if (!e || !s || !out || (n && !bs)) return KP_EINVAL;
  if (int rc = refuse_out_of_tree(e, s)) return rc;
  auto& A = e->aff;
  A.status.assign(n, KP_STATUS_OK);
  A.err.assign(n, KP_ERR_NONE);
  A.arg.assign(n, 0);
  A.idx.assign(n, -1);
  A.attempts.assign(n, 0);
  // per binding: current term, first error seen, and its final (offset, count) in `pool`
  std::vector<uint32_t> cur(n, 0);
  std::vector<uint8_t> have_first(n, 0);
  std::vector<uint64_t> f_off(n, 0), f_cnt(n, 0);
  std::vector<uint32_t> pool_idx;
  std::vector<int32_t> pool_rep;
  std::vector<uint64_t> pending(n);
  for (uint64_t i = 0; i < n; i++) {
    pending[i] = i;
    const kp_binding& b = bs[i];
    if (b.n_cluster_affinities == 0) continue;
    cur[i] = affinity_index_of(b);
    if (b.has_reschedule_triggered_at && b.has_last_scheduled_time &&
        b.reschedule_triggered_at_ns > b.last_scheduled_time_ns)  // util.RescheduleRequired (binding.go:118-127)
      cur[i] = 0;
  }
  uint32_t rounds = 0;
  std::vector<kp_binding> sub;
  while (!pending.empty()) {
    rounds++;
    sub.resize(pending.size());
    for (size_t j = 0; j < pending.size(); j++) {
      sub[j] = bs[pending[j]];
      if (sub[j].n_cluster_affinities)  // updatedStatus.SchedulerObservedAffinityName (scheduler.go:640)
        sub[j].observed_affinity_name = sub[j].cluster_affinities[cur[pending[j]]].affinity_name;
    }
    kp_batch* bt = nullptr;
    int rc = kp_batch_create(e, s, sub.data(), sub.size(), &bt);
    if (rc) return rc;
    kp_results r{};
    rc = kp_schedule_batch(e, bt, &r);
    if (rc) {
      kp_batch_destroy(bt);
      return rc;
    }
    std::vector<uint64_t> next;
    for (size_t j = 0; j < pending.size(); j++) {
      const uint64_t i = pending[j];
      const kp_binding& b = bs[i];
      A.attempts[i]++;
      const bool ok = r.status[j] == KP_STATUS_OK;
      if (ok || b.n_cluster_affinities == 0) {
        A.status[i] = r.status[j];
        A.err[i] = r.err_code[j];
        A.arg[i] = r.err_arg[j];
        if (b.n_cluster_affinities && ok) A.idx[i] = (int32_t)cur[i];
        f_off[i] = pool_idx.size();
        f_cnt[i] = r.offsets[j + 1] - r.offsets[j];
        pool_idx.insert(pool_idx.end(), r.cluster_idx + r.offsets[j], r.cluster_idx + r.offsets[j + 1]);
        pool_rep.insert(pool_rep.end(), r.replicas + r.offsets[j], r.replicas + r.offsets[j + 1]);
        continue;
      }
      if (!have_first[i]) {  // firstErr (scheduler.go:646-649)
        have_first[i] = 1;
        A.status[i] = r.status[j];
        A.err[i] = r.err_code[j];
        A.arg[i] = r.err_arg[j];
      }
      if (++cur[i] < b.n_cluster_affinities) next.push_back(i);
    }
    kp_batch_destroy(bt);
    pending.swap(next);
  }
  A.offsets.assign(n + 1, 0);
  uint64_t tot = 0;
  for (uint64_t i = 0; i < n; i++) {
    A.offsets[i] = tot;
    tot += f_cnt[i];
  }
  A.offsets[n] = tot;
  A.cidx.resize(std::max<uint64_t>(1, tot));
  A.rep.resize(std::max<uint64_t>(1, tot));
  for (uint64_t i = 0; i < n; i++)
    for (uint64_t k = 0; k < f_cnt[i]; k++) {
      A.cidx[A.offsets[i] + k] = pool_idx[f_off[i] + k];
      A.rep[A.offsets[i] + k] = pool_rep[f_off[i] + k];
    }
  out->results.n_bindings = n;
  out->results.status = A.status.data();
  out->results.err_code = A.err.data();
  out->results.err_arg = A.arg.data();
  out->results.offsets = A.offsets.data();
  out->results.cluster_idx = A.cidx.data();
  out->results.replicas = A.rep.data();
  out->results.n_targets = tot;
  out->affinity_index = A.idx.data();
  out->attempts = A.attempts.data();
  out->rounds = rounds;
  return KP_OK;
}
