// spread_selftest.hip — test-only library (libkp_spreadtest.so): the engine's
// spread-selection device code (kp_paths.h) run over caller-given candidate lists,
// so the reference's spread tables (tests/golden/spread.json, transcribed from
// pkg/scheduler/core/spreadconstraint/*_test.go) can state arbitrary cluster
// scores, which no binding can produce through kp_schedule_batch (the in-tree
// score sum is 0 or 100). Never linked into libkp.so.
//
// Each entry runs either on the GPU (one 256-thread workgroup, GpuBlk, gfx950) or
// on the host (CpuBlk, the engine's host-build block), over the same template
// bodies the select kernels instantiate:
//   kpst_group_score     calcGroupScore / calcGroupScoreForDuplicate per group
//                        (region_a_fast or region_a; group_clusters.go:156-351)
//   kpst_select_groups   selectGroups (select_groups_dev; select_groups.go:102-224)
//   kpst_select_region   selectBestClustersByRegion: selectGroups over the given
//                        region scores, then the heads + top-up (region_b;
//                        select_clusters_by_region.go:25-64)
//   kpst_select_cluster  selectBestClustersByCluster incl. the swap step
//                        (sel_cluster_fast; select_clusters_by_cluster.go:25-102)
//   kpst_sort            sortClusters order of the keys (place_sorted; util.go:43-61)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "kp_paths.h"

using namespace kp;

namespace {

enum : int { OP_SCORE_FAST = 0, OP_SCORE_WALK = 1, OP_GROUPS = 2, OP_REGION = 3, OP_CLUSTER = 4, OP_SORT = 5 };

struct Case {
  int op, n, R;
  SnapView s;
  BatchView bv;
  BindHdr h;
  const uint64_t* keys;   // [n] sortClusters keys (sort_key), rank in the low bits
  const int16_t* reg;     // [n] group (region) index of candidate i, -1 none
  const RegionOut* gin;   // [R] OP_GROUPS / OP_REGION: (clusters, score) per group
  RegionOut* rout;        // [R] OP_SCORE_*: the group scores
  int32_t* sel;           // [R] selected group ids (path order)
  Item* items;            // [2 * kSmallMax] the selected clusters
  int32_t* res;           // [4]: n (or -1), status, err, nsel
  int64_t* arg;           // [1]
  uint64_t* start;        // [1] (sink)
  uint32_t* count;        // [1] (sink)
};

// Workspace (LDS on the device, a host buffer on the host).
size_t ws_bytes(int R, int Cp) {
  const size_t r8 = 8 * (size_t)R, r4 = 4 * (size_t)((R + 3) & ~3);
  return kRedBytes + 1024 + sizeof(Item) * 2 * kSmallMax + 8 * 2 * kSmallMax + r8 + r4 + 8 * r8 + 4 * r4 + 8 * (size_t)Cp +
         2 * (size_t)Cp + 64;
}

template <class BLK>
KP_HD void run_case(const BLK& B, unsigned char* ws, const Case& c) {
  const int R = c.R, Cp = c.s.Cp;
  unsigned char* p = ws + kRedBytes;
  uint32_t* hist = (uint32_t*)p;
  p += 1024;
  Item* items = (Item*)p;
  p += sizeof(Item) * 2 * kSmallMax;
  uint64_t* keys = (uint64_t*)p;
  p += 8 * 2 * kSmallMax;
  unsigned long long* heads = (unsigned long long*)p;
  p += 8 * (size_t)R;
  int32_t* rs = (int32_t*)p;
  p += 4 * (size_t)((R + 3) & ~3);
  RegionLds L;
  int64_t* q = (int64_t*)p;
  L.minkey = (unsigned long long*)q;
  L.last = (unsigned long long*)(q + R);
  L.sumAvail = q + 2 * R;
  L.sumScore = q + 3 * R;
  L.dscore = q + 4 * R;
  L.wsum = q + 5 * R;
  L.wscore = q + 6 * R;
  L.amin = q + 7 * R;
  p += 8 * 8 * (size_t)R;
  int32_t* q4 = (int32_t*)p;
  const int R4 = (R + 3) & ~3;
  L.cnt = q4;
  L.dvalid = q4 + R4;
  L.wcnt = q4 + 2 * R4;
  L.done = q4 + 3 * R4;
  p += 4 * 4 * (size_t)R4;
  Cands cd;
  cd.r = (uint32_t*)p;
  cd.v = (int32_t*)(cd.r + Cp);
  cd.g = (int16_t*)(cd.v + Cp);
  cd.F = c.n;
  for (int i = B.tid(); i < c.n; i += B.nth()) {
    put_ckey(cd, i, c.keys[i]);
    cd.g[i] = c.reg ? c.reg[i] : (int16_t)-1;
  }
  B.sync();
  SelCtx x;
  x.s = &c.s;
  x.bv = &c.bv;
  x.h = &c.h;
  x.b = 0;
  x.frow = nullptr;
  // AllocatableReplicas by rank (item_from_key -> est_at): the caller's buffer holds
  // the alloc row right after the region index row
  x.erow = c.s.region_idx + Cp;
  x.mrep = kInt32Max;
  x.merge = false;
  x.tgt_bits = nullptr;
  x.sink.status = c.res + 1;
  x.sink.err = c.res + 2;
  x.sink.arg = c.arg;
  x.sink.start = c.start;
  x.sink.count = c.count;
  x.dbg = nullptr;
  int n = -1;
  switch (c.op) {
    case OP_SCORE_FAST:
      if (!region_a_fast<BLK, true>(B, x, cd, L, c.rout)) {
        if (B.tid() == 0) c.res[0] = -2;  // (beyond the staging: the caller asked for the fast form)
        return;
      }
      n = 0;
      break;
    case OP_SCORE_WALK:
      region_a<BLK, true>(B, x, cd, L, c.rout);
      n = 0;
      break;
    case OP_GROUPS:
      if (B.tid() == 0) c.res[3] = select_groups_dev(c.gin, R, c.h.region_min, c.h.region_max, c.h.cluster_min, c.sel);
      n = 0;
      break;
    case OP_REGION: {
      if (B.tid() == 0) c.res[3] = select_groups_dev(c.gin, R, c.h.region_min, c.h.region_max, c.h.cluster_min, c.sel);
      B.sync();
      const int nsel = c.res[3];
      if (nsel < 0) {
        if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, -nsel, 0);
        break;
      }
      region_b<BLK, true>(B, x, cd, c.sel, nsel, hist, heads, rs, items, keys, nullptr, 0, 0, &n);
      break;
    }
    case OP_CLUSTER:
      if (!sel_cluster_fast<BLK, true>(B, x, cd, hist, items, keys, nullptr, 0, 0, &n)) n = -3;
      break;
    case OP_SORT:
      for (int i = B.tid(); i < c.n; i += B.nth()) keys[i] = c.keys[i];
      B.sync();
      place_sorted(B, x, keys, c.n, items);
      n = c.n;
      break;
  }
  B.sync();
  for (int i = B.tid(); i < n; i += B.nth()) c.items[i] = items[i];
  if (B.tid() == 0) c.res[0] = n;
}

}  // namespace

extern "C" __global__ void __launch_bounds__(256) k_spread_case(Case c) {
  extern __shared__ __align__(16) unsigned char smem[];
  run_case(GpuBlk{(int64_t*)smem}, smem, c);
}

namespace {

// Device buffer helpers: every failure returns -1000 - hipError (a test-only library).
struct Dev {
  std::vector<void*> ptrs;
  int rc = 0;
  template <class T>
  T* put(const T* src, size_t n) {
    void* d = nullptr;
    if (rc || hipMalloc(&d, sizeof(T) * (n ? n : 1)) != hipSuccess) {
      rc = -1001;
      return nullptr;
    }
    ptrs.push_back(d);
    if (src && n && hipMemcpy(d, src, sizeof(T) * n, hipMemcpyHostToDevice) != hipSuccess) rc = -1002;
    else if (!src && hipMemset(d, 0, sizeof(T) * (n ? n : 1)) != hipSuccess) rc = -1003;
    return (T*)d;
  }
  template <class T>
  void get(T* dst, const T* src, size_t n) {
    if (!rc && n && hipMemcpy(dst, src, sizeof(T) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = -1004;
  }
  ~Dev() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

// Runs one case. keys/reg: n candidates; region_idx/alloc: by rank, Cp entries each.
int run(int gpu, Case c, const uint64_t* keys, const int16_t* reg, const int32_t* region_idx, const int32_t* alloc,
        const RegionOut* gin, RegionOut* rout, int32_t* sel, Item* items, int32_t* res, int64_t* arg) {
  const int Cp = c.s.Cp, R = c.R;
  std::vector<int32_t> ridx_alloc(2 * (size_t)Cp);
  for (int i = 0; i < Cp; i++) {
    ridx_alloc[i] = region_idx ? region_idx[i] : -1;
    ridx_alloc[Cp + i] = alloc ? alloc[i] : 0;
  }
  res[0] = -1;
  res[1] = res[2] = 0;
  res[3] = 0;
  *arg = 0;
  uint64_t start = 0;
  uint32_t count = 0;
  const size_t wsb = ws_bytes(R, Cp);
  if (!gpu) {
    std::vector<int64_t> ws(wsb / 8 + 1);
    c.keys = keys;
    c.reg = reg;
    c.s.region_idx = ridx_alloc.data();
    c.gin = gin;
    c.rout = rout;
    c.sel = sel;
    c.items = items;
    c.res = res;
    c.arg = arg;
    c.start = &start;
    c.count = &count;
    run_case(CpuBlk{ws.data()}, (unsigned char*)ws.data(), c);
    return 0;
  }
  Dev d;
  c.keys = d.put(keys, (size_t)c.n);
  c.reg = d.put(reg, (size_t)c.n);
  c.s.region_idx = d.put(ridx_alloc.data(), ridx_alloc.size());
  c.gin = d.put(gin, (size_t)R);
  c.rout = d.put<RegionOut>(nullptr, (size_t)R);
  c.sel = d.put<int32_t>(nullptr, (size_t)R);
  c.items = d.put<Item>(nullptr, 2 * (size_t)kSmallMax);
  c.res = d.put(res, 4);
  c.arg = d.put(arg, 1);
  c.start = d.put<uint64_t>(nullptr, 1);
  c.count = d.put<uint32_t>(nullptr, 1);
  if (d.rc) return d.rc;
  if (wsb > 64 * 1024 &&
      hipFuncSetAttribute((const void*)k_spread_case, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wsb) != hipSuccess)
    return -1005;
  hipLaunchKernelGGL(k_spread_case, dim3(1), dim3(256), wsb, 0, c);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -1006;
  d.get(res, c.res, 4);
  d.get(arg, c.arg, 1);
  if (rout) d.get(rout, c.rout, (size_t)R);
  if (sel) d.get(sel, c.sel, (size_t)R);
  if (items && res[0] > 0) d.get(items, c.items, (size_t)res[0]);
  return d.rc;
}

Case base_case(int op, int n, int R, int Cp) {
  Case c;
  memset(&c, 0, sizeof c);
  c.op = op;
  c.n = n;
  c.R = R;
  c.s.C = Cp;
  c.s.Cp = Cp;
  c.s.W = (Cp + 63) / 64;
  c.s.n_regions = R;
  return c;
}

}  // namespace

extern "C" {

// One candidate of a ClusterDetailInfo list (group_clusters.go:353-378): its name
// rank (the clusters of one case are renumbered by name), Score, OverflowOrder,
// AvailableReplicas and AllocatableReplicas, and its group (region) index.
typedef struct kpst_cand {
  uint32_t rank;
  int32_t score;
  int32_t ovf;
  int32_t group;
  int64_t avail;
  int32_t alloc;
  int32_t pad;
} kpst_cand;

static void cands_in(const kpst_cand* cs, int n, int Cp, std::vector<uint64_t>* keys, std::vector<int16_t>* reg,
                     std::vector<int32_t>* ridx, std::vector<int32_t>* alloc) {
  keys->resize(n);
  reg->resize(n);
  ridx->assign(Cp, -1);
  alloc->assign(Cp, 0);
  for (int i = 0; i < n; i++) {
    (*keys)[i] = sort_key(cs[i].ovf, cs[i].score, cs[i].avail, cs[i].rank);
    (*reg)[i] = (int16_t)cs[i].group;
    (*ridx)[cs[i].rank] = cs[i].group;
    (*alloc)[cs[i].rank] = cs[i].alloc;
  }
}

static int cp_of(const kpst_cand* cs, int n) {
  int m = 1;
  for (int i = 0; i < n; i++)
    if ((int)cs[i].rank + 1 > m) m = (int)cs[i].rank + 1;
  return (m + 63) / 64 * 64;
}

// calcGroupScore per group: scores[g] for every group g < R. dup: the Duplicated
// formula (calcGroupScoreForDuplicate); walk: region_a (every group walked) instead
// of region_a_fast. Returns 0, or < 0 on a device error.
int kpst_group_score(int gpu, int walk, const kpst_cand* cs, int n, int R, int32_t replicas, int dup,
                     int64_t min_groups, int64_t cluster_min, int64_t* scores, int32_t* counts) {
  const int Cp = cp_of(cs, n);
  std::vector<uint64_t> keys;
  std::vector<int16_t> reg;
  std::vector<int32_t> ridx, alloc;
  cands_in(cs, n, Cp, &keys, &reg, &ridx, &alloc);
  Case c = base_case(walk ? OP_SCORE_WALK : OP_SCORE_FAST, n, R, Cp);
  c.h.replicas = replicas;
  c.h.flags = dup ? BF_GROUP_DUP : 0u;
  c.h.region_min = min_groups;
  c.h.cluster_min = cluster_min;
  std::vector<RegionOut> rout(R);
  int32_t res[4];
  int64_t arg;
  const int rc = run(gpu, c, keys.data(), reg.data(), ridx.data(), alloc.data(), nullptr, rout.data(), nullptr,
                     nullptr, res, &arg);
  if (rc) return rc;
  if (res[0] < 0) return res[0];
  for (int g = 0; g < R; g++) {
    scores[g] = rout[g].score;
    counts[g] = rout[g].count;
  }
  return 0;
}

// selectGroups over groups 0..R-1 (ids = name order): values (cluster counts) and
// weights (group scores). Returns the selected count (ids in out, path order) or
// -KP_ERR_* / the device-DFS budget code.
int kpst_select_groups(int gpu, const int32_t* values, const int64_t* weights, int R, int64_t min_groups,
                       int64_t max_groups, int64_t target, int32_t* out) {
  std::vector<RegionOut> gin(R);
  for (int g = 0; g < R; g++) gin[g] = RegionOut{values[g], 0, weights[g]};
  Case c = base_case(OP_GROUPS, 0, R, 64);
  c.h.region_min = min_groups;
  c.h.region_max = max_groups;
  c.h.cluster_min = target;
  int32_t res[4];
  int64_t arg;
  const int rc = run(gpu, c, nullptr, nullptr, nullptr, nullptr, gin.data(), nullptr, out, nullptr, res, &arg);
  return rc ? rc : res[3];
}

// selectBestClustersByRegion with the regions' scores given (RegionInfo.Score):
// out = ranks of the selected clusters (heads in path order, then the rest in
// sortClusters order). Returns their count, or -err (KP_ERR_*) for the reference's
// errors.
int kpst_select_region(int gpu, const kpst_cand* cs, int n, int R, const int64_t* region_scores, int64_t region_min,
                       int64_t region_max, int64_t cluster_min, int64_t cluster_max, uint32_t* out) {
  const int Cp = cp_of(cs, n);
  std::vector<uint64_t> keys;
  std::vector<int16_t> reg;
  std::vector<int32_t> ridx, alloc;
  cands_in(cs, n, Cp, &keys, &reg, &ridx, &alloc);
  std::vector<RegionOut> gin(R);
  for (int g = 0; g < R; g++) gin[g] = RegionOut{0, 0, region_scores[g]};
  for (int i = 0; i < n; i++)
    if (cs[i].group >= 0) gin[cs[i].group].count++;
  Case c = base_case(OP_REGION, n, R, Cp);
  c.h.region_min = region_min;
  c.h.region_max = region_max;
  c.h.cluster_min = cluster_min;
  c.h.cluster_max = cluster_max;
  std::vector<int32_t> sel(R);
  std::vector<Item> items(2 * kSmallMax);
  int32_t res[4];
  int64_t arg;
  const int rc = run(gpu, c, keys.data(), reg.data(), ridx.data(), alloc.data(), gin.data(), nullptr, sel.data(),
                     items.data(), res, &arg);
  if (rc) return rc;
  if (res[0] < 0) return res[1] ? -res[2] : -1;
  for (int i = 0; i < res[0]; i++) out[i] = items[i].rank;
  return res[0];
}

// selectBestClustersByCluster (need_replicas -1: resources ignored). Returns the
// selected count (ranks in out, in the order AssignReplicas receives them) or -err.
int kpst_select_cluster(int gpu, const kpst_cand* cs, int n, int64_t cluster_min, int64_t cluster_max,
                        int32_t need_replicas, uint32_t* out) {
  const int Cp = cp_of(cs, n);
  std::vector<uint64_t> keys;
  std::vector<int16_t> reg;
  std::vector<int32_t> ridx, alloc;
  cands_in(cs, n, Cp, &keys, &reg, &ridx, &alloc);
  Case c = base_case(OP_CLUSTER, n, 1, Cp);
  c.h.cluster_min = cluster_min;
  c.h.cluster_max = cluster_max;
  c.h.need_replicas = need_replicas;
  std::vector<Item> items(2 * kSmallMax);
  int32_t res[4];
  int64_t arg;
  const int rc = run(gpu, c, keys.data(), reg.data(), ridx.data(), alloc.data(), nullptr, nullptr, nullptr,
                     items.data(), res, &arg);
  if (rc) return rc;
  if (res[0] < 0) return res[1] ? -res[2] : -1;
  for (int i = 0; i < res[0]; i++) out[i] = items[i].rank;
  return res[0];
}

// sortClusters order (util.go:43-61) of the candidates' keys: ranks in out.
int kpst_sort(int gpu, const kpst_cand* cs, int n, uint32_t* out) {
  if (n > 2 * kSmallMax) return -1;
  const int Cp = cp_of(cs, n);
  std::vector<uint64_t> keys;
  std::vector<int16_t> reg;
  std::vector<int32_t> ridx, alloc;
  cands_in(cs, n, Cp, &keys, &reg, &ridx, &alloc);
  Case c = base_case(OP_SORT, n, 1, Cp);
  std::vector<Item> items(2 * kSmallMax);
  int32_t res[4];
  int64_t arg;
  const int rc = run(gpu, c, keys.data(), reg.data(), ridx.data(), alloc.data(), nullptr, nullptr, nullptr,
                     items.data(), res, &arg);
  if (rc) return rc;
  for (int i = 0; i < res[0]; i++) out[i] = items[i].rank;
  return res[0];
}

// The key's fields read back (the 7-bit score field): for the layout tests.
uint64_t kpst_sort_key(int32_t ovf, int64_t score, int64_t avail, uint32_t rank) {
  return sort_key(ovf, score, avail, rank);
}
void kpst_key_fields(uint64_t k, int32_t* ovf, int64_t* score, int64_t* avail, uint32_t* rank) {
  *ovf = key_ovf(k);
  *score = key_score(k);
  *avail = key_avail(k);
  *rank = key_rank(k);
}

}  // extern "C"
