// synth.cpp — seeded synthetic Karmada universes as kp_api.h
// structs, for the benchmark and the large parity tests (libkpsynth.so).
//
// Every cluster and every binding draws from its own splitmix64 stream keyed by
// (seed, kind, index), so any binding range [lo, hi) can be generated alone and
// is identical to the same range of the full universe (one range per rank).
//
// Workloads (config ids follow BASELINE.json "configs"):
//   1  C=10,   B=1k:  50% Duplicated, 50% Divided/Weighted/DynamicWeight
//   2  C=1k,   B=100k: affinity + tolerations, StaticWeight (4 label rules, weights 1-4)
//   3  C=5k,   B=100k: ResourceModels (8 grades), 50% DynamicWeight, 50% Aggregated
//   4  C=5k:   spread constraints (region+cluster / cluster / zone / provider)
//   5  C=10k,  B=1M:  mix of 2-4 by binding index
//   6  "edge": every branch of the path (overflow tiers, multi-term affinities,
//      reschedule, scale-down, duplicates, non-workloads, odd strategies) at small C.
//   7  "ties": clusters in three identical capacity classes, mostly Aggregated,
//      so equal AvailableReplicas straddle the Aggregated cut (sort.Sort's
//      permutation of equal keys decides; SURVEY hazard H2), parity only.
//   8  "wrap": clusters whose estimates approach MaxInt32 (pods ~1-2.1e9, huge
//      resources, model-grade counts near 2^31), so the int32 sums of
//      GetSumOfReplicas, dynamicDivideReplicas and the Aggregated prefix wrap
//      (SURVEY hazard H5), StaticWeight weights >= 2^31, spec.Clusters replicas
//      near 2^31 and seat counts up to MaxInt32; parity only.
//  10  "distinct": config 3 with every binding's requests drawn independently (cpu
//      milli uniform over [100, 4000], memory MiB over [128, 16384]), so nearly every
//      binding is its own estimator class; performance only.
//  11  "min0": config-4 clusters and spread constraints whose MinGroups are 0 (region
//      and cluster), so calcGroupScore divides Replicas by 0 (+Inf, or NaN at
//      Replicas 0, both MinInt64 on amd64: SURVEY hazard H4, group_clusters.go:
//      248-249) on Divided bindings; parity only.
//   9  "templates": multi-template workloads (spec.Components) for the
//      MultiplePodTemplatesScheduling gate: most carry a cluster spread constraint
//      with MinGroups = MaxGroups = 1 (isMultiTemplateSchedulingApplicable), over
//      config-3 clusters with resource models; parity only.
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kp/kp_api.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
  int64_t range(int64_t lo, int64_t hi) { return lo + (int64_t)below((uint64_t)(hi - lo + 1)); }  // inclusive
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  bool p(double x) { return unit() < x; }
};
uint64_t key(uint64_t seed, uint64_t kind, uint64_t i) {
  Rng r(seed * 0x100000001b3ull ^ (kind << 56) ^ (i * 0x9e3779b97f4a7c15ull));
  r.next();
  return r.next();
}

struct Arena {
  std::vector<std::unique_ptr<char[]>> chunks;
  size_t used = 0, cap = 0;
  void* raw(size_t bytes) {
    bytes = (bytes + 15) & ~(size_t)15;
    if (used + bytes > cap) {
      cap = std::max<size_t>(bytes, (size_t)4 << 20);
      chunks.emplace_back(new char[cap]);
      used = 0;
    }
    void* p = chunks.back().get() + used;
    used += bytes;
    memset(p, 0, bytes);
    return p;
  }
  template <class T>
  T* alloc(size_t n) {
    return n ? (T*)raw(sizeof(T) * n) : nullptr;
  }
};

}  // namespace

struct kps_world {
  Arena a;
  std::deque<std::string> strs;
  std::unordered_map<std::string, kp_str> interned;
  std::vector<kp_cluster> clusters;
  std::vector<kp_binding> bindings;
  uint32_t C = 0;
  int config = 0;
  uint64_t seed = 0;

  kp_str s(const std::string& v) {
    auto it = interned.find(v);
    if (it != interned.end()) return it->second;
    strs.push_back(v);
    kp_str k{strs.back().data(), (uint32_t)strs.back().size()};
    interned.emplace(v, k);
    return k;
  }
  kp_str u(const std::string& v) {  // unique (not interned)
    char* p = a.alloc<char>(v.size() + 1);
    memcpy(p, v.data(), v.size());
    return kp_str{p, (uint32_t)v.size()};
  }
  std::string cname(uint32_t i) const {
    char b[32];
    snprintf(b, sizeof b, C > 99999 ? "member-%07u" : "member-%05u", i);
    return b;
  }
};

namespace {

const char* kProviders[] = {"aws", "gcp", "azure"};
const int kRegions = 16, kKeys = 16, kVals = 8, kGvks = 64;

std::string lkey(int k) {
  char b[48];
  snprintf(b, sizeof b, "topology.example.io/k%02d", k);
  return b;
}
std::string lval(int v) { return "v" + std::to_string(v); }
std::string region(int r) {
  char b[16];
  snprintf(b, sizeof b, "region-%02d", r);
  return b;
}
std::string zone(int r, int z) { return region(r) + "-" + (char)('a' + z); }
void gvk(int g, std::string* gv, std::string* kind) {
  if (g == 0) {
    *gv = "apps/v1";
    *kind = "Deployment";
    return;
  }
  char b[48];
  snprintf(b, sizeof b, "g%02d.example.io/v1", g);
  *gv = b;
  *kind = "Kind" + std::to_string(g);
}

void gen_cluster(kps_world& w, uint32_t i, kp_cluster& c) {
  Rng r(key(w.seed, 1, i));
  const int cfg = w.config == 10 ? 3 : (w.config == 11 ? 4 : w.config);  // configs 10 / 11: config-3 / 4 clusters
  c.name = w.s(w.cname(i));
  // labels: 8 distinct keys of 16
  c.labels = w.a.alloc<kp_label>(8);
  c.n_labels = 8;
  int ks[kKeys];
  for (int k = 0; k < kKeys; k++) ks[k] = k;
  for (int k = 0; k < 8; k++) {
    int j = k + (int)r.below(kKeys - k);
    std::swap(ks[k], ks[j]);
    const_cast<kp_label*>(c.labels)[k] = kp_label{w.s(lkey(ks[k])), w.s(lval((int)r.below(kVals)))};
  }
  int reg = (int)r.below(kRegions);
  c.provider = w.s(kProviders[r.below(3)]);
  c.region = w.s(region(reg));
  int nz = 1 + (int)r.below(2);
  kp_str* zs = w.a.alloc<kp_str>(nz);
  int z0 = (int)r.below(4);
  for (int z = 0; z < nz; z++) zs[z] = w.s(zone(reg, (z0 + z) % 4));
  c.zones = zs;
  c.n_zones = nz;
  c.zone = zs[0];
  if (cfg == 4 && r.p(0.02)) {  // a few clusters without region / zones (filtered by spread presence)
    c.region = kp_str{nullptr, 0};
    c.n_zones = 0;
  }
  // taints
  kp_taint* ts = w.a.alloc<kp_taint>(2);
  int nt = 0;
  if (r.p(0.20)) ts[nt++] = kp_taint{w.s("dedicated"), w.s("gpu"), w.s("NoSchedule")};
  if (r.p(0.05)) ts[nt++] = kp_taint{w.s("maint"), w.s(""), w.s("NoExecute")};
  if (r.p(0.05)) ts[nt++] = kp_taint{w.s("soft"), w.s("x"), w.s("PreferNoSchedule")};
  c.taints = ts;
  c.n_taints = nt > 2 ? 2 : nt;
  // API enablements
  kp_api_enablement* ae = w.a.alloc<kp_api_enablement>(kGvks);
  int na = 0;
  for (int g = 0; g < kGvks; g++) {
    if (g != 0 && !r.p(0.95)) continue;
    std::string gv, kind;
    gvk(g, &gv, &kind);
    ae[na++] = kp_api_enablement{w.s(gv), w.s(kind)};
  }
  c.api_enablements = ae;
  c.n_api_enablements = na;
  // resource summary
  c.has_resource_summary = 1;
  const bool gpu = cfg == 3 || cfg == 5 || cfg == 6 || cfg == 9;
  int nres = gpu ? 5 : 4;
  kp_resource* al = w.a.alloc<kp_resource>(nres);
  kp_resource* ad = w.a.alloc<kp_resource>(nres);
  int64_t cpu = r.range(500, 4000), memg = r.range(2048, 16384), pods = r.range(1100, 11000),
          eph = r.range(10, 100), gpus = r.range(0, 64);
  double f = 0.7 * r.unit();
  if (cfg == 6 && r.p(0.2)) f = 0.999;  // nearly full clusters
  if (cfg == 7) {  // three capacity classes, nothing allocated: estimates tie in large groups
    cpu = 1000 * (1 + (int64_t)r.below(3));
    memg = 16384;
    pods = 11000;
    eph = 100;
    f = 0;
  }
  if (cfg == 8) {  // estimates near MaxInt32: the pod count binds (getAllowedPodNumber)
    cpu = 100000000;
    memg = (int64_t)1 << 30;
    pods = r.range(1000000000, 2147483000);
    eph = 1000000;
    f = r.p(0.5) ? 0 : 0.001 * r.unit();
  }
  al[0] = {w.s("cpu"), w.s(std::to_string(cpu))};
  al[1] = {w.s("memory"), w.s(std::to_string(memg) + "Gi")};
  al[2] = {w.s("pods"), w.s(std::to_string(pods))};
  al[3] = {w.s("ephemeral-storage"), w.s(std::to_string(eph) + "Ti")};
  ad[0] = {w.s("cpu"), w.s(std::to_string((int64_t)(cpu * 1000 * f)) + "m")};
  ad[1] = {w.s("memory"), w.s(std::to_string((int64_t)(memg * 1024 * f)) + "Mi")};
  ad[2] = {w.s("pods"), w.s(std::to_string((int64_t)(pods * f)))};
  ad[3] = {w.s("ephemeral-storage"), w.s(std::to_string((int64_t)(eph * 1024 * f)) + "Gi")};
  if (gpu) {
    al[4] = {w.s("nvidia.com/gpu"), w.s(std::to_string(gpus))};
    ad[4] = {w.s("nvidia.com/gpu"), w.s(std::to_string((int64_t)(gpus * f)))};
  }
  c.allocatable = al;
  c.n_allocatable = nres;
  c.allocated = ad;
  c.n_allocated = nres;
  if (cfg == 6 && r.p(0.05)) c.has_resource_summary = 0;
  if (cfg == 6 && r.p(0.03)) c.deleting = 1;
  // resource models: 8 grades over (cpu, memory) with monotone mins
  if (cfg == 3 || cfg == 5 || cfg == 9 || (cfg == 6 && r.p(0.5)) || (cfg == 8 && r.p(0.3))) {
    const int K = 8;
    kp_resource_model* rm = w.a.alloc<kp_resource_model>(K);
    kp_allocatable_modeling* am = w.a.alloc<kp_allocatable_modeling>(K);
    for (int g = 0; g < K; g++) {
      kp_model_range* rg = w.a.alloc<kp_model_range>(2);
      int64_t c0 = (int64_t)1 << g, c1 = (int64_t)1 << (g + 1);
      rg[0] = {w.s("cpu"), w.s(std::to_string(c0)), w.s(std::to_string(c1))};
      rg[1] = {w.s("memory"), w.s(std::to_string(4 * c0) + "Gi"), w.s(std::to_string(4 * c1) + "Gi")};
      rm[g] = {(uint32_t)g, rg, 2};
      am[g] = {(uint32_t)g, cfg == 8 ? r.range((int64_t)1 << 29, 2147483647) : r.range(0, 64)};
    }
    c.resource_models = rm;
    c.n_resource_models = K;
    c.allocatable_modelings = am;
    c.n_allocatable_modelings = K;
  }
}

const char* kCpu[] = {"100m", "250m", "500m", "1", "2", "4"};
const char* kMem[] = {"128Mi", "256Mi", "512Mi", "1Gi", "2Gi", "4Gi", "8Gi"};

kp_cluster_affinity label_in(kps_world& w, Rng& r, int nvals) {
  kp_cluster_affinity a{};
  a.has_label_selector = 1;
  kp_requirement* rq = w.a.alloc<kp_requirement>(1);
  kp_str* vs = w.a.alloc<kp_str>(nvals);
  int v0 = (int)r.below(kVals);
  for (int i = 0; i < nvals; i++) vs[i] = w.s(lval((v0 + i) % kVals));
  rq[0] = kp_requirement{w.s(lkey((int)r.below(kKeys))), w.s("In"), vs, (uint32_t)nvals};
  a.match_expressions = rq;
  a.n_match_expressions = 1;
  return a;
}

// 1..kmax components (workv1alpha2.Component) with small replica counts and requests.
void gen_components(kps_world& w, Rng& r, kp_binding& b, int kmax) {
  const int K = 1 + (int)r.below(kmax);
  kp_component* cs = w.a.alloc<kp_component>(K);
  for (int k = 0; k < K; k++) {
    cs[k].name = w.s("comp-" + std::to_string(k));
    cs[k].replicas = (int32_t)r.range(r.p(0.05) ? 0 : 1, 4);
    cs[k].has_replica_requirements = r.p(0.9);
    if (cs[k].has_replica_requirements) {
      const int nq = r.p(0.15) ? 3 : 2;
      kp_resource* rq = w.a.alloc<kp_resource>(nq);
      rq[0] = {w.s("cpu"), w.s(kCpu[r.below(6)])};
      rq[1] = {w.s("memory"), w.s(kMem[r.below(7)])};
      if (nq == 3) rq[2] = {w.s("nvidia.com/gpu"), w.s("1")};
      cs[k].resource_request = rq;
      cs[k].n_resource_request = nq;
    }
  }
  b.components = cs;
  b.n_components = K;
}
// a cluster spread constraint MinGroups = MaxGroups = 1 (+ sometimes a region one)
void one_cluster_spread(kps_world& w, Rng& r, kp_binding& b) {
  kp_spread_constraint* sc = w.a.alloc<kp_spread_constraint>(2);
  int n = 0;
  if (r.p(0.15)) sc[n++] = {w.s("region"), {}, 2, 1};
  sc[n++] = {w.s("cluster"), {}, 1, 1};
  b.spread_constraints = sc;
  b.n_spread_constraints = n;
}

void gen_binding(kps_world& w, uint64_t i, kp_binding& b) {
  Rng r(key(w.seed, 2, i));
  int cfg = w.config;
  if (cfg == 5) cfg = 2 + (int)(i % 3);
  const bool distinct = cfg == 10;  // config 10: config 3 with per-binding requests
  if (distinct) cfg = 3;
  const uint32_t C = w.C;
  char ub[40];
  snprintf(ub, sizeof ub, "%08x-%04x-4%03x-%04x-%012llx", (unsigned)r.next(), (unsigned)(r.next() & 0xffff),
           (unsigned)(r.next() & 0xfff), (unsigned)((r.next() & 0x3fff) | 0x8000),
           (unsigned long long)(r.next() & 0xffffffffffffull));
  b.uid = w.u(ub);
  char nb[32];
  snprintf(nb, sizeof nb, "app-%07llu", (unsigned long long)i);
  b.name = w.u(nb);
  b.namespace_ = w.s("default");
  std::string gv = "apps/v1", kind = "Deployment";
  if (r.p(0.2)) gvk(1 + (int)r.below(kGvks - 1), &gv, &kind);
  b.api_version = w.s(gv);
  b.kind = w.s(kind);
  b.replicas = (int32_t)std::floor(std::exp(r.unit() * std::log(1000.0)));
  if (b.replicas < 1) b.replicas = 1;
  b.has_replica_requirements = 1;
  int nreq = (cfg == 3 && r.p(0.1)) ? 3 : 2;
  kp_resource* rq = w.a.alloc<kp_resource>(nreq);
  if (distinct) {  // cpu milli uniform over [100, 4000], memory MiB uniform over [128, 16384]
    char cb[24], mb[24];
    snprintf(cb, sizeof cb, "%dm", (int)r.range(100, 4000));
    snprintf(mb, sizeof mb, "%dMi", (int)r.range(128, 16384));
    rq[0] = {w.s("cpu"), w.s(cb)};
    rq[1] = {w.s("memory"), w.s(mb)};
  } else {
    rq[0] = {w.s("cpu"), w.s(kCpu[r.below(6)])};
    rq[1] = {w.s("memory"), w.s(kMem[r.below(7)])};
  }
  if (nreq == 3) rq[2] = {w.s("nvidia.com/gpu"), w.s("1")};
  b.resource_request = rq;
  b.n_resource_request = nreq;
  // placement: affinity + tolerations
  if (r.p(0.7)) {
    b.has_cluster_affinity = 1;
    b.cluster_affinity = label_in(w, r, 1 + (int)r.below(4));
  }
  if (r.p(0.5)) {
    kp_toleration* t = w.a.alloc<kp_toleration>(1);
    t[0] = {w.s("dedicated"), w.s("Equal"), w.s("gpu"), w.s("NoSchedule")};
    b.tolerations = t;
    b.n_tolerations = 1;
  }
  b.has_replica_scheduling = 1;
  b.replica_scheduling_type = w.s("Divided");
  b.replica_division_preference = w.s("Weighted");
  b.has_weight_preference = 1;
  b.dynamic_weight = w.s("AvailableReplicas");
  if (cfg == 1) {
    if (r.p(0.5)) {
      b.replica_scheduling_type = w.s("Duplicated");
      b.replica_division_preference = kp_str{nullptr, 0};
      b.has_weight_preference = 0;
      b.dynamic_weight = kp_str{nullptr, 0};
    }
  } else if (cfg == 2) {
    b.dynamic_weight = kp_str{nullptr, 0};
    kp_static_weight* sw = w.a.alloc<kp_static_weight>(4);
    for (int k = 0; k < 4; k++) {
      kp_cluster_affinity a{};
      a.has_label_selector = 1;
      kp_label* ml = w.a.alloc<kp_label>(1);
      ml[0] = kp_label{w.s(lkey((int)r.below(kKeys))), w.s(lval((int)r.below(kVals)))};
      a.match_labels = ml;
      a.n_match_labels = 1;
      sw[k] = kp_static_weight{a, 1 + k};
    }
    b.static_weights = sw;
    b.n_static_weights = 4;
  } else if (cfg == 3) {
    if (r.p(0.5)) {
      b.replica_division_preference = w.s("Aggregated");
      b.has_weight_preference = 0;
      b.dynamic_weight = kp_str{nullptr, 0};
    }
  } else if (cfg == 4) {
    double x = r.unit();
    kp_spread_constraint* sc = w.a.alloc<kp_spread_constraint>(2);
    if (x < 0.70) {
      sc[0] = {w.s("region"), {}, 3, 2};
      sc[1] = {w.s("cluster"), {}, 8, 4};
      b.n_spread_constraints = 2;
    } else if (x < 0.90) {
      sc[0] = {w.s("cluster"), {}, 8, 1};
      b.n_spread_constraints = 1;
    } else if (x < 0.95) {
      sc[0] = {w.s("zone"), {}, 3, 1};
      b.n_spread_constraints = 1;
    } else {
      sc[0] = {w.s("provider"), {}, 2, 1};
      b.n_spread_constraints = 1;
    }
    b.spread_constraints = sc;
  } else if (cfg == 11) {
    const double x = r.unit();
    kp_spread_constraint* sc = w.a.alloc<kp_spread_constraint>(2);
    if (x < 0.45) {
      sc[0] = {w.s("region"), {}, 2 + (int64_t)r.below(2), 0};
      sc[1] = {w.s("cluster"), {}, 8, r.p(0.5) ? 0 : 4};
      b.n_spread_constraints = 2;
    } else if (x < 0.65) {
      sc[0] = {w.s("cluster"), {}, 6, 2};  // (cluster first: the map keeps the last per field)
      sc[1] = {w.s("region"), {}, 2, 0};
      b.n_spread_constraints = 2;
    } else if (x < 0.75) {
      sc[0] = {w.s("region"), {}, 3, 0};  // region only: no cluster MaxGroups
      b.n_spread_constraints = 1;
    } else if (x < 0.9) {
      sc[0] = {w.s("cluster"), {}, 8, 0};
      b.n_spread_constraints = 1;
    } else {
      sc[0] = {w.s("region"), {}, 3, 1};
      sc[1] = {w.s("cluster"), {}, 8, 3};
      b.n_spread_constraints = 2;
    }
    b.spread_constraints = sc;
    const double y = r.unit();
    if (y < 0.4) {
      b.replica_division_preference = w.s("Aggregated");
      b.has_weight_preference = 0;
      b.dynamic_weight = kp_str{nullptr, 0};
    } else if (y < 0.55) {
      b.replica_scheduling_type = w.s("Duplicated");
    } else if (y < 0.6) {
      b.replicas = 0;  // Replicas / MinGroups = 0 / 0: NaN
    }
  }
  // previous placement (20%) and eviction (5%)
  if (r.p(0.2) && C > 0) {
    int n = 1 + (int)r.below(std::min<uint32_t>(5, C));
    kp_target_cluster* tc = w.a.alloc<kp_target_cluster>(n);
    uint32_t c0 = (uint32_t)r.below(C);
    for (int k = 0; k < n; k++) tc[k] = {w.s(w.cname((c0 + 7 * k) % C)), (int32_t)r.range(0, b.replicas)};
    b.clusters = tc;
    b.n_clusters = n;
  }
  if (r.p(0.05) && C > 0) {
    kp_str* ev = w.a.alloc<kp_str>(1);
    ev[0] = w.s(w.cname((uint32_t)r.below(C)));
    b.eviction_from = ev;
    b.n_eviction_from = 1;
  }
  if (cfg == 8) {
    double x = r.unit();
    b.has_cluster_affinity = r.p(0.5) ? b.has_cluster_affinity : 0;
    if (x < 0.35) {
      // DynamicWeight
    } else if (x < 0.7) {
      b.replica_division_preference = w.s("Aggregated");
      b.has_weight_preference = 0;
      b.dynamic_weight = kp_str{nullptr, 0};
    } else if (x < 0.88) {  // StaticWeight, weights around and beyond 2^31
      b.dynamic_weight = kp_str{nullptr, 0};
      const int64_t kW[] = {1, 5, 2147483647, 2147483648ll, 3000000000ll, (int64_t)1 << 40};
      const int n = 1 + (int)r.below(3);
      kp_static_weight* sw = w.a.alloc<kp_static_weight>(n);
      for (int k = 0; k < n; k++) sw[k] = kp_static_weight{label_in(w, r, 2 + (int)r.below(5)), kW[r.below(6)]};
      b.static_weights = sw;
      b.n_static_weights = n;
    } else {
      b.replica_scheduling_type = w.s("Duplicated");
    }
    const double y = r.unit();
    b.replicas = y < 0.6 ? (int32_t)r.range(1, 1000000) : (y < 0.9 ? (int32_t)r.range(100000000, 2147483647)
                                                                      : (int32_t)r.range(1, 20));
    if (r.p(0.4) && C > 0) {  // previous placement: sums of spec.Clusters wrap
      int n = 1 + (int)r.below(std::min<uint32_t>(4, C));
      kp_target_cluster* tc = w.a.alloc<kp_target_cluster>(n);
      uint32_t c0 = (uint32_t)r.below(C);
      for (int k = 0; k < n; k++)
        tc[k] = {w.s(w.cname((c0 + 5 * k) % C)), (int32_t)(r.p(0.6) ? r.range(600000000, 2147483647) : r.range(0, 1000))};
      b.clusters = tc;
      b.n_clusters = n;
    } else {
      b.clusters = nullptr;
      b.n_clusters = 0;
    }
    if (r.p(0.1)) {
      b.has_reschedule_triggered_at = 1;
      b.has_last_scheduled_time = 1;
      b.reschedule_triggered_at_ns = 2000;
      b.last_scheduled_time_ns = 1000;
    }
    b.n_resource_request = 2;
    kp_resource* rq = w.a.alloc<kp_resource>(2);
    rq[0] = {w.s("cpu"), w.s(r.p(0.8) ? "1m" : "2")};
    rq[1] = {w.s("memory"), w.s(r.p(0.8) ? "1Ki" : "1Gi")};
    b.resource_request = rq;
    return;
  }
  if (cfg == 9) {
    gen_components(w, r, b, 4);
    const double x = r.unit();
    if (x < 0.7) one_cluster_spread(w, r, b);
    else if (x < 0.85) {
      kp_spread_constraint* sc = w.a.alloc<kp_spread_constraint>(1);
      sc[0] = {w.s("cluster"), {}, 3, 1};
      b.spread_constraints = sc;
      b.n_spread_constraints = 1;
    }
    const double y = r.unit();
    if (y < 0.25) {
      b.replica_scheduling_type = w.s("Duplicated");
    } else if (y < 0.55) {
      b.replica_division_preference = w.s("Aggregated");
      b.has_weight_preference = 0;
      b.dynamic_weight = kp_str{nullptr, 0};
    } else if (y < 0.6) {
      b.has_replica_scheduling = 0;
    }
    if (r.p(0.3)) b.replicas = 0;  // spec.Replicas is not set for most multi-template kinds
    if (r.p(0.2)) b.has_replica_requirements = 0;
    return;
  }
  if (cfg == 7) {
    b.replica_division_preference = w.s(r.p(0.8) ? "Aggregated" : "Weighted");
    if (r.p(0.7)) b.has_cluster_affinity = 0;  // keep most clusters feasible
    b.replicas = (int32_t)r.range(1, 400000);
    if (r.p(0.1)) {  // reschedule triggered: fresh with prior placement
      b.has_reschedule_triggered_at = 1;
      b.has_last_scheduled_time = 1;
      b.reschedule_triggered_at_ns = 2000;
      b.last_scheduled_time_ns = 1000;
    }
    if (b.n_clusters > 0)
      for (uint32_t k = 0; k < b.n_clusters; k++)
        const_cast<kp_target_cluster*>(b.clusters)[k].replicas = (int32_t)r.range(0, b.replicas / 4 + 1);
    return;
  }
  if (cfg != 6) return;
  // ---- edge workload: perturb everything the path branches on ----
  double x = r.unit();
  if (x < 0.06) {  // non-workload
    b.replicas = 0;
    b.has_replica_requirements = r.p(0.5);
  } else if (x < 0.10) {
    b.replicas = (int32_t)r.range(0, 3);
  } else if (x < 0.14) {
    gen_components(w, r, b, 3);
  }
  double y = r.unit();
  if (y < 0.15) {
    b.replica_scheduling_type = w.s("Duplicated");
  } else if (y < 0.35) {
    b.replica_division_preference = w.s("Aggregated");
  } else if (y < 0.55) {
    b.dynamic_weight = kp_str{nullptr, 0};  // StaticWeight
    if (r.p(0.5)) {
      int n = 1 + (int)r.below(4);
      kp_static_weight* sw = w.a.alloc<kp_static_weight>(n);
      for (int k = 0; k < n; k++) sw[k] = kp_static_weight{label_in(w, r, 1 + (int)r.below(3)), r.range(0, 5)};
      b.static_weights = sw;
      b.n_static_weights = n;
    } else if (r.p(0.3)) {
      b.has_weight_preference = 0;
    }
  } else if (y < 0.58) {
    b.replica_division_preference = w.s("Bogus");
  } else if (y < 0.60) {
    b.has_replica_scheduling = 0;
  }
  if (r.p(0.15)) {  // reschedule triggered
    b.has_reschedule_triggered_at = 1;
    b.has_last_scheduled_time = 1;
    b.reschedule_triggered_at_ns = 2000;
    b.last_scheduled_time_ns = r.p(0.7) ? 1000 : 3000;
  }
  if (r.p(0.25) && C > 0) {  // previous placement incl. scale-down / duplicates
    int n = 1 + (int)r.below(std::min<uint32_t>(12, C));
    kp_target_cluster* tc = w.a.alloc<kp_target_cluster>(n);
    for (int k = 0; k < n; k++)
      tc[k] = {w.s(w.cname((uint32_t)r.below(C))), (int32_t)r.range(0, std::max(1, b.replicas))};
    b.clusters = tc;
    b.n_clusters = n;
  }
  if (r.p(0.2)) {  // multi-term affinities with overflow
    b.has_cluster_affinity = 0;
    int nt = 1 + (int)r.below(3);
    kp_affinity_term* at = w.a.alloc<kp_affinity_term>(nt);
    for (int k = 0; k < nt; k++) {
      at[k].affinity_name = w.s("term-" + std::to_string(k));
      at[k].affinity = label_in(w, r, 1 + (int)r.below(3));
      int no = (int)r.below(3);
      kp_cluster_affinity* ov = w.a.alloc<kp_cluster_affinity>(no);
      for (int j = 0; j < no; j++) ov[j] = label_in(w, r, 1 + (int)r.below(4));
      at[k].overflow = ov;
      at[k].n_overflow = no;
    }
    b.cluster_affinities = at;
    b.n_cluster_affinities = nt;
    double z = r.unit();
    if (z < 0.8) b.observed_affinity_name = at[r.below(nt)].affinity_name;
    else if (z < 0.9) b.observed_affinity_name = w.s("missing");
  }
  if (r.p(0.1)) {  // cluster name lists / excludes
    kp_cluster_affinity a{};
    int n = 1 + (int)r.below(6);
    kp_str* ns = w.a.alloc<kp_str>(n);
    for (int k = 0; k < n; k++) ns[k] = w.s(w.cname((uint32_t)r.below(C + 2)));
    if (r.p(0.5)) {
      a.cluster_names = ns;
      a.n_cluster_names = n;
    } else {
      a.exclude_clusters = ns;
      a.n_exclude_clusters = n;
    }
    b.has_cluster_affinity = 1;
    b.cluster_affinity = a;
    b.n_cluster_affinities = 0;
  }
  if (b.n_components > 0 && r.p(0.6)) {
    one_cluster_spread(w, r, b);
  } else if (r.p(0.25)) {  // spread constraints
    double z = r.unit();
    kp_spread_constraint* sc = w.a.alloc<kp_spread_constraint>(2);
    if (z < 0.4) {
      sc[0] = {w.s("region"), {}, r.range(1, 4), r.range(0, 3)};
      sc[1] = {w.s("cluster"), {}, r.range(1, 12), r.range(0, 6)};
      b.n_spread_constraints = 2;
    } else if (z < 0.8) {
      sc[0] = {w.s("cluster"), {}, r.range(0, 12), r.range(0, 6)};
      b.n_spread_constraints = 1;
    } else {
      sc[0] = {w.s(r.p(0.5) ? "zone" : "provider"), {}, 2, 1};
      b.n_spread_constraints = 1;
    }
    b.spread_constraints = sc;
  }
  if (r.p(0.1)) {  // tolerate everything / nothing
    kp_toleration* t = w.a.alloc<kp_toleration>(1);
    t[0] = {kp_str{nullptr, 0}, w.s("Exists"), kp_str{nullptr, 0}, kp_str{nullptr, 0}};
    b.tolerations = t;
    b.n_tolerations = 1;
  }
  if (r.p(0.05)) b.n_resource_request = 0;
  // ReplicaRequirements.NodeClaim: the model path still answers (accurate.go:155-177,
  // scheduling_simulator_components.go:149-153)
  if (b.has_replica_requirements && r.p(0.15)) b.has_node_claim = 1;
}

}  // namespace

extern "C" {

// Generates clusters [0, n_clusters) and bindings [b_lo, b_hi) of the universe.
int kps_create(int config, uint64_t seed, uint32_t n_clusters, uint64_t b_lo, uint64_t b_hi, kps_world** out) {
  if (!out || b_hi < b_lo) return -1;
  auto* w = new kps_world();
  w->config = config;
  w->seed = seed;
  w->C = n_clusters;
  w->clusters.resize(n_clusters);
  for (uint32_t i = 0; i < n_clusters; i++) {
    memset(&w->clusters[i], 0, sizeof(kp_cluster));
    gen_cluster(*w, i, w->clusters[i]);
  }
  w->bindings.resize(b_hi - b_lo);
  for (uint64_t i = b_lo; i < b_hi; i++) {
    memset(&w->bindings[i - b_lo], 0, sizeof(kp_binding));
    gen_binding(*w, i, w->bindings[i - b_lo]);
  }
  *out = w;
  return 0;
}
void kps_destroy(kps_world* w) { delete w; }
const kp_cluster* kps_clusters(const kps_world* w, uint64_t* n) {
  *n = w->clusters.size();
  return w->clusters.data();
}
const kp_binding* kps_bindings(const kps_world* w, uint64_t* n) {
  *n = w->bindings.size();
  return w->bindings.data();
}

// spec.Replicas of bindings [b_lo, b_hi) (the §8(e) shard cost model), without
// keeping them: each binding is generated into a scratch world and dropped.
int kps_replicas(int config, uint64_t seed, uint32_t n_clusters, uint64_t b_lo, uint64_t b_hi, int32_t* out) {
  if (!out || b_hi < b_lo) return -1;
  kps_world w;
  w.config = config;
  w.seed = seed;
  w.C = n_clusters;
  for (uint64_t i = b_lo; i < b_hi; i++) {
    if (((i - b_lo) & 4095) == 0) w.a = Arena();  // release the previous chunk's strings
    kp_binding b;
    memset(&b, 0, sizeof(b));
    gen_binding(w, i, b);
    out[i - b_lo] = b.replicas;
  }
  return 0;
}

}  // extern "C"
