// oracle.cpp — CPU restatement of Karmada's genericScheduler.Schedule path.
//
// TEST INFRASTRUCTURE ONLY (see oracle.h). Every function cites the Go source it
// restates; paths are relative to /root/reference. Go semantics that matter for
// bit-exact parity are reproduced explicitly: int32 wrap-around, float64
// priorities, amd64 float->int conversion, Quantity rounding, container/heap and
// sort.Sort (pdqsort) behaviour. Where Go iterates a map and the result depends
// on the order only through a multiset (SURVEY.md hazard H1), a fixed order is
// used and results are compared as multisets.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace {

using std::string;
using std::vector;
typedef __int128 i128;
typedef int64_t i64;
typedef int32_t i32;

string S(const kp_str& s) { return (s.ptr && s.len) ? string(s.ptr, s.len) : string(); }

// int32 arithmetic with Go wrap-around semantics.
inline i32 add32(i32 a, i32 b) { return (i32)((uint32_t)a + (uint32_t)b); }
inline i32 sub32(i32 a, i32 b) { return (i32)((uint32_t)a - (uint32_t)b); }
inline i64 add64(i64 a, i64 b) { return (i64)((uint64_t)a + (uint64_t)b); }
inline i64 mul64(i64 a, i64 b) { return (i64)((uint64_t)a * (uint64_t)b); }

// ===========================================================================
// resource.Quantity (vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go)
// Exact value kept as a multiple of 1e-9 (ParseQuantity rounds to Nano,
// quantity.go:365-370) in a 128-bit integer.
// ===========================================================================
struct Quantity {
  i128 nano = 0;
  int fmt = 0;  // resource.Format: 0 DecimalSI, 1 BinarySI, 2 DecimalExponent (quantity.go:113-119)
};

i128 pow10_128(int k) {
  i128 r = 1;
  for (int i = 0; i < k; i++) r *= 10;
  return r;
}

// Value()/MilliValue(): "rounded up to the nearest integer away from 0"
// (quantity.go:813-835, math.go:166-199).
i64 scaled_away(i128 nano, i128 div) {
  if (nano >= 0) return (i64)((nano + div - 1) / div);
  return -(i64)(((-nano) + div - 1) / div);
}
inline i64 QValue(const Quantity& q) { return scaled_away(q.nano, (i128)1000000000); }
inline i64 QMilli(const Quantity& q) { return scaled_away(q.nano, (i128)1000000); }

const i128 kQMax = (i128)1 << 100;  // beyond this we refuse (never produced by real objects)

// ParseQuantity (quantity.go:161-394).
bool ParseQuantity(const string& str, Quantity* out) {
  if (str.empty()) return false;
  if (str == "0") {  // quantity.go: the "0" fast path is DecimalSI
    out->nano = 0;
    out->fmt = 0;
    return true;
  }
  bool positive = true;
  size_t pos = 0, end = str.size();
  string num, denom, suf;
  if (pos < end) {
    if (str[0] == '-') {
      positive = false;
      pos++;
    } else if (str[0] == '+') {
      pos++;
    }
  }
  // strip leading zeros
  bool done = false;
  for (size_t i = pos;; i++) {
    if (i >= end) {
      num = "0";
      done = true;
      break;
    }
    if (str[i] == '0') pos++;
    else break;
  }
  if (!done) {
    size_t i = pos;
    for (;; i++) {
      if (i >= end) {
        num = str.substr(pos, end - pos);
        done = true;
        break;
      }
      if (!(str[i] >= '0' && str[i] <= '9')) {
        num = str.substr(pos, i - pos);
        pos = i;
        break;
      }
    }
    if (!done) {
      if (num.empty()) num = "0";
      if (pos < end && str[pos] == '.') {
        pos++;
        size_t j = pos;
        for (;; j++) {
          if (j >= end) {
            denom = str.substr(pos, end - pos);
            done = true;
            break;
          }
          if (!(str[j] >= '0' && str[j] <= '9')) {
            denom = str.substr(pos, j - pos);
            pos = j;
            break;
          }
        }
      }
    } else if (num.empty()) {
      num = "0";
    }
    if (!done) {
      size_t suffixStart = pos;
      const char* sufchars = "eEinumkKMGTP";
      bool reached_end = false;
      for (size_t k = pos;; k++) {
        if (k >= end) {
          suf = str.substr(suffixStart);
          reached_end = true;
          break;
        }
        if (!strchr(sufchars, str[k])) {
          pos = k;
          break;
        }
      }
      if (!reached_end) {
        if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
        for (size_t k = pos;; k++) {
          if (k >= end) {
            suf = str.substr(suffixStart);
            break;
          }
          if (!(str[k] >= '0' && str[k] <= '9')) return false;  // ErrFormatWrong
        }
      }
    }
  }
  // quantitySuffixer.interpret (suffix.go)
  int base = 10;
  i64 exponent = 0;
  bool binary = false;
  int fmt = 0;
  static const std::map<string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0},  {"k", 3},
                                            {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  static const std::map<string, int> bin = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30},
                                            {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  auto d = dec.find(suf);
  if (d != dec.end()) {
    exponent = d->second;
  } else {
    auto b = bin.find(suf);
    if (b != bin.end()) {
      base = 2;
      exponent = b->second;
      binary = true;
      fmt = 1;
    } else if (suf.size() > 1 && (suf[0] == 'E' || suf[0] == 'e')) {
      // strconv.ParseInt(suffix[1:], 10, 64), then int32(parsed)
      const char* p = suf.c_str() + 1;
      char* endp = nullptr;
      errno = 0;
      long long v = strtoll(p, &endp, 10);
      if (errno != 0 || *endp != 0 || endp == p) return false;
      if (p[0] == ' ') return false;
      exponent = (i32)v;
      fmt = 2;
    } else {
      return false;  // ErrSuffix
    }
  }
  // value = num.denom * base^exponent, rounded away from zero to 1e-9.
  string digits = num + denom;
  i128 m = 0;
  for (char c : digits) {
    if (m > kQMax) return false;
    m = m * 10 + (c - '0');
  }
  i128 nano;
  if (base == 10) {
    i64 sc = 9 + exponent - (i64)denom.size();
    if (sc >= 0) {
      if (sc > 36) {
        if (m != 0) return false;
        nano = 0;
      } else {
        nano = m * pow10_128((int)sc);
        if (m != 0 && nano / pow10_128((int)sc) != m) return false;
      }
    } else {
      i64 k = -sc;
      if (k > 36) {
        nano = (m != 0) ? 1 : 0;
      } else {
        i128 div = pow10_128((int)k);
        nano = (m + div - 1) / div;  // round up magnitude
      }
    }
  } else {
    // binary: num.denom * 2^exp ; exact scale of denom then multiply
    i128 v = m;
    for (i64 i = 0; i < exponent; i++) {
      v *= 2;
      if (v > kQMax * 1000) return false;
    }
    i64 sc = 9 - (i64)denom.size();
    if (sc >= 0) {
      nano = v * pow10_128((int)sc);
    } else {
      i128 div = pow10_128((int)-sc);
      nano = (v + div - 1) / div;
    }
    // BinarySI cap at maxAllowed (quantity.go:373-376)
    i128 cap = (i128)INT64_MAX * 1000000000;
    if (nano > cap) nano = cap;
    (void)binary;
  }
  if (nano > kQMax) return false;
  out->nano = positive ? nano : -nano;
  out->fmt = fmt;
  return true;
}

// ===========================================================================
// Validation (vendor/k8s.io/apimachinery/pkg/api/validate/content/{kube,dns}.go)
// ===========================================================================
inline bool isAlnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
inline bool isLowerAlnum(char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }

// "(" + [A-Za-z0-9] + [-A-Za-z0-9_.]* ")?" + [A-Za-z0-9]
bool matchLabelKeyFmt(const string& s) {
  if (s.empty()) return false;
  if (!isAlnum(s.front()) || !isAlnum(s.back())) return false;
  for (char c : s)
    if (!(isAlnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
// dns1123SubdomainFmt: label(\.label)*, label = [a-z0-9]([-a-z0-9]*[a-z0-9])?
bool isDNS1123Subdomain(const string& s) {
  if (s.size() > 253) return false;
  if (s.empty()) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    string lab = s.substr(start, dot == string::npos ? string::npos : dot - start);
    if (lab.empty()) return false;
    if (!isLowerAlnum(lab.front()) || !isLowerAlnum(lab.back())) return false;
    for (char c : lab)
      if (!(isLowerAlnum(c) || c == '-')) return false;
    if (dot == string::npos) break;
    start = dot + 1;
  }
  return true;
}
// content.IsLabelKey (kube.go)
bool IsLabelKey(const string& v) {
  size_t slash = v.find('/');
  string name;
  if (slash == string::npos) {
    name = v;
  } else {
    if (v.find('/', slash + 1) != string::npos) return false;
    string prefix = v.substr(0, slash);
    name = v.substr(slash + 1);
    if (prefix.empty()) return false;
    if (!isDNS1123Subdomain(prefix)) return false;
  }
  if (name.empty() || name.size() > 63) return false;
  return matchLabelKeyFmt(name);
}
// content.IsLabelValue
bool IsLabelValue(const string& v) {
  if (v.size() > 63) return false;
  if (v.empty()) return true;
  return matchLabelKeyFmt(v);
}
// strconv.ParseInt(s, 10, 64)
bool ParseInt64(const string& s, i64* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c == '_') return false;
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (i64)(-(i128)v) : (i64)v;
  return true;
}

// ===========================================================================
// Object model (Go objects)
// ===========================================================================
typedef std::map<string, Quantity> ResourceList;
struct Taint {
  string key, value, effect;
};
struct Toleration {
  string key, op, value, effect;
};
struct Req {
  string key, op;
  vector<string> values;
};
struct Affinity {
  bool has_ls = false;
  std::map<string, string> match_labels;
  vector<Req> exprs;
  bool has_fs = false;
  vector<Req> fexprs;
  vector<string> names, exclude;
};
struct Term {
  string name;
  Affinity aff;
  vector<Affinity> overflow;
};
struct Spread {
  string field, label;
  i64 max = 0, min = 0;
};
struct StaticWeight {
  Affinity target;
  i64 weight = 0;
};
struct TargetCluster {
  string name;
  i32 replicas = 0;
};
struct RModelRange {
  string name;
  Quantity min, max;
};
struct RModel {
  uint32_t grade = 0;
  vector<RModelRange> ranges;
};
struct AllocModel {
  uint32_t grade = 0;
  i64 count = 0;
};
struct Cluster {
  int idx = -1;
  string name;
  bool deleting = false;
  std::map<string, string> labels;
  string provider, region, zone;
  vector<string> zones;
  vector<Taint> taints;
  vector<std::pair<string, string>> apis;
  vector<RModel> models;
  bool has_summary = false;
  ResourceList allocatable, allocated, allocating;
  vector<AllocModel> modelings;
};
struct Component {
  i32 replicas = 0;
  bool has_rr = false;
  ResourceList request;
};
// workv1alpha2.Component (binding_types.go:89-98): one pod template of a
// multi-template workload (Replicas + ReplicaRequirements.ResourceRequest).
struct Binding {
  string uid, api_version, kind, ns, name;
  i32 replicas = 0;
  bool has_rr = false, has_node_claim = false;
  ResourceList request;
  uint32_t n_components = 0;
  vector<Component> comps;  // spec.Components (empty when the caller passed counts only)
  vector<TargetCluster> clusters;
  vector<string> eviction;
  bool has_rta = false, has_lst = false;
  i64 rta = 0, lst = 0;
  string observed;
  bool has_ca = false;
  Affinity ca;
  vector<Term> cas;
  vector<Toleration> tolerations;
  vector<Spread> spreads;
  bool has_rs = false;
  string rs_type, rs_div;
  bool has_wp = false;
  vector<StaticWeight> sw;
  string dyn;
  bool bad = false;  // an input quantity failed to parse
};
struct Options {
  bool empty_workload_propagation = false;
  bool models_gate = true;
  bool multi_templates = false;  // MultiplePodTemplatesScheduling (features.go, alpha, default off)
  uint32_t plugins = KP_PLUGIN_ALL;
};

bool parseList(const kp_resource* r, uint32_t n, ResourceList* out) {
  bool ok = true;
  for (uint32_t i = 0; i < n; i++) {
    Quantity q;
    if (!ParseQuantity(S(r[i].quantity), &q)) ok = false;
    (*out)[S(r[i].name)] = q;
  }
  return ok;
}

Affinity convAffinity(const kp_cluster_affinity& a) {
  Affinity o;
  o.has_ls = a.has_label_selector;
  for (uint32_t i = 0; i < a.n_match_labels; i++) o.match_labels[S(a.match_labels[i].key)] = S(a.match_labels[i].value);
  auto conv = [](const kp_requirement* r, uint32_t n, vector<Req>* out) {
    for (uint32_t i = 0; i < n; i++) {
      Req q;
      q.key = S(r[i].key);
      q.op = S(r[i].op);
      for (uint32_t j = 0; j < r[i].n_values; j++) q.values.push_back(S(r[i].values[j]));
      out->push_back(q);
    }
  };
  conv(a.match_expressions, a.n_match_expressions, &o.exprs);
  o.has_fs = a.has_field_selector;
  conv(a.field_expressions, a.n_field_expressions, &o.fexprs);
  for (uint32_t i = 0; i < a.n_cluster_names; i++) o.names.push_back(S(a.cluster_names[i]));
  for (uint32_t i = 0; i < a.n_exclude_clusters; i++) o.exclude.push_back(S(a.exclude_clusters[i]));
  return o;
}

Cluster convCluster(const kp_cluster& c, int idx, bool* ok) {
  Cluster o;
  o.idx = idx;
  o.name = S(c.name);
  o.deleting = c.deleting;
  for (uint32_t i = 0; i < c.n_labels; i++) o.labels[S(c.labels[i].key)] = S(c.labels[i].value);
  o.provider = S(c.provider);
  o.region = S(c.region);
  o.zone = S(c.zone);
  for (uint32_t i = 0; i < c.n_zones; i++) o.zones.push_back(S(c.zones[i]));
  for (uint32_t i = 0; i < c.n_taints; i++) o.taints.push_back({S(c.taints[i].key), S(c.taints[i].value), S(c.taints[i].effect)});
  for (uint32_t i = 0; i < c.n_api_enablements; i++)
    o.apis.push_back({S(c.api_enablements[i].group_version), S(c.api_enablements[i].kind)});
  for (uint32_t i = 0; i < c.n_resource_models; i++) {
    RModel m;
    m.grade = c.resource_models[i].grade;
    for (uint32_t j = 0; j < c.resource_models[i].n_ranges; j++) {
      RModelRange r;
      r.name = S(c.resource_models[i].ranges[j].name);
      if (!ParseQuantity(S(c.resource_models[i].ranges[j].min), &r.min)) *ok = false;
      if (c.resource_models[i].ranges[j].max.len && !ParseQuantity(S(c.resource_models[i].ranges[j].max), &r.max)) *ok = false;
      m.ranges.push_back(r);
    }
    o.models.push_back(m);
  }
  o.has_summary = c.has_resource_summary;
  if (!parseList(c.allocatable, c.n_allocatable, &o.allocatable)) *ok = false;
  if (!parseList(c.allocated, c.n_allocated, &o.allocated)) *ok = false;
  if (!parseList(c.allocating, c.n_allocating, &o.allocating)) *ok = false;
  for (uint32_t i = 0; i < c.n_allocatable_modelings; i++)
    o.modelings.push_back({c.allocatable_modelings[i].grade, c.allocatable_modelings[i].count});
  return o;
}

Binding convBinding(const kp_binding& b) {
  Binding o;
  o.uid = S(b.uid);
  o.api_version = S(b.api_version);
  o.kind = S(b.kind);
  o.ns = S(b.namespace_);
  o.name = S(b.name);
  o.replicas = b.replicas;
  o.has_rr = b.has_replica_requirements;
  o.has_node_claim = b.has_node_claim;
  if (!parseList(b.resource_request, b.n_resource_request, &o.request)) o.bad = true;
  o.n_components = b.n_components;
  if (b.components)
    for (uint32_t i = 0; i < b.n_components; i++) {
      Component k;
      k.replicas = b.components[i].replicas;
      k.has_rr = b.components[i].has_replica_requirements != 0;
      if (!parseList(b.components[i].resource_request, b.components[i].n_resource_request, &k.request)) o.bad = true;
      o.comps.push_back(k);
    }
  for (uint32_t i = 0; i < b.n_clusters; i++) o.clusters.push_back({S(b.clusters[i].name), b.clusters[i].replicas});
  for (uint32_t i = 0; i < b.n_eviction_from; i++) o.eviction.push_back(S(b.eviction_from[i]));
  o.has_rta = b.has_reschedule_triggered_at;
  o.has_lst = b.has_last_scheduled_time;
  o.rta = b.reschedule_triggered_at_ns;
  o.lst = b.last_scheduled_time_ns;
  o.observed = S(b.observed_affinity_name);
  o.has_ca = b.has_cluster_affinity;
  if (o.has_ca) o.ca = convAffinity(b.cluster_affinity);
  for (uint32_t i = 0; i < b.n_cluster_affinities; i++) {
    Term t;
    t.name = S(b.cluster_affinities[i].affinity_name);
    t.aff = convAffinity(b.cluster_affinities[i].affinity);
    for (uint32_t j = 0; j < b.cluster_affinities[i].n_overflow; j++)
      t.overflow.push_back(convAffinity(b.cluster_affinities[i].overflow[j]));
    o.cas.push_back(t);
  }
  for (uint32_t i = 0; i < b.n_tolerations; i++)
    o.tolerations.push_back({S(b.tolerations[i].key), S(b.tolerations[i].op), S(b.tolerations[i].value), S(b.tolerations[i].effect)});
  for (uint32_t i = 0; i < b.n_spread_constraints; i++)
    o.spreads.push_back({S(b.spread_constraints[i].spread_by_field), S(b.spread_constraints[i].spread_by_label),
                         b.spread_constraints[i].max_groups, b.spread_constraints[i].min_groups});
  o.has_rs = b.has_replica_scheduling;
  o.rs_type = S(b.replica_scheduling_type);
  o.rs_div = S(b.replica_division_preference);
  o.has_wp = b.has_weight_preference;
  for (uint32_t i = 0; i < b.n_static_weights; i++)
    o.sw.push_back({convAffinity(b.static_weights[i].target), b.static_weights[i].weight});
  o.dyn = S(b.dynamic_weight);
  return o;
}

Options convOptions(const kp_options* o) {
  Options r;
  if (o) {
    r.empty_workload_propagation = o->enable_empty_workload_propagation;
    r.models_gate = o->customized_cluster_resource_modeling;
    r.multi_templates = o->multiple_pod_templates_scheduling;
    r.plugins = o->enabled_plugins;
  }
  return r;
}

// ===========================================================================
// Label selectors (vendor/k8s.io/apimachinery/pkg/labels/selector.go:150-300,
// pkg/apis/meta/v1/helpers.go:36-74; pkg/util/lifted/nodeaffinity.go:36-71)
// ===========================================================================
struct Requirement {
  string key, op;  // op in {In, NotIn, Exists, DoesNotExist, Gt, Lt}; Equals folded into In
  vector<string> values;
};
typedef std::map<string, string> LabelSet;

// labels.NewRequirement validation (selector.go:150-230)
bool NewRequirement(const string& key, const string& op, const vector<string>& vals) {
  bool ok = IsLabelKey(key);
  if (op == "In" || op == "NotIn") {
    if (vals.empty()) ok = false;
  } else if (op == "=" || op == "==" || op == "!=") {
    if (vals.size() != 1) ok = false;
  } else if (op == "Exists" || op == "DoesNotExist") {
    if (!vals.empty()) ok = false;
  } else if (op == "Gt" || op == "Lt") {
    if (vals.size() != 1) ok = false;
    for (auto& v : vals) {
      i64 x;
      if (!ParseInt64(v, &x)) ok = false;
    }
  } else {
    ok = false;
  }
  for (auto& v : vals)
    if (!IsLabelValue(v)) ok = false;
  return ok;
}

// Requirement.Matches (selector.go:247-292)
bool ReqMatches(const Requirement& r, const LabelSet& ls) {
  auto it = ls.find(r.key);
  bool exists = it != ls.end();
  auto has = [&](const string& v) {
    for (auto& x : r.values)
      if (x == v) return true;
    return false;
  };
  if (r.op == "In" || r.op == "=" || r.op == "==") {
    if (!exists) return false;
    return has(it->second);
  }
  if (r.op == "NotIn" || r.op == "!=") {
    if (!exists) return true;
    return !has(it->second);
  }
  if (r.op == "Exists") return exists;
  if (r.op == "DoesNotExist") return !exists;
  if (r.op == "Gt" || r.op == "Lt") {
    if (!exists) return false;
    i64 lv;
    if (!ParseInt64(it->second, &lv)) return false;
    if (r.values.size() != 1) return false;
    i64 rv;
    if (!ParseInt64(r.values[0], &rv)) return false;
    return (r.op == "Gt" && lv > rv) || (r.op == "Lt" && lv < rv);
  }
  return false;
}

// metav1.LabelSelectorAsSelector; returns false on error. `everything` set
// when the selector has no requirements.
bool LabelSelectorAsSelector(const Affinity& a, vector<Requirement>* reqs) {
  for (auto& kv : a.match_labels) {
    if (!NewRequirement(kv.first, "=", {kv.second})) return false;
    reqs->push_back({kv.first, "=", {kv.second}});
  }
  for (auto& e : a.exprs) {
    string op;
    if (e.op == "In") op = "In";
    else if (e.op == "NotIn") op = "NotIn";
    else if (e.op == "Exists") op = "Exists";
    else if (e.op == "DoesNotExist") op = "DoesNotExist";
    else return false;
    if (!NewRequirement(e.key, op, e.values)) return false;
    reqs->push_back({e.key, op, e.values});
  }
  return true;
}

// lifted.NodeSelectorRequirementsAsSelector (nodeaffinity.go:36-71)
bool NodeSelectorRequirementsAsSelector(const vector<Req>& nsm, vector<Requirement>* reqs) {
  bool ok = true;
  for (auto& e : nsm) {
    string op;
    if (e.op == "In") op = "In";
    else if (e.op == "NotIn") op = "NotIn";
    else if (e.op == "Exists") op = "Exists";
    else if (e.op == "DoesNotExist") op = "DoesNotExist";
    else if (e.op == "Gt") op = "Gt";
    else if (e.op == "Lt") op = "Lt";
    else {
      ok = false;
      continue;
    }
    if (!NewRequirement(e.key, op, e.values)) ok = false;
    reqs->push_back({e.key, op, e.values});
  }
  return ok;
}

// util.matchZones (pkg/util/selector.go:208-235)
bool matchZones(const Req& e, const vector<string>& zones) {
  auto contains = [&](const string& z) {
    for (auto& v : e.values)
      if (v == z) return true;
    return false;
  };
  if (e.op == "In") {
    if (zones.empty()) return false;
    for (auto& z : zones)
      if (contains(z)) return true;
    return false;
  }
  if (e.op == "NotIn") {
    for (auto& z : zones)
      if (contains(z)) return false;
    return true;
  }
  if (e.op == "Exists") return !zones.empty();
  if (e.op == "DoesNotExist") return zones.empty();
  return false;
}

// util.ClusterMatches (pkg/util/selector.go:97-155)
bool ClusterMatches(const Cluster& c, const Affinity& a) {
  for (auto& x : a.exclude)
    if (x == c.name) return false;
  if (a.has_ls) {
    vector<Requirement> reqs;  // compiled per call, as the reference does (selector.go:116)
    if (!LabelSelectorAsSelector(a, &reqs)) return false;
    for (auto& r : reqs)
      if (!ReqMatches(r, c.labels)) return false;
  }
  if (a.has_fs) {
    vector<Req> others;
    for (auto& e : a.fexprs) {
      if (e.key != "zone") {
        others.push_back(e);
        continue;
      }
      if (!matchZones(e, c.zones)) return false;
    }
    if (!others.empty()) {
      vector<Requirement> reqs;
      if (!NodeSelectorRequirementsAsSelector(others, &reqs)) return false;
      LabelSet fields;  // extractClusterFields (selector.go:193-205)
      if (!c.provider.empty()) fields["provider"] = c.provider;
      if (!c.region.empty()) fields["region"] = c.region;
      for (auto& r : reqs)
        if (!ReqMatches(r, fields)) return false;
    }
  }
  if (a.names.empty()) return true;
  for (auto& n : a.names)
    if (n == c.name) return true;
  return false;
}

// ===========================================================================
// Binding helpers (pkg/apis/work/v1alpha2/binding_types_helper.go, pkg/util/binding.go)
// ===========================================================================
bool TargetContains(const Binding& b, const string& name) {
  for (auto& t : b.clusters)
    if (t.name == name) return true;
  return false;
}
i32 AssignedReplicasForCluster(const Binding& b, const string& name) {
  for (auto& t : b.clusters)
    if (t.name == name) return t.replicas;
  return 0;
}
bool IsWorkload(const Binding& b) { return b.replicas > 0 || b.has_rr || b.n_components >= 1; }
i32 GetSumOfReplicas(const vector<TargetCluster>& v) {
  i32 s = 0;
  for (auto& t : v) s = add32(s, t.replicas);
  return s;
}
bool RescheduleRequired(const Binding& b) {
  if (!b.has_rta) return false;
  if (!b.has_lst) return false;
  return b.rta > b.lst;
}
// util.MergeTargetClusters (pkg/util/binding.go:91-115)
vector<TargetCluster> MergeTargetClusters(const vector<TargetCluster>& oldc, vector<TargetCluster> newc) {
  if (oldc.empty()) return newc;
  if (newc.empty()) return oldc;
  std::map<string, i32> oldMap;
  vector<string> order;
  for (auto& c : oldc) {
    if (!oldMap.count(c.name)) order.push_back(c.name);
    oldMap[c.name] = c.replicas;
  }
  for (auto& c : newc) {
    auto it = oldMap.find(c.name);
    if (it != oldMap.end()) {
      c.replicas = add32(c.replicas, it->second);
      oldMap.erase(it);
    }
  }
  for (auto& n : order) {  // map order in Go (hazard H1): multiset-equivalent
    auto it = oldMap.find(n);
    if (it != oldMap.end()) newc.push_back({n, it->second});
  }
  return newc;
}

// ===========================================================================
// Filter / score plugins (pkg/scheduler/framework/plugins/*)
// ===========================================================================
// schema.FromAPIVersionAndKind + GroupVersion().String() (group_version.go:211-226,300-305)
string GroupVersionString(const string& apiVersion) {
  string group, version;
  if (apiVersion.empty() || apiVersion == "/") {
  } else {
    size_t n = std::count(apiVersion.begin(), apiVersion.end(), '/');
    if (n == 0) {
      version = apiVersion;
    } else if (n == 1) {
      size_t i = apiVersion.find('/');
      group = apiVersion.substr(0, i);
      version = apiVersion.substr(i + 1);
    }
  }
  if (!group.empty()) return group + "/" + version;
  return version;
}

// apienablement.Filter (api_enablement.go:51-78) + Cluster.APIEnablement (cluster_helper.go:46-67)
bool FilterAPIEnablement(const Binding& b, const Cluster& c) {
  if (TargetContains(b, c.name)) return true;
  string gv = GroupVersionString(b.api_version);
  for (auto& p : c.apis)
    if (p.first == gv && p.second == b.kind) return true;
  return false;  // APIDisabled or APIUnknown
}

// Toleration.ToleratesTaint with comparison operators disabled (toleration.go:52-77)
bool ToleratesTaint(const Toleration& t, const Taint& taint) {
  if (!t.effect.empty() && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
  if (t.op == "Exists") return true;
  return false;  // Lt/Gt disabled (enableComparisonOperators=false), unknown ops
}

// tainttoleration.Filter (taint_toleration.go:53-84) + FindMatchingUntoleratedTaint (helpers.go:79-102)
bool FilterTaintToleration(const Binding& b, const Cluster& c) {
  if (TargetContains(b, c.name)) return true;
  for (auto& taint : c.taints) {
    if (!(taint.effect == "NoSchedule" || taint.effect == "NoExecute")) continue;
    bool tol = false;
    for (auto& t : b.tolerations)
      if (ToleratesTaint(t, taint)) {
        tol = true;
        break;
      }
    if (!tol) return false;
  }
  return true;
}

// clusteraffinity.Filter (cluster_affinity.go:51-94)
bool FilterClusterAffinity(const Binding& b, const Cluster& c) {
  vector<const Affinity*> affinities;
  if (b.has_ca) {
    affinities.push_back(&b.ca);
  } else {
    for (auto& term : b.cas) {
      if (term.name != b.observed) continue;
      affinities.push_back(&term.aff);
      if (IsWorkload(b))
        for (auto& o : term.overflow) affinities.push_back(&o);
      break;
    }
  }
  if (!affinities.empty()) {
    for (auto* a : affinities)
      if (ClusterMatches(c, *a)) return true;
    return false;
  }
  return true;
}

// spreadconstraint.Filter (spread_constraint.go:49-66)
bool FilterSpreadConstraint(const Binding& b, const Cluster& c) {
  for (auto& sc : b.spreads) {
    if (sc.field == "provider" && c.provider.empty()) return false;
    else if (sc.field == "region" && c.region.empty()) return false;
    else if (sc.field == "zone" && c.zones.empty()) return false;
  }
  return true;
}

// clustereviction.Filter (cluster_eviction.go:50-57)
bool FilterClusterEviction(const Binding& b, const Cluster& c) {
  for (auto& e : b.eviction)
    if (e == c.name) return false;
  return true;
}

// RunFilterPlugins (runtime/framework.go:93-105); canonical order (hazard H1).
uint32_t RunFilterPlugins(const Binding& b, const Cluster& c, const Options& o) {
  if ((o.plugins & KP_PLUGIN_API_ENABLEMENT) && !FilterAPIEnablement(b, c)) return KP_PLUGIN_API_ENABLEMENT;
  if ((o.plugins & KP_PLUGIN_TAINT_TOLERATION) && !FilterTaintToleration(b, c)) return KP_PLUGIN_TAINT_TOLERATION;
  if ((o.plugins & KP_PLUGIN_CLUSTER_AFFINITY) && !FilterClusterAffinity(b, c)) return KP_PLUGIN_CLUSTER_AFFINITY;
  if ((o.plugins & KP_PLUGIN_SPREAD_CONSTRAINT) && !FilterSpreadConstraint(b, c)) return KP_PLUGIN_SPREAD_CONSTRAINT;
  if ((o.plugins & KP_PLUGIN_CLUSTER_EVICTION) && !FilterClusterEviction(b, c)) return KP_PLUGIN_CLUSTER_EVICTION;
  return 0;
}

// The Result of RunFilterPlugins as a kp_filter_reasons word (KP_REASON_* | arg << 8):
// findClustersThatFit's skip of deleting clusters (generic_scheduler.go:138-142), then
// the first failing plugin's reason (api_enablement.go:77, taint_toleration.go:83 with
// the FindMatchingUntoleratedTaint taint among the NoSchedule/NoExecute ones,
// cluster_affinity.go:89, spread_constraint.go:55-62 per constraint in spec order,
// cluster_eviction.go:53).
uint32_t RunFilterPluginsReason(const Binding& b, const Cluster& c, const Options& o) {
  if (c.deleting) return 255;
  if ((o.plugins & KP_PLUGIN_API_ENABLEMENT) && !FilterAPIEnablement(b, c)) return 1;
  if ((o.plugins & KP_PLUGIN_TAINT_TOLERATION) && !TargetContains(b, c.name)) {
    uint32_t k = 0;
    for (auto& taint : c.taints) {
      if (!(taint.effect == "NoSchedule" || taint.effect == "NoExecute")) continue;
      bool tol = false;
      for (auto& t : b.tolerations) tol = tol || ToleratesTaint(t, taint);
      if (!tol) return 2u | k << 8;
      k++;
    }
  }
  if ((o.plugins & KP_PLUGIN_CLUSTER_AFFINITY) && !FilterClusterAffinity(b, c)) return 3;
  if (o.plugins & KP_PLUGIN_SPREAD_CONSTRAINT) {
    for (auto& sc : b.spreads) {
      if (sc.field == "provider" && c.provider.empty()) return 4;
      if (sc.field == "region" && c.region.empty()) return 5;
      if (sc.field == "zone" && c.zones.empty()) return 6;
    }
  }
  if ((o.plugins & KP_PLUGIN_CLUSTER_EVICTION) && !FilterClusterEviction(b, c)) return 7;
  return 0;
}

// RunScorePlugins summed (framework.go:126-170, generic_scheduler.go:185-191):
// ClusterLocality (cluster_locality.go:50-61) + ClusterAffinity = 0 (cluster_affinity.go:97-100)
i64 ScoreCluster(const Binding& b, const Cluster& c, const Options& o) {
  i64 s = 0;
  if (o.plugins & KP_PLUGIN_CLUSTER_LOCALITY) {
    if (!b.clusters.empty() && TargetContains(b, c.name)) s += 100;
  }
  return s;
}

// ===========================================================================
// GeneralEstimator (pkg/estimator/client/general.go)
// ===========================================================================
const i64 kMaxPodsPerNode = 110;  // general.go:41

// lifted.IsScalarResourceName (pkg/util/lifted/resourcename.go:31-34, corev1helpers.go:39-82)
bool IsNativeResource(const string& n) {
  return n.find('/') == string::npos || n.find("kubernetes.io/") != string::npos;
}
bool IsExtendedResourceName(const string& n) {
  if (IsNativeResource(n) || n.rfind("requests.", 0) == 0) return false;
  return IsLabelKey("requests." + n);  // IsQualifiedName == IsLabelKey
}
bool IsScalarResourceName(const string& n) {
  return IsExtendedResourceName(n) || n.rfind("hugepages-", 0) == 0 ||
         n.find("kubernetes.io/") != string::npos || n.rfind("attachable-volumes-", 0) == 0;
}

// util.Resource (pkg/util/resource.go:30-248)
struct Resource {
  i64 MilliCPU = 0, Memory = 0, EphemeralStorage = 0, AllowedPodNumber = 0;
  std::map<string, i64> Scalar;
  void Add(const ResourceList& rl) {
    for (auto& kv : rl) {
      const string& n = kv.first;
      if (n == "cpu") MilliCPU = add64(MilliCPU, QMilli(kv.second));
      else if (n == "memory") Memory = add64(Memory, QValue(kv.second));
      else if (n == "pods") AllowedPodNumber = add64(AllowedPodNumber, QValue(kv.second));
      else if (n == "ephemeral-storage") EphemeralStorage = add64(EphemeralStorage, QValue(kv.second));
      else if (IsScalarResourceName(n)) Scalar[n] = add64(Scalar[n], QValue(kv.second));
    }
  }
  // MaxDivided over the ResourceList() of a request resource (resource.go:191-220)
  i64 MaxDivided(const Resource& req) const {
    i64 res = INT64_MAX;
    if (req.MilliCPU > 0) res = std::min(res, MilliCPU / req.MilliCPU);
    if (req.Memory > 0) res = std::min(res, Memory / req.Memory);
    if (req.EphemeralStorage > 0) res = std::min(res, EphemeralStorage / req.EphemeralStorage);
    for (auto& kv : req.Scalar) {
      if (kv.second <= 0) continue;
      if (!IsScalarResourceName(kv.first)) continue;
      auto it = Scalar.find(kv.first);
      i64 have = it == Scalar.end() ? 0 : it->second;
      res = std::min(res, have / kv.second);
    }
    res = std::min(res, AllowedPodNumber);
    return res;
  }
  // SubResource (resource.go:96-115): clamp at zero
  void Sub(const Resource& rr) {
    MilliCPU = std::max<i64>(MilliCPU - rr.MilliCPU, 0);
    Memory = std::max<i64>(Memory - rr.Memory, 0);
    EphemeralStorage = std::max<i64>(EphemeralStorage - rr.EphemeralStorage, 0);
    AllowedPodNumber = std::max<i64>(AllowedPodNumber - rr.AllowedPodNumber, 0);
    for (auto& kv : rr.Scalar) {
      auto it = Scalar.find(kv.first);
      if (it != Scalar.end()) it->second = std::max<i64>(it->second - kv.second, 0);
    }
  }
};

// getAllowedPodNumber (general.go:445-463)
i64 getAllowedPodNumber(const Cluster& c) {
  i64 a = 0, b = 0, d = 0;
  auto pods = [](const ResourceList& rl) -> i64 {
    auto it = rl.find("pods");
    return it == rl.end() ? 0 : QValue(it->second);
  };
  a = pods(c.allocatable);
  b = pods(c.allocated);
  d = pods(c.allocating);
  i64 allowed = a - b - d;
  if (allowed <= 0) return 0;
  return allowed;
}

// getMaximumReplicasBasedOnClusterSummary (general.go:465-505)
i64 getMaximumReplicasBasedOnClusterSummary(const Cluster& c, const ResourceList& req) {
  i64 maximum = INT64_MAX;
  for (auto& kv : req) {
    i64 requested = QValue(kv.second);
    if (requested <= 0) continue;
    auto al = c.allocatable.find(kv.first);
    if (al == c.allocatable.end()) return 0;
    Quantity avail = al->second;
    auto ad = c.allocated.find(kv.first);
    if (ad != c.allocated.end()) avail.nano -= ad->second.nano;
    auto ag = c.allocating.find(kv.first);
    if (ag != c.allocating.end()) avail.nano -= ag->second.nano;
    i64 availableQuantity = QValue(avail);
    if (availableQuantity <= 0) return 0;
    if (kv.first == "cpu") {
      requested = QMilli(kv.second);
      availableQuantity = QMilli(avail);
    }
    i64 m = availableQuantity / requested;
    if (m < maximum) maximum = m;
  }
  return maximum;
}

// buildModelNodes (general.go:296-361): returns false on error.
struct ModelNode {
  Resource alloc;
};
bool buildModelNodes(const Cluster& c, vector<std::pair<Resource, i64>>* groups) {
  if (!c.has_summary) return false;
  if (c.models.empty()) return false;
  std::map<uint32_t, ResourceList> caps;
  for (auto& m : c.models) {
    ResourceList tmpl;
    for (auto& r : m.ranges) tmpl[r.name] = r.min;
    Quantity pods;
    pods.nano = (i128)kMaxPodsPerNode * 1000000000;
    tmpl["pods"] = pods;
    caps[m.grade] = tmpl;
  }
  std::map<uint32_t, i64> counts;
  for (auto& a : c.modelings) {
    if (a.count < 0) return false;
    counts[a.grade] += a.count;
  }
  for (auto& kv : caps) {  // grades ascending (sort.Ints)
    auto it = counts.find(kv.first);
    i64 cnt = it == counts.end() ? 0 : it->second;
    if (cnt == 0) continue;
    Resource r;
    r.Add(kv.second);
    groups->push_back({r, cnt});
  }
  return true;
}

// getMaximumReplicasBasedOnResourceModels (general.go:507-553) with the
// SchedulingSimulator (scheduling_simulator_components.go:51-130).
bool getMaximumReplicasBasedOnResourceModels(const Cluster& c, const Binding& b, int mode, i64* out) {
  vector<std::pair<Resource, i64>> groups;
  if (!buildModelNodes(c, &groups)) return false;
  Resource req;
  req.Add(b.request);
  req.AllowedPodNumber = 1;  // requiredPerReplica.AllowedPodNumber = 1
  // ResourceList() keeps only positive fields; MaxDivided ignores the rest.
  Resource reqPos;
  reqPos.MilliCPU = req.MilliCPU > 0 ? req.MilliCPU : 0;
  reqPos.Memory = req.Memory > 0 ? req.Memory : 0;
  reqPos.EphemeralStorage = req.EphemeralStorage > 0 ? req.EphemeralStorage : 0;
  reqPos.AllowedPodNumber = 1;
  for (auto& kv : req.Scalar)
    if (kv.second > 0) reqPos.Scalar[kv.first] = kv.second;
  if (mode == KPO_FAITHFUL) {
    // Literal first-fit loop: one complete set (1 replica) per iteration,
    // scanning nodes from the first one, until no node fits or MaxInt32.
    vector<Resource> nodes;
    for (auto& g : groups)
      for (i64 i = 0; i < g.second; i++) nodes.push_back(g.first);
    i32 complete = 0;
    while (complete < INT32_MAX) {
      bool placed = false;
      for (auto& n : nodes) {
        i64 alloc = n.MaxDivided(reqPos);
        if (alloc == 0) continue;
        if (alloc > 1) alloc = 1;
        Resource sub = reqPos;
        sub.MilliCPU *= alloc;
        sub.Memory *= alloc;
        sub.EphemeralStorage *= alloc;
        sub.AllowedPodNumber *= alloc;
        for (auto& kv : sub.Scalar) kv.second *= alloc;
        n.Sub(sub);
        placed = true;
        break;
      }
      if (!placed) break;
      complete++;
    }
    *out = complete;
  } else {
    // Closed form: each identical node absorbs exactly
    // its initial MaxDivided; total capped by the MaxInt32 upper bound.
    i128 total = 0;
    for (auto& g : groups) total += (i128)g.first.MaxDivided(reqPos) * g.second;
    if (total > INT32_MAX) total = INT32_MAX;
    *out = (i64)total;
  }
  return true;
}

// GeneralEstimator.maxAvailableReplicas (general.go:66-108), assumed workloads empty.
i32 maxAvailableReplicas(const Cluster& c, const Binding& b, const Options& o, int mode) {
  if (!c.has_summary) return 0;
  i64 maximum = getAllowedPodNumber(c);
  if (maximum <= 0) return 0;
  if (!b.has_rr) return (i32)maximum;
  // A NodeClaim does not divert the model path: toPBReplicaRequirements converts
  // it without error (accurate.go:155-177) and MatchNode accepts every model node,
  // which carries no Node object (scheduling_simulator_components.go:149-153).
  if (o.models_gate && !c.modelings.empty()) {
    i64 num;
    if (getMaximumReplicasBasedOnResourceModels(c, b, mode, &num)) {
      if (num < maximum) maximum = num;
      return (i32)maximum;
    }
  }
  i64 num = getMaximumReplicasBasedOnClusterSummary(c, b.request);
  if (num < maximum) maximum = num;
  return (i32)maximum;
}

// ===========================================================================
// GeneralEstimator.MaxAvailableComponentSets (general.go:154-292), assumed
// workloads empty (SchedulingOvercommitProtection off).
// ===========================================================================

// quantityAsInt64 (general.go:417-427): DecimalSI / DecimalExponent -> MilliValue,
// BinarySI -> Value.
i64 quantityAsInt64(const Quantity& q) { return q.fmt == 1 ? QValue(q) : QMilli(q); }
// Quantity.Sub: a zero receiver takes the subtrahend's format (quantity.go Sub).
void QSub(Quantity& a, const Quantity& y) {
  if (a.nano == 0) a.fmt = y.fmt;
  a.nano -= y.nano;
}
i64 wrapmul(i64 a, i64 b) { return (i64)((uint64_t)a * (uint64_t)b); }
i32 toI32(i64 v) { return (i32)(uint32_t)(uint64_t)v; }  // int32(x) of an int64

// util.Resource of a per-replica request (requiredPerReplica, AllowedPodNumber = 1)
// and the positive part MaxDivided reads (Resource.ResourceList keeps fields > 0).
void replicaRequest(const Component& k, Resource* req, Resource* pos) {
  *req = Resource();
  if (k.has_rr) req->Add(k.request);
  req->AllowedPodNumber = 1;
  *pos = Resource();
  pos->MilliCPU = req->MilliCPU > 0 ? req->MilliCPU : 0;
  pos->Memory = req->Memory > 0 ? req->Memory : 0;
  pos->EphemeralStorage = req->EphemeralStorage > 0 ? req->EphemeralStorage : 0;
  pos->AllowedPodNumber = 1;
  for (auto& kv : req->Scalar)
    if (kv.second > 0) pos->Scalar[kv.first] = kv.second;
}
Resource scaled(const Resource& r, i64 f) {  // Clone().Multiply(f) (resource.go:77-93)
  Resource o = r;
  o.MilliCPU = wrapmul(o.MilliCPU, f);
  o.Memory = wrapmul(o.Memory, f);
  o.EphemeralStorage = wrapmul(o.EphemeralStorage, f);
  o.AllowedPodNumber = wrapmul(o.AllowedPodNumber, f);
  for (auto& kv : o.Scalar) kv.second = wrapmul(kv.second, f);
  return o;
}

// SchedulingSimulator.SimulateScheduling (scheduling_simulator_components.go:51-131)
// over the model nodes of `groups`, literally: every node, every set, first fit.
i32 simulateFF(const vector<std::pair<Resource, i64>>& groups, const vector<Component>& comps, i32 upper) {
  vector<Resource> nodes;
  for (auto& g : groups)
    for (i64 i = 0; i < g.second; i++) nodes.push_back(g.first);
  vector<Resource> req(comps.size()), pos(comps.size());
  for (size_t k = 0; k < comps.size(); k++) replicaRequest(comps[k], &req[k], &pos[k]);
  i32 complete = 0;
  while (complete < upper) {
    bool ok = true;
    for (size_t k = 0; k < comps.size() && ok; k++) {  // scheduleComponentSet
      i32 remaining = comps[k].replicas;
      bool done = false;
      for (auto& n : nodes) {  // scheduleComponent
        i64 alloc = n.MaxDivided(pos[k]);
        if (alloc == 0) continue;
        if ((i64)remaining < alloc) alloc = remaining;
        n.Sub(scaled(req[k], alloc));
        remaining -= (i32)alloc;
        if (remaining == 0) {
          done = true;
          break;
        }
      }
      if (!done && remaining != 0) ok = false;
    }
    if (!ok) break;
    complete++;
  }
  return complete;
}

// The same simulation over runs of identical nodes (the engine's device form):
// identical consecutive nodes absorb the same amount, so a run of cnt nodes that
// each take m replicas is one step, and a partial fill splits a run into at most
// three. Runs before ptr[k] can no longer hold component k (capacity only drops),
// so each component's scan resumes there. Same answer as simulateFF.
i32 simulateRuns(const vector<std::pair<Resource, i64>>& groups, const vector<Component>& comps, i32 upper) {
  struct Run {
    Resource cap;
    i64 cnt;
  };
  vector<Run> runs;
  for (auto& g : groups)
    if (g.second > 0) runs.push_back({g.first, g.second});
  const size_t K = comps.size();
  vector<Resource> req(K), pos(K);
  for (size_t k = 0; k < K; k++) replicaRequest(comps[k], &req[k], &pos[k]);
  vector<size_t> ptr(K, 0);
  i32 complete = 0;
  while (complete < upper) {
    bool ok = true;
    for (size_t k = 0; k < K && ok; k++) {
      i64 rem = comps[k].replicas;
      if (rem == 0) continue;  // succeeds at the first node that fits or at the end
      bool lead = true;
      size_t i = ptr[k];
      for (; i < runs.size() && rem > 0; i++) {
        const i64 m = runs[i].cap.MaxDivided(pos[k]);
        if (m <= 0) {
          if (lead) ptr[k] = i + 1;
          continue;
        }
        lead = false;
        const i128 all = (i128)m * runs[i].cnt;
        if ((i128)rem >= all) {
          runs[i].cap.Sub(scaled(req[k], m));
          rem -= (i64)all;
          continue;
        }
        const i64 q = rem / m, r = rem % m, rest = runs[i].cnt - q - (r > 0 ? 1 : 0);
        vector<Run> parts;
        if (q > 0) {
          Run a = runs[i];
          a.cap.Sub(scaled(req[k], m));
          a.cnt = q;
          parts.push_back(a);
        }
        if (r > 0) {
          Run b = runs[i];
          b.cap.Sub(scaled(req[k], r));
          b.cnt = 1;
          parts.push_back(b);
        }
        if (rest > 0) {
          Run c = runs[i];
          c.cnt = rest;
          parts.push_back(c);
        }
        const size_t add = parts.size() - 1;
        runs.erase(runs.begin() + i);
        runs.insert(runs.begin() + i, parts.begin(), parts.end());
        for (size_t j = 0; j < K; j++)
          if (j != k && ptr[j] > i) ptr[j] += add;
        rem = 0;
      }
      if (rem > 0) ok = false;
    }
    if (!ok) break;
    complete++;
  }
  return complete;
}

// maxAvailableComponentSets (general.go:163-199) with resourceBoundedSets,
// applyResourceModelBound and getMaximumSetsBasedOnResourceModels (:218-292).
i32 maxAvailableComponentSets(const Cluster& c, const vector<Component>& comps, const Options& o, int mode) {
  if (!c.has_summary) return 0;
  std::map<string, i64> available;  // availableResourceMap (general.go:403-415)
  for (auto& kv : c.allocatable) {
    Quantity a = kv.second;
    auto ad = c.allocated.find(kv.first);
    if (ad != c.allocated.end()) QSub(a, ad->second);
    auto ag = c.allocating.find(kv.first);
    if (ag != c.allocating.end()) QSub(a, ag->second);
    available[kv.first] = quantityAsInt64(a);
  }
  const i64 allowedPods = getAllowedPodNumber(c);
  if (allowedPods <= 0) return 0;
  i64 podsPerSet = 0;  // podsInSet
  for (auto& k : comps) podsPerSet += (i64)k.replicas;
  if (podsPerSet <= 0) return toI32(allowedPods);
  const i32 podBound = toI32(allowedPods / podsPerSet);
  std::map<string, i64> perSet;  // perSetRequirement
  for (auto& k : comps) {
    if (!k.has_rr) continue;
    for (auto& kv : k.request) perSet[kv.first] = (i64)((uint64_t)perSet[kv.first] + (uint64_t)wrapmul(quantityAsInt64(kv.second), k.replicas));
  }
  i32 maxSets = podBound;  // resourceBoundedSets
  bool allZero = true;
  for (auto& kv : perSet) allZero = allZero && kv.second == 0;
  if (!perSet.empty() && !allZero) {
    for (auto& kv : perSet) {
      if (kv.second <= 0) continue;
      auto it = available.find(kv.first);
      const i64 av = it == available.end() ? 0 : it->second;
      if (av <= 0) return 0;
      const i32 rb = toI32(av / kv.second);
      if (rb < maxSets) maxSets = rb;
    }
  }
  // applyResourceModelBound
  if (!o.models_gate || c.modelings.empty()) return maxSets;
  vector<std::pair<Resource, i64>> groups;
  if (!buildModelNodes(c, &groups)) return maxSets;  // error -> the summary bound
  const i32 num = mode == KPO_FAITHFUL ? simulateFF(groups, comps, maxSets) : simulateRuns(groups, comps, maxSets);
  return num < maxSets ? num : maxSets;
}

// isMultiTemplateSchedulingApplicable (core/estimation.go:43-65): components present and a
// cluster spread constraint with MinGroups == MaxGroups == 1.
bool multiTemplateApplicable(const Binding& b) {
  if (b.n_components == 0) return false;
  for (auto& sc : b.spreads)
    if (sc.field == "cluster" && sc.min == 1 && sc.max == 1) return true;
  return false;
}
bool useComponentSets(const Binding& b, const Options& o) { return o.multi_templates && multiTemplateApplicable(b); }

// calAvailableReplicas (pkg/scheduler/core/util.go:57-110) with the general estimator only.
vector<TargetCluster> calAvailableReplicas(const vector<const Cluster*>& clusters, const Binding& b, const Options& o,
                                           int mode) {
  vector<TargetCluster> out(clusters.size());
  for (size_t i = 0; i < clusters.size(); i++) {
    out[i].name = clusters[i]->name;
    out[i].replicas = INT32_MAX;
  }
  if (b.replicas == 0 && b.n_components == 0) return out;
  // runReplicaEstimator (util.go:113-118): with the MultiplePodTemplatesScheduling gate
  // and isMultiTemplateSchedulingApplicable, MaxAvailableComponentSets answers
  // (calculateMultiTemplateAvailableSets, estimation.go:77-113; the general estimator
  // answers every cluster, never UnauthenticReplica).
  const bool sets = useComponentSets(b, o);
  for (size_t i = 0; i < clusters.size(); i++) {
    i32 r = sets ? maxAvailableComponentSets(*clusters[i], b.comps, o, mode) : maxAvailableReplicas(*clusters[i], b, o, mode);
    if (r != -1 && out[i].replicas > r) out[i].replicas = r;  // mergeReplicaResults (util.go:157-170)
  }
  for (auto& t : out)
    if (t.replicas == INT32_MAX) t.replicas = b.replicas;
  return out;
}

// ===========================================================================
// Go sort.Sort (pdqsort, sort/zsortinterface.go, go1.26) on TargetClustersList
// (division_algorithm.go:31-36). Parity for n > 12 is unpinned.
// ===========================================================================
struct TCList {
  vector<TargetCluster>* a;
  bool Less(int i, int j) const { return (*a)[i].replicas > (*a)[j].replicas; }
  void Swap(int i, int j) { std::swap((*a)[i], (*a)[j]); }
};
template <class D>
void insertionSort(D& d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
}
template <class D>
void siftDown(D& d, int lo, int hi, int first) {
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
void heapSort(D& d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) {
    d.Swap(first, first + i);
    siftDown(d, lo, i, first);
  }
}
int bitsLen(uint64_t x) {
  int n = 0;
  while (x) {
    n++;
    x >>= 1;
  }
  return n;
}
template <class D>
void breakPatterns(D& d, int a, int b) {
  int length = b - a;
  if (length >= 8) {
    uint64_t r = (uint64_t)length;
    uint64_t modulus = 1ull << bitsLen((uint64_t)length);
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
template <class D>
void order2(D& d, int& a, int& b, int& swaps) {
  if (d.Less(b, a)) {
    swaps++;
    std::swap(a, b);
  }
}
template <class D>
int median(D& d, int a, int b, int c, int& swaps) {
  order2(d, a, b, swaps);
  order2(d, b, c, swaps);
  order2(d, a, b, swaps);
  return b;
}
template <class D>
int medianAdjacent(D& d, int a, int& swaps) {
  return median(d, a - 1, a, a + 1, swaps);
}
enum { kUnknownHint = 0, kIncreasingHint = 1, kDecreasingHint = 2 };
template <class D>
int choosePivot(D& d, int a, int b, int* hint) {
  int l = b - a;
  int swaps = 0;
  int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
  if (l >= 8) {
    if (l >= 50) {
      i = medianAdjacent(d, i, swaps);
      j = medianAdjacent(d, j, swaps);
      k = medianAdjacent(d, k, swaps);
    }
    j = median(d, i, j, k, swaps);
  }
  *hint = swaps == 0 ? kIncreasingHint : (swaps == 12 ? kDecreasingHint : kUnknownHint);
  return j;
}
template <class D>
void reverseRange(D& d, int a, int b) {
  int i = a, j = b - 1;
  while (i < j) {
    d.Swap(i, j);
    i++;
    j--;
  }
}
template <class D>
bool partialInsertionSort(D& d, int a, int b) {
  int i = a + 1;
  for (int step = 0; step < 5; step++) {
    while (i < b && !d.Less(i, i - 1)) i++;
    if (i == b) return true;
    if (b - a < 50) return false;
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
  return false;
}
template <class D>
int partitionEqual(D& d, int a, int b, int pivot) {
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
  return i;
}
template <class D>
int partition(D& d, int a, int b, int pivot, bool* already) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  while (i <= j && d.Less(i, a)) i++;
  while (i <= j && !d.Less(j, a)) j--;
  if (i > j) {
    d.Swap(j, a);
    *already = true;
    return j;
  }
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
  *already = false;
  return j;
}
template <class D>
void pdqsort(D& d, int a, int b, int limit) {
  bool wasBalanced = true, wasPartitioned = true;
  for (;;) {
    int length = b - a;
    if (length <= 12) {
      insertionSort(d, a, b);
      return;
    }
    if (limit == 0) {
      heapSort(d, a, b);
      return;
    }
    if (!wasBalanced) {
      breakPatterns(d, a, b);
      limit--;
    }
    int hint;
    int pivot = choosePivot(d, a, b, &hint);
    if (hint == kDecreasingHint) {
      reverseRange(d, a, b);
      pivot = (b - 1) - (pivot - a);
      hint = kIncreasingHint;
    }
    if (wasBalanced && wasPartitioned && hint == kIncreasingHint) {
      if (partialInsertionSort(d, a, b)) return;
    }
    if (a > 0 && !d.Less(a - 1, pivot)) {
      a = partitionEqual(d, a, b, pivot);
      continue;
    }
    bool already;
    int mid = partition(d, a, b, pivot, &already);
    wasPartitioned = already;
    int leftLen = mid - a, rightLen = b - mid;
    int balanceThreshold = length / 8;
    if (leftLen < rightLen) {
      wasBalanced = leftLen >= balanceThreshold;
      pdqsort(d, a, mid, limit);
      a = mid + 1;
    } else {
      wasBalanced = rightLen >= balanceThreshold;
      pdqsort(d, mid + 1, b, limit);
      b = mid;
    }
  }
}
void SortTargetClustersList(vector<TargetCluster>& v) {
  int n = (int)v.size();
  if (n <= 1) return;
  TCList d{&v};
  pdqsort(d, 0, n, bitsLen((uint64_t)n));
}

// ===========================================================================
// Webster / Dispenser (pkg/util/helper/webstermethod.go, binding.go:51-183)
// ===========================================================================
struct Party {
  string name;
  i64 votes = 0;
  i32 seats = 0;
};
uint32_t fnv32a(const string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) {
    h ^= c;
    h *= 16777619u;
  }
  return h;
}
// tie_mode: 0 = WebsterPriorityQueue default (seats, name asc), 1 = name asc (UID even/empty), 2 = name desc (UID odd)
struct WebsterPQ {
  vector<Party> P;
  int tie_mode = 0;
  // float64(Votes) / float64(2*Seats+1), the int32 expression wrapping as in Go.
  static double prio(const Party& p) { return (double)p.votes / (double)add32((i32)(2u * (uint32_t)p.seats), 1); }
  bool Less(int i, int j) const {
    double ip = prio(P[i]);
    double jp = prio(P[j]);
    if (ip == jp) {
      if (P[i].seats != P[j].seats) return P[i].seats < P[j].seats;
      if (tie_mode == 2) return P[i].name > P[j].name;
      return P[i].name < P[j].name;
    }
    return ip > jp;
  }
  void Swap(int i, int j) { std::swap(P[i], P[j]); }
  // container/heap
  void down(int i0, int n) {
    int i = i0;
    for (;;) {
      int j1 = 2 * i + 1;
      if (j1 >= n || j1 < 0) break;
      int j = j1;
      int j2 = j1 + 1;
      if (j2 < n && Less(j2, j1)) j = j2;
      if (!Less(j, i)) break;
      Swap(i, j);
      i = j;
    }
  }
  void up(int j) {
    for (;;) {
      int i = (j - 1) / 2;
      if (i == j || !Less(j, i)) break;
      Swap(i, j);
      j = i;
    }
  }
  void init() {
    int n = (int)P.size();
    for (int i = n / 2 - 1; i >= 0; i--) down(i, n);
  }
  Party pop() {
    int n = (int)P.size() - 1;
    Swap(0, n);
    down(0, n);
    Party x = P.back();
    P.pop_back();
    return x;
  }
  void push(const Party& x) {
    P.push_back(x);
    up((int)P.size() - 1);
  }
};
// FAST mode only (g_webster_fast, set by kpo_schedule's workers for KPO_FAST): seats
// the first S heap pops at once. The heap pops a strict total order of the elements
// (party i, seat k) keyed by (v_i/(2k+1) desc, k asc, name), a party's elements in k
// order, so for any t >= 0 the elements with priority > t are
// exactly the first S pops when their count S <= newSeats; the heap then runs the
// remaining newSeats - S pops from there. Elements with k >= 2^30 (2*Seats+1 wraps
// in int32, webstermethod.go:60-61) are left to the heap. Only for fresh parties
// (no initial seats) with non-negative votes; tests/test_oracle_synth.py checks it
// against the literal loop.
thread_local bool g_webster_fast = false;
i32 websterPreseat(vector<Party>& P, i32 N, int tie_mode) {
  if (N <= 64) return 0;
  i64 V = 0;
  int npos = 0, nzero = 0, ipos = -1;
  for (size_t i = 0; i < P.size(); i++) {
    if (P[i].seats != 0) return 0;
    V += P[i].votes > 0 ? P[i].votes : 0;
    if (P[i].votes > 0) npos++, ipos = (int)i;
    nzero += P[i].votes == 0;
  }
  const i64 kCap = (i64)1 << 30;
  auto ahead = [&](int a, int b) { return tie_mode == 2 ? P[a].name > P[b].name : P[a].name < P[b].name; };
  if (npos <= 1 && (i64)N > (i64)npos * kCap) {
    // Every positive party's first 2^30 elements have positive priority; after them
    // its denominator 2*Seats+1 wraps negative in int32. The rest R goes, in heap
    // order, to the zero-vote parties (priority 0; ties by seats then name: a round
    // robin in name order), else to the positive party's wrapped seats while they
    // stay above the best negative head v_j (a tie goes to fewer seats: j), then to
    // j, whose priority only rises once it holds a seat.
    if (ipos >= 0) P[ipos].seats = (i32)kCap;
    i64 R = (i64)N - (i64)npos * kCap;
    if (nzero) {
      vector<int> z;
      for (size_t i = 0; i < P.size(); i++)
        if (P[i].votes == 0) z.push_back((int)i);
      std::sort(z.begin(), z.end(), ahead);
      for (size_t j = 0; j < z.size(); j++) P[z[j]].seats = (i32)(R / nzero + ((i64)j < R % nzero ? 1 : 0));
      return N;
    }
    int jn = -1;
    for (size_t j = 0; j < P.size(); j++)
      if (P[j].votes < 0 && (jn < 0 || P[j].votes > P[jn].votes || (P[j].votes == P[jn].votes && ahead((int)j, jn))))
        jn = (int)j;
    if (ipos >= 0) {
      i64 m = 0;  // wrapped seats k = 2^30 + m while WebsterPQ::prio stays above v_j (literal, one by one)
      for (; m < R; m++) {
        Party q = P[ipos];
        q.seats = (i32)(kCap + m);
        if (jn >= 0 && !(WebsterPQ::prio(q) > (double)P[jn].votes)) break;
      }
      P[ipos].seats = (i32)(kCap + m);
      R -= m;
    }
    if (R > 0 && jn >= 0) P[jn].seats = (i32)R;
    return N;
  }
  if (npos == 0) return 0;
  auto count = [&](i64 v, double t) -> i64 {  // #{k < 2^30 : fl(v/(2k+1)) > t}
    if (v <= 0 || !((double)v > t)) return 0;
    double q = ((double)v / t - 1.0) / 2.0;
    i64 k = q >= (double)(kCap - 1) ? kCap - 1 : (q < 0 ? 0 : (i64)q);
    while (k > 0 && !((double)v / (double)(2 * k + 1) > t)) k--;
    while (k + 1 < kCap && (double)v / (double)(2 * (k + 1) + 1) > t) k++;
    return k + 1;
  };
  auto total = [&](double t) {
    i64 S = 0;
    for (auto& p : P) S += p.votes > 0 ? count(p.votes, t) : 0;
    return S;
  };
  // t_hi: count <= N; t_lo: count > N (or 0); bisect so that the heap's share is
  // about the tie group at the N-th priority
  double hi = (double)V / (2.0 * (double)N), lo = 0;
  for (int it = 0; it < 200 && total(hi) > (i64)N; it++) {
    lo = hi;
    hi *= 1.5;
  }
  if (total(hi) > (i64)N) return 0;
  for (int it = 0; it < 64 && lo < hi && (i64)N - total(hi) > 4 * (i64)P.size() + 64; it++) {
    const double mid = lo + (hi - lo) / 2;
    if (mid <= lo || mid >= hi) break;
    if (total(mid) <= (i64)N) hi = mid;
    else lo = mid;
  }
  i64 S = 0;
  for (auto& p : P) {
    p.seats = p.votes > 0 ? (i32)count(p.votes, hi) : 0;
    S += p.seats;
  }
  return (i32)S;
}
int tieModeForUID(const string& uid) {
  if (uid.empty()) return 1;
  return (fnv32a(uid) & 1) ? 2 : 1;
}
// AllocateWebsterSeats (webstermethod.go:112-161); maps given as ordered
// (name,value) lists with Go map-assignment semantics (later entries win).
vector<Party> AllocateWebsterSeats(i32 newSeats, const vector<std::pair<string, i64>>& partyVotes,
                                   const vector<std::pair<string, i32>>& initial, int tie_mode) {
  std::map<string, Party> parties;
  for (auto& kv : initial) parties[kv.first] = Party{kv.first, 0, kv.second};
  for (auto& kv : partyVotes) {
    auto it = parties.find(kv.first);
    if (it != parties.end()) it->second.votes = kv.second;
    else parties[kv.first] = Party{kv.first, kv.second, 0};
  }
  WebsterPQ pq;
  pq.tie_mode = tie_mode;
  for (auto& kv : parties) pq.P.push_back(kv.second);
  if (pq.P.empty()) return {};
  i32 preseated = g_webster_fast ? websterPreseat(pq.P, newSeats, tie_mode) : 0;
  pq.init();
  for (i32 remaining = newSeats - preseated; remaining > 0; remaining--) {
    Party p = pq.pop();
    p.seats = add32(p.seats, 1);
    pq.push(p);
  }
  std::sort(pq.P.begin(), pq.P.end(), [](const Party& a, const Party& b) { return a.name < b.name; });
  return pq.P;
}
struct WeightInfo {
  string name;
  i64 weight = 0;
  i32 last = 0;
};
// Dispenser.AllocateByWeight with init == nil (binding.go:94-115).
vector<TargetCluster> DispenserAllocate(i32 numReplicas, const vector<TargetCluster>& init, const string& uid,
                                        const vector<WeightInfo>& w) {
  vector<TargetCluster> result = init;
  if (numReplicas == 0 && !result.empty()) return result;  // Done()
  i64 sum = 0;
  for (auto& x : w) sum = add64(sum, x.weight);
  if (sum == 0) return result;
  vector<std::pair<string, i32>> initial;
  for (auto& c : result) initial.push_back({c.name, c.replicas});
  vector<std::pair<string, i64>> votes;
  for (auto& x : w) votes.push_back({x.name, x.weight});
  auto parties = AllocateWebsterSeats(numReplicas, votes, initial, tieModeForUID(uid));
  vector<TargetCluster> out;
  for (auto& p : parties) out.push_back({p.name, p.seats});
  return out;
}
// SpreadReplicasByTargetClusters (binding.go:157-183)
vector<TargetCluster> SpreadReplicasByTargetClusters(i32 num, const vector<TargetCluster>& tcs,
                                                     const vector<TargetCluster>& init, const string& uid) {
  vector<WeightInfo> w;
  for (auto& t : tcs) {
    i32 last = 0;
    for (auto& s : init)
      if (t.name == s.name) {
        last = s.replicas;
        break;
      }
    w.push_back({t.name, (i64)t.replicas, last});
  }
  return DispenserAllocate(num, init, uid, w);
}

// ===========================================================================
// Spread constraints (pkg/scheduler/core/spreadconstraint)
// ===========================================================================
struct DetailInfo {  // ClusterDetailInfo (group_clusters.go:78-93)
  string name;
  i64 score = 0;
  i32 overflow = 0;
  i64 available = 0;
  const Cluster* cluster = nullptr;
  i32 allocatable = 0;
};
// sortClusters (spreadconstraint/util.go:43-61) with the AvailableReplicas tie-break
bool lessDetailAvail(const DetailInfo& a, const DetailInfo& b) {
  if (a.overflow != b.overflow) return a.overflow < b.overflow;
  if (a.score != b.score) return a.score > b.score;
  if (a.available != b.available) return a.available > b.available;
  return a.name < b.name;
}
struct RegionInfo {
  string name;
  i64 score = 0;
  i64 available = 0;
  vector<DetailInfo> clusters;
};
struct GroupInfoAll {
  std::map<string, RegionInfo> regions;
  bool has_regions = false;
  vector<DetailInfo> clusters;
};
const i64 kWeightUnit = 1000;  // group_clusters.go:154

string ReplicaSchedulingType(const Binding& b) {  // propagation_helper.go:40-46
  if (!b.has_rs) return "Duplicated";
  return b.rs_type;
}
bool shouldIgnoreSpreadConstraint(const Binding& b) {  // select_clusters.go:57-69
  if (b.has_rs && b.rs_type == "Divided" && b.rs_div == "Weighted" &&
      (!b.has_wp || (!b.sw.empty() && b.dyn.empty())))
    return true;
  return false;
}
bool shouldIgnoreAvailableResource(const Binding& b) {  // select_clusters.go:71-80
  return !b.has_rs || b.rs_type == "Duplicated";
}
bool isTopologyIgnored(const Binding& b) {  // group_clusters.go:506-514
  if (b.spreads.empty() || (b.spreads.size() == 1 && b.spreads[0].field == "cluster")) return true;
  return shouldIgnoreSpreadConstraint(b);
}
// calcGroupScoreForDuplicate (group_clusters.go:156-236)
i64 calcGroupScoreForDuplicate(const vector<DetailInfo>& clusters, const Binding& b) {
  i64 target = b.replicas;
  i64 valid = 0, sumValid = 0;
  for (auto& c : clusters)
    if (c.available >= target) {
      valid++;
      sumValid += c.score;
    }
  if (valid == 0) return 0;
  return mul64(valid, kWeightUnit) + sumValid / valid;
}
// int64(math.Ceil(float64/float64)) with amd64 conversion of NaN/Inf/out-of-range (hazard H4)
std::atomic<uint64_t> g_h4_hits{0};  // conversions that took the NaN/Inf branch (tests count them)
i64 goCeilDivToInt64(i32 a, i64 b) {
  double q = std::ceil((double)a / (double)b);
  if (std::isnan(q) || q >= 9223372036854775808.0 || q < -9223372036854775808.0) {
    g_h4_hits.fetch_add(1, std::memory_order_relaxed);
    return INT64_MIN;
  }
  return (i64)q;
}
// calcGroupScore (group_clusters.go:238-351)
i64 calcGroupScore(const vector<DetailInfo>& clusters, const Binding& b, i64 minGroups) {
  if (ReplicaSchedulingType(b) == "Duplicated") return calcGroupScoreForDuplicate(clusters, b);
  i64 targetReplica = goCeilDivToInt64(b.replicas, minGroups);
  i64 clusterMinGroups = 0;
  for (auto& sc : b.spreads)
    if (sc.field == "cluster") clusterMinGroups = sc.min;
  if (clusterMinGroups < minGroups) clusterMinGroups = minGroups;
  i64 sumAvail = 0, sumScore = 0, valid = 0;
  for (auto& c : clusters) {
    sumAvail = add64(sumAvail, c.available);
    sumScore = add64(sumScore, c.score);
    valid++;
    if (valid >= clusterMinGroups && sumAvail >= targetReplica) break;
  }
  if (sumAvail < targetReplica) {
    sumAvail = mul64(sumAvail, kWeightUnit);
    return add64(sumAvail, sumScore / (i64)clusters.size());
  }
  targetReplica = mul64(targetReplica, kWeightUnit);
  return add64(targetReplica, sumScore / valid);
}
bool hasSpreadField(const Binding& b, const string& f) {  // IsSpreadConstraintExisted (util.go:33-41)
  for (auto& s : b.spreads)
    if (s.field == f) return true;
  return false;
}
// getClusterOverflowOrder (group_clusters.go:517-543)
i32 getClusterOverflowOrder(const Cluster& c, const Binding& b) {
  if (b.has_ca || b.cas.empty()) return 0;
  const Term* term = nullptr;
  for (auto& t : b.cas)
    if (t.name == b.observed) {
      term = &t;
      break;
    }
  if (term) {
    if (ClusterMatches(c, term->aff)) return 0;
    for (size_t i = 0; i < term->overflow.size(); i++)
      if (ClusterMatches(c, term->overflow[i])) return (i32)(i + 1);
  }
  return 1000;
}
// GroupClustersWithScore (group_clusters.go:103-149) + generateClustersInfo (:353-378)
// + generateRegionInfo (:418-457). Zone/provider infos are computed by the
// reference but never read by selection, so they are skipped.
GroupInfoAll GroupClustersWithScore(const vector<std::pair<const Cluster*, i64>>& scored, const Binding& b,
                                    const vector<i32>* est_override, const Options& o, int mode) {
  GroupInfoAll info;
  vector<const Cluster*> cl;
  for (auto& s : scored) {
    DetailInfo d;
    d.name = s.first->name;
    d.score = s.second;
    d.cluster = s.first;
    d.overflow = getClusterOverflowOrder(*s.first, b);
    info.clusters.push_back(d);
    cl.push_back(s.first);
  }
  vector<TargetCluster> reps;
  if (est_override) {
    for (size_t i = 0; i < cl.size(); i++) reps.push_back({cl[i]->name, (*est_override)[i]});
  } else {
    reps = calAvailableReplicas(cl, b, o, mode);
  }
  for (size_t i = 0; i < reps.size(); i++) {
    info.clusters[i].available = (i64)reps[i].replicas + (i64)AssignedReplicasForCluster(b, reps[i].name);
    info.clusters[i].allocatable = reps[i].replicas;
  }
  std::sort(info.clusters.begin(), info.clusters.end(), lessDetailAvail);  // strict total order
  if (!isTopologyIgnored(b) && hasSpreadField(b, "region")) {
    info.has_regions = true;
    for (auto& ci : info.clusters) {
      const string& r = ci.cluster->region;
      if (r.empty()) continue;
      auto& ri = info.regions[r];
      ri.name = r;
      ri.clusters.push_back(ci);
      ri.available += ci.available;
    }
    i64 minGroups = 0;
    for (auto& sc : b.spreads)
      if (sc.field == "region") minGroups = sc.min;
    for (auto& kv : info.regions) kv.second.score = calcGroupScore(kv.second.clusters, b, minGroups);
  }
  return info;
}

// select_groups.go
struct GroupInfo {
  string name;
  i64 value = 0;
  i64 weight = 0;
};
struct DfsPath {
  int id = 0;
  vector<const GroupInfo*> groups;
  i64 weight = 0;
  i64 value = 0;
};
vector<const GroupInfo*> selectGroups(vector<GroupInfo>& groupsIn, i64 minC, i64 maxC, i64 target) {
  if (groupsIn.empty()) return {};
  vector<const GroupInfo*> groups;
  for (auto& g : groupsIn) groups.push_back(&g);
  // findFeasiblePaths (select_groups.go:146-190)
  if (groups.size() > 1) {
    std::sort(groups.begin(), groups.end(), [](const GroupInfo* a, const GroupInfo* b) {
      if (a->value != b->value) return a->value < b->value;
      if (a->weight != b->weight) return a->weight > b->weight;
      return a->name < b->name;
    });
  }
  vector<DfsPath> paths;
  DfsPath root;
  std::function<void(i64, int)> dfs = [&](i64 sum, int begin) {
    if (sum >= target && (i64)root.groups.size() >= minC && (i64)root.groups.size() <= maxC) {
      root.id++;  // dfsPath.next (select_groups.go:41-55)
      DfsPath r = root;
      for (auto* g : r.groups) {
        r.weight += g->weight;
        r.value += g->value;
      }
      std::sort(r.groups.begin(), r.groups.end(), [](const GroupInfo* a, const GroupInfo* b) {
        if (a->weight != b->weight) return a->weight > b->weight;
        return a->name < b->name;
      });
      paths.push_back(r);
      return;
    }
    if ((i64)root.groups.size() >= maxC) return;
    for (int i = begin; i < (int)groups.size(); i++) {
      sum += groups[i]->value;
      root.groups.push_back(groups[i]);
      dfs(sum, i + 1);
      if ((i64)groups.size() == minC) break;
      sum -= groups[i]->value;
      root.groups.pop_back();
    }
  };
  dfs(0, 0);
  if (paths.empty()) return {};
  // prioritizePaths (select_groups.go:200-224)
  if (paths.size() == 1) return paths[0].groups;
  std::sort(paths.begin(), paths.end(), [](const DfsPath& a, const DfsPath& b) {
    if (a.weight != b.weight) return a.weight > b.weight;
    if (a.value != b.value) return a.value > b.value;
    return a.id < b.id;
  });
  const DfsPath* fin = &paths[0];
  for (size_t i = 1; i < paths.size(); i++) {
    const DfsPath& sub = paths[i];
    bool match = sub.groups.size() < fin->groups.size();
    if (match)
      for (size_t k = 0; k < sub.groups.size(); k++)
        if (fin->groups[k]->name != sub.groups[k]->name) {
          match = false;
          break;
        }
    if (match) fin = &paths[i];
  }
  return fin->groups;
}

struct SelectResult {
  vector<DetailInfo> clusters;
  int err = KP_ERR_NONE;
  i64 arg = 0;
};
// selectBestClustersByRegion (select_clusters_by_region.go:25-64)
SelectResult selectByRegion(const std::map<string, Spread>& scm, GroupInfoAll& info) {
  SelectResult res;
  Spread regionC = scm.count("region") ? scm.at("region") : Spread{};
  Spread clusterC = scm.count("cluster") ? scm.at("cluster") : Spread{};
  if ((i64)info.regions.size() < regionC.min) {
    res.err = KP_ERR_REGION_MIN_GROUPS;
    return res;
  }
  vector<GroupInfo> groups;
  for (auto& kv : info.regions) groups.push_back({kv.second.name, (i64)kv.second.clusters.size(), kv.second.score});
  auto sel = selectGroups(groups, regionC.min, regionC.max, clusterC.min);
  if (sel.empty()) {
    res.err = KP_ERR_REGION_CLUSTER_MIN;
    return res;
  }
  vector<DetailInfo> candidates, selected;
  for (auto* g : sel) {
    auto& r = info.regions[g->name];
    selected.push_back(r.clusters[0]);
    for (size_t i = 1; i < r.clusters.size(); i++) candidates.push_back(r.clusters[i]);
  }
  i64 needCnt = std::min<i64>((i64)(candidates.size() + selected.size()), clusterC.max);
  i64 restCnt = needCnt - (i64)selected.size();
  if (restCnt > 0) {
    std::sort(candidates.begin(), candidates.end(), lessDetailAvail);
    for (i64 i = 0; i < restCnt; i++) selected.push_back(candidates[i]);
  }
  res.clusters = selected;
  return res;
}
// selectBestClustersByCluster (select_clusters_by_cluster.go:25-102)
SelectResult selectByCluster(const Spread& sc, GroupInfoAll& info, i32 needReplicas) {
  SelectResult res;
  i64 total = (i64)info.clusters.size();
  if (total < sc.min) {
    res.err = KP_ERR_CLUSTER_MIN_GROUPS;
    return res;
  }
  i64 needCnt = std::min<i64>(total, sc.max);
  if (needCnt < 0) needCnt = 0;  // Go would panic on a negative slice bound
  if (needReplicas == -1) {
    res.clusters.assign(info.clusters.begin(), info.clusters.begin() + needCnt);
    return res;
  }
  vector<DetailInfo>& all = info.clusters;  // ret/rest alias the same backing array
  auto check = [&](void) {
    i64 t = 0;
    for (i64 i = 0; i < needCnt; i++) t += all[i].available;
    return t >= (i64)needReplicas;
  };
  i64 upd = needCnt - 1;
  while (!check() && upd >= 0) {
    i64 maxv = all[upd].available;
    i64 id = -1;
    for (i64 i = needCnt; i < total; i++)
      if (maxv < all[i].available) {
        id = i;
        maxv = all[i].available;
      }
    if (id == -1) {
      upd--;
      continue;
    }
    std::swap(all[upd], all[id]);
    upd--;
  }
  if (!check() || needCnt == 0) {
    res.err = KP_ERR_CLUSTER_RESOURCE;
    res.arg = needCnt;
    return res;
  }
  res.clusters.assign(all.begin(), all.begin() + needCnt);
  return res;
}
// SelectBestClusters (select_clusters.go:28-55)
SelectResult SelectBestClusters(const Binding& b, GroupInfoAll& info, i32 needReplicas) {
  if (b.spreads.empty() || shouldIgnoreSpreadConstraint(b)) {
    SelectResult r;
    r.clusters = info.clusters;
    return r;
  }
  if (shouldIgnoreAvailableResource(b)) needReplicas = -1;
  std::map<string, Spread> scm;
  for (auto& s : b.spreads) scm[s.field] = s;
  if (scm.count("region")) return selectByRegion(scm, info);
  if (scm.count("cluster")) return selectByCluster(scm["cluster"], info, needReplicas);
  SelectResult r;
  r.err = KP_ERR_SPREAD_UNSUPPORTED;
  return r;
}

// ===========================================================================
// Assignment (pkg/scheduler/core/{common,assignment,division_algorithm}.go)
// ===========================================================================
struct AssignResult {
  vector<TargetCluster> targets;
  int status = KP_STATUS_OK;
  int err = KP_ERR_NONE;
  i64 arg = 0;
};
enum Strategy { kNone, kDuplicated, kAggregated, kStatic, kDynamic };
Strategy strategyOf(const Binding& b) {  // newAssignState (assignment.go:95-123)
  string t = ReplicaSchedulingType(b);
  if (t == "Duplicated") return kDuplicated;
  if (t == "Divided") {
    if (b.rs_div == "Aggregated") return kAggregated;
    if (b.rs_div == "Weighted") {
      if (b.has_wp && !b.dyn.empty()) return kDynamic;
      return kStatic;
    }
  }
  return kNone;
}
vector<TargetCluster> removeZero(const vector<TargetCluster>& v) {  // util.go:189-197
  vector<TargetCluster> o;
  for (auto& t : v)
    if (t.replicas > 0) o.push_back(t);
  return o;
}
// dynamicDivideReplicas (division_algorithm.go:75-101)
bool dynamicDivide(Strategy st, const Binding& b, vector<TargetCluster>& available, i32 availableReplicas,
                   i32 target, vector<TargetCluster>& scheduled, AssignResult* out, int errcode) {
  if (availableReplicas < target) {
    out->status = KP_STATUS_UNSCHEDULABLE;
    out->err = errcode;
    out->arg = availableReplicas;
    return false;
  }
  if (st == kAggregated) {
    // resortAvailableClusters (assignment.go:151-178)
    std::set<string> prior;
    for (auto& c : scheduled)
      if (c.replicas > 0) prior.insert(c.name);
    if (!prior.empty()) {
      vector<TargetCluster> prev, left;
      for (auto& c : available) (prior.count(c.name) ? prev : left).push_back(c);
      prev.insert(prev.end(), left.begin(), left.end());
      available = prev;
    }
    i32 sum = 0;
    for (size_t i = 0; i < available.size(); i++) {
      sum = add32(sum, available[i].replicas);
      if (sum >= target) {
        available.resize(i + 1);
        break;
      }
    }
  } else if (st != kDynamic) {
    out->status = KP_STATUS_ERROR;
    out->err = KP_ERR_UNDEFINED_STRATEGY;
    return false;
  }
  out->targets = MergeTargetClusters(scheduled, SpreadReplicasByTargetClusters(target, available, {}, b.uid));
  return true;
}
// The assignFuncMap strategies (assignment.go:31-38,180-244) without the final
// removeZeroReplicasCluster. force_scale_up=true runs buildScheduledClusters +
// dynamicScaleUp directly (the Test_dynamicScaleUp entry).
AssignResult assignByStrategy(const vector<DetailInfo>& cands, const Binding& spec, bool force_scale_up = false) {
  AssignResult r;
  Strategy st = strategyOf(spec);
  if (st == kNone) {
    r.status = KP_STATUS_ERROR;
    r.err = KP_ERR_UNSUPPORTED_STRATEGY;
    return r;
  }
  vector<TargetCluster> res;
  if (st == kDuplicated) {  // assignment.go:181-187
    for (auto& c : cands) res.push_back({c.name, spec.replicas});
  } else if (st == kStatic) {  // assignment.go:199-211 + division_algorithm.go:38-72
    vector<WeightInfo> list;
    if (!spec.has_wp) {  // getDefaultWeightPreference: one rule {ClusterNames:[name]} weight 1 per candidate
      for (auto& c : cands) list.push_back({c.name, 1, AssignedReplicasForCluster(spec, c.name)});
    } else {
      for (auto& c : cands) {
        i64 w = 0;
        for (auto& rule : spec.sw)
          if (ClusterMatches(*c.cluster, rule.target)) w = std::max<i64>(w, rule.weight);
        if (w > 0) list.push_back({c.name, w, AssignedReplicasForCluster(spec, c.name)});
      }
    }
    i64 sum = 0;
    for (auto& x : list) sum = add64(sum, x.weight);
    if (sum == 0)
      for (auto& c : cands) list.push_back({c.name, 1, 0});
    res = DispenserAllocate(spec.replicas, {}, spec.uid, list);
  } else {  // assignByDynamicStrategy (assignment.go:213-244)
    std::set<string> candSet;
    for (auto& c : cands) candSet.insert(c.name);
    vector<TargetCluster> scheduled;  // buildScheduledClusters (assignment.go:125-142)
    for (auto& c : spec.clusters)
      if (candSet.count(c.name)) scheduled.push_back(c);
    i32 assigned = GetSumOfReplicas(scheduled);
    if (!force_scale_up && RescheduleRequired(spec)) {  // dynamicFreshScale (division_algorithm.go:139-166)
      vector<TargetCluster> avail;
      for (auto& c : cands) avail.push_back({c.name, c.allocatable});
      for (auto& s : scheduled)
        for (auto& a : avail)
          if (a.name == s.name) {
            a.replicas = add32(a.replicas, s.replicas);
            break;
          }
      SortTargetClustersList(avail);
      vector<TargetCluster> none;
      if (!dynamicDivide(st, spec, avail, GetSumOfReplicas(avail), spec.replicas, none, &r, KP_ERR_FRESH_NOT_ENOUGH))
        return r;
      res = r.targets;
    } else if (!force_scale_up && assigned > spec.replicas) {  // dynamicScaleDown (:103-119)
      vector<TargetCluster> avail = scheduled;
      SortTargetClustersList(avail);
      vector<TargetCluster> none;
      if (!dynamicDivide(st, spec, avail, GetSumOfReplicas(avail), spec.replicas, none, &r,
                         KP_ERR_SCALE_DOWN_NOT_ENOUGH))
        return r;
      res = r.targets;
    } else if (force_scale_up || assigned < spec.replicas) {  // dynamicScaleUp (:121-136)
      vector<TargetCluster> avail;
      for (auto& c : cands) avail.push_back({c.name, c.allocatable});
      SortTargetClustersList(avail);
      if (!dynamicDivide(st, spec, avail, GetSumOfReplicas(avail), sub32(spec.replicas, assigned), scheduled, &r,
                         KP_ERR_SCALE_UP_NOT_ENOUGH))
        return r;
      res = r.targets;
    } else {
      res = scheduled;
    }
  }
  r.targets = res;
  return r;
}
// assignReplicasToClusters (common.go:141-154)
AssignResult assignReplicasToClusters(const vector<DetailInfo>& cands, const Binding& spec) {
  AssignResult r = assignByStrategy(cands, spec);
  if (r.status == KP_STATUS_OK) r.targets = removeZero(r.targets);
  return r;
}
bool enableOverflow(const Binding& b) {  // common.go:156-170
  if (b.has_ca || b.cas.empty() || b.observed.empty()) return false;
  for (auto& t : b.cas)
    if (t.name == b.observed && !t.overflow.empty()) return true;
  return false;
}
// AssignReplicas (common.go:51-83) + assignWorkloadReplicas (:97-139)
AssignResult AssignReplicas(const vector<DetailInfo>& clusters, const Binding& spec) {
  AssignResult r;
  if (clusters.empty()) {
    r.status = KP_STATUS_ERROR;
    r.err = KP_ERR_NO_CLUSTERS;
    return r;
  }
  if ((spec.replicas > 0 || spec.has_rr) && spec.n_components <= 1) {
    if (enableOverflow(spec)) {
      std::map<int, vector<DetailInfo>> tiers;
      std::map<int, i64> tierAvail;
      int maxOrder = 0;
      for (auto& c : clusters) {
        tiers[c.overflow].push_back(c);
        tierAvail[c.overflow] += c.available;
        if (c.overflow > maxOrder) maxOrder = c.overflow;
      }
      vector<TargetCluster> fin;
      i32 remaining = spec.replicas;
      Binding copy = spec;
      for (int i = 0; i <= maxOrder; i++) {
        if (tiers[i].empty()) continue;
        copy.replicas = (i32)std::min<i64>((i64)remaining, tierAvail[i]);
        AssignResult t = assignReplicasToClusters(tiers[i], copy);
        if (t.status != KP_STATUS_OK) return t;
        fin.insert(fin.end(), t.targets.begin(), t.targets.end());
        remaining = sub32(remaining, copy.replicas);
        if (remaining <= 0) break;
      }
      if (remaining > 0) {
        r.status = KP_STATUS_UNSCHEDULABLE;
        r.err = KP_ERR_OVERFLOW_NOT_ENOUGH;
        return r;
      }
      r.targets = fin;
      return r;
    }
    return assignReplicasToClusters(clusters, spec);
  }
  for (auto& c : clusters) r.targets.push_back({c.name, 0});
  return r;
}

// ===========================================================================
// genericScheduler.Schedule (pkg/scheduler/core/generic_scheduler.go:71-116)
// ===========================================================================
struct World {
  vector<Cluster> clusters;
  Options opts;
  bool ok = true;
  std::map<string, int> index;
};
struct ScheduleOut {
  int status = KP_STATUS_OK;
  int err = KP_ERR_NONE;
  i64 arg = 0;
  vector<std::pair<int, i32>> targets;  // (cluster idx, replicas)
};
ScheduleOut Schedule(const World& w, const Binding& b, int mode) {
  ScheduleOut out;
  if (b.bad) {
    out.status = KP_STATUS_ERROR;
    return out;
  }
  // g.schedulerCache.Snapshot(): List + DeepCopy of every cluster (cache.go:124-139)
  vector<Cluster> deep;
  const vector<Cluster>* snap = &w.clusters;
  if (mode != KPO_FAST) {
    deep = w.clusters;
    snap = &deep;
  }
  // findClustersThatFit (generic_scheduler.go:119-163)
  vector<const Cluster*> feasible;
  for (auto& c : *snap) {
    if (c.deleting) continue;
    if (RunFilterPlugins(b, c, w.opts) == 0) feasible.push_back(&c);
  }
  if (feasible.empty()) {
    out.status = KP_STATUS_FIT_ERROR;
    out.err = KP_ERR_FIT;
    out.arg = (i64)snap->size();
    return out;
  }
  // prioritizeClusters (:166-194)
  vector<std::pair<const Cluster*, i64>> scored;
  for (auto* c : feasible) scored.push_back({c, ScoreCluster(b, *c, w.opts)});
  // selectClusters -> SelectClusters (common.go:34-48)
  GroupInfoAll info = GroupClustersWithScore(scored, b, nullptr, w.opts, mode);
  // SelectClusters (common.go:34-48): a multi-template workload is placed as one set,
  // so it needs 1 available replica (:42-46)
  SelectResult sel = SelectBestClusters(b, info, useComponentSets(b, w.opts) ? 1 : b.replicas);
  if (sel.err != KP_ERR_NONE) {
    out.status = KP_STATUS_ERROR;
    out.err = sel.err;
    out.arg = sel.arg;
    return out;
  }
  // assignReplicas (common.go:51-83)
  AssignResult ar = AssignReplicas(sel.clusters, b);
  if (ar.status != KP_STATUS_OK) {
    out.status = ar.status;
    out.err = ar.err;
    out.arg = ar.arg;
    return out;
  }
  vector<TargetCluster> result = ar.targets;
  if (w.opts.empty_workload_propagation) {  // attachZeroReplicasCluster (util.go:174-186)
    std::set<string> have;
    for (auto& t : result) have.insert(t.name);
    for (auto& c : sel.clusters)
      if (!have.count(c.name)) result.push_back({c.name, 0});
  }
  for (auto& t : result) {
    auto it = w.index.find(t.name);
    out.targets.push_back({it == w.index.end() ? -1 : it->second, t.replicas});
  }
  return out;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
struct kpo_world {
  World w;
};

extern "C" {

kpo_world* kpo_world_create(const kp_cluster* clusters, uint64_t n, const kp_options* opts) {
  auto* k = new kpo_world();
  k->w.opts = convOptions(opts);
  for (uint64_t i = 0; i < n; i++) {
    bool ok = true;
    k->w.clusters.push_back(convCluster(clusters[i], (int)i, &ok));
    if (!ok) k->w.ok = false;
    k->w.index[k->w.clusters.back().name] = (int)i;
  }
  return k;
}

void kpo_world_destroy(kpo_world* w) { delete w; }

}  // extern "C"

namespace {
// Runs fn(i) for i in [0, n) on n_threads host threads.
template <class F>
void ParallelFor(uint64_t n, int n_threads, F fn) {
  if (n_threads <= 1) {
    for (uint64_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<uint64_t> next(0);
  vector<std::thread> th;
  for (int t = 0; t < n_threads; t++)
    th.emplace_back([&]() {
      for (;;) {
        uint64_t i = next.fetch_add(1);
        if (i >= n) break;
        fn(i);
      }
    });
  for (auto& t : th) t.join();
}

// getAffinityIndex (pkg/scheduler/helper.go:99-110).
uint32_t GetAffinityIndex(const kp_binding& b) {
  string obs = S(b.observed_affinity_name);
  if (obs.empty()) return 0;
  for (uint32_t i = 0; i < b.n_cluster_affinities; i++)
    if (S(b.cluster_affinities[i].affinity_name) == obs) return i;
  return 0;
}

// Scheduler.scheduleResourceBindingWithClusterAffinities (pkg/scheduler/scheduler.go:618-684):
// try the terms from the observed one on; the first success wins; when every term
// fails the FIRST error is the binding's result (FitError -> empty result patched,
// other errors returned as is; both are "no targets" here). *aff = the term index
// that succeeded, or -1 (SchedulerObservedAffinityName left unchanged).
// Bindings with no ClusterAffinities take scheduleResourceBinding (scheduler.go:584-585).
// The StaticWeight WeightPreference mutation (assignment.go:202-204) happens
// only on an attempt that then succeeds, so it is never seen by a later term here.
ScheduleOut ScheduleWithAffinities(const World& w, const kp_binding& b0, int mode, int32_t* aff, int32_t* attempts) {
  *aff = -1;
  *attempts = 1;
  if (b0.n_cluster_affinities == 0) return Schedule(w, convBinding(b0), mode);
  uint32_t idx = GetAffinityIndex(b0);
  if (b0.has_reschedule_triggered_at && b0.has_last_scheduled_time &&
      b0.reschedule_triggered_at_ns > b0.last_scheduled_time_ns)  // util.RescheduleRequired (binding.go:118-127)
    idx = 0;
  ScheduleOut first;
  bool have_first = false;
  *attempts = 0;
  for (; idx < b0.n_cluster_affinities; idx++) {
    kp_binding b = b0;
    b.observed_affinity_name = b0.cluster_affinities[idx].affinity_name;
    ScheduleOut o = Schedule(w, convBinding(b), mode);
    (*attempts)++;
    if (o.status == KP_STATUS_OK) {
      *aff = (int32_t)idx;
      return o;
    }
    if (!have_first) {
      first = o;
      have_first = true;
    }
  }
  first.targets.clear();
  return first;
}

kpo_results* PackResults(const vector<ScheduleOut>& res) {
  const uint64_t n = res.size();
  auto* r = (kpo_results*)calloc(1, sizeof(kpo_results));
  r->n = n;
  r->status = (int32_t*)malloc(sizeof(int32_t) * (n + 1));
  r->err_code = (int32_t*)malloc(sizeof(int32_t) * (n + 1));
  r->err_arg = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  r->offsets = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t tot = 0;
  for (uint64_t i = 0; i < n; i++) tot += res[i].targets.size();
  r->cluster_idx = (uint32_t*)malloc(sizeof(uint32_t) * (tot + 1));
  r->replicas = (int32_t*)malloc(sizeof(int32_t) * (tot + 1));
  uint64_t o = 0;
  for (uint64_t i = 0; i < n; i++) {
    r->status[i] = res[i].status;
    r->err_code[i] = res[i].err;
    r->err_arg[i] = res[i].arg;
    r->offsets[i] = o;
    for (auto& t : res[i].targets) {
      r->cluster_idx[o] = (uint32_t)t.first;
      r->replicas[o] = t.second;
      o++;
    }
  }
  r->offsets[n] = o;
  r->n_targets = o;
  return r;
}
}  // namespace

extern "C" {

int kpo_schedule(kpo_world* k, const kp_binding* b, uint64_t n, int mode, int n_threads, kpo_results** outp) {
  vector<ScheduleOut> res(n);
  ParallelFor(n, n_threads, [&](uint64_t i) {
    g_webster_fast = mode == KPO_FAST;
    res[i] = Schedule(k->w, convBinding(b[i]), mode);
  });
  *outp = PackResults(res);
  return 0;
}

int kpo_schedule_affinities(kpo_world* k, const kp_binding* b, uint64_t n, int mode, int n_threads,
                            kpo_results** outp, int32_t* affinity_index, int32_t* attempts) {
  vector<ScheduleOut> res(n);
  ParallelFor(n, n_threads, [&](uint64_t i) {
    g_webster_fast = mode == KPO_FAST;
    res[i] = ScheduleWithAffinities(k->w, b[i], mode, &affinity_index[i], &attempts[i]);
  });
  *outp = PackResults(res);
  return 0;
}

void kpo_results_free(kpo_results* r) {
  if (!r) return;
  free(r->status);
  free(r->err_code);
  free(r->err_arg);
  free(r->offsets);
  free(r->cluster_idx);
  free(r->replicas);
  free(r);
}

int kpo_quantity(const char* s, uint32_t len, int milli, int64_t* out) {
  Quantity q;
  if (!ParseQuantity(string(s, len), &q)) return -1;
  *out = milli ? QMilli(q) : QValue(q);
  return 0;
}

int kpo_cluster_matches(const kp_cluster* c, const kp_cluster_affinity* a) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  return ClusterMatches(cl, convAffinity(*a)) ? 1 : 0;
}

uint32_t kpo_filter(const kp_cluster* c, const kp_binding* b, const kp_options* opts) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  return RunFilterPlugins(convBinding(*b), cl, convOptions(opts));
}
static bool convComponents(const kp_component* comps, uint32_t n, vector<Component>* v);
int32_t kpo_max_available_component_sets(const kp_cluster* c, const kp_component* comps, uint32_t n,
                                         const kp_options* opts, int mode) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  vector<Component> v;
  if (!convComponents(comps, n, &v)) return -1;
  return maxAvailableComponentSets(cl, v, convOptions(opts), mode);
}
static bool convComponents(const kp_component* comps, uint32_t n, vector<Component>* v) {
  v->assign(n, Component());
  for (uint32_t i = 0; i < n; i++) {
    (*v)[i].replicas = comps[i].replicas;
    (*v)[i].has_rr = comps[i].has_replica_requirements != 0;
    if (!parseList(comps[i].resource_request, comps[i].n_resource_request, &(*v)[i].request)) return false;
  }
  return true;
}
int32_t kpo_max_sets_models(const kp_cluster* c, const kp_component* comps, uint32_t n, int32_t upper, int mode) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  vector<Component> v;
  if (!convComponents(comps, n, &v)) return -2;
  vector<std::pair<Resource, i64>> groups;
  if (!buildModelNodes(cl, &groups)) return -1;  // getMaximumSetsBasedOnResourceModels' error
  return mode == KPO_FAITHFUL ? simulateFF(groups, v, upper) : simulateRuns(groups, v, upper);
}
int32_t kpo_simulate_sets(const kp_cluster* nodes, uint32_t n_nodes, const kp_component* comps, uint32_t n,
                          int32_t upper, int mode) {
  vector<std::pair<Resource, i64>> groups;
  for (uint32_t i = 0; i < n_nodes; i++) {  // createNodeInfo: Allocatable = NewResource(allocatable)
    ResourceList rl;
    if (!parseList(nodes[i].allocatable, nodes[i].n_allocatable, &rl)) return -2;
    Resource r;
    r.Add(rl);
    groups.push_back({r, 1});
  }
  vector<Component> v;
  if (!convComponents(comps, n, &v)) return -2;
  return mode == KPO_FAITHFUL ? simulateFF(groups, v, upper) : simulateRuns(groups, v, upper);
}
uint32_t kpo_filter_reason(const kp_cluster* c, const kp_binding* b, const kp_options* opts) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  return RunFilterPluginsReason(convBinding(*b), cl, convOptions(opts));
}

int64_t kpo_score(const kp_cluster* c, const kp_binding* b, const kp_options* opts) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  return ScoreCluster(convBinding(*b), cl, convOptions(opts));
}

int32_t kpo_max_available_replicas(const kp_cluster* c, const kp_binding* b, const kp_options* opts, int mode) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  return maxAvailableReplicas(cl, convBinding(*b), convOptions(opts), mode);
}


int kpo_estimator_part(const kp_cluster* c, const kp_binding* b, const kp_options* opts, int part, int mode,
                       int64_t* out) {
  bool ok = true;
  Cluster cl = convCluster(*c, 0, &ok);
  Binding bb = convBinding(*b);
  Options o = convOptions(opts);
  switch (part) {
    case 0:
      *out = maxAvailableReplicas(cl, bb, o, mode);
      return 0;
    case 1: {
      i64 v = -1;
      bool r = getMaximumReplicasBasedOnResourceModels(cl, bb, mode, &v);
      *out = r ? v : -1;
      return r ? 0 : -1;
    }
    case 2:
      *out = getMaximumReplicasBasedOnClusterSummary(cl, bb.request);
      return 0;
    case 3:
      *out = getAllowedPodNumber(cl);
      return 0;
  }
  return -1;
}

void kpo_set_webster_fast(int on) { g_webster_fast = on != 0; }
static vector<TargetCluster> convTargets(const kp_target_cluster* t, uint32_t n) {
  vector<TargetCluster> v;
  for (uint32_t i = 0; i < n; i++) v.push_back({S(t[i].name), t[i].replicas});
  return v;
}
int32_t kpo_sum_replicas(const kp_target_cluster* t, uint32_t n) { return GetSumOfReplicas(convTargets(t, n)); }
int kpo_merge_target_clusters(const kp_target_cluster* old_t, uint32_t n_old, const kp_target_cluster* new_t,
                              uint32_t n_new, const kp_target_cluster* names, uint32_t n_names, int32_t* out_idx,
                              int32_t* out_rep, uint32_t out_cap) {
  auto r = MergeTargetClusters(convTargets(old_t, n_old), convTargets(new_t, n_new));
  uint32_t k = 0;
  for (auto& t : r) {
    if (k >= out_cap) break;
    int32_t idx = -1;
    for (uint32_t j = 0; j < n_names; j++)
      if (S(names[j].name) == t.name) idx = (int32_t)j;
    out_idx[k] = idx;
    out_rep[k] = t.replicas;
    k++;
  }
  return (int)r.size();
}
int kpo_reschedule_required(const kp_binding* b) { return RescheduleRequired(convBinding(*b)) ? 1 : 0; }
int kpo_allocate_webster(int32_t new_seats, const kp_str* vote_names, const int64_t* votes, uint32_t n_votes,
                         const kp_str* init_names, const int32_t* init_seats, uint32_t n_init, int tie_mode,
                         kp_str uid, int32_t* out_seats, uint32_t out_cap) {
  vector<std::pair<string, i64>> pv;
  for (uint32_t i = 0; i < n_votes; i++) pv.push_back({S(vote_names[i]), votes[i]});
  vector<std::pair<string, i32>> ia;
  for (uint32_t i = 0; i < n_init; i++) ia.push_back({S(init_names[i]), init_seats[i]});
  int tm = tie_mode;
  if (tm < 0) tm = tieModeForUID(S(uid));
  auto parties = AllocateWebsterSeats(new_seats, pv, ia, tm);
  for (size_t i = 0; i < parties.size() && i < out_cap; i++) out_seats[i] = parties[i].seats;
  return (int)parties.size();
}

int kpo_spread_replicas(int32_t num, const kp_target_cluster* tcs, uint32_t n, const kp_target_cluster* init,
                        uint32_t n_init, kp_str uid, kp_target_cluster* out, uint32_t out_cap) {
  vector<TargetCluster> t, in;
  for (uint32_t i = 0; i < n; i++) t.push_back({S(tcs[i].name), tcs[i].replicas});
  for (uint32_t i = 0; i < n_init; i++) in.push_back({S(init[i].name), init[i].replicas});
  auto r = SpreadReplicasByTargetClusters(num, t, in, S(uid));
  // map names back to input string views
  for (size_t i = 0; i < r.size() && i < out_cap; i++) {
    out[i].replicas = r[i].replicas;
    out[i].name = kp_str{nullptr, 0};
    for (uint32_t j = 0; j < n; j++)
      if (S(tcs[j].name) == r[i].name) out[i].name = tcs[j].name;
    if (!out[i].name.ptr)
      for (uint32_t j = 0; j < n_init; j++)
        if (S(init[j].name) == r[i].name) out[i].name = init[j].name;
  }
  return (int)r.size();
}

int kpo_assign_replicas(const kpo_candidate* cands, uint32_t n, const kp_cluster* clusters, uint32_t n_clusters,
                        const kp_binding* b, int level, int32_t* err_code, int64_t* err_arg, kp_target_cluster* out,
                        uint32_t out_cap) {
  vector<Cluster> cl;
  for (uint32_t i = 0; i < n_clusters; i++) {
    bool ok = true;
    cl.push_back(convCluster(clusters[i], (int)i, &ok));
  }
  vector<DetailInfo> d;
  for (uint32_t i = 0; i < n; i++) {
    DetailInfo x;
    x.name = S(cands[i].name);
    x.score = cands[i].score;
    x.overflow = cands[i].overflow_order;
    x.available = cands[i].available_replicas;
    x.allocatable = cands[i].allocatable_replicas;
    x.cluster = (cands[i].cluster >= 0 && (uint32_t)cands[i].cluster < n_clusters) ? &cl[cands[i].cluster] : nullptr;
    d.push_back(x);
  }
  Binding bb = convBinding(*b);
  AssignResult r = level == 0 ? AssignReplicas(d, bb) : assignByStrategy(d, bb, level == 2);
  *err_code = r.err;
  *err_arg = r.arg;
  if (r.status != KP_STATUS_OK) return -r.status;
  for (size_t i = 0; i < r.targets.size() && i < out_cap; i++) {
    out[i].replicas = r.targets[i].replicas;
    out[i].name = kp_str{nullptr, 0};
    for (uint32_t j = 0; j < n; j++)
      if (S(cands[j].name) == r.targets[i].name) out[i].name = cands[j].name;
    if (!out[i].name.ptr)
      for (uint32_t j = 0; j < b->n_clusters; j++)
        if (S(b->clusters[j].name) == r.targets[i].name) out[i].name = b->clusters[j].name;
  }
  return (int)r.targets.size();
}

int kpo_select_groups(const kp_str* names, const int64_t* values, const int64_t* weights, uint32_t n, int64_t min_c,
                      int64_t max_c, int64_t target, uint32_t* out) {
  vector<GroupInfo> g;
  for (uint32_t i = 0; i < n; i++) g.push_back({S(names[i]), values[i], weights[i]});
  auto sel = selectGroups(g, min_c, max_c, target);
  for (size_t i = 0; i < sel.size(); i++) out[i] = (uint32_t)(sel[i] - &g[0]);
  return (int)sel.size();
}

// calcGroupScore's conversions that took hazard H4's NaN/Inf branch since the last reset
// (the parity tests check that a workload exercised it).
uint64_t kpo_h4_hits(int reset) {
  return reset ? g_h4_hits.exchange(0) : g_h4_hits.load();
}

int64_t kpo_calc_group_score(const kpo_candidate* cands, uint32_t n, const kp_binding* b, int64_t min_groups) {
  vector<DetailInfo> d;
  for (uint32_t i = 0; i < n; i++) {
    DetailInfo x;
    x.name = S(cands[i].name);
    x.score = cands[i].score;
    x.overflow = cands[i].overflow_order;
    x.available = cands[i].available_replicas;
    x.allocatable = cands[i].allocatable_replicas;
    d.push_back(x);
  }
  return calcGroupScore(d, convBinding(*b), min_groups);
}

int kpo_select_clusters(const kp_cluster* clusters, const int64_t* scores, const int32_t* avail, uint32_t n,
                        const kp_binding* b, int32_t need_replicas, uint32_t* out, uint32_t out_cap) {
  vector<Cluster> cl;
  for (uint32_t i = 0; i < n; i++) {
    bool ok = true;
    cl.push_back(convCluster(clusters[i], (int)i, &ok));
  }
  Binding bb = convBinding(*b);
  vector<std::pair<const Cluster*, i64>> scored;
  vector<i32> est;
  for (uint32_t i = 0; i < n; i++) {
    scored.push_back({&cl[i], scores[i]});
    est.push_back(avail[i]);
  }
  Options o;
  GroupInfoAll info = GroupClustersWithScore(scored, bb, &est, o, KPO_FAST);
  SelectResult r = SelectBestClusters(bb, info, need_replicas);
  if (r.err != KP_ERR_NONE) return -r.err;
  for (size_t i = 0; i < r.clusters.size() && i < out_cap; i++) out[i] = (uint32_t)r.clusters[i].cluster->idx;
  return (int)r.clusters.size();
}

namespace {
DetailInfo detail_of(const kpo_candidate& c) {
  DetailInfo x;
  x.name = S(c.name);
  x.score = c.score;
  x.overflow = c.overflow_order;
  x.available = c.available_replicas;
  x.allocatable = c.allocatable_replicas;
  return x;
}
}  // namespace

void kpo_sort_clusters(const kpo_candidate* c, uint32_t n, int with_avail, uint32_t* order) {
  vector<uint32_t> idx(n);
  for (uint32_t i = 0; i < n; i++) idx[i] = i;
  vector<DetailInfo> d;
  for (uint32_t i = 0; i < n; i++) d.push_back(detail_of(c[i]));
  // sortClusters (spreadconstraint/util.go:43-61): overflow asc, score desc, [avail desc], name asc
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
    if (with_avail) return lessDetailAvail(d[a], d[b]);
    if (d[a].overflow != d[b].overflow) return d[a].overflow < d[b].overflow;
    if (d[a].score != d[b].score) return d[a].score > d[b].score;
    return d[a].name < d[b].name;
  });
  for (uint32_t i = 0; i < n; i++) order[i] = idx[i];
}

int kpo_group_clusters(const kp_cluster* clusters, const int64_t* scores, uint32_t n, const kp_binding* b,
                       int32_t avail, uint32_t* order, int32_t* groups) {
  vector<Cluster> cl;
  for (uint32_t i = 0; i < n; i++) {
    bool ok = true;
    cl.push_back(convCluster(clusters[i], (int)i, &ok));
  }
  Binding bb = convBinding(*b);
  vector<std::pair<const Cluster*, i64>> scored;
  vector<i32> est(n, avail);
  for (uint32_t i = 0; i < n; i++) scored.push_back({&cl[i], scores[i]});
  Options o;
  GroupInfoAll info = GroupClustersWithScore(scored, bb, &est, o, KPO_FAST);
  for (size_t i = 0; i < info.clusters.size(); i++) order[i] = (uint32_t)info.clusters[i].cluster->idx;
  // generateZoneInfo / generateProviderInfo (group_clusters.go:380-504): computed by the
  // reference but never read by the selection; their group counts for the unit test
  std::set<string> zones, providers;
  if (!isTopologyIgnored(bb)) {
    for (auto& ci : info.clusters) {
      if (hasSpreadField(bb, "zone"))
        for (auto& z : ci.cluster->zones) zones.insert(z);
      if (hasSpreadField(bb, "provider") && !ci.cluster->provider.empty()) providers.insert(ci.cluster->provider);
    }
  }
  groups[0] = (int32_t)zones.size();
  groups[1] = (int32_t)info.regions.size();
  groups[2] = (int32_t)providers.size();
  return (int)info.clusters.size();
}

int kpo_select_by_region(const kp_str* region_names, const int64_t* region_scores, const uint32_t* off,
                         uint32_t n_regions, const kpo_candidate* cands, int64_t rmin, int64_t rmax, int64_t cmin,
                         int64_t cmax, uint32_t* out) {
  GroupInfoAll info;
  info.has_regions = true;
  std::map<string, vector<uint32_t>> members;
  for (uint32_t r = 0; r < n_regions; r++) {
    RegionInfo ri;
    ri.name = S(region_names[r]);
    ri.score = region_scores[r];
    for (uint32_t k = off[r]; k < off[r + 1]; k++) {
      DetailInfo d = detail_of(cands[k]);
      d.allocatable = (int32_t)k;  // (carries the candidate index through the selection)
      ri.clusters.push_back(d);
      ri.available += d.available;
    }
    info.regions[ri.name] = ri;
  }
  std::map<string, Spread> scm;
  scm["region"] = Spread{"region", "", rmax, rmin};
  scm["cluster"] = Spread{"cluster", "", cmax, cmin};
  SelectResult res = selectByRegion(scm, info);
  if (res.err != KP_ERR_NONE) return -res.err;
  for (size_t i = 0; i < res.clusters.size(); i++) out[i] = (uint32_t)res.clusters[i].allocatable;
  return (int)res.clusters.size();
}

int kpo_select_best(const kpo_candidate* cands, uint32_t n, const kp_binding* b, int32_t need_replicas,
                    uint32_t* out) {
  GroupInfoAll info;
  for (uint32_t i = 0; i < n; i++) {
    DetailInfo d = detail_of(cands[i]);
    d.allocatable = (int32_t)i;
    info.clusters.push_back(d);
  }
  SelectResult res = SelectBestClusters(convBinding(*b), info, need_replicas);
  if (res.err != KP_ERR_NONE) return -res.err;
  for (size_t i = 0; i < res.clusters.size(); i++) out[i] = (uint32_t)res.clusters[i].allocatable;
  return (int)res.clusters.size();
}

int kpo_dynamic_divide(const kp_target_cluster* avail, uint32_t n, int32_t available_replicas, int32_t target,
                       int strategy, const kp_binding* b, int32_t* err_code, kp_target_cluster* out, uint32_t out_cap) {
  vector<TargetCluster> av;
  for (uint32_t i = 0; i < n; i++) av.push_back({S(avail[i].name), avail[i].replicas});
  vector<TargetCluster> scheduled;
  AssignResult r;
  const Strategy st = strategy == 2 ? kAggregated : (strategy == 1 ? kDynamic : kNone);
  if (!dynamicDivide(st, convBinding(*b), av, available_replicas, target, scheduled, &r,
                     KP_ERR_FRESH_NOT_ENOUGH)) {
    *err_code = r.err;
    return -r.status;
  }
  *err_code = KP_ERR_NONE;
  for (size_t i = 0; i < r.targets.size() && i < out_cap; i++) {
    out[i].replicas = r.targets[i].replicas;
    out[i].name = kp_str{nullptr, 0};
    for (uint32_t j = 0; j < n; j++)
      if (S(avail[j].name) == r.targets[i].name) out[i].name = avail[j].name;
  }
  return (int)r.targets.size();
}

void kpo_sort_target_clusters(int32_t* replicas, uint32_t* ids, uint32_t n) {
  vector<TargetCluster> v(n);
  for (uint32_t i = 0; i < n; i++) {
    v[i].replicas = replicas[i];
    v[i].name = std::to_string(ids[i]);
  }
  SortTargetClustersList(v);
  for (uint32_t i = 0; i < n; i++) {
    replicas[i] = v[i].replicas;
    ids[i] = (uint32_t)std::stoul(v[i].name);
  }
}

uint32_t kpo_fnv32a(const char* s, uint32_t len) { return fnv32a(string(s, len)); }


// ---------------------------------------------------------------------------
// Member-cluster nodes
// ---------------------------------------------------------------------------
static ResourceList rl_of(const kp_resource* r, uint32_t n, bool* ok) {
  ResourceList m;
  for (uint32_t i = 0; i < n; i++) {
    Quantity q;
    if (!ParseQuantity(S(r[i].quantity), &q)) *ok = false;
    m[S(r[i].name)] = q;
  }
  return m;
}

// modeling.searchLastLessElement (modeling.go:123-145)
static int SearchLastLessElement(const vector<Quantity>& nums, const Quantity& target) {
  int low = 0, high = (int)nums.size() - 1;
  while (low <= high) {
    int mid = low + ((high - low) >> 1);
    int diff1 = nums[mid].nano < target.nano ? -1 : (nums[mid].nano > target.nano ? 1 : 0);
    int diff2 = 0;
    if (mid != (int)nums.size() - 1)
      diff2 = nums[mid + 1].nano < target.nano ? -1 : (nums[mid + 1].nano > target.nano ? 1 : 0);
    if (diff1 < 1) {
      if (mid == (int)nums.size() - 1 || diff2 == 1) return mid;
      low = mid + 1;
    } else {
      high = mid - 1;
    }
  }
  return -1;
}

// getAllocatableModelings (cluster_status_controller.go:642-677) with
// modeling.InitSummary (modeling.go:75-102), getIndex (:112-121) and
// AddToResourceSummary (:163-223; only the per-grade Quantity is observable).
int kpo_model_grades(const kp_resource_model* models, uint32_t n_models, const kp_node* nodes, uint64_t n_nodes,
                     int64_t* out) {
  if (n_models == 0) return 0;
  vector<string> rsName;
  vector<ResourceList> rsList;
  bool ok = true;
  for (uint32_t g = 0; g < n_models; g++) {
    ResourceList tmp;
    for (uint32_t j = 0; j < models[g].n_ranges; j++) {
      const kp_model_range& it = models[g].ranges[j];
      if (rsName.size() != models[g].n_ranges) rsName.push_back(S(it.name));
      Quantity q;
      if (!ParseQuantity(S(it.min), &q)) ok = false;
      tmp[S(it.name)] = q;
    }
    rsList.push_back(tmp);
  }
  if (!ok) return -1;
  if (!rsName.empty() && !rsList.empty() && rsName.size() != rsList[0].size()) return -1;  // InitSummary error
  if (rsName.empty()) return -1;  // getIndex -> MaxInt: RMs[MaxInt] panics
  vector<vector<Quantity>> sortings(rsName.size());
  for (size_t g = 0; g < rsList.size(); g++)
    for (size_t i = 0; i < rsName.size(); i++) {
      auto it = rsList[g].find(rsName[i]);
      sortings[i].push_back(it == rsList[g].end() ? Quantity() : it->second);
    }
  for (uint32_t g = 0; g < n_models; g++) out[g] = 0;
  for (uint64_t k = 0; k < n_nodes; k++) {
    const kp_node& nd = nodes[k];
    ResourceList alloc = rl_of(nd.allocatable, nd.n_allocatable, &ok);
    if (!ok) return -1;
    // getNodeAvailable (:613-639); nodePodResourcesMap has no entry without pods
    if (nd.n_pods > 0) {
      Resource pr;
      pr.Add(rl_of(nd.requested, nd.n_requested, &ok));
      ResourceList pods1;
      pods1["pods"].nano = (i128)nd.n_pods * 1000000000;
      pr.Add(pods1);  // AddResourcePods
      ResourceList al;  // Resource.ResourceList (resource.go:250-280)
      if (pr.MilliCPU > 0) al["cpu"] = Quantity{(i128)pr.MilliCPU * 1000000, 0};
      if (pr.Memory > 0) al["memory"] = Quantity{(i128)pr.Memory * 1000000000, 1};
      if (pr.EphemeralStorage > 0) al["ephemeral-storage"] = Quantity{(i128)pr.EphemeralStorage * 1000000000, 1};
      if (pr.AllowedPodNumber > 0) al["pods"] = Quantity{(i128)pr.AllowedPodNumber * 1000000000, 0};
      for (auto& kv : pr.Scalar)
        if (kv.second > 0) al[kv.first] = Quantity{(i128)kv.second * 1000000000, kv.first.rfind("hugepages-", 0) == 0 ? 1 : 0};
      auto podsv = [](const ResourceList& m) {
        auto it = m.find("pods");
        return it == m.end() ? (i64)0 : QValue(it->second);
      };
      if (podsv(alloc) - podsv(al) <= 0) break;  // nodeAvailable == nil: the walk stops
      for (auto& kv : al) {
        auto it = alloc.find(kv.first);
        if (it != alloc.end()) it->second.nano -= kv.second.nano;  // Quantity.Sub
      }
    }
    int index = INT32_MAX;  // getIndex
    for (size_t i = 0; i < rsName.size(); i++) {
      auto it = alloc.find(rsName[i]);
      int t = SearchLastLessElement(sortings[i], it == alloc.end() ? Quantity() : it->second);
      if (t < index) index = t;
    }
    if (index == -1) continue;  // no appropriate grade
    out[index] += 1;
  }
  return 0;
}

// ---- estimator server node matching (estimator/server/nodes/filter.go:38-99) ----
// nodeaffinity.RequiredNodeAffinity (vendor/k8s.io/component-helpers/scheduling/
// corev1/nodeaffinity/nodeaffinity.go:39-333): the nodeSelector as
// labels.SelectorFromSet, and the required terms as a LazyErrorNodeSelector.
struct NodeTerm {
  bool parse_err = false;
  bool has_labels = false, has_fields = false;
  vector<Requirement> labels;
  vector<std::pair<string, std::pair<bool, string>>> fields;  // key, (In?, value)
};
struct RequiredNodeAffinity {
  bool has_selector = false;
  LabelSet selector;
  bool has_affinity = false;
  vector<NodeTerm> terms;
};
// GetRequiredNodeAffinity (filter.go:38-57; nodeaffinity.go:306-319)
RequiredNodeAffinity GetRequiredNodeAffinity(const kp_node_claim* c) {
  RequiredNodeAffinity a;
  if (!c) return a;
  for (uint32_t j = 0; j < c->n_node_selector; j++) a.selector[S(c->node_selector[j].key)] = S(c->node_selector[j].value);
  a.has_selector = !a.selector.empty();
  if (!c->has_node_affinity) return a;  // UnmarshalNodeAffinity: no bytes -> nil
  a.has_affinity = true;
  for (uint32_t t = 0; t < c->n_node_affinity_terms; t++) {  // NewLazyErrorNodeSelector
    const kp_node_selector_term& term = c->node_affinity_terms[t];
    if (term.n_match_expressions == 0 && term.n_match_fields == 0) continue;  // isEmptyNodeSelectorTerm
    NodeTerm nt;
    if (term.n_match_expressions) {  // nodeSelectorRequirementsAsSelector (:213-250)
      nt.has_labels = true;
      vector<Req> rs;
      for (uint32_t q = 0; q < term.n_match_expressions; q++) {
        const kp_requirement& r = term.match_expressions[q];
        Req x{S(r.key), S(r.op), {}};
        for (uint32_t j = 0; j < r.n_values; j++) x.values.push_back(S(r.values[j]));
        rs.push_back(x);
      }
      if (!NodeSelectorRequirementsAsSelector(rs, &nt.labels)) nt.parse_err = true;
    }
    if (term.n_match_fields) {  // nodeSelectorRequirementsAsFieldSelector (:257-289)
      nt.has_fields = true;
      for (uint32_t q = 0; q < term.n_match_fields; q++) {
        const kp_requirement& r = term.match_fields[q];
        const string op = S(r.op);
        if ((op != "In" && op != "NotIn") || r.n_values != 1) {
          nt.parse_err = true;
          continue;
        }
        nt.fields.push_back({S(r.key), {op == "In", S(r.values[0])}});
      }
    }
    a.terms.push_back(nt);
  }
  return a;
}
// RequiredNodeAffinity.Match (nodeaffinity.go:321-333) with errors ignored
// (IsNodeAffinityMatched, filter.go:60-64).
bool NodeAffinityMatches(const RequiredNodeAffinity& a, const kp_node& nd) {
  LabelSet labels;
  for (uint32_t j = 0; j < nd.n_labels; j++) labels[S(nd.labels[j].key)] = S(nd.labels[j].value);
  if (a.has_selector)
    for (auto& kv : a.selector) {
      auto it = labels.find(kv.first);
      if (it == labels.end() || it->second != kv.second) return false;
    }
  if (!a.has_affinity) return true;
  std::map<string, string> fields;  // extractNodeFields
  if (nd.name.len) fields["metadata.name"] = S(nd.name);
  for (auto& t : a.terms) {  // LazyErrorNodeSelector.Match: any term
    if (t.parse_err) continue;
    bool ok = true;
    if (t.has_labels)
      for (auto& r : t.labels) ok = ok && ReqMatches(r, labels);
    if (ok && t.has_fields && !fields.empty())
      for (auto& f : t.fields) {
        auto it = fields.find(f.first);
        const string v = it == fields.end() ? string() : it->second;
        ok = ok && ((v == f.second.second) == f.second.first);
      }
    if (ok) return true;
  }
  return false;
}
// IsTolerationMatched (filter.go:66-92)
bool TolerationMatches(const kp_node& nd, const vector<Toleration>& tols) {
  const Taint unsched{"node.kubernetes.io/unschedulable", "", "NoSchedule"};
  bool tolUnsched = false;
  for (auto& t : tols) tolUnsched = tolUnsched || ToleratesTaint(t, unsched);
  if (nd.unschedulable && !tolUnsched) return false;
  for (uint32_t j = 0; j < nd.n_taints; j++) {
    const Taint taint{S(nd.taints[j].key), S(nd.taints[j].value), S(nd.taints[j].effect)};
    if (!(taint.effect == "NoSchedule" || taint.effect == "NoExecute")) continue;
    bool tol = false;
    for (auto& t : tols) tol = tol || ToleratesTaint(t, taint);
    if (!tol) return false;
  }
  return true;
}
vector<Toleration> TolerationsOf(const kp_node_claim* c) {
  vector<Toleration> tols;
  if (c)
    for (uint32_t j = 0; j < c->n_tolerations; j++) {
      const kp_toleration& t = c->tolerations[j];
      tols.push_back(Toleration{S(t.key), S(t.op), S(t.value), S(t.effect)});
    }
  return tols;
}
// getNodeAvailableResource (noderesource.go:135-144)
static bool NodeAvailable(const kp_node& nd, Resource* rest) {
  bool ok = true;
  Resource rq;
  rest->Add(rl_of(nd.allocatable, nd.n_allocatable, &ok));
  rq.Add(rl_of(nd.requested, nd.n_requested, &ok));
  rest->Sub(rq);
  rest->AllowedPodNumber = std::max<i64>(rest->AllowedPodNumber - (i64)nd.n_pods, 0);
  return ok;
}

// SchedulingSimulator (scheduling_simulator_components.go:26-131) over the nodes'
// available resources, literally: each set places every component first-fit from
// the first node, one scan per component per set.
struct NodeSimulator {
  const kp_node* nodes;
  uint64_t n;
  vector<Resource> avail;  // node.Allocatable after getNodeAvailableResource
  struct Comp {
    Resource per;  // requiredPerReplica
    RequiredNodeAffinity aff;
    vector<Toleration> tols;
    int32_t replicas;
  };
  bool init(const kp_node* ns, uint64_t nn) {
    nodes = ns;
    n = nn;
    avail.assign(nn, Resource());
    for (uint64_t i = 0; i < nn; i++)
      if (!NodeAvailable(nodes[i], &avail[i])) return false;
    return true;
  }
  static bool comps_of(const kp_node_component* comps, uint32_t K, vector<Comp>* out) {
    out->assign(K, Comp());
    for (uint32_t k = 0; k < K; k++) {
      bool ok = true;
      Comp& c = (*out)[k];
      if (comps[k].has_replica_requirements) {
        c.per.Add(rl_of(comps[k].resource_request, comps[k].n_resource_request, &ok));
        if (!ok) return false;
        c.aff = GetRequiredNodeAffinity(comps[k].node_claim);
        c.tols = TolerationsOf(comps[k].node_claim);
      }
      c.per.AllowedPodNumber = 1;
      c.replicas = comps[k].replicas;
    }
    return true;
  }
  static Resource multiply(Resource r, i64 f) {  // Resource.Multiply (resource.go:77-94), wrapping
    auto m = [f](i64 v) { return (i64)((uint64_t)v * (uint64_t)f); };
    r.MilliCPU = m(r.MilliCPU);
    r.Memory = m(r.Memory);
    r.EphemeralStorage = m(r.EphemeralStorage);
    r.AllowedPodNumber = m(r.AllowedPodNumber);
    for (auto& kv : r.Scalar) kv.second = m(kv.second);
    return r;
  }
  bool scheduleComponent(const Comp& c) {  // (:95-131)
    int32_t remaining = c.replicas;
    for (uint64_t i = 0; i < n; i++) {
      if (!(NodeAffinityMatches(c.aff, nodes[i]) && TolerationMatches(nodes[i], c.tols))) continue;
      i64 allocatable = avail[i].MaxDivided(c.per);
      if (allocatable == 0) continue;
      if ((i64)remaining < allocatable) allocatable = remaining;
      avail[i].Sub(multiply(c.per, allocatable));
      remaining = (int32_t)(uint32_t)((uint32_t)remaining - (uint32_t)(int32_t)allocatable);
      if (remaining == 0) return true;
    }
    return remaining == 0;
  }
  int32_t SimulateScheduling(const vector<Comp>& cs, int32_t upperBound) {  // (:51-77)
    int32_t complete = 0;
    while (complete < upperBound) {
      bool ok = true;
      for (size_t k = 0; k < cs.size() && ok; k++) ok = scheduleComponent(cs[k]);
      if (!ok) break;
      complete++;
      bool any = false;  // a set of zero-replica components repeats to the bound unchanged
      for (auto& c : cs) any = any || c.replicas != 0;
      if (!any) return upperBound;
    }
    return complete;
  }
  // the assumed-workload deduction (noderesource.go:95-113,166-185)
  bool deduct(const kp_assumed_workload* assumed, uint32_t n_assumed) {
    for (uint32_t w = 0; w < n_assumed; w++) {
      if (assumed[w].n_components == 0) continue;
      vector<Comp> cs;
      if (!comps_of(assumed[w].components, assumed[w].n_components, &cs)) return false;
      SimulateScheduling(cs, 1);
    }
    return true;
  }
};

// nodeResourceEstimator.Estimate (noderesource.go:70-131): the assumed workloads
// deducted, then MatchNode (scheduling_simulator_components.go:149-156) and the
// int32 sum of MaxDivided over the nodes' available resources.
int kpo_node_max_replicas(const kp_node* nodes, uint64_t n_nodes, const kp_resource* request, uint32_t n_request,
                          const kp_node_claim* claim, const kp_assumed_workload* assumed, uint32_t n_assumed,
                          int32_t* out) {
  *out = 0;
  bool ok = true;
  Resource req;
  req.Add(rl_of(request, n_request, &ok));
  if (!ok) return -1;
  NodeSimulator sim;
  if (!sim.init(nodes, n_nodes) || !sim.deduct(assumed, n_assumed)) return -1;
  const RequiredNodeAffinity aff = GetRequiredNodeAffinity(claim);
  const vector<Toleration> tols = TolerationsOf(claim);
  uint32_t res = 0;  // atomic.AddInt32 wraps
  for (uint64_t k = 0; k < n_nodes; k++) {
    if (!(NodeAffinityMatches(aff, nodes[k]) && TolerationMatches(nodes[k], tols))) continue;
    res += (uint32_t)(int32_t)sim.avail[k].MaxDivided(req);
  }
  *out = (int32_t)res;
  return 0;
}

// nodeResourceEstimator.EstimateComponents (noderesource.go:146-190):
// SimulateScheduling(components, MaxInt32) after the deduction; MaxInt32 for an
// empty component list.
int kpo_node_max_component_sets(const kp_node* nodes, uint64_t n_nodes, const kp_node_component* comps, uint32_t K,
                                const kp_assumed_workload* assumed, uint32_t n_assumed, int32_t* out) {
  *out = 0;
  if (K == 0) {
    *out = INT32_MAX;
    return 0;
  }
  NodeSimulator sim;
  if (!sim.init(nodes, n_nodes) || !sim.deduct(assumed, n_assumed)) return -1;
  vector<NodeSimulator::Comp> cs;
  if (!NodeSimulator::comps_of(comps, K, &cs)) return -1;
  *out = sim.SimulateScheduling(cs, INT32_MAX);
  return 0;
}
}  // extern "C"
