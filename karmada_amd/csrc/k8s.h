// k8s.h — host-side restatements of the Kubernetes value semantics the packer
// needs (vendor/k8s.io/apimachinery @ v0.36.2, as vendored by the reference):
//   resource.Quantity parsing and Value()/MilliValue() rounding
//     (api/resource/quantity.go:161-394, 813-835; math.go:166-199)
//   label key / value validation (api/validate/content/kube.go, dns.go)
//   strconv.ParseInt base 10
#pragma once
#include <stdint.h>

#include <cstring>
#include <string>
#include <string_view>

namespace kp {
namespace k8s {

typedef __int128 i128;

// Exact quantity value in units of 1e-9 (ParseQuantity rounds to Nano away from zero).
struct Qty {
  i128 nano = 0;
  int fmt = 0;  // resource.Format: 0 DecimalSI, 1 BinarySI, 2 DecimalExponent
};

inline i128 p10(int k) {
  i128 r = 1;
  while (k-- > 0) r *= 10;
  return r;
}
inline int64_t round_away(i128 nano, i128 div) {
  if (nano >= 0) return (int64_t)((nano + div - 1) / div);
  return -(int64_t)(((-nano) + div - 1) / div);
}
inline int64_t value(const Qty& q) { return round_away(q.nano, (i128)1000000000); }
inline int64_t milli(const Qty& q) { return round_away(q.nano, (i128)1000000); }
// quantityAsInt64 (estimator/client/general.go:417-427): DecimalSI/DecimalExponent ->
// MilliValue, BinarySI -> Value
inline int64_t as_int64(const Qty& q) { return q.fmt == 1 ? value(q) : milli(q); }
// Quantity.Sub: a zero receiver takes the subtrahend's format
inline void qsub(Qty& a, const Qty& y) {
  if (a.nano == 0) a.fmt = y.fmt;
  a.nano -= y.nano;
}

inline bool parse_quantity(std::string_view str, Qty* out) {
  if (str.empty()) return false;
  if (str == "0") {
    out->nano = 0;
    out->fmt = 0;
    return true;
  }
  size_t pos = 0, end = str.size();
  bool positive = true;
  if (str[0] == '-' || str[0] == '+') {
    positive = str[0] != '-';
    pos = 1;
  }
  while (pos < end && str[pos] == '0') pos++;
  std::string_view num, denom, suf;
  size_t i = pos;
  while (i < end && str[i] >= '0' && str[i] <= '9') i++;
  num = str.substr(pos, i - pos);
  if (num.empty()) num = "0";
  pos = i;
  if (pos < end && str[pos] == '.') {
    pos++;
    size_t j = pos;
    while (j < end && str[j] >= '0' && str[j] <= '9') j++;
    denom = str.substr(pos, j - pos);
    pos = j;
  }
  if (pos < end) {  // suffix: [eEinumkKMGTP]* [+-]? digits*
    size_t k = pos;
    while (k < end && strchr("eEinumkKMGTP", str[k])) k++;
    size_t q = k;
    if (q < end && (str[q] == '+' || str[q] == '-')) q++;
    while (q < end && str[q] >= '0' && str[q] <= '9') q++;
    if (q != end) return false;
    suf = str.substr(pos);
  }
  int64_t ex = 0;
  bool binary = false;
  static const char* dec[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int dece[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bin[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool found = false;
  for (int t = 0; t < 10 && !found; t++)
    if (suf == dec[t]) {
      ex = dece[t];
      found = true;
    }
  for (int t = 0; t < 6 && !found; t++)
    if (suf == bin[t]) {
      ex = 10 * (t + 1);
      binary = true;
      found = true;
    }
  int fmt = binary ? 1 : 0;
  if (!found) {
    if (suf.size() > 1 && suf.size() < 32 && (suf[0] == 'e' || suf[0] == 'E')) {
      char buf[32];
      memcpy(buf, suf.data() + 1, suf.size() - 1);
      buf[suf.size() - 1] = 0;
      char* e = nullptr;
      long long v = strtoll(buf, &e, 10);
      if (e == buf || *e) return false;
      ex = (int32_t)v;
      fmt = 2;
    } else {
      return false;
    }
  }
  const i128 lim = (i128)1 << 100;
  i128 m = 0;
  for (std::string_view part : {num, denom})
    for (char c : part) {
      if (m > lim) return false;
      m = m * 10 + (c - '0');
    }
  i128 nano;
  if (!binary) {
    int64_t sc = 9 + ex - (int64_t)denom.size();
    if (sc >= 0) {
      if (sc > 30 && m != 0) return false;
      nano = m * p10((int)(sc > 30 ? 0 : sc));
      if (m != 0 && nano / p10((int)sc) != m) return false;
    } else {
      int64_t k = -sc;
      nano = k > 36 ? (m != 0 ? 1 : 0) : (m + p10((int)k) - 1) / p10((int)k);
    }
  } else {
    i128 v = m;
    for (int64_t t = 0; t < ex; t++) {
      v *= 2;
      if (v > lim * 1000) return false;
    }
    int64_t sc = 9 - (int64_t)denom.size();
    nano = sc >= 0 ? v * p10((int)sc) : (v + p10((int)-sc) - 1) / p10((int)-sc);
    const i128 cap = (i128)INT64_MAX * 1000000000;  // BinarySI maxAllowed (quantity.go:373-376)
    if (nano > cap) nano = cap;
  }
  if (nano > lim) return false;
  out->nano = positive ? nano : -nano;
  out->fmt = fmt;
  return true;
}

inline bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
inline bool lower_alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }
inline bool label_fmt(std::string_view s) {
  if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
inline bool dns1123_subdomain(std::string_view s) {
  if (s.empty() || s.size() > 253) return false;
  size_t st = 0;
  for (;;) {
    size_t d = s.find('.', st);
    std::string_view l = s.substr(st, d == std::string_view::npos ? std::string_view::npos : d - st);
    if (l.empty() || !lower_alnum(l.front()) || !lower_alnum(l.back())) return false;
    for (char c : l)
      if (!(lower_alnum(c) || c == '-')) return false;
    if (d == std::string_view::npos) return true;
    st = d + 1;
  }
}
inline bool label_key(std::string_view v) {  // content.IsLabelKey
  size_t sl = v.find('/');
  std::string_view name = v;
  if (sl != std::string_view::npos) {
    if (v.find('/', sl + 1) != std::string_view::npos) return false;
    std::string_view pre = v.substr(0, sl);
    name = v.substr(sl + 1);
    if (pre.empty() || !dns1123_subdomain(pre)) return false;
  }
  if (name.empty() || name.size() > 63) return false;
  return label_fmt(name);
}
inline bool label_value(std::string_view v) {  // content.IsLabelValue
  if (v.size() > 63) return false;
  return v.empty() || label_fmt(v);
}
inline bool parse_int64(std::string_view s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    if (s.size() == 1) return false;
    i = 1;
  }
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(i128)v) : (int64_t)v;
  return true;
}
// lifted.IsScalarResourceName (pkg/util/lifted/resourcename.go:31-34, corev1helpers.go:39-82)
inline bool scalar_resource(const std::string& n) {
  bool native = n.find('/') == std::string::npos || n.find("kubernetes.io/") != std::string::npos;
  bool extended = !native && n.rfind("requests.", 0) != 0 && label_key(std::string("requests.") + n);
  return extended || n.rfind("hugepages-", 0) == 0 || n.find("kubernetes.io/") != std::string::npos ||
         n.rfind("attachable-volumes-", 0) == 0;
}
inline uint32_t fnv32a(const char* p, size_t n) {
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n; i++) {
    h ^= (unsigned char)p[i];
    h *= 16777619u;
  }
  return h;
}

}  // namespace k8s
}  // namespace kp
