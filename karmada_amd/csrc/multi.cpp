// multi.cpp — the multi-GPU engine behind the C-ABI (kp_multi_*, kp_api.h).
//
// One scheduler process owns N devices (SURVEY §8(b) Threading, §8(e)): one
// kp_engine per device (its own HIP streams), the cluster snapshot packed once on
// the first device and replicated onto the others by device-to-device copies over
// xGMI (kp_snapshot_replicate), and each batch cut into contiguous binding shards
// by the §8(e) cost model, one shard per device. Bindings schedule independently
// against one snapshot (no assume/reserve step under the default feature gates),
// so the shards run concurrently — one host thread per device packs its shard and
// drives its engine — with no cross-device exchange on the data path; the shard
// results are merged into one CSR in binding order.
//
// Replaces the single worker of the reference scheduler (pkg/scheduler/scheduler.go:327
// `go wait.Until(s.worker, ...)`), whose scheduleNext loop schedules one binding at a
// time against the cache snapshot.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kp/kp_api.h"

struct kp_multi {
  std::vector<kp_engine*> eng;
  std::vector<int> devices;
  std::string err;
};

struct kp_multi_snapshot {
  kp_multi* m = nullptr;
  std::vector<kp_snapshot*> rep;  // replica per device (rep[0] packed, the others copied)
  uint64_t n_clusters = 0;
  // set when an update failed on some device: the replicas may then describe different
  // cluster states, so batches on it are refused (KP_ESTATE) until it is rebuilt
  bool invalid = false;
  ~kp_multi_snapshot() {
    for (auto* s : rep) kp_snapshot_destroy(s);
  }
};

struct kp_multi_batch {
  const kp_multi_snapshot* snap = nullptr;
  std::vector<uint64_t> start;  // shard d = bindings [start[d], start[d + 1])
  std::vector<kp_batch*> shard;
  // merged results (kp_multi_schedule)
  std::vector<int32_t> status, err;
  std::vector<int64_t> arg;
  std::vector<uint64_t> offsets;
  std::vector<uint32_t> cidx;
  std::vector<int32_t> rep;
  ~kp_multi_batch() {
    for (auto* b : shard) kp_batch_destroy(b);
  }
};

namespace {

// Runs fn(d) for every device d on its own host thread; the first failing device's
// error (prefixed with its device id) goes to m->err.
template <class F>
int each_device(kp_multi* m, F fn) {
  const size_t n = m->eng.size();
  std::vector<int> rc(n, KP_OK);
  if (n == 1) {
    rc[0] = fn(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t d = 0; d < n; d++) th.emplace_back([&, d] { rc[d] = fn((int)d); });
    for (auto& t : th) t.join();
  }
  for (size_t d = 0; d < n; d++)
    if (rc[d] != KP_OK) {
      m->err = "device " + std::to_string(m->devices[d]) + ": " + kp_last_error(m->eng[d]);
      return rc[d];
    }
  return KP_OK;
}

}  // namespace

extern "C" {

int kp_multi_create(const int* devices, uint32_t n, kp_multi** out) {
  if (!devices || n == 0 || !out) return KP_EINVAL;
  auto m = std::make_unique<kp_multi>();
  const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
  for (uint32_t d = 0; d < n; d++) {
    for (uint32_t q = 0; q < d; q++)
      if (devices[q] == devices[d]) return KP_EINVAL;  // one engine per device
    kp_engine* e = nullptr;
    const int rc = kp_engine_create(devices[d], &e);
    if (rc != KP_OK) {
      for (auto* x : m->eng) kp_engine_destroy(x);
      return rc;
    }
    m->eng.push_back(e);
    m->devices.push_back(devices[d]);
  }
  // the devices pack their shards concurrently: split the host threads between them
  const int per = (int)std::max(1u, std::min(16u, hc / n));
  for (auto* e : m->eng) (void)kp_engine_set_threads(e, per);
  *out = m.release();
  return KP_OK;
}

void kp_multi_destroy(kp_multi* m) {
  if (!m) return;
  for (auto* e : m->eng) kp_engine_destroy(e);
  delete m;
}

const char* kp_multi_last_error(const kp_multi* m) { return m ? m->err.c_str() : "null multi engine"; }

uint32_t kp_multi_devices(const kp_multi* m) { return m ? (uint32_t)m->eng.size() : 0u; }

kp_engine* kp_multi_engine(kp_multi* m, uint32_t i) { return m && i < m->eng.size() ? m->eng[i] : nullptr; }

int kp_multi_snapshot_create(kp_multi* m, const kp_cluster* clusters, uint64_t n, const kp_options* opts,
                             kp_multi_snapshot** out) {
  if (!m || !out || (n && !clusters)) return KP_EINVAL;
  auto s = std::make_unique<kp_multi_snapshot>();
  s->m = m;
  s->n_clusters = n;
  s->rep.assign(m->eng.size(), nullptr);
  int rc = kp_snapshot_create(m->eng[0], clusters, n, opts, &s->rep[0]);
  if (rc != KP_OK) {
    m->err = std::string("device ") + std::to_string(m->devices[0]) + ": " + kp_last_error(m->eng[0]);
    return rc;
  }
  for (size_t d = 1; d < m->eng.size(); d++) {
    rc = kp_snapshot_replicate(m->eng[d], s->rep[0], &s->rep[d]);
    if (rc != KP_OK) {
      m->err = std::string("device ") + std::to_string(m->devices[d]) + ": " + kp_last_error(m->eng[d]);
      return rc;
    }
  }
  *out = s.release();
  return KP_OK;
}

// Cluster events on every replica (kp_snapshot_update per device, in parallel); the
// replicas stay identical because each applies the same rows to the same columns.
int kp_multi_snapshot_update(kp_multi* m, kp_multi_snapshot* s, const kp_cluster* clusters, uint64_t n,
                             int* dict_grew) {
  if (!m || !s || s->m != m || (n && !clusters)) return KP_EINVAL;
  if (s->invalid) {
    m->err = "multi snapshot is invalid after a failed update on one device: rebuild it";
    return KP_ESTATE;
  }
  std::vector<int> grew(m->eng.size(), 0);
  const int rc = each_device(m, [&](int d) { return kp_snapshot_update(m->eng[d], s->rep[d], clusters, n, &grew[d]); });
  if (rc != KP_OK) s->invalid = true;  // the other devices may have applied it
  if (dict_grew) *dict_grew = grew[0];
  return rc;
}

void kp_multi_snapshot_destroy(kp_multi_snapshot* s) { delete s; }

kp_snapshot* kp_multi_snapshot_replica(kp_multi_snapshot* s, uint32_t i) {
  return s && i < s->rep.size() ? s->rep[i] : nullptr;
}

// Shard cuts at equal prefix sums of the §8(e) per-binding cost C + Replicas·log2 C
// (the candidate count F_b is bounded by C before the filter runs).
int kp_multi_shard_cuts(const kp_binding* bindings, uint64_t n, uint64_t n_clusters, uint32_t n_shards,
                        uint64_t* starts) {
  if (!starts || n_shards == 0 || (n && !bindings)) return KP_EINVAL;
  const double lg = std::log2((double)std::max<uint64_t>(2, n_clusters));
  std::vector<double> pre(n + 1, 0.0);
  for (uint64_t i = 0; i < n; i++)
    pre[i + 1] = pre[i] + (double)n_clusters + (double)std::max<int32_t>(0, bindings[i].replicas) * lg;
  starts[0] = 0;
  uint64_t j = 0;
  for (uint32_t d = 1; d < n_shards; d++) {
    const double want = pre[n] * (double)d / (double)n_shards;
    while (j < n && pre[j] < want) j++;
    starts[d] = std::max(j, starts[d - 1]);
  }
  starts[n_shards] = n;
  return KP_OK;
}

int kp_multi_batch_create(kp_multi* m, const kp_multi_snapshot* s, const kp_binding* bindings, uint64_t n,
                          kp_multi_batch** out) {
  if (!m || !s || s->m != m || !out || (n && !bindings)) return KP_EINVAL;
  if (s->invalid) {
    m->err = "multi snapshot is invalid after a failed update on one device: rebuild it";
    return KP_ESTATE;
  }
  const uint32_t D = (uint32_t)m->eng.size();
  auto b = std::make_unique<kp_multi_batch>();
  b->snap = s;
  b->start.assign(D + 1, 0);
  (void)kp_multi_shard_cuts(bindings, n, s->n_clusters, D, b->start.data());
  b->shard.assign(D, nullptr);
  const int rc = each_device(m, [&](int d) {
    return kp_batch_create(m->eng[d], s->rep[d], bindings + b->start[d], b->start[d + 1] - b->start[d], &b->shard[d]);
  });
  if (rc != KP_OK) return rc;
  *out = b.release();
  return KP_OK;
}

void kp_multi_batch_destroy(kp_multi_batch* b) { delete b; }

int kp_multi_batch_shards(const kp_multi_batch* b, uint64_t* starts) {
  if (!b || !starts) return KP_EINVAL;
  std::copy(b->start.begin(), b->start.end(), starts);
  return KP_OK;
}

int kp_multi_schedule(kp_multi* m, kp_multi_batch* b, kp_results* out) {
  if (!m || !b || !out || b->snap->m != m) return KP_EINVAL;
  if (b->snap->invalid) {
    m->err = "multi snapshot is invalid after a failed update on one device: rebuild it";
    return KP_ESTATE;
  }
  const uint32_t D = (uint32_t)m->eng.size();
  std::vector<kp_results> r(D);
  int rc = each_device(m, [&](int d) { return kp_schedule_batch(m->eng[d], b->shard[d], &r[d]); });
  if (rc != KP_OK) return rc;
  const uint64_t B = b->start[D];
  std::vector<uint64_t> tbase(D + 1, 0);
  for (uint32_t d = 0; d < D; d++) tbase[d + 1] = tbase[d] + r[d].n_targets;
  b->status.resize(B);
  b->err.resize(B);
  b->arg.resize(B);
  b->offsets.resize(B + 1);
  b->cidx.resize(std::max<uint64_t>(1, tbase[D]));
  b->rep.resize(std::max<uint64_t>(1, tbase[D]));
  // each device's part copied by its own thread
  rc = each_device(m, [&](int d) {
    const uint64_t lo = b->start[d], nb = b->start[d + 1] - lo, t0 = tbase[d];
    if (nb) {
      memcpy(b->status.data() + lo, r[d].status, 4 * nb);
      memcpy(b->err.data() + lo, r[d].err_code, 4 * nb);
      memcpy(b->arg.data() + lo, r[d].err_arg, 8 * nb);
      for (uint64_t i = 0; i < nb; i++) b->offsets[lo + i] = t0 + r[d].offsets[i];
    }
    if (r[d].n_targets) {
      memcpy(b->cidx.data() + t0, r[d].cluster_idx, 4 * r[d].n_targets);
      memcpy(b->rep.data() + t0, r[d].replicas, 4 * r[d].n_targets);
    }
    return KP_OK;
  });
  b->offsets[B] = tbase[D];
  out->n_bindings = B;
  out->status = b->status.data();
  out->err_code = b->err.data();
  out->err_arg = b->arg.data();
  out->offsets = b->offsets.data();
  out->cluster_idx = b->cidx.data();
  out->replicas = b->rep.data();
  out->n_targets = tbase[D];
  return rc;
}

}  // extern "C"
