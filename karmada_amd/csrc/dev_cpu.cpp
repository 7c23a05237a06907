// dev_cpu.cpp — TEST-ONLY host implementation of kp_dev.h (libkp_cpusim.so).
//
// Runs the kernel bodies of kp_kernels.h with the 1-thread CpuBlk policy, one
// "workgroup" at a time per host thread, so tests/ can check the engine's
// orchestration and kernel logic against the oracle without a GPU. It is never
// linked into libkp.so and the product loader (karmada_amd/engine.py) never
// loads it.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "kp_dev.h"
#include "kp_sets.h"
#include "kp_kernels.h"
#include "kp_top.h"

namespace kp {
namespace dev {

namespace {
int threads() {
  const char* e = getenv("KP_CPUSIM_THREADS");
  int n = e ? atoi(e) : 1;
  return n < 1 ? 1 : n;
}
// GPU LDS is not zeroed at launch and keeps whatever the previous workgroup on
// the CU left: every "workgroup" here starts from a poison pattern (0xA5 bytes,
// KP_CPUSIM_POISON=0 turns it off), so a read of LDS the kernel never wrote
// gives garbage here as it would on the device, not a convenient zero.
bool poison() {
  static const bool on = [] {
    const char* e = getenv("KP_CPUSIM_POISON");
    return !(e && e[0] == '0');
  }();
  return on;
}
// Runs fn(blk, smem) for blk in [0, n) on the configured host threads.
template <class F>
void grid(int n, size_t smem_bytes, F fn) {
  int T = threads();
  if (T > n) T = n;
  std::atomic<int> next(0);
  const bool pz = poison();
  auto work = [&]() {
    std::vector<int64_t> smem((smem_bytes + kRedBytes + 7) / 8);
    for (;;) {
      int b = next.fetch_add(1);
      if (b >= n) break;
      if (pz) memset(smem.data(), 0xA5, smem.size() * 8);
      fn(b, (unsigned char*)smem.data());
    }
  };
  if (T <= 1) {
    work();
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back(work);
  for (auto& t : th) t.join();
}
struct Ev {
  double ms;
};
}  // namespace

// Emulated devices (the multi-device engine's tests): KP_CPUSIM_DEVICES, default 8.
int device_count() {
  const char* e = getenv("KP_CPUSIM_DEVICES");
  const int n = e ? atoi(e) : 8;
  return n < 1 ? 1 : n;
}
int set_device(int) { return 0; }
size_t max_lds_per_block(int) { return 160 * 1024; }
const char* last_error() { return "cpusim error"; }
int stream_create(stream_t* s) {
  *s = (void*)1;
  return 0;
}
void stream_destroy(stream_t) {}
int sync(stream_t) { return 0; }
int event_create(event_t* e) {
  *e = new Ev{0};
  return 0;
}
void event_destroy(event_t e) { delete (Ev*)e; }
int event_record(event_t e, stream_t) {
  ((Ev*)e)->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  return 0;
}
int stream_wait(stream_t, event_t) { return 0; }
int event_sync(event_t) { return 0; }
float event_ms(event_t a, event_t b) { return (float)(((Ev*)b)->ms - ((Ev*)a)->ms); }
// Device memory is poisoned like LDS: a pooled arena block on the GPU holds the
// previous batch's data, so nothing may rely on a zeroed allocation.
int alloc(void** p, size_t bytes) {
  *p = malloc(bytes ? bytes : 1);
  if (*p && poison()) memset(*p, 0xA5, bytes ? bytes : 1);
  return *p ? 0 : -1;
}
void release(void* p) { free(p); }
int host_alloc(void** p, size_t bytes) { return alloc(p, bytes); }
void host_release(void* p) { free(p); }
int h2d(void* dst, const void* src, size_t bytes, stream_t) {
  if (bytes) memcpy(dst, src, bytes);
  return 0;
}
int d2h(void* dst, const void* src, size_t bytes, stream_t) {
  if (bytes) memcpy(dst, src, bytes);
  return 0;
}
int peer_copy(void* dst, int, const void* src, int, size_t bytes, stream_t) {
  if (bytes) memcpy(dst, src, bytes);
  return 0;
}
int fill(void* dst, int value, size_t bytes, stream_t) {
  if (bytes) memset(dst, value, bytes);
  return 0;
}

int pair(stream_t, const SnapView& s, const BatchView& bv, const int32_t* list, int b0, int nb, uint64_t* fmask,
         int32_t* est, int64_t* score, int est_mode, int md_cap, size_t smem, int fast) {
  grid(nb, smem, [&](int blk, unsigned char* sm) {
    const CpuBlk B{(int64_t*)sm};
    switch (fast) {
      case EST_MIXED: body_pair<EST_MIXED>(B, blk, sm, s, bv, list, b0, fmask, est, score, est_mode, md_cap); break;
      case EST_SUMMARY: body_pair<EST_SUMMARY>(B, blk, sm, s, bv, list, b0, fmask, est, score, est_mode, md_cap); break;
      case EST_MODEL8: body_pair<EST_MODEL8>(B, blk, sm, s, bv, list, b0, fmask, est, score, est_mode, md_cap); break;
      case EST_MODEL16: body_pair<EST_MODEL16>(B, blk, sm, s, bv, list, b0, fmask, est, score, est_mode, md_cap); break;
      default: body_pair<EST_GENERIC>(B, blk, sm, s, bv, list, b0, fmask, est, score, est_mode, md_cap);
    }
  });
  return 0;
}

int est_class(stream_t, const SnapView& s, const BatchView& bv, const int32_t* rep, int n_rows, int32_t* rows,
              int fast, const int32_t* klist, const uint64_t* fmask) {
  grid(n_rows, 4 * kTmplDense + (fmask ? 4 * (size_t)s.Cp : 0), [&](int i, unsigned char* sm) {
    const CpuBlk B{(int64_t*)sm};
    const int k = klist ? klist[i] : i;
    switch (fast) {
      case EST_MIXED: body_est_class<EST_MIXED>(B, k, sm, s, bv, rep, rows, fmask); break;
      case EST_SUMMARY: body_est_class<EST_SUMMARY>(B, k, sm, s, bv, rep, rows, fmask); break;
      case EST_MODEL8: body_est_class<EST_MODEL8>(B, k, sm, s, bv, rep, rows, fmask); break;
      case EST_MODEL16: body_est_class<EST_MODEL16>(B, k, sm, s, bv, rep, rows, fmask); break;
      default: break;
    }
  });
  return fast == EST_MIXED || fast == EST_SUMMARY || fast == EST_MODEL8 || fast == EST_MODEL16 ? 0 : -1;
}

int filter(stream_t, const SnapView& s, const BatchView& bv, uint64_t* fmask) {
  grid(bv.B, 0, [&](int b, unsigned char* sm) { body_filter(CpuBlk{(int64_t*)sm}, b, s, bv, fmask); });
  return 0;
}

int select(stream_t, int which, const KArgs& a, size_t smem, int cap, const SelectExtra& x) {
  switch (which) {
    case SEL_LAUNCH_ALL: {
      const int n = a.n_dev ? (int)*a.n_dev : a.n;
      const size_t need = kRedBytes + 4 * (size_t)((((a.s.Cp + 31) >> 5) + 3) & ~3) + 8 * (size_t)a.s.Cp + 3072 +
                          8 * (size_t)sel_all_ecap(a.s.Cp) + 64;
      grid(n, need > smem ? need : smem,
           [&](int blk, unsigned char* sm) { body_select_all(CpuBlk{(int64_t*)sm}, blk, sm, a); });
      break;
    }
    case SEL_LAUNCH_ALL_STREAM:
      grid(a.n_dev ? (int)*a.n_dev : a.n, smem,
           [&](int blk, unsigned char* sm) { body_select_all_stream(CpuBlk{(int64_t*)sm}, blk, sm, a); });
      break;
    case SEL_LAUNCH_CLUSTER:
      grid(a.n_dev ? (int)*a.n_dev : a.n, smem, [&](int j, unsigned char* sm) {
        body_select_cluster(CpuBlk{(int64_t*)sm}, a.sub ? a.sub[j] : j, sm, a, cap);
      });
      break;
    case SEL_LAUNCH_REGION_A:
      grid(a.n_dev ? (int)*a.n_dev : a.n, smem, [&](int j, unsigned char* sm) {
        body_region_a(CpuBlk{(int64_t*)sm}, a.sub ? a.sub[j] : j, sm, a, x.rout, x.rstat);
      });
      break;
    case SEL_LAUNCH_REGION_B:
      grid(a.n_dev ? (int)*a.n_dev : a.n, smem, [&](int j, unsigned char* sm) {
        body_region_b(CpuBlk{(int64_t*)sm}, a.sub ? a.sub[j] : j, sm, a, x.rsel, x.rnsel, x.rout, cap);
      });
      break;
    case SEL_LAUNCH_SLOW: {
      // On the GPU the flagged list's order is the order of the device atomics that
      // appended it, so which bindings follow each other in one workgroup's slot
      // varies from run to run. KP_CPUSIM_SLOW_SHUFFLE=<seed> permutes the list and
      // KP_CPUSIM_SLOW_GRID=<g> narrows the grid, to replay such orders here.
      if (const char* sh = getenv("KP_CPUSIM_SLOW_SHUFFLE")) {
        uint64_t r = (uint64_t)atoll(sh) * 0x9E3779B97F4A7C15ull + 1;
        const int ns = (int)std::min<uint32_t>(a.stats[0], (uint32_t)a.n);
        for (int i = ns - 1; i > 0; i--) {
          r ^= r << 13, r ^= r >> 7, r ^= r << 17;
          std::swap(a.slow_ids[i], a.slow_ids[(int)(r % (uint64_t)(i + 1))]);
        }
      }
      int g = x.grid;
      if (const char* sg = getenv("KP_CPUSIM_SLOW_GRID")) g = std::max(1, std::min(g, atoi(sg)));
      grid(g, smem, [&](int blk, unsigned char* sm) {
        body_slow(CpuBlk{(int64_t*)sm}, blk, g, sm, a, x.scratch, x.slot_bytes, cap, x.lds_area, x.lds_sort);
      });
      break;
    }
    default:
      return -1;
  }
  return 0;
}

int class_order(stream_t, const SnapView& s, const int32_t* rows, int n_rows, uint64_t* ord, int64_t* tot,
                int32_t* ok) {
  int P = 1;
  while (P < s.C) P <<= 1;
  grid(n_rows, 8 * (size_t)P, [&](int k, unsigned char* sm) {
    body_class_order(CpuBlk{(int64_t*)sm}, k, (uint64_t*)(sm + kRedBytes), P, s, rows, ord, tot, ok);
  });
  return 0;
}

int select_top(stream_t, const KArgs& a, const TopArgs& t, size_t slice, int) {
  grid(a.n_dev ? (int)*a.n_dev : a.n, slice, [&](int blk, unsigned char* sm) { body_select_top(CpuBlk{(int64_t*)sm}, blk, sm, a, t); });
  return 0;
}
int select_top_wg(stream_t, const KArgs& a, const TopArgs& t, size_t smem) {
  grid(a.n, smem, [&](int blk, unsigned char* sm) {
    body_select_top_wg(CpuBlk{(int64_t*)sm}, CpuBlk{(int64_t*)top_wg_slice(sm)}, blk, sm, a, t);
  });
  return 0;
}

int region_groups(stream_t, const RegionOut* rout, const int32_t* rstat, const BindHdr* hdr, const int32_t* list,
                  int n, int R, int32_t* rsel, int32_t* rnsel, uint32_t* nhost) {
  for (int j = 0; j < n; j++) {
    const int32_t k = region_groups_one(rout + (size_t)j * R, rstat[j], hdr[list[j]], R, rsel + (size_t)j * R);
    if (k == kGroupsHost) ++*nhost;
    rnsel[j] = k;
  }
  return 0;
}

int component_sets(stream_t, const SnapView& s, const SetsArgs* A, const int32_t* ranks, const int64_t* off,
                   uint64_t n, int64_t* scratch, int32_t* out) {
  for (uint64_t i = 0; i < n; i++) body_sets(s, A, ranks, off, i, scratch, out);
  return 0;
}

int sets_rows(stream_t, const SnapView& s, const SetsArgs* A, const int64_t* off, int64_t* scratch, int32_t* row,
              uint32_t* ovf) {
  for (int r = 0; r < s.C; r++) body_sets_row(s, *A, off, r, scratch, row, ovf);
  return 0;
}

int rows_from_class(stream_t, const SnapView& s, const BatchView& bv, const int32_t* list, int n, const int32_t* bcls,
                    const int32_t* cls_rows, const uint64_t* fmask, int32_t* est) {
  grid(n, 0, [&](int blk, unsigned char* sm) {
    body_rows_from_class(CpuBlk{(int64_t*)sm}, blk, s, bv, list, bcls, cls_rows, fmask, est);
  });
  return 0;
}

int grades(stream_t, const GradesArgs& A) {
  for (uint64_t i = 0; i < A.n; i++) body_grades(A, i);
  return 0;
}

int node_est(stream_t, const NodeEstArgs& A) {
  uint32_t s = 0;
  for (uint64_t i = 0; i < A.v.n; i++) s += (uint32_t)node_replicas(A, i);
  *A.sum += s;
  return 0;
}

int spread_order(stream_t, const KArgs& a, const OrderArgs& o, size_t slice) {
  grid(a.n, slice, [&](int blk, unsigned char* sm) { body_spread_order(CpuBlk{(int64_t*)sm}, blk, sm, a, o); });
  return 0;
}

int region_a_order(stream_t, const KArgs& a, RegionOut* rout, int32_t* rstat, int32_t* fb, uint32_t* fb_n,
                   size_t slice) {
  grid(a.n, slice, [&](int blk, unsigned char* sm) {
    body_region_a_order(CpuBlk{(int64_t*)sm}, blk, sm, a, rout, rstat, fb, fb_n);
  });
  return 0;
}

int select_static(stream_t, const KArgs& a, size_t slice) {
  grid(a.n, slice, [&](int blk, unsigned char* sm) { body_select_static(CpuBlk{(int64_t*)sm}, blk, sm, a); });
  return 0;
}

int node_match(stream_t, const NodeView& v, const ClaimProg* P, int K, uint8_t* match) {
  const uint64_t n = v.n * (uint64_t)K;
  for (uint64_t i = 0; i < n; i++) body_node_match(v, P, i, match);
  return 0;
}

int node_sets(stream_t, const NodeSetsArgs* A) {
  int64_t red[2];
  kp::node_sets(CpuBlk{red}, *A);
  return 0;
}

int reasons(stream_t, const SnapView& s, const BatchView& bv, int b0, int nb, uint32_t* out) {
  const uint64_t n = (uint64_t)nb * (uint64_t)s.C;
  for (uint64_t i = 0; i < n; i++) body_reasons(s, bv, b0, i, out);
  return 0;
}

int offsets(stream_t, const int32_t* status, const uint32_t* count, int n, uint64_t* off, uint64_t* part) {
  int64_t red[8];
  const int nb = (n + kOffChunk - 1) / kOffChunk;
  for (int k = 0; k < nb; k++) body_offsets_a(CpuBlk{red}, k, status, count, n, off, part);
  for (int k = 0; k < nb; k++) body_offsets_b(CpuBlk{red}, k, nb, n, off, part);
  return 0;
}

int compact(stream_t, const uint64_t* start, const uint32_t* count, const uint64_t* offsets, const uint32_t* in_idx,
            const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n, const uint32_t* perm, uint32_t* h_idx,
            int32_t* h_rep, uint64_t h_cap) {
  int64_t red[8];
  for (int b = 0; b < n; b++)
    body_compact(CpuBlk{red}, b, start, count, offsets, in_idx, in_rep, out_idx, out_rep, n, perm, h_idx, h_rep, h_cap);
  return 0;
}
int host_device_ptr(void* host, void** dev) {
  *dev = host;
  return 0;
}

}  // namespace dev
}  // namespace kp

// ---------------------------------------------------------------------------
// Test-only entry points into single kernel helpers (tests/test_cpusim_units.py)
// ---------------------------------------------------------------------------
extern "C" {

// webster_par over n parties with the given votes (>= 0, < 2^31) and ranks
// (name order); seats per party into out. ecap: enumeration capacity (0 =
// bisection only).
int kpsim_webster(const int32_t* votes, const uint32_t* ranks, int n, int32_t N, int desc, int ecap, int32_t* out) {
  using namespace kp;
  std::vector<uint32_t> r(n);
  std::vector<int32_t> v(n);
  for (int i = 0; i < n; i++) {
    r[i] = ranks[i];
    v[i] = votes[i];
  }
  std::vector<uint32_t> hist(256);
  std::vector<unsigned long long> wh(256);
  std::vector<uint64_t> buf(ecap > 0 ? ecap : 1);
  SelScratch ss{hist.data(), wh.data(), buf.data(), ecap};
  int64_t red[8];
  CpuBlk B{red};
  auto parties = [&](auto fn) {
    for (int i = 0; i < n; i++) fn(r[i], (int64_t)v[i]);
  };
  WebRes w = webster_par(B, parties, N, desc != 0, ss);
  for (int i = 0; i < n; i++) out[i] = web_seats(w, v[i], r[i]);
  return w.mode;
}

// webster_serial (k_slow's exact AllocateWebsterSeats) over n parties with int64
// votes of any sign and ranks (name order); seats per party into out.
void kpsim_webster_serial(const int64_t* votes, const uint32_t* ranks, int n, int32_t N, int desc, int32_t* out) {
  std::vector<int32_t> heap(n > 0 ? n : 1);
  kp::webster_serial(ranks, votes, out, heap.data(), n, N, desc != 0);
}

// MergeTargetClusters (pkg/util/binding.go:91-115) as SerialAssign::merge does it:
// old = (on, orr)[0, no), new = (nn, nr)[0, nw); result into (out_n, out_r), returns
// its length (<= no + nw).
int kpsim_merge_targets(const uint32_t* on, const int32_t* orr, int no, const uint32_t* nn, const int32_t* nr, int nw,
                        uint32_t* out_n, int32_t* out_r) {
  using namespace kp;
  const int cap = no + nw + 1;
  std::vector<unsigned char> mem(serial_scratch_bytes(cap));
  SerialScratch sc = serial_scratch_carve(mem.data(), cap);
  for (int i = 0; i < no; i++) sc.sn[i] = on[i], sc.sr[i] = orr[i];
  for (int i = 0; i < nw; i++) sc.tn[i] = nn[i], sc.tr[i] = nr[i];
  SelCtx x{};
  SerialAssign sa{x, sc, false};
  const int k = sa.merge(no, nw);
  for (int i = 0; i < k; i++) out_n[i] = sc.tn[i], out_r[i] = sc.tr[i];
  return k;
}

// wsel_max over values (>= 0): largest v* with sum{v_i >= v*} >= target.
int64_t kpsim_wsel_max(const int32_t* vals, int n, int64_t target) {
  using namespace kp;
  std::vector<unsigned long long> wh(256);
  int64_t red[8];
  CpuBlk B{red};
  auto vs = [&](auto fn) {
    for (int i = 0; i < n; i++) fn((int64_t)vals[i]);
  };
  return wsel_max(B, wh.data(), vs, target);
}

// select_groups_dev over n regions (ids 0..n-1 in name order; value = #clusters,
// 0 = region absent; weight = group score). Returns the count or -KP_ERR_*.
int kpsim_select_groups(const int32_t* values, const int64_t* weights, int n, int64_t min_c, int64_t max_c,
                        int64_t target, int32_t* out) {
  using namespace kp;
  std::vector<RegionOut> ro(n);
  for (int r = 0; r < n; r++) ro[r] = RegionOut{values[r], 0, weights[r]};
  return select_groups_dev(ro.data(), n, min_c, max_c, target, out);
}

// Go sort.Sort over (name, rep)[0, n): mode 0 = the serial emulation
// (pdqsort_go), mode 1 = the wave form (PdqWave, one lane). Returns 1 if the
// wave form emulated it (0: it declined), in place.
int kpsim_sort_tcl(uint32_t* name, int32_t* rep, int n, int mode) {
  using namespace kp;
  if (mode == 0) {
    sort_tcl(name, rep, n);
    return 1;
  }
  std::vector<unsigned char> lds(pdq_wave_bytes(n));
  int64_t red[8];
  CpuBlk B{red};
  PdqWave<CpuBlk> pw = pdq_carve(B, lds.data(), n);
  for (int i = 0; i < n; i++) {
    pw.name[i] = name[i];
    pw.rep[i] = rep[i];
  }
  if (!pw.run(n)) return 0;
  for (int i = 0; i < n; i++) {
    name[i] = pw.name[i];
    rep[i] = pw.rep[i];
  }
  return 1;
}

}  // extern "C"
