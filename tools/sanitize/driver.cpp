// driver.cpp — sanitizer run of the engine's host code (test infrastructure).
//
// Builds engine.cpp + dev_cpu.cpp (the kernel bodies on host threads: the CPU-sim
// device layer), the synthetic universes (synth.cpp) and the oracle (oracle.cpp)
// into one program, instrumented with ThreadSanitizer or AddressSanitizer +
// UndefinedBehaviorSanitizer (tools/sanitize/Makefile). It schedules seeded
// universes of every workload with KP_CPUSIM_THREADS concurrent "workgroups" and
// checks each binding against the oracle (status, error, argument, multiset of
// targets). Exit code 0 = no mismatch (the sanitizers abort on their own findings).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <tuple>
#include <vector>

#include "../../include/kp/kp_api.h"
#include "../../oracle/oracle.h"

struct kps_world;
extern "C" {
int kps_create(int config, uint64_t seed, uint32_t n_clusters, uint64_t b_lo, uint64_t b_hi, kps_world** out);
void kps_destroy(kps_world* w);
const kp_cluster* kps_clusters(const kps_world* w, uint64_t* n);
const kp_binding* kps_bindings(const kps_world* w, uint64_t* n);
}

typedef std::vector<std::pair<uint32_t, int32_t>> Targets;

static Targets targets_of(const uint64_t* off, const uint32_t* idx, const int32_t* rep, uint64_t i) {
  Targets t;
  for (uint64_t k = off[i]; k < off[i + 1]; k++) t.push_back({idx[k], rep[k]});
  std::sort(t.begin(), t.end());
  return t;
}

static int run_case(kp_engine* e, int config, uint64_t seed, uint32_t C, uint64_t B, bool multi) {
  kps_world* w = nullptr;
  if (kps_create(config, seed, C, 0, B, &w)) return 1;
  uint64_t nc = 0, nb = 0;
  const kp_cluster* cl = kps_clusters(w, &nc);
  const kp_binding* bs = kps_bindings(w, &nb);
  kp_options o{};
  o.customized_cluster_resource_modeling = 1;
  o.multiple_pod_templates_scheduling = multi ? 1 : 0;
  o.enabled_plugins = KP_PLUGIN_ALL;
  kp_snapshot* s = nullptr;
  kp_batch* b = nullptr;
  kp_results r{};
  int bad = 0;
  if (kp_snapshot_create(e, cl, nc, &o, &s) || kp_batch_create(e, s, bs, nb, &b) || kp_schedule_batch(e, b, &r)) {
    fprintf(stderr, "config %d: engine error: %s\n", config, kp_last_error(e));
    bad = 1;
  } else {
    kpo_world* ow = kpo_world_create(cl, nc, &o);
    kpo_results* want = nullptr;
    kpo_schedule(ow, bs, nb, KPO_FAST, 4, &want);
    for (uint64_t i = 0; i < nb; i++) {
      const bool same = r.status[i] == want->status[i] && r.err_code[i] == want->err_code[i] &&
                        r.err_arg[i] == want->err_arg[i] &&
                        targets_of(r.offsets, r.cluster_idx, r.replicas, i) ==
                            targets_of(want->offsets, want->cluster_idx, want->replicas, i);
      if (!same && bad++ < 3) fprintf(stderr, "config %d seed %llu binding %llu differs\n", config,
                                      (unsigned long long)seed, (unsigned long long)i);
    }
    kpo_results_free(want);
    kpo_world_destroy(ow);
  }
  if (b) kp_batch_destroy(b);
  if (s) kp_snapshot_destroy(s);
  kps_destroy(w);
  printf("config %d seed %llu: %llu bindings x %u clusters, %d mismatches\n", config, (unsigned long long)seed,
         (unsigned long long)nb, C, bad);
  return bad ? 1 : 0;
}

int main() {
  kp_engine* e = nullptr;
  if (kp_engine_create(0, &e)) return 2;
  int fails = 0;
  const std::vector<std::tuple<int, uint64_t, uint32_t, uint64_t, bool>> cases = {
      {3, 3, 120, 200, false}, {4, 4, 200, 300, false}, {6, 6, 150, 600, false}, {6, 9, 257, 300, true},
      {7, 17, 200, 300, false}, {8, 4, 64, 150, false}, {9, 1, 150, 300, true}, {2, 2, 200, 200, false},
  };
  for (auto& c : cases) fails += run_case(e, std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c), std::get<4>(c));
  kp_engine_destroy(e);
  printf("%s\n", fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
