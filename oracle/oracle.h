/*
 * oracle.h — CPU restatement of Karmada's genericScheduler.Schedule path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the checker for the HIP engine and
 * the CPU baseline of bench.py. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product (karmada_amd/, libkp.so)
 * never links or calls it.
 *
 * The restatement follows the Go sources of /root/reference (cited file:line in
 * oracle.cpp) over the object model of include/kp/kp_api.h. Parity pinning:
 * the reference is Go and no Go toolchain exists here, so the
 * oracle is pinned by the reference's own table-driven tests, transcribed into
 * tests/golden/ JSON files (see tests/test_oracle_golden.py).
 *
 * Modes:
 *   KPO_FAITHFUL — the reference's algorithmic shape: per-call snapshot deep
 *                  copy (cache.go:124-139), per-pair selector compile
 *                  (selector.go:116), first-fit simulator loop
 *                  (scheduling_simulator_components.go:51-130), heap Webster
 *                  (webstermethod.go:112-161), Go pdqsort emulation.
 *   KPO_FAST     — same results; no per-call deep copy and the closed-form grade
 *                  walk instead of the FF loop.
 *   KPO_REFSHAPE — KPO_FAITHFUL except the FF loop, which is replaced by its
 *                  closed form: the CPU baseline where the FF loop is
 *                  intractable (config 3), a lower bound on the reference's cost.
 */
#ifndef KPO_ORACLE_H
#define KPO_ORACLE_H

#include <stdint.h>

#include "../include/kp/kp_api.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { KPO_FAITHFUL = 0, KPO_FAST = 1, KPO_REFSHAPE = 2 };

typedef struct kpo_world kpo_world;

typedef struct kpo_results {
  uint64_t n;
  int32_t* status;
  int32_t* err_code;
  int64_t* err_arg;
  uint64_t* offsets; /* n+1 */
  uint32_t* cluster_idx;
  int32_t* replicas;
  uint64_t n_targets;
} kpo_results;

/* A ClusterDetailInfo (spreadconstraint/group_clusters.go:78-93) for unit hooks. */
typedef struct kpo_candidate {
  kp_str name;
  int64_t score;
  int32_t overflow_order;
  int64_t available_replicas;
  int32_t allocatable_replicas;
  int32_t cluster; /* index into the hook's cluster array, or -1 */
} kpo_candidate;

kpo_world* kpo_world_create(const kp_cluster* clusters, uint64_t n, const kp_options* opts);
void kpo_world_destroy(kpo_world* w);

/* Schedule bindings with `n_threads` host threads (<=0: 1). */
int kpo_schedule(kpo_world* w, const kp_binding* b, uint64_t n, int mode, int n_threads,
                 kpo_results** out);
/* Scheduler.scheduleResourceBindingWithClusterAffinities (scheduler.go:618-684) per binding:
 * affinity_index[i] = term that succeeded or -1, attempts[i] = Schedule calls made. */
int kpo_schedule_affinities(kpo_world* w, const kp_binding* b, uint64_t n, int mode, int n_threads,
                            kpo_results** out, int32_t* affinity_index, int32_t* attempts);
void kpo_results_free(kpo_results* r);

/* ---- unit hooks used by the golden-vector tests ---- */
int kpo_quantity(const char* s, uint32_t len, int milli, int64_t* out); /* 0 ok, -1 parse error */
int kpo_cluster_matches(const kp_cluster* c, const kp_cluster_affinity* a);
/* Filter plugins in canonical order; returns 0 when the cluster fits, else the
 * KP_PLUGIN_* bit of the first failing plugin. */
uint32_t kpo_filter(const kp_cluster* c, const kp_binding* b, const kp_options* opts);
/* GeneralEstimator.maxAvailableComponentSets (general.go:163-292) for one cluster;
 * mode FAITHFUL runs the literal first-fit over every model node, FAST the run form. */
int32_t kpo_max_available_component_sets(const kp_cluster* c, const kp_component* comps, uint32_t n,
                                         const kp_options* opts, int mode);
/* getMaximumSetsBasedOnResourceModels (general.go:262-292): -1 on its error. */
int32_t kpo_max_sets_models(const kp_cluster* c, const kp_component* comps, uint32_t n, int32_t upper, int mode);
/* SchedulingSimulator.SimulateScheduling over explicit nodes (each node = a cluster
 * struct's resource_summary.allocatable, createNodeInfo of the reference's test). */
int32_t kpo_simulate_sets(const kp_cluster* nodes, uint32_t n_nodes, const kp_component* comps, uint32_t n,
                          int32_t upper, int mode);
/* The same pair as a kp_filter_reasons word (KP_REASON_* | arg << 8). */
uint32_t kpo_filter_reason(const kp_cluster* c, const kp_binding* b, const kp_options* opts);
int64_t kpo_score(const kp_cluster* c, const kp_binding* b, const kp_options* opts);
int32_t kpo_max_available_replicas(const kp_cluster* c, const kp_binding* b,
                                   const kp_options* opts, int mode);
/* GeneralEstimator pieces: part 0 maxAvailableReplicas, 1 getMaximumReplicasBased-
 * OnResourceModels (returns -1 on error), 2 ...OnClusterSummary, 3 getAllowedPodNumber. */
int kpo_estimator_part(const kp_cluster* c, const kp_binding* b, const kp_options* opts, int part,
                       int mode, int64_t* out);
/* helper.AllocateWebsterSeats; parties = union of names in votes/init, output is in
 * ascending name order: out_seats[k] for the k-th distinct name. Returns #parties. */
int kpo_allocate_webster(int32_t new_seats, const kp_str* vote_names, const int64_t* votes,
                         uint32_t n_votes, const kp_str* init_names, const int32_t* init_seats,
                         uint32_t n_init, int tie_mode, kp_str uid, int32_t* out_seats,
                         uint32_t out_cap);
/* The calling thread's AllocateWebsterSeats: 0 = the literal heap loop (default), 1 = the
 * FAST form (threshold-preseated, then the heap; kpo_schedule's KPO_FAST workers use it). */
void kpo_set_webster_fast(int on);
/* util.GetSumOfReplicas (pkg/util/binding.go:72-78, int32 wrapping). */
int32_t kpo_sum_replicas(const kp_target_cluster* t, uint32_t n);
/* util.MergeTargetClusters (binding.go:91-115): result entries as indices into `names`
 * (-1 if absent) + replicas; returns the result length. */
int kpo_merge_target_clusters(const kp_target_cluster* old_t, uint32_t n_old, const kp_target_cluster* new_t,
                              uint32_t n_new, const kp_target_cluster* names, uint32_t n_names, int32_t* out_idx,
                              int32_t* out_rep, uint32_t out_cap);
/* util.RescheduleRequired (binding.go:117-127) of the binding's two timestamps. */
int kpo_reschedule_required(const kp_binding* b);
/* helper.SpreadReplicasByTargetClusters / Dispenser.AllocateByWeight;
 * returns #targets written (name order), names as indices into `tcs`. */
int kpo_spread_replicas(int32_t num, const kp_target_cluster* tcs, uint32_t n,
                        const kp_target_cluster* init, uint32_t n_init, kp_str uid,
                        kp_target_cluster* out, uint32_t out_cap);
/* core.AssignReplicas (level 0), the strategy function alone (level 1) or
 * buildScheduledClusters+dynamicScaleUp (level 2) over explicit candidates;
 * `clusters` backs StaticWeight ClusterMatches (candidate.cluster indexes it).
 * Returns #targets, or -status on error. */
int kpo_assign_replicas(const kpo_candidate* cands, uint32_t n, const kp_cluster* clusters,
                        uint32_t n_clusters, const kp_binding* b, int level, int32_t* err_code,
                        int64_t* err_arg, kp_target_cluster* out, uint32_t out_cap);
/* spreadconstraint.selectGroups: returns #selected; out = indices into input. */
int kpo_select_groups(const kp_str* names, const int64_t* values, const int64_t* weights,
                      uint32_t n, int64_t min_c, int64_t max_c, int64_t target, uint32_t* out);
/* spreadconstraint.(GroupClustersInfo).calcGroupScore. */
uint64_t kpo_h4_hits(int reset);
int64_t kpo_calc_group_score(const kpo_candidate* cands, uint32_t n, const kp_binding* b,
                             int64_t min_groups);
/* GroupClustersWithScore + SelectBestClusters from a scored cluster list with
 * precomputed estimator answers; returns #selected (candidate indices) or <0 =
 * -KP_ERR_*. */
int kpo_select_clusters(const kp_cluster* clusters, const int64_t* scores, const int32_t* avail,
                        uint32_t n, const kp_binding* b, int32_t need_replicas, uint32_t* out,
                        uint32_t out_cap);
/* sortClusters (spreadconstraint/util.go:43-61): candidate indices in sorted order;
 * with_avail adds the AvailableReplicas comparison of generateClustersInfo
 * (group_clusters.go:370-375). */
void kpo_sort_clusters(const kpo_candidate* c, uint32_t n, int with_avail, uint32_t* order);
/* GroupClustersWithScore (group_clusters.go:103-149) with a calAvailableReplicasFunc
 * answering `avail` for every cluster: order = cluster indices in info.Clusters
 * order; groups = {#zones, #regions, #providers}. Returns n. */
int kpo_group_clusters(const kp_cluster* clusters, const int64_t* scores, uint32_t n, const kp_binding* b,
                       int32_t avail, uint32_t* order, int32_t* groups);
/* selectBestClustersByRegion (select_clusters_by_region.go:25-64) over a given
 * GroupClustersInfo: region r has its clusters at candidates [off[r], off[r+1]).
 * Returns #selected (candidate indices in out) or -KP_ERR_*. */
int kpo_select_by_region(const kp_str* region_names, const int64_t* region_scores, const uint32_t* off,
                         uint32_t n_regions, const kpo_candidate* cands, int64_t rmin, int64_t rmax, int64_t cmin,
                         int64_t cmax, uint32_t* out);
/* SelectBestClusters (select_clusters.go:28-55) over a given GroupClustersInfo.Clusters
 * list (in its order, no regions). Returns #selected or -KP_ERR_*. */
int kpo_select_best(const kpo_candidate* cands, uint32_t n, const kp_binding* b, int32_t need_replicas,
                    uint32_t* out);
/* dynamicDivideReplicas (division_algorithm.go:75-101) over an explicit availableClusters
 * list (no scheduled clusters); strategy 1 = DynamicWeight, 2 = Aggregated, other =
 * undefined. Returns #targets or -status (err_code = KP_ERR_*). */
int kpo_dynamic_divide(const kp_target_cluster* avail, uint32_t n, int32_t available_replicas, int32_t target,
                       int strategy, const kp_binding* b, int32_t* err_code, kp_target_cluster* out, uint32_t out_cap);
/* Go 1.26 sort.Sort emulation on TargetClustersList (Less = Replicas desc). */
void kpo_sort_target_clusters(int32_t* replicas, uint32_t* ids, uint32_t n);
uint32_t kpo_fnv32a(const char* s, uint32_t len);
/* getAllocatableModelings' grade counts (0 ok, -1 InitSummary error) and
 * nodeResourceEstimator.Estimate's sum (0 ok, -1 parse error, -2 node affinity). */
int kpo_model_grades(const kp_resource_model* models, uint32_t n_models, const kp_node* nodes, uint64_t n_nodes,
                     int64_t* out);
int kpo_node_max_replicas(const kp_node* nodes, uint64_t n_nodes, const kp_resource* request, uint32_t n_request,
                          const kp_node_claim* claim, const kp_assumed_workload* assumed, uint32_t n_assumed,
                          int32_t* out);
int kpo_node_max_component_sets(const kp_node* nodes, uint64_t n_nodes, const kp_node_component* comps, uint32_t K,
                                const kp_assumed_workload* assumed, uint32_t n_assumed, int32_t* out);

#ifdef __cplusplus
}
#endif

#endif
