/*
 * kp_api.h — C-ABI of the MI355X batched placement engine ("kp") for Karmada's
 * scheduling hot path (genericScheduler.Schedule).
 *
 * Two layers live in this header:
 *
 *   1. The OBJECT MODEL: plain C structs that mirror the subset of the Karmada
 *      API types the placement path reads. A cgo shim fills them from the Go
 *      objects; the Python test harness fills them through
 *      ctypes. Field names follow the Go/JSON names of the reference types:
 *        kp_cluster          <- clusterv1alpha1.Cluster
 *                               (pkg/apis/cluster/v1alpha1/types.go:43-377)
 *        kp_binding          <- workv1alpha2.ResourceBindingSpec + Status subset
 *                               (pkg/apis/work/v1alpha2/binding_types.go:71-300,443-467)
 *        kp_cluster_affinity <- policyv1alpha1.ClusterAffinity
 *                               (pkg/apis/policy/v1alpha1/propagation_types.go:445-772)
 *      Strings are (ptr,len) views; slices are (ptr,count). Nothing is retained
 *      after a call returns (cgo pointer rules): the engine copies/packs inputs.
 *
 *   2. The ENTRY POINTS (kp_*), each replacing a reference interface:
 *        kp_schedule_batch          <- core.ScheduleAlgorithm.Schedule
 *                                      (pkg/scheduler/core/generic_scheduler.go:37-49,71-116)
 *        kp_filter_batch            <- framework.FilterPlugin.Filter for the in-tree filter set
 *                                      (pkg/scheduler/framework/interface.go:85-98,
 *                                       pkg/scheduler/framework/runtime/framework.go:93-122)
 *        kp_filter_reasons          <- framework.FitError's Diagnosis (framework/types.go:56-90)
 *        kp_score_batch             <- framework.ScorePlugin.Score summed by RunScorePlugins
 *                                      (pkg/scheduler/framework/interface.go:215-232,
 *                                       pkg/scheduler/framework/runtime/framework.go:126-170)
 *        kp_max_available_replicas  <- estimatorclient.ReplicaEstimator.MaxAvailableReplicas
 *                                      for the GeneralEstimator
 *                                      (pkg/estimator/client/interface.go:39-71,
 *                                       pkg/estimator/client/general.go:57-108)
 *        kp_max_available_component_sets <- ReplicaEstimator.MaxAvailableComponentSets
 *                                      (general.go:154-292)
 *        kp_model_grades            <- getAllocatableModelings over modeling.AddToResourceSummary
 *                                      (pkg/controllers/status/cluster_status_controller.go:642-677)
 *        kp_node_max_replicas       <- noderesource.nodeResourceEstimator.Estimate (estimator server,
 *                                      pkg/estimator/server/framework/plugins/noderesource)
 *        kp_node_max_component_sets <- noderesource.nodeResourceEstimator.EstimateComponents
 *        kp_snapshot_create         <- cache.Cache.Snapshot (pkg/scheduler/cache/cache.go:124-139)
 *        kp_schedule_affinities     <- Scheduler.scheduleResourceBindingWithClusterAffinities
 *                                      (pkg/scheduler/scheduler.go:584-585,618-684)
 *
 * Return convention: 0 = OK, <0 = KP_E* ; kp_last_error() gives the text.
 * No exceptions cross the ABI. An engine handle is not re-entrant.
 */
#ifndef KP_API_H
#define KP_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KP_ABI_VERSION 14

/* ------------------------------------------------------------------------- */
/* Object model                                                              */
/* ------------------------------------------------------------------------- */

typedef struct kp_str {
  const char* ptr;
  uint32_t len;
} kp_str;

/* map[string]string entry (labels, matchLabels). */
typedef struct kp_label {
  kp_str key;
  kp_str value;
} kp_label;

/* metav1.LabelSelectorRequirement / corev1.NodeSelectorRequirement. `op` is the
 * operator string exactly as in the API ("In", "NotIn", "Exists", ...). */
typedef struct kp_requirement {
  kp_str key;
  kp_str op;
  const kp_str* values;
  uint32_t n_values;
} kp_requirement;

/* policyv1alpha1.ClusterAffinity (propagation_types.go). */
typedef struct kp_cluster_affinity {
  uint8_t has_label_selector; /* LabelSelector != nil */
  const kp_label* match_labels;
  uint32_t n_match_labels;
  const kp_requirement* match_expressions;
  uint32_t n_match_expressions;
  uint8_t has_field_selector; /* FieldSelector != nil */
  const kp_requirement* field_expressions;
  uint32_t n_field_expressions;
  const kp_str* cluster_names;
  uint32_t n_cluster_names;
  const kp_str* exclude_clusters;
  uint32_t n_exclude_clusters;
} kp_cluster_affinity;

/* policyv1alpha1.ClusterAffinityTerm: {AffinityName, ClusterAffinity, OverflowAffinities}. */
typedef struct kp_affinity_term {
  kp_str affinity_name;
  kp_cluster_affinity affinity;
  const kp_cluster_affinity* overflow; /* OverflowAffinities[i].ClusterAffinity */
  uint32_t n_overflow;
} kp_affinity_term;

/* corev1.Toleration (TolerationSeconds is irrelevant for placement). */
typedef struct kp_toleration {
  kp_str key;
  kp_str op; /* "", "Equal", "Exists", "Lt", "Gt", ... */
  kp_str value;
  kp_str effect;
} kp_toleration;

/* corev1.Taint. */
typedef struct kp_taint {
  kp_str key;
  kp_str value;
  kp_str effect;
} kp_taint;

/* policyv1alpha1.SpreadConstraint (MaxGroups/MinGroups are Go `int`). */
typedef struct kp_spread_constraint {
  kp_str spread_by_field; /* "cluster" | "region" | "zone" | "provider" | "" */
  kp_str spread_by_label;
  int64_t max_groups;
  int64_t min_groups;
} kp_spread_constraint;

/* policyv1alpha1.StaticClusterWeight. */
typedef struct kp_static_weight {
  kp_cluster_affinity target;
  int64_t weight;
} kp_static_weight;

/* corev1.ResourceList entry: name + resource.Quantity string ("100m", "2Gi", ...). */
typedef struct kp_resource {
  kp_str name;
  kp_str quantity;
} kp_resource;

/* workv1alpha2.TargetCluster (Components omitted: multi-template gate is off). */
typedef struct kp_target_cluster {
  kp_str name;
  int32_t replicas;
} kp_target_cluster;

/* workv1alpha2.Component (pkg/apis/work/v1alpha2/binding_types.go): one pod template
 * of a multi-template workload; ReplicaRequirements.ResourceRequest only (the
 * NodeClaim never filters the estimator's model nodes, which carry no Node object,
 * scheduling_simulator_components.go:149-153). */
typedef struct kp_component {
  kp_str name;
  int32_t replicas;
  uint8_t has_replica_requirements;
  const kp_resource* resource_request;
  uint32_t n_resource_request;
} kp_component;

/* ResourceBindingSpec + the status fields Schedule reads. */
typedef struct kp_binding {
  kp_str uid; /* spec.Resource.UID: FNV tie-break (pkg/util/helper/binding.go:117-144) */
  kp_str api_version;
  kp_str kind;
  kp_str namespace_;
  kp_str name;
  int32_t replicas;
  uint8_t has_replica_requirements; /* spec.ReplicaRequirements != nil */
  uint8_t has_node_claim;           /* ReplicaRequirements.NodeClaim != nil: no effect on the
                                       general estimator (a NodeClaim converts without error and
                                       every model node matches it, accurate.go:155-177,
                                       scheduling_simulator_components.go:149-153) */
  const kp_resource* resource_request;
  uint32_t n_resource_request;
  uint32_t n_components; /* len(spec.Components) */
  const kp_component* components; /* spec.Components (binding_types.go:89-98): read only with the
                                     MultiplePodTemplatesScheduling gate on, for bindings
                                     isMultiTemplateSchedulingApplicable accepts
                                     (core/estimation.go:43-65); NULL there -> KP_EINVAL */
  const kp_target_cluster* clusters; /* spec.Clusters (previous result) */
  uint32_t n_clusters;
  const kp_str* eviction_from; /* spec.GracefulEvictionTasks[].FromCluster */
  uint32_t n_eviction_from;
  uint8_t has_reschedule_triggered_at;
  uint8_t has_last_scheduled_time;
  int64_t reschedule_triggered_at_ns; /* unix nanoseconds */
  int64_t last_scheduled_time_ns;
  kp_str observed_affinity_name; /* status.SchedulerObservedAffinityName */
  /* spec.Placement */
  uint8_t has_cluster_affinity;
  kp_cluster_affinity cluster_affinity;
  const kp_affinity_term* cluster_affinities;
  uint32_t n_cluster_affinities;
  const kp_toleration* tolerations; /* ClusterTolerations */
  uint32_t n_tolerations;
  const kp_spread_constraint* spread_constraints;
  uint32_t n_spread_constraints;
  uint8_t has_replica_scheduling;
  kp_str replica_scheduling_type;     /* "Duplicated" | "Divided" */
  kp_str replica_division_preference; /* "Aggregated" | "Weighted" */
  uint8_t has_weight_preference;
  const kp_static_weight* static_weights;
  uint32_t n_static_weights;
  kp_str dynamic_weight; /* "AvailableReplicas" | "" */
} kp_binding;

/* Cluster.Status.APIEnablements flattened to (GroupVersion, Resources[].Kind) pairs. */
typedef struct kp_api_enablement {
  kp_str group_version;
  kp_str kind;
} kp_api_enablement;

/* clusterv1alpha1.ResourceModelRange / ResourceModel / AllocatableModeling. */
typedef struct kp_model_range {
  kp_str name;
  kp_str min;
  kp_str max;
} kp_model_range;

typedef struct kp_resource_model {
  uint32_t grade;
  const kp_model_range* ranges;
  uint32_t n_ranges;
} kp_resource_model;

typedef struct kp_allocatable_modeling {
  uint32_t grade;
  int64_t count;
} kp_allocatable_modeling;

/* clusterv1alpha1.Cluster subset. */
typedef struct kp_cluster {
  kp_str name;
  uint8_t deleting; /* !DeletionTimestamp.IsZero() */
  const kp_label* labels;
  uint32_t n_labels;
  kp_str provider;
  kp_str region;
  kp_str zone;
  const kp_str* zones;
  uint32_t n_zones;
  const kp_taint* taints;
  uint32_t n_taints;
  const kp_api_enablement* api_enablements;
  uint32_t n_api_enablements;
  const kp_resource_model* resource_models; /* Spec.ResourceModels */
  uint32_t n_resource_models;
  uint8_t has_resource_summary; /* Status.ResourceSummary != nil */
  const kp_resource* allocatable;
  uint32_t n_allocatable;
  const kp_resource* allocated;
  uint32_t n_allocated;
  const kp_resource* allocating;
  uint32_t n_allocating;
  const kp_allocatable_modeling* allocatable_modelings;
  uint32_t n_allocatable_modelings;
} kp_cluster;


/* In-tree plugin names (pkg/scheduler/framework/plugins/registry.go:33-50). */
enum {
  KP_PLUGIN_API_ENABLEMENT = 1u << 0,
  KP_PLUGIN_TAINT_TOLERATION = 1u << 1,
  KP_PLUGIN_CLUSTER_AFFINITY = 1u << 2,
  KP_PLUGIN_SPREAD_CONSTRAINT = 1u << 3,
  KP_PLUGIN_CLUSTER_LOCALITY = 1u << 4,
  KP_PLUGIN_CLUSTER_EVICTION = 1u << 5,
  KP_PLUGIN_ALL = 0x3fu
};

/* Flags and gates that change results (cmd/scheduler/app/options/options.go:130-165,
 * pkg/features/features.go:162-189). */
typedef struct kp_options {
  uint8_t enable_empty_workload_propagation;   /* --enable-empty-workload-propagation */
  uint8_t customized_cluster_resource_modeling; /* feature gate, default on */
  uint8_t multiple_pod_templates_scheduling;    /* feature gate MultiplePodTemplatesScheduling, alpha, default off */
  uint32_t enabled_plugins;                     /* KP_PLUGIN_* bitmask (--plugins) */
  /* Filter or score plugins the scheduler's registry holds beyond the in-tree set
   * (app.WithPlugin, cmd/scheduler/app/scheduler.go:90). RunFilterPlugins and
   * RunScorePlugins (runtime/framework.go:93-170) run every registered plugin, so
   * the batch path, which computes the in-tree set only, would place differently:
   * kp_schedule_batch, kp_schedule_affinities and kp_multi_schedule return
   * KP_ENOTSUP for a snapshot with n_out_of_tree_plugins > 0. The per-pair entry
   * points (kp_filter_reasons, kp_score_batch, kp_max_available_replicas) still
   * answer for the in-tree set, for the framework to combine with the others. */
  uint32_t n_out_of_tree_plugins;
} kp_options;

/* ------------------------------------------------------------------------- */
/* Results                                                                   */
/* ------------------------------------------------------------------------- */

/* Error class of one Schedule call (framework/types.go:61-99). */
enum {
  KP_STATUS_OK = 0,
  KP_STATUS_FIT_ERROR = 1,     /* *framework.FitError */
  KP_STATUS_UNSCHEDULABLE = 2, /* *framework.UnschedulableError (possibly wrapped) */
  KP_STATUS_ERROR = 3          /* any other error */
};

/* The reference error site that produced a non-OK status. */
enum {
  KP_ERR_NONE = 0,
  KP_ERR_FIT = 1,                    /* generic_scheduler.go:84-89; arg = NumAllClusters */
  KP_ERR_REGION_MIN_GROUPS = 2,      /* select_clusters_by_region.go:30-32 */
  KP_ERR_REGION_CLUSTER_MIN = 3,     /* select_clusters_by_region.go:37-39 */
  KP_ERR_CLUSTER_MIN_GROUPS = 4,     /* select_clusters_by_cluster.go:28-30 */
  KP_ERR_CLUSTER_RESOURCE = 5,       /* select_clusters_by_cluster.go:39-41; arg = needCnt */
  KP_ERR_SPREAD_UNSUPPORTED = 6,     /* select_clusters.go:54 */
  KP_ERR_NO_CLUSTERS = 7,            /* common.go:55-57 */
  KP_ERR_UNSUPPORTED_STRATEGY = 8,   /* common.go:143-148 */
  KP_ERR_OVERFLOW_NOT_ENOUGH = 9,    /* common.go:132-134 */
  KP_ERR_FRESH_NOT_ENOUGH = 10,      /* assignment.go:218-221 wrapping division_algorithm.go:76-78; arg = available */
  KP_ERR_SCALE_DOWN_NOT_ENOUGH = 11, /* assignment.go:228-231; arg = available */
  KP_ERR_SCALE_UP_NOT_ENOUGH = 12,   /* assignment.go:236-239; arg = available */
  KP_ERR_UNDEFINED_STRATEGY = 13,    /* division_algorithm.go:97-99 */
  KP_ERR_RESULT_CAPACITY = 14,       /* engine limit, no reference site: a serial result list
                                        outgrew the batch's result pool (arg = its length);
                                        never expected, reported instead of written */
  KP_ERR_SETS_CAPACITY = 15,         /* engine limit, no reference site: the binding's
                                        MaxAvailableComponentSets simulation needed more than
                                        the device's node runs in one cluster (arg = the
                                        cluster's caller index); only that binding fails */
  KP_ERR_OVERFLOW_TERMS = 16         /* engine limit, no reference site: the observed
                                        ClusterAffinities term plus its overflow affinities
                                        number more than 63, the orders the sortClusters key
                                        holds (getClusterOverflowOrder, common.go:156-170,
                                        takes any number); arg = that count */
};

/* Per-batch results, engine-owned, valid until the next call on the engine.
 * Targets of binding b are entries [offsets[b], offsets[b+1]) of cluster_idx /
 * replicas; cluster_idx indexes the caller's cluster array given to
 * kp_snapshot_create. Order inside one binding follows the reference where it
 * is deterministic; compare as a multiset (test/helper/scheduler.go:26-40). */
typedef struct kp_results {
  uint64_t n_bindings;
  const int32_t* status;   /* KP_STATUS_* */
  const int32_t* err_code; /* KP_ERR_* */
  const int64_t* err_arg;
  const uint64_t* offsets; /* n_bindings + 1 */
  const uint32_t* cluster_idx;
  const int32_t* replicas;
  uint64_t n_targets;
} kp_results;

/* Results of kp_schedule_affinities, engine-owned like kp_results. `results` holds
 * each binding's final Schedule outcome: the first successful term's targets, or,
 * when every term failed, the FIRST term's error class/code/arg with no targets
 * (scheduler.go:657-673). affinity_index[b] = the ClusterAffinities index that
 * succeeded (its AffinityName becomes Status.SchedulerObservedAffinityName,
 * scheduler.go:676-678), or -1 when the observed name stays as it was (all terms
 * failed, or the binding has no ClusterAffinities). attempts[b] = Schedule calls
 * made for binding b. rounds = batched passes run (1 + the largest retry depth). */
typedef struct kp_affinity_results {
  kp_results results;
  const int32_t* affinity_index;
  const int32_t* attempts;
  uint32_t rounds;
} kp_affinity_results;

/* Per-stage timing of the last kp_schedule_batch call (milliseconds, host clock
 * around device work; kernel-only numbers come from rocprof). */
typedef struct kp_stage_times {
  double pair_ms;      /* filter + estimate stage: k_est_class + k_filter, or the pair kernel */
  double select_ms;    /* candidate/group/select/divide kernels after the filter stage */
  double host_ms;      /* host group-combination (region DFS) */
  double copy_ms;      /* device -> host result copies */
  double total_ms;
  float pair_kernel_ms;   /* filter + estimate stage kernels (HIP events) */
  float select_kernel_ms; /* select kernels after the filter stage (HIP events) */
  uint64_t n_slow;        /* bindings that took the exact serial path */
  uint32_t pair_launches; /* filter-stage kernel launches (2: k_est_class + k_filter, 1: pair kernel) */
  uint32_t pair_kind;     /* estimator instance: 0 generic, 1 mixed, 2 summary-only, 8/16 model-only */
  float filter_kernel_ms; /* k_filter alone (HIP events), 0 with the pair kernel */
  uint32_t bits;          /* 1: bitset filter + estimator-class rows; 0: per-binding pair rows */
  float sel_all_kernel_ms; /* the two-kernel path's SEL_ALL select kernel alone (HIP events) */
  uint32_t n_sel_all;      /* bindings of the SEL_ALL select kernel (SelectBestClusters selects all) */
  uint32_t n_classes;      /* estimator-class rows computed (bits == 1; row 0 = non-workload) */
  uint32_t n_top;          /* SEL_ALL bindings given to k_select_top (deciding-candidate subsets) */
  uint32_t n_top_fallback; /* of those, the ones it handed to the full-candidate kernel */
  float top_kernel_ms;     /* k_select_top alone (HIP events on its stream), 0 when it did not run */
  uint32_t n_cluster;       /* cluster-spread bindings (selectBestClustersByCluster) */
  uint32_t n_cluster_order; /* of those, the ones selected over their estimator-class order */
  float cluster_kernel_ms;  /* the cluster-spread select kernel alone (HIP events on its stream) */
  uint32_t n_region;        /* region-spread bindings (selectBestClustersByRegion) */
  uint32_t n_region_order;  /* of those, the ones whose final selection walked their estimator-class order */
} kp_stage_times;

/* ------------------------------------------------------------------------- */
/* Entry points                                                              */
/* ------------------------------------------------------------------------- */

typedef struct kp_engine kp_engine;
typedef struct kp_snapshot kp_snapshot;
typedef struct kp_batch kp_batch;

enum {
  KP_OK = 0,
  KP_EINVAL = -1,
  KP_ENOMEM = -2,
  KP_EDEVICE = -3,
  KP_ENOTSUP = -4,
  KP_ESTATE = -5
};

int kp_abi_version(void);

/* Creates an engine bound to HIP device `device` (one HIP stream). */
int kp_engine_create(int device, kp_engine** out);
void kp_engine_destroy(kp_engine* e);
const char* kp_last_error(const kp_engine* e);

/* Packs a cluster list (cache.Snapshot) into the device SoA layout and uploads it.
 * Replaces the per-Schedule List+DeepCopy (cache.go:124-139) by one upload. */
int kp_snapshot_create(kp_engine* e, const kp_cluster* clusters, uint64_t n_clusters,
                       const kp_options* opts, kp_snapshot** out);
void kp_snapshot_destroy(kp_snapshot* s);
/* Applies cluster events to a snapshot in place: `clusters` are new versions of
 * clusters already in it (matched by name). Only those rows are re-packed; the
 * device copy is refreshed. This replaces re-snapshotting all clusters on every
 * informer event (cache.go:124-139, event_handler.go:314-378). *dict_grew = 1
 * when the update added names, keys, GVKs or resources to the snapshot's
 * dictionaries or changed its set of regions: batches packed before the call
 * must then be re-created (their compiled selectors resolve strings against the
 * old dictionaries; their region buffers are sized by the region count), and
 * kp_schedule_batch returns KP_ESTATE for a region-spread batch whose region
 * count no longer matches; otherwise they stay valid. Adding or removing
 * clusters needs kp_snapshot_create. */
int kp_snapshot_update(kp_engine* e, kp_snapshot* s, const kp_cluster* clusters, uint64_t n_clusters,
                       int* dict_grew);
/* Packed snapshot as one relocatable byte image (for RCCL broadcast) and back. */
int kp_snapshot_export(const kp_snapshot* s, const void** bytes, uint64_t* n_bytes);
int kp_snapshot_import(kp_engine* e, const void* bytes, uint64_t n_bytes, kp_snapshot** out);

/* Packs a batch of bindings against a snapshot and uploads them to HBM. */
int kp_batch_create(kp_engine* e, const kp_snapshot* s, const kp_binding* bindings,
                    uint64_t n_bindings, kp_batch** out);
void kp_batch_destroy(kp_batch* b);

/* ---- packed-record reuse across scheduling cycles --------------------------------
 * The scheduler re-runs Schedule for bindings whose spec did not change: Duplicated and
 * non-workload bindings on every reconcile, bindings with terminating target clusters,
 * requeued failures (pkg/scheduler/scheduler.go:437-468); a changed spec moves
 * metadata.generation. A kp_pack_cache keeps each binding's packed record (its binding
 * header and pool slices, snapshot ids resolved) keyed by (metadata.uid,
 * metadata.generation), and kp_batch_create_keyed copies a record instead of re-packing
 * the binding when the key matches and so do the status fields the record depends on
 * (status.schedulerObservedAffinityName, spec.rescheduleTriggeredAt,
 * status.lastScheduledTime, compared field by field). Records are tied to the snapshot's
 * dictionaries: a different snapshot, or a kp_snapshot_update that grew them
 * (dict_grew = 1), empties the cache. The batch is byte-for-byte the one
 * kp_batch_create packs from the same bindings. A cache is used by one call at a time. */
typedef struct kp_pack_cache kp_pack_cache;
typedef struct kp_binding_key {
  kp_str uid;         /* metadata.uid */
  int64_t generation; /* metadata.generation */
} kp_binding_key;
typedef struct kp_pack_cache_stats {
  uint64_t hits, misses; /* over the cache's lifetime */
  uint64_t entries;      /* records held */
  uint64_t last_hits;    /* of the last kp_batch_create_keyed */
} kp_pack_cache_stats;
/* max_entries: records kept (0: 4M); past it the cache is emptied before the next batch. */
int kp_pack_cache_create(uint64_t max_entries, kp_pack_cache** out);
void kp_pack_cache_destroy(kp_pack_cache* c);
int kp_pack_cache_get_stats(const kp_pack_cache* c, kp_pack_cache_stats* out);
/* Diagnostic: a 64-bit digest of a batch's packed host image (binding headers, pools,
 * routes, and each binding's estimator class as its first binding), equal for two
 * batches exactly when they pack the same records (the tests compare keyed and fresh). */
int kp_batch_digest(const kp_batch* b, uint64_t* out);
/* kp_batch_create with keys[i] for bindings[i] (keys[i].uid empty: never cached). */
int kp_batch_create_keyed(kp_engine* e, const kp_snapshot* s, const kp_binding* bindings,
                          const kp_binding_key* keys, uint64_t n_bindings, kp_pack_cache* cache,
                          kp_batch** out);

/* genericScheduler.Schedule for every binding of the batch. */
int kp_schedule_batch(kp_engine* e, kp_batch* b, kp_results* out);
/* kp_schedule_batch in two halves, for a caller that keeps batches in flight (a scheduler
 * draining its queue): _submit queues the batch's kernels and per-binding read-backs on the
 * engine's stream (it waits only where the region chain's host step does) and returns;
 * _collect waits for them, copies the CSR back and fills *out exactly as kp_schedule_batch
 * does. A batch holds one submitted call at a time (KP_ESTATE otherwise); an engine may hold
 * several submitted batches, collected in any order. Submitting the next batch before
 * collecting the last keeps the GPU queue fed while the host reads results back. Not with
 * kp_engine_set_profile (KP_EINVAL). */
int kp_schedule_batch_submit(kp_engine* e, kp_batch* b);
int kp_schedule_batch_collect(kp_engine* e, kp_batch* b, kp_results* out);

/* Scheduler.scheduleResourceBindingWithClusterAffinities (scheduler.go:618-684),
 * batched: bindings with n_cluster_affinities > 0 start at getAffinityIndex of their
 * observed name (helper.go:99-110; index 0 when util.RescheduleRequired), and every
 * binding whose term failed is re-packed with the next term's name and scheduled
 * again in the next round, all failing bindings of a round in one batch. Bindings
 * without ClusterAffinities run once (scheduleResourceBinding, scheduler.go:584-600). */
int kp_schedule_affinities(kp_engine* e, const kp_snapshot* s, const kp_binding* bindings, uint64_t n_bindings,
                           kp_affinity_results* out);

/* FilterPlugin boundary: feasibility of every (binding, cluster) pair after
 * RunFilterPlugins (+ the skip-deleting rule of findClustersThatFit).
 * out_mask: n_bindings * ceil(n_clusters/64) words, bit c%64 of word c/64 set
 * when cluster c (caller order) fits. */
int kp_filter_batch(kp_engine* e, kp_batch* b, uint64_t* out_mask);

/* FitError diagnosis (framework/types.go:56-90; findClustersThatFit,
 * generic_scheduler.go:119-163): per pair the Result of RunFilterPlugins
 * (runtime/framework.go:93-105, plugins in canonical order), n_bindings*n_clusters
 * words in caller cluster order: bits [7:0] = KP_REASON_*, bits [31:8] = argument.
 * KP_REASON_FIT pairs fit; KP_REASON_DELETING clusters are skipped before the
 * plugins run and are absent from Diagnosis.ClusterToResultMap. The argument of
 * KP_REASON_TAINT is the index of the untolerated taint among the cluster's
 * NoSchedule/NoExecute taints in spec.taints order (FindMatchingUntoleratedTaint);
 * 0 otherwise. */
enum {
  KP_REASON_FIT = 0,
  KP_REASON_API = 1,             /* api_enablement.go:77 "cluster(s) did not have the API resource" */
  KP_REASON_TAINT = 2,           /* taint_toleration.go:83 "cluster(s) had untolerated taint {%s}" */
  KP_REASON_AFFINITY = 3,        /* cluster_affinity.go:89 "...did not match the placement cluster affinity constraint" */
  KP_REASON_SPREAD_PROVIDER = 4, /* spread_constraint.go:57 "cluster(s) did not have provider property" */
  KP_REASON_SPREAD_REGION = 5,   /* spread_constraint.go:59 "cluster(s) did not have region property" */
  KP_REASON_SPREAD_ZONES = 6,    /* spread_constraint.go:61 "cluster(s) did not have zones property" */
  KP_REASON_EVICTION = 7,        /* cluster_eviction.go:53 "cluster(s) is in the process of eviction" */
  KP_REASON_DELETING = 255       /* generic_scheduler.go:138-142 (skipped) */
};
int kp_filter_reasons(kp_engine* e, kp_batch* b, uint32_t* out_reasons);

/* ScorePlugin boundary: summed score (RunScorePlugins) per pair; n_bindings*n_clusters. */
int kp_score_batch(kp_engine* e, kp_batch* b, int64_t* out_scores);

/* ReplicaEstimator boundary (GeneralEstimator.MaxAvailableReplicas): for binding
 * `binding` of the batch and the given caller cluster indices, writes the
 * estimator answer per cluster in input order (general.go:57-64). */
int kp_max_available_replicas(kp_engine* e, kp_batch* b, uint64_t binding,
                              const uint32_t* cluster_idx, uint64_t n, int32_t* out);

/* ReplicaEstimator.MaxAvailableComponentSets for the GeneralEstimator
 * (estimator/client/general.go:154-292): for one component list (one set = every
 * component's Replicas), the number of complete sets each cluster cluster_idx[i]
 * (caller order) holds, written to out[i]: the pod and resource-summary bounds
 * (quantityAsInt64 by each Quantity's format), then, with the
 * CustomizedClusterResourceModeling gate and models, the first-fit simulation over
 * the model-grade nodes (SchedulingSimulator.SimulateScheduling,
 * scheduling_simulator_components.go:51-131). Assumed workloads are empty
 * (SchedulingOvercommitProtection off). KP_ENOTSUP when the snapshot's options
 * have the MultiplePodTemplatesScheduling gate off (the scheduler then never calls
 * it, core/util.go:113-118), or when a cluster's simulation exceeds the device
 * run capacity (kp_last_error says which). */
int kp_max_available_component_sets(kp_engine* e, const kp_snapshot* s, const kp_component* components,
                                    uint32_t n_components, const uint32_t* cluster_idx, uint64_t n, int32_t* out);

/* ---- member-cluster nodes ------------------------------------
 * A member cluster's node as the cluster status controller and the estimator
 * server see it: corev1.Node plus the non-terminal pods bound to it. `requested`
 * is their summed effective requests (util.Resource.AddPodRequest: cpu, memory,
 * ephemeral-storage and scalar resources), n_pods their count. */
typedef struct kp_node {
  kp_str name;
  const kp_label* labels;
  uint32_t n_labels;
  const kp_taint* taints;
  uint32_t n_taints;
  int32_t unschedulable; /* node.Spec.Unschedulable */
  const kp_resource* allocatable; /* node.Status.Allocatable */
  uint32_t n_allocatable;
  const kp_resource* requested;
  uint32_t n_requested;
  uint32_t n_pods;
} kp_node;

/* The resource-model grade histogram of a cluster: getAllocatableModelings
 * (controllers/status/cluster_status_controller.go:642-677) over
 * modeling.InitSummary / AddToResourceSummary (pkg/modeling/modeling.go:75-223).
 * Each node's available resources (getNodeAvailable, :613-639; the walk stops at
 * the first node with no pod room, as the reference's `break` does) go to the grade
 * getIndex picks (searchLastLessElement per resource name, the minimum over names);
 * out_counts[k] = AllocatableModeling.Count of models[k]. KP_EINVAL for
 * InitSummary's error and for models without ranges. Replaces the Go function
 * getAllocatableModelings. */
int kp_model_grades(kp_engine* e, const kp_resource_model* models, uint32_t n_models, const kp_node* nodes,
                    uint64_t n_nodes, int64_t* out_counts);

/* corev1.NodeSelectorTerm of a required node affinity: MatchExpressions over node
 * labels (In, NotIn, Exists, DoesNotExist, Gt, Lt) and MatchFields over the node's
 * fields (metadata.name; In / NotIn with exactly one value). */
typedef struct kp_node_selector_term {
  const kp_requirement* match_expressions;
  uint32_t n_match_expressions;
  const kp_requirement* match_fields;
  uint32_t n_match_fields;
} kp_node_selector_term;

/* pb.NodeClaim of the estimator request (pkg/estimator/pb): nodeSelector,
 * tolerations and the required node affinity. has_node_affinity != 0 when
 * NodeAffinityBytes decodes to a NodeSelector (pb/helpers.go:40-55); its terms are
 * ORed (nodeaffinity.LazyErrorNodeSelector.Match), a term that fails to parse or is
 * empty never matches, and a selector with no usable term matches no node. */
typedef struct kp_node_claim {
  const kp_label* node_selector;
  uint32_t n_node_selector;
  const kp_toleration* tolerations;
  uint32_t n_tolerations;
  int32_t has_node_affinity;
  const kp_node_selector_term* node_affinity_terms;
  uint32_t n_node_affinity_terms;
} kp_node_claim;

/* pb.Component of an estimator server request: Replicas and ReplicaRequirements
 * (ResourceRequest, NodeClaim). has_replica_requirements == 0: nil requirements
 * (only the pod count is required, every node matches). */
typedef struct kp_node_component {
  int32_t replicas;
  uint8_t has_replica_requirements;
  const kp_resource* resource_request;
  uint32_t n_resource_request;
  const kp_node_claim* node_claim; /* NULL: no NodeClaim */
} kp_node_component;

/* pb.AssumedWorkload: a workload admitted but possibly not yet visible in node
 * accounting, deducted first (one set, SimulateScheduling(components, 1)). */
typedef struct kp_assumed_workload {
  const kp_node_component* components;
  uint32_t n_components;
} kp_assumed_workload;

/* The accurate estimator's per-node path: nodeResourceEstimator.Estimate
 * (estimator/server/framework/plugins/noderesource/noderesource.go:70-131): the
 * assumed workloads deducted in order (one first-fit set each), then the sum over
 * the nodes that MatchNode accepts (nodeSelector, required node affinity,
 * tolerations incl. the unschedulable taint; filter.go:38-99) of int32(MaxDivided)
 * of the node's available resources (allocatable - requested, clamped at 0; pods =
 * allocatable pods - n_pods, util/resource.go:96-115,221-248; noderesource.go:
 * 135-144) for `request`. claim may be NULL (no NodeClaim). *out = the int32 sum
 * (Go's atomic int32 adds wrap). Replaces AccurateSchedulerEstimatorServer.
 * EstimateReplicas for one request (estimate.go:33-76; 0 when there are no nodes). */
int kp_node_max_replicas(kp_engine* e, const kp_node* nodes, uint64_t n_nodes, const kp_resource* request,
                         uint32_t n_request, const kp_node_claim* claim, const kp_assumed_workload* assumed,
                         uint32_t n_assumed, int32_t* out);

/* The accurate estimator's component-set path: nodeResourceEstimator.EstimateComponents
 * (noderesource.go:146-190): the assumed workloads deducted as above, then the
 * first-fit simulation (SchedulingSimulator.SimulateScheduling,
 * scheduling_simulator_components.go:51-131) of complete component sets over the
 * nodes' available resources, each component placed on the nodes that MatchNode
 * accepts for its NodeClaim, up to MaxInt32 sets. n_components == 0 -> *out =
 * MaxInt32 (noNodeConstraint, the reference's Noopperation result); otherwise *out
 * = the set count (0 = the reference's Unschedulable "no enough resources").
 * KP_ENOTSUP past 16 components per set, 64 in all, 16 assumed workloads or 7
 * distinct requested resources. */
int kp_node_max_component_sets(kp_engine* e, const kp_node* nodes, uint64_t n_nodes,
                               const kp_node_component* components, uint32_t n_components,
                               const kp_assumed_workload* assumed, uint32_t n_assumed, int32_t* out);

/* Last schedule call's stage timings. */
int kp_last_stage_times(const kp_engine* e, kp_stage_times* out);

/* Per-kernel times of the last kp_schedule_batch, with profiling on
 * (kp_engine_set_profile(e, 1): an event pair around every launch on its own
 * stream; off by default). One entry per kernel name: the summed HIP-event time of
 * its launches, their count, and the bindings (or class rows) they covered. */
typedef struct kp_kernel_time {
  char name[32];
  float ms;
  uint32_t launches;
  uint64_t units;
} kp_kernel_time;
int kp_engine_set_profile(kp_engine* e, int on);
/* *n_out = the number of entries; at most `cap` are written to out. */
int kp_last_kernel_times(const kp_engine* e, kp_kernel_time* out, uint32_t cap, uint32_t* n_out);

/* Host threads an engine packs a batch on (kp_batch_create); default: the
 * hardware threads, at most 16. */
int kp_engine_set_threads(kp_engine* e, int n_threads);

/* A replica of snapshot `src` (of another engine, on another device) on engine e's
 * device: the packed device image copied device to device (hipMemcpyPeer, over xGMI
 * between the GPUs of one node) instead of re-packed and re-uploaded. The replica
 * schedules exactly as `src` does. */
int kp_snapshot_replicate(kp_engine* e, const kp_snapshot* src, kp_snapshot** out);

/* ---- one scheduler process over N GPUs (SURVEY §8(b) Threading, §8(e)) ------------
 * Replaces the reference scheduler's single worker (pkg/scheduler/scheduler.go:327):
 * a kp_multi owns one engine per device (own HIP streams); its snapshot is packed on
 * the first device and replicated onto the others (kp_snapshot_replicate); a batch
 * is cut into contiguous binding shards at equal prefix sums of the §8(e) cost
 * C + Replicas*log2 C, one per device; kp_multi_schedule runs the shards
 * concurrently (one host thread per device, no cross-device traffic) and returns one
 * CSR in binding order, identical to kp_schedule_batch over the whole batch on one
 * device. Result buffers belong to the batch and stay valid until its next
 * kp_multi_schedule or destruction. Verified on the host build (several simulated
 * devices, tests/test_multi.py) and on one physical GPU only: the cross-device
 * replication (hipMemcpyPeerAsync) has not run on two or more GPUs yet. */
typedef struct kp_multi kp_multi;
typedef struct kp_multi_snapshot kp_multi_snapshot;
typedef struct kp_multi_batch kp_multi_batch;

int kp_multi_create(const int* devices, uint32_t n_devices, kp_multi** out);
void kp_multi_destroy(kp_multi* m);
const char* kp_multi_last_error(const kp_multi* m);
uint32_t kp_multi_devices(const kp_multi* m);
/* The engine of the i-th device (stage times, diagnosis entry points); owned by m. */
kp_engine* kp_multi_engine(kp_multi* m, uint32_t i);

int kp_multi_snapshot_create(kp_multi* m, const kp_cluster* clusters, uint64_t n_clusters, const kp_options* opts,
                             kp_multi_snapshot** out);
/* kp_snapshot_update on every replica (same semantics, same dict_grew). If it fails on
 * any device the others may already have applied the rows, so the multi snapshot is
 * marked invalid: this call, kp_multi_batch_create and kp_multi_schedule on it return
 * KP_ESTATE until it is destroyed and created again. */
int kp_multi_snapshot_update(kp_multi* m, kp_multi_snapshot* s, const kp_cluster* clusters, uint64_t n_clusters,
                             int* dict_grew);
void kp_multi_snapshot_destroy(kp_multi_snapshot* s);
/* The i-th device's replica; owned by s. */
kp_snapshot* kp_multi_snapshot_replica(kp_multi_snapshot* s, uint32_t i);

/* The shard cuts kp_multi_batch_create uses: starts[0..n_shards], starts[0] = 0,
 * starts[n_shards] = n_bindings. */
int kp_multi_shard_cuts(const kp_binding* bindings, uint64_t n_bindings, uint64_t n_clusters, uint32_t n_shards,
                        uint64_t* starts);
int kp_multi_batch_create(kp_multi* m, const kp_multi_snapshot* s, const kp_binding* bindings, uint64_t n_bindings,
                          kp_multi_batch** out);
void kp_multi_batch_destroy(kp_multi_batch* b);
/* The batch's shard cuts (n_devices + 1 entries). */
int kp_multi_batch_shards(const kp_multi_batch* b, uint64_t* starts);
/* genericScheduler.Schedule for every binding, the shards on their devices at once. */
int kp_multi_schedule(kp_multi* m, kp_multi_batch* b, kp_results* out);

#ifdef __cplusplus
}
#endif

#endif /* KP_API_H */
