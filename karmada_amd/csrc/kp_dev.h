// kp_dev.h — the device interface engine.cpp runs on.
//
// libkp.so implements it with HIP on gfx950 (kernels.hip). The test-only
// libkp_cpusim.so implements it on the host (dev_cpu.cpp) by running the same
// kernel bodies (kp_kernels.h) with a 1-thread block policy, so the engine's
// orchestration and kernel logic can be checked without a GPU. The CPU build
// is never linked into libkp.so.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "kp_launch.h"

namespace kp {
struct SetsArgs;
struct TopArgs;
struct OrderArgs;
struct RegionOut;
struct GradesArgs;
struct NodeEstArgs;
struct NodeView;
struct ClaimProg;
struct NodeSetsArgs;
namespace dev {

typedef void* stream_t;
typedef void* event_t;

int device_count();
int set_device(int device);
size_t max_lds_per_block(int device);
const char* last_error();  // text of the last failing call

int stream_create(stream_t* s);
void stream_destroy(stream_t s);
int sync(stream_t s);
int event_create(event_t* e);
void event_destroy(event_t e);
int event_record(event_t e, stream_t s);
int event_sync(event_t e);  // host waits for e
int stream_wait(stream_t s, event_t e);  // s waits for e (no host block)
float event_ms(event_t a, event_t b);

int alloc(void** p, size_t bytes);
void release(void* p);
// Page-locked host memory: the result copy-back DMAs straight into it.
int host_alloc(void** p, size_t bytes);
void host_release(void* p);
int h2d(void* dst, const void* src, size_t bytes, stream_t s);  // stream-ordered
int d2h(void* dst, const void* src, size_t bytes, stream_t s);
int fill(void* dst, int value, size_t bytes, stream_t s);
// Device-to-device copy between GPUs (xGMI peer copy; same device: a local copy).
int peer_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, stream_t s);

// fast: the estimator instance (EST_*); other than EST_GENERIC only for batches
// that meet pair_fast_ok.
// Pair rows of bindings list[b0 + i] (or b0 + i when list is null), i < nb.
int pair(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* list, int b0, int nb, uint64_t* fmask,
         int32_t* est, int64_t* score, int est_mode, int md_cap, size_t smem, int fast = 0);
// Estimator-class rows: rows[k][Cp] for k = klist[i] (k = i when klist is null), i < n_rows
// (body_est_class; row 0 MaxInt32), class k's representative binding rep[k]; fast = EST_*
// kind (not EST_GENERIC). fmask set: only the entries of the representative's feasible
// clusters (the singleton classes of a batch without class orders, after k_filter).
int est_class(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* rep, int n_rows, int32_t* rows,
              int fast, const int32_t* klist = nullptr, const uint64_t* fmask = nullptr);
// Feasibility rows fmask[b][W] of every binding by bitset algebra (body_filter;
// requires s.n_bits > 0).
int filter(stream_t st, const SnapView& s, const BatchView& bv, uint64_t* fmask);
int select(stream_t st, int which, const KArgs& a, size_t smem, int cap, const SelectExtra& x);
// Estimator-class orders for k_select_top: ord[k][i] = (estimate << 32 | rank) of
// rows[k] sorted by estimate desc, rank asc; tot[k] its sum; ok[k] whether it can be
// walked (body_class_order). C <= 16384.
int class_order(stream_t st, const SnapView& s, const int32_t* rows, int n_rows, uint64_t* ord, int64_t* tot,
                int32_t* ok);
// SEL_ALL DynamicWeight / Aggregated bindings a.list[0, a.n) over their deciding
// candidates (body_select_top), `slice` bytes of LDS per binding; the others are
// appended to t.fb.
// (a.n_dev set: the list's length is on the device, a.n its capacity; max_grid > 0
// bounds the grid, whose waves then stride over the list)
int select_top(stream_t st, const KArgs& a, const TopArgs& t, size_t slice, int max_grid = 0);
// k_select_top_wg: one workgroup per binding (the large-subset bindings), smem = top_wg_lds_bytes
int select_top_wg(stream_t st, const KArgs& a, const TopArgs& t, size_t smem);
// selectGroups for n region bindings (one thread each): rsel/rnsel as the host
// step writes them; *nhost counts the bindings left to the host (kGroupsHost).
int region_groups(stream_t st, const RegionOut* rout, const int32_t* rstat, const BindHdr* hdr, const int32_t* list,
                  int n, int R, int32_t* rsel, int32_t* rnsel, uint32_t* nhost);
// kp_max_available_component_sets: out[i] = sets_one for cluster rank ranks[i]
// (A, ranks and off in device memory; cluster i's runs at scratch[off[i], off[i+1])).
int component_sets(stream_t st, const SnapView& s, const SetsArgs* A, const int32_t* ranks, const int64_t* off,
                   uint64_t n, int64_t* scratch, int32_t* out);
// Component-set class row: row[r] = sets_one for every cluster rank r < C (cluster r's
// runs at scratch[off[r], off[r+1])); *ovf = 1 when a simulation outgrew its runs.
int sets_rows(stream_t st, const SnapView& s, const SetsArgs* A, const int64_t* off, int64_t* scratch, int32_t* row,
              uint32_t* ovf);
// Pair-row mode: est[b][c] of the n bindings list[i] rebuilt from their class rows
// (cal_merge_bf with spec.Replicas on feasible clusters, 0 elsewhere, as pair_eval writes).
int rows_from_class(stream_t st, const SnapView& s, const BatchView& bv, const int32_t* list, int n,
                    const int32_t* bcls, const int32_t* cls_rows, const uint64_t* fmask, int32_t* est);
// kp_model_grades: A.counts[grade] += 1 per node (body_grades); A's arrays in device memory.
int grades(stream_t st, const GradesArgs& A);
// kp_node_max_replicas: *A.sum += int32 sum of node_replicas over the nodes (wrapping).
int node_est(stream_t st, const NodeEstArgs& A);
// StaticWeight SEL_ALL bindings a.list[0, a.n) at class level (body_select_static),
// one wave each with `slice` bytes of LDS.
int select_static(stream_t st, const KArgs& a, size_t slice);
// Spread selections over the estimator-class orders (body_spread_order), one wave
// per binding, `slice` bytes of LDS each; unfinished list positions go to o.fb.
int spread_order(stream_t st, const KArgs& a, const OrderArgs& o, size_t slice);
// Region stage A of the order-eligible bindings (body_region_a_order), one wave per
// binding; the other list positions go to fb.
int region_a_order(stream_t st, const KArgs& a, RegionOut* rout, int32_t* rstat, int32_t* fb, uint32_t* fb_n,
                   size_t slice);
// kp_node_max_component_sets: match[k * n + j] = MatchNode(node j, P[k]) (P in
// device memory), then the first-fit set simulation by one wave (A in device memory).
int node_match(stream_t st, const NodeView& v, const ClaimProg* P, int K, uint8_t* match);
int node_sets(stream_t st, const NodeSetsArgs* A);
// kp_filter_reasons: out[(b - b0) * C + r] = pair_reason of binding b in [b0, b0 + nb), cluster rank r.
int reasons(stream_t st, const SnapView& s, const BatchView& bv, int b0, int nb, uint32_t* out);
// CSR offsets[n + 1] of the per-binding results (counts of OK bindings), on the device;
// part: ceil(n / kOffChunk) u64 of scratch.
int offsets(stream_t st, const int32_t* status, const uint32_t* count, int n, uint64_t* off, uint64_t* part);
// (in_idx holds snapshot ranks; out_idx gets perm[rank], the caller's cluster index)
// h_idx / h_rep (device addresses of page-locked host buffers, h_cap entries each): the
// CSR entries below h_cap are also written there, over the bus, by the kernel itself.
int compact(stream_t st, const uint64_t* start, const uint32_t* count, const uint64_t* offsets, const uint32_t* in_idx,
            const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n, const uint32_t* perm,
            uint32_t* h_idx = nullptr, int32_t* h_rep = nullptr, uint64_t h_cap = 0);
// The device address of page-locked host memory from host_alloc (the same on the host build).
int host_device_ptr(void* host, void** dev);

}  // namespace dev
}  // namespace kp
