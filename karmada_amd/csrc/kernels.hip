// kernels.hip — CDNA4 (gfx950) kernels of the batched placement engine.
//
// k_pair          one workgroup per binding; each wave64 evaluates 64 consecutive
//                 clusters (coalesced SoA columns), emits their feasibility as one
//                 u64 ballot word and the calAvailableReplicas answer per cluster.
// k_select_all    SEL_ALL bindings: block-parallel assignment (Webster threshold
//                 search, Aggregated cut) over the candidates compacted in LDS.
// k_select_cluster / k_region_a / k_region_b   spread-constraint selection.
// k_slow          persistent workgroups: exact serial emulation for flagged bindings.
#include <hip/hip_runtime.h>

#include "kp_launch.h"
#include "kp_paths.h"

using namespace kp;

namespace {

__device__ __forceinline__ SelCtx make_ctx(const KArgs& a, int b, const uint32_t* tgt_bits) {
  SelCtx x;
  x.s = &a.s;
  x.bv = &a.bv;
  x.h = &a.bv.hdr[b];
  x.b = b;
  x.frow = a.fmask + (size_t)b * a.s.W;
  x.erow = a.est + (size_t)b * a.s.Cp;
  x.tgt_bits = tgt_bits;
  x.sink = a.sink;
  return x;
}

// LDS bitset of the binding's spec.Clusters ranks (TargetContains, locality).
__device__ void build_bits(const GpuBlk& B, uint32_t* bits, int words, const int32_t* pool, int off, int cnt,
                           int stride) {
  for (int i = B.tid(); i < words; i += B.nth()) bits[i] = 0;
  B.sync();
  for (int j = B.tid(); j < cnt; j += B.nth()) {
    int r = pool[off + stride * j];
    atomicOr(&bits[r >> 5], 1u << (r & 31));
  }
  B.sync();
}

__device__ bool pre_checks(const GpuBlk& B, const SelCtx& x, int F) {
  // status of bindings that never reach selection
  if (x.h->flags & BF_BAD) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_NONE, 0);
    return true;
  }
  if (F == 0) {  // FitError (generic_scheduler.go:84-89)
    if (B.tid() == 0) sink_error(x, KP_STATUS_FIT_ERROR, KP_ERR_FIT, x.s->C);
    return true;
  }
  return false;
}

}  // namespace

// ---------------------------------------------------------------------------
// Pair stage
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_pair(SnapView s, BatchView bv, int b0, uint64_t* fmask,
                                                         int32_t* est, int64_t* score, int est_mode, int md_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  const int b = b0 + blockIdx.x;
  const BindHdr h = bv.hdr[b];
  const int words = (s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + 512);
  uint32_t* evict = tgt + words;
  int32_t* md = (int32_t*)(evict + words);
  build_bits(B, tgt, words, bv.ipool, h.tgt_off, h.tgt_cnt, 2);
  build_bits(B, evict, words, bv.ipool, h.evict_off, h.evict_cnt, 1);
  const bool use_md = s.n_tmpl <= md_cap && (h.flags & BF_HAS_RR);
  if (use_md) {
    for (int t = B.tid(); t < s.n_tmpl; t += B.nth()) md[t] = template_md(s, bv, h, t);
    B.sync();
  }
  uint64_t* frow = fmask + (size_t)b * s.W;
  int32_t* erow = est + (size_t)b * s.Cp;
  const int lane = threadIdx.x & 63;
  for (int base = 0; base < s.Cp; base += blockDim.x) {
    const int c = base + threadIdx.x;
    bool fit = false;
    int32_t e = 0;
    if (est_mode == 0) {
      fit = pair_feasible(s, bv, h, c, tgt, evict);
      if (fit) e = cal_available(s, bv, h, c, use_md ? md : nullptr);
    } else if (c < s.C) {  // raw GeneralEstimator answers for every cluster
      e = general_estimate(s, bv, h, c, use_md ? md : nullptr);
      fit = true;
    }
    const uint64_t m = __ballot(fit);
    if (lane == 0 && (c >> 6) < s.W) frow[c >> 6] = m;
    if (c < s.Cp) erow[c] = e;
    if (score && c < s.C) {
      int64_t sc = 0;
      if ((h.enabled & KP_PLUGIN_CLUSTER_LOCALITY) && h.n_targets_all > 0 && h.tgt_cnt > 0 && bit_test(tgt, c)) sc = 100;
      score[(size_t)b * s.C + c] = sc;
    }
  }
}

// ---------------------------------------------------------------------------
// Select stage: SEL_ALL (and spread-unsupported / FitError reporting)
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_select_all(KArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  if ((int)blockIdx.x >= a.n) return;
  const int b = a.list[blockIdx.x];
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + 512);
  Cands cd;
  cd.r = tgt + words;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  const bool weights = h->strategy == ST_STATIC && h->sel == SEL_ALL;
  cd.F = gather(B, x, cd, weights);
  if (pre_checks(B, x, cd.F)) return;
  if (h->sel == SEL_ERR_UNSUPPORTED) {  // select_clusters.go:54
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, KP_ERR_SPREAD_UNSUPPORTED, 0);
    return;
  }
  if (!sel_all_fast(B, x, cd)) {
    if (B.tid() == 0) {
      a.slow[b] = 1;
      a.sink.count[b] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Select stage: SEL_CLUSTER
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_select_cluster(KArgs a, int scratch_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  if ((int)blockIdx.x >= a.n) return;
  const int b = a.list[blockIdx.x];
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* hist = (uint32_t*)(smem + 512);
  Item* items = (Item*)(smem + 512 + 1024);
  uint64_t* keys = (uint64_t*)(items + 2 * kSmallMax);
  uint32_t* tgt = (uint32_t*)(keys + 2 * kSmallMax);
  unsigned char* area = (unsigned char*)(tgt + ((words + 3) & ~3));
  Cands cd;
  cd.r = (uint32_t*)area;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  cd.F = gather(B, x, cd, false);
  if (pre_checks(B, x, cd.F)) return;
  if (!sel_cluster_fast(B, x, cd, hist, items, keys, area, scratch_cap)) {
    if (B.tid() == 0) {
      a.slow[b] = 1;
      a.sink.count[b] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Region stage A: per-region count and group score for the host selectGroups.
// rout: [n][n_regions]
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_region_a(KArgs a, RegionOut* rout, int32_t* rstat) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  if ((int)blockIdx.x >= a.n) return;
  const int b = a.list[blockIdx.x];
  const int words = (a.s.Cp + 31) >> 5;
  const int R = a.s.n_regions;
  unsigned char* p = smem + 512;
  RegionLds L;
  L.minkey = (unsigned long long*)p;
  p += 8 * R;
  L.last = (unsigned long long*)p;
  p += 8 * R;
  L.sumAvail = (int64_t*)p;
  p += 8 * R;
  L.sumScore = (int64_t*)p;
  p += 8 * R;
  L.dscore = (int64_t*)p;
  p += 8 * R;
  L.wsum = (int64_t*)p;
  p += 8 * R;
  L.wscore = (int64_t*)p;
  p += 8 * R;
  L.amin = (int64_t*)p;
  p += 8 * R;
  L.cnt = (int32_t*)p;
  p += 4 * R;
  L.dvalid = (int32_t*)p;
  p += 4 * R;
  L.wcnt = (int32_t*)p;
  p += 4 * R;
  L.done = (int32_t*)p;
  p += 4 * R;
  uint32_t* tgt = (uint32_t*)p;
  p += 4 * ((words + 3) & ~3);
  Cands cd;
  cd.r = (uint32_t*)p;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  cd.F = gather(B, x, cd, false);
  if (pre_checks(B, x, cd.F)) {
    if (B.tid() == 0) rstat[blockIdx.x] = -1;  // final status already written
    return;
  }
  region_a(B, x, cd, L, rout + (size_t)blockIdx.x * R);
  if (B.tid() == 0) rstat[blockIdx.x] = 0;
}

// Region stage B. rsel: [n][n_regions] selected region ids (path order), rnsel[n]:
// count, or -KP_ERR_* when the host group selection failed.
extern "C" __global__ void __launch_bounds__(256) k_region_b(KArgs a, const int32_t* rsel, const int32_t* rnsel,
                                                             int scratch_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  if ((int)blockIdx.x >= a.n) return;
  const int b = a.list[blockIdx.x];
  const int nsel = rnsel[blockIdx.x];
  const int words = (a.s.Cp + 31) >> 5;
  const int R = a.s.n_regions;
  unsigned char* p = smem + 512;
  uint32_t* hist = (uint32_t*)p;
  p += 1024;
  Item* items = (Item*)p;
  p += sizeof(Item) * 2 * kSmallMax;
  uint64_t* keys = (uint64_t*)p;
  p += 8 * 2 * kSmallMax;
  unsigned long long* heads = (unsigned long long*)p;
  p += 8 * R;
  int32_t* rs = (int32_t*)p;
  p += 4 * ((R + 3) & ~3);
  uint32_t* tgt = (uint32_t*)p;
  p += 4 * ((words + 3) & ~3);
  Cands cd;
  cd.r = (uint32_t*)p;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  const BindHdr* h = &a.bv.hdr[b];
  if (nsel == -1000) return;  // stage A already reported the final status
  build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
  SelCtx x = make_ctx(a, b, tgt);
  if (nsel < 0) {
    if (B.tid() == 0) sink_error(x, KP_STATUS_ERROR, -nsel, 0);
    return;
  }
  cd.F = gather(B, x, cd, false);
  region_b(B, x, cd, rsel + (size_t)blockIdx.x * R, nsel, hist, heads, rs, items, keys, p, scratch_cap);
}

// ---------------------------------------------------------------------------
// Exact serial path: candidates fully sorted by the sortClusters key in global
// scratch, then the Go algorithm on thread 0 (Aggregated ties with the pdqsort
// emulation, scale-down, overflow tiers, duplicates, wrap-around).
// Persistent grid: block k handles list entries k, k+grid, ...
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_slow(KArgs a, unsigned char* scratch, size_t slot_bytes,
                                                         int scratch_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  GpuBlk B{(int64_t*)smem};
  const int words = (a.s.Cp + 31) >> 5;
  uint32_t* tgt = (uint32_t*)(smem + 512);
  unsigned char* mine = scratch + (size_t)blockIdx.x * slot_bytes;
  // slot layout: cand r/v [Cp] | keys [P] | items [Cp] | pos [Cp] | serial scratch
  int P = 1;
  while (P < a.s.Cp) P <<= 1;
  Cands cd;
  cd.r = (uint32_t*)mine;
  cd.v = (int32_t*)(cd.r + a.s.Cp);
  uint64_t* keys = (uint64_t*)(cd.v + a.s.Cp);
  Item* items = (Item*)(keys + P);
  int32_t* pos = (int32_t*)(items + a.s.Cp);
  unsigned char* ser = (unsigned char*)(pos + a.s.Cp);
  for (int i = B.tid(); i < a.s.Cp; i += B.nth()) pos[i] = -1;
  for (int idx = blockIdx.x; idx < a.n; idx += gridDim.x) {
    const int b = a.list[idx];
    if (!a.slow[b]) continue;
    const BindHdr* h = &a.bv.hdr[b];
    build_bits(B, tgt, words, a.bv.ipool, h->tgt_off, h->tgt_cnt, 2);
    SelCtx x = make_ctx(a, b, tgt);
    cd.F = gather(B, x, cd, false);
    const int F = cd.F;
    for (int i = B.tid(); i < P; i += B.nth()) keys[i] = i < F ? cand_key(x, cd, i, cd.v[i]) : ~0ull;
    B.sync();
    for (int k = 2; k <= P; k <<= 1)  // bitonic sort (ascending)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = B.tid(); i < P; i += B.nth()) {
          int l = i ^ j;
          if (l > i) {
            uint64_t ki = keys[i], kl = keys[l];
            bool up = (i & k) == 0;
            if ((ki > kl) == up) {
              keys[i] = kl;
              keys[l] = ki;
            }
          }
        }
        __threadfence_block();
        B.sync();
      }
    for (int i = B.tid(); i < F; i += B.nth()) items[i] = item_from_key(x, keys[i]);
    __threadfence_block();
    B.sync();
    if (B.tid() == 0) {
      SerialScratch sc = serial_scratch_carve(ser, scratch_cap);
      sc.pos = pos;
      int n = F;
      bool err = false;
      if (h->sel == SEL_CLUSTER) {  // selectBestClustersByCluster on the sorted list
        if ((int64_t)F < h->cluster_min) {
          sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_MIN_GROUPS, 0);
          err = true;
        } else {
          int64_t needCnt = (int64_t)F < h->cluster_max ? (int64_t)F : h->cluster_max;
          if (needCnt < 0) needCnt = 0;
          if (h->need_replicas != -1) {
            auto check = [&]() {
              int64_t t = 0;
              for (int i = 0; i < needCnt; i++) t += items[i].avail;
              return t >= (int64_t)h->need_replicas;
            };
            int64_t upd = needCnt - 1;
            while (!check() && upd >= 0) {
              int64_t mv = items[upd].avail;
              int64_t id = -1;
              for (int64_t i = needCnt; i < F; i++)
                if (mv < items[i].avail) {
                  id = i;
                  mv = items[i].avail;
                }
              if (id < 0) {
                upd--;
                continue;
              }
              Item t = items[upd];
              items[upd] = items[id];
              items[id] = t;
              upd--;
            }
            if (!check() || needCnt == 0) {
              sink_error(x, KP_STATUS_ERROR, KP_ERR_CLUSTER_RESOURCE, needCnt);
              err = true;
            }
          }
          n = (int)needCnt;
        }
      }
      if (!err) {
        SerialAssign sa{x, sc, (h->flags & BF_UID_DESC) != 0};
        SerialOut o = sa.run(items, n);
        sink_serial(x, sc, o);
      }
      a.slow[b] = 0;
    }
    B.sync();
  }
}

// Gathers per-binding results into CSR order (offsets computed on the host).
extern "C" __global__ void k_compact(const uint64_t* start, const uint32_t* count, const uint64_t* offsets,
                                     const uint32_t* in_idx, const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep,
                                     int n) {
  int b = blockIdx.x;
  if (b >= n) return;
  uint64_t s = start[b], o = offsets[b];
  uint32_t c = count[b];
  for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
    out_idx[o + i] = in_idx[s + i];
    out_rep[o + i] = in_rep[s + i];
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
namespace kp {

hipError_t launch_pair(hipStream_t st, const SnapView& s, const BatchView& bv, int b0, int nb, uint64_t* fmask,
                       int32_t* est, int64_t* score, int est_mode, int md_cap, size_t smem) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair, dim3(nb), dim3(kBlock), smem, st, s, bv, b0, fmask, est, score, est_mode, md_cap);
  return hipGetLastError();
}

hipError_t launch_select(hipStream_t st, int which, const KArgs& a, size_t smem, int cap, const SelectExtra& x) {
  if (a.n <= 0) return hipSuccess;
  switch (which) {
    case SEL_LAUNCH_ALL:
      hipLaunchKernelGGL(k_select_all, dim3(a.n), dim3(kBlock), smem, st, a);
      break;
    case SEL_LAUNCH_CLUSTER:
      hipLaunchKernelGGL(k_select_cluster, dim3(a.n), dim3(kBlock), smem, st, a, cap);
      break;
    case SEL_LAUNCH_REGION_A:
      hipLaunchKernelGGL(k_region_a, dim3(a.n), dim3(kBlock), smem, st, a, x.rout, x.rstat);
      break;
    case SEL_LAUNCH_REGION_B:
      hipLaunchKernelGGL(k_region_b, dim3(a.n), dim3(kBlock), smem, st, a, x.rsel, x.rnsel, cap);
      break;
    case SEL_LAUNCH_SLOW:
      hipLaunchKernelGGL(k_slow, dim3(x.grid), dim3(kBlock), smem, st, a, x.scratch, x.slot_bytes, cap);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_compact(hipStream_t st, const uint64_t* start, const uint32_t* count, const uint64_t* offsets,
                          const uint32_t* in_idx, const int32_t* in_rep, uint32_t* out_idx, int32_t* out_rep, int n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compact, dim3(n), dim3(64), 0, st, start, count, offsets, in_idx, in_rep, out_idx, out_rep, n);
  return hipGetLastError();
}

}  // namespace kp
