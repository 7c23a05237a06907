"""Benchmark: ResourceBindings scheduled/sec through the HIP placement engine.

Workload (BASELINE.json metric config, configs[2]): 100k bindings x 5k clusters,
GeneralEstimator with 8 resource-model grades, 50% DynamicWeight / 50%
Aggregated (synthetic universe of SURVEY.md §8(d), seed 3). A step = one
kp_schedule_batch over the whole batch: filter -> score -> estimate -> select ->
divide, results copied back to the host as CSR. Packed inputs are resident in
HBM before the timed region; `end_to_end_value` times binding packing + upload +
schedule together (the snapshot is packed once per cache generation). Multi-GPU:
one process per GPU, each schedules its own contiguous binding range of the
universe against its own snapshot replica (weak scaling, no data-path
collective); the per-rank CSR results are all-gathered after the timed region.

In flight: --inflight engines (default 4), each with its own HIP streams and its
own copy of the batch, are driven by as many host threads, so one batch's host
steps and result copy-back overlap another batch's kernels (a scheduler keeping
several batches in flight); `serial_value` is one batch at a time. The lane
threads issue the warm-up steps themselves and keep going: the timed region
starts at the (W x lanes)-th completion, with every lane mid-stream, and ends at
the K-th completion after it, before any lane runs dry. So K timed steps measure
the steady state, not the pipeline's fill and drain (each lane's step in flight
at the end finishes untimed).

Roofline: the dominant kernel of the step (by its HIP-event time) against HBM
peak with compulsory bytes, plus the counter-derived DRAM bytes
(FETCH_SIZE x2 on gfx950 + WRITE_SIZE) and VALU issue fraction of the same
kernel from the committed PMC summary (profiles/r03_pmc_config<N>.json, else r02).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

# Hardware queues per process (read once, when the HIP runtime starts; nothing here has
# touched the GPU yet). HIP maps a process's streams onto GPU_MAX_HW_QUEUES in-order
# hardware queues (4 by default, what the GPU boxes export); streams that share a queue
# run in order. The bench keeps the environment's setting (KP_HW_QUEUES overrides it)
# and sizes the engines' streams to it (KP_STREAMS, main(); DESIGN.md §5 "Round 6").
if os.environ.get("KP_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, int(os.environ["KP_HW_QUEUES"]))))

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 instruction per 2 cycles per SIMD
# at 2.4 GHz (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # 1228.8 G wave-instructions/s
# Per-binding input record: BindHdr (160 B) + its pool slices (~96 B on these workloads)
B_BIND = 256
# pair kernel instance per kp_stage_times.pair_kind (kp_algo.h EST_*)
PAIR_KERNELS = {0: "k_pair", 1: "k_pair_fast", 2: "k_pair_fast_summary", 8: "k_pair_fast_m8", 16: "k_pair_fast_m16"}


def compulsory_bytes(n_bind, n_all, n_clusters, n_targets, snap_bytes, n_classes):
    """Compulsory HBM bytes per launch.
    bits mode (n_classes > 0):
      filter stage = snapshot (incl. its bitset rows) once + binding records + the
                     feasibility row (Cp/8) written per binding + the estimator-class
                     rows (4*Cp each) written once;
      k_select_all = its bindings' records and feasibility rows read back, the class
                     rows once, their results (cluster u32 + replicas i32 per target,
                     status/err/arg/start/count per binding).
    pair-row mode: the pair kernel writes a 4*Cp est row per binding and k_select_all
    reads it back."""
    Cp = (n_clusters + 63) // 64 * 64
    if n_classes:
        cls = 4.0 * Cp * n_classes
        pair = snap_bytes + n_bind * (B_BIND + Cp / 8.0) + cls
        sel = n_all * (B_BIND + Cp / 8.0 + 28) + cls + 8.0 * n_targets
    else:
        row = 4.0 * Cp + Cp / 8.0
        pair = snap_bytes + n_bind * (B_BIND + row)
        sel = n_all * (B_BIND + row + 28) + 8.0 * n_targets
    return pair, sel


def kernel_bytes(name, units, Cp, n_classes, n_bind, n_targets, snap_bytes, R, orders=True):
    """Compulsory HBM bytes of one kernel over the units (bindings or class rows) its
    launches covered: the records and feasibility rows it must read
    (256 + Cp/8 B per binding), the class rows (4 B/cluster) and orders (8 B/cluster)
    it reads once, the results it writes (8 B per target, 28 B per binding).
    orders=False: the batch built no class orders (k_select_top thresholds each
    binding's votes by a histogram instead, kp_top.h), so only the class rows count."""
    if units == 0 and name not in ("k_offsets", "k_compact"):
        return 0.0  # (an empty fallback list: the launch found nothing to do)
    rec = B_BIND + Cp / 8.0
    share = n_targets * units / max(1, n_bind)  # its bindings' share of the targets
    if name.startswith("k_est_class"):
        return snap_bytes + 4.0 * Cp * units
    if name.startswith("k_pair"):
        return snap_bytes + units * (B_BIND + Cp / 8.0 + 4.0 * Cp)
    if name == "k_filter":
        return units * rec
    if name == "k_class_order":
        return 12.0 * Cp * units
    if name in ("k_select_top", "k_select_top_wg"):
        return units * (rec + 28) + (12.0 if orders else 4.0) * Cp * n_classes + 8.0 * share
    if name == "k_select_static":
        return units * (rec + 28) + 8.0 * share
    if name in ("k_spread_order", "k_region_a_order"):
        return units * (rec + 28) + 12.0 * Cp * n_classes + 8.0 * share
    if name == "k_region_groups":
        return units * (B_BIND + 16.0 * max(1, R))
    if name == "k_slow":
        return units * (rec + 4.0 * Cp + 28) + 8.0 * share
    if name == "k_offsets":
        return n_bind * 16.0
    if name == "k_compact":
        return n_bind * 20.0 + 16.0 * n_targets
    # k_select_all*, k_select_cluster*, k_region_a*, k_region_b*: the bindings' records,
    # feasibility rows and class rows, their results
    return units * (rec + 28) + 4.0 * Cp * n_classes + 8.0 * share


def load_pmc(config, kernel):
    """Per-launch PMC figures of `kernel` from the committed summary (same bench
    command, default sizes): {hbm_bytes (FETCH_SIZE*2 + WRITE_SIZE), valu_insts, ...}."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # the newest summary that holds the kernel
        try:
            with open(os.path.join(ROOT, "profiles", f"{rnd}_pmc_config{config}.json")) as f:
                k = json.load(f).get("kernels", {}).get(kernel)
        except (OSError, ValueError):
            continue
        if k:
            return k
    return None


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on
    (sched_getaffinity), capped by its cgroup CPU quota (cpu.max) when one is set,
    or KP_CPU_THREADS."""
    if os.environ.get("KP_CPU_THREADS"):
        return max(1, int(os.environ["KP_CPU_THREADS"]))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(u, opts, budget_s):
    """Oracle (faithful C++ restatement, REFSHAPE mode) on a bounded sample, rank 0 only,
    at 1 thread and at every CPU the process may use."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    threads = cpu_threads()
    out = {}
    for th, share in ((1, 0.35), (threads, 0.65)):
        n = 16
        while True:
            n = min(n, u.n_bindings)
            ba, _ = u.binding_slice(0, n)
            t0 = time.perf_counter()
            O.schedule_c(u.clusters, u.n_clusters, ba, n, opts, O.REFSHAPE, th)
            dt = time.perf_counter() - t0
            if dt >= budget_s * share / 3 or n >= u.n_bindings:
                break
            n *= 2
        out[th] = (n / dt, n, dt)
    rate, n, dt = out[threads]
    r1, n1, dt1 = out[1]
    return {
        "value": round(rate, 2), "unit": "ResourceBindings/s", "cores": threads, "kind": "port",
        "sample": (f"{n} bindings of the same workload in {dt:.1f}s on {threads} threads "
                   f"(1 thread: {r1:.2f}/s over {n1} bindings in {dt1:.1f}s); oracle REFSHAPE mode = "
                   "faithful restatement with per-binding snapshot deep copy, FF loop replaced by its "
                   "closed form (the literal FF loop is intractable here), so a lower bound on the "
                   "reference's cost"),
        "single_thread_value": round(r1, 3),
        "os_cpu_count": os.cpu_count(),
    }


def timed_gaps(clock, n_warm, steps, cap=64):
    """Intervals between consecutive completions inside the timed window (ms), with the
    lane that completed; at most `cap` of them."""
    st = clock["stamps"]
    lo = max(0, n_warm - 1)
    out = []
    for i in range(lo + 1, min(len(st), n_warm + steps)):
        out.append([round(1e3 * (st[i][0] - st[i - 1][0]), 3), st[i][1]])
    return out[:cap]


def parity_check(u, results, opts, n_check, seed):
    """Oracle (FAST mode) on n_check bindings sampled from the timed batch, compared
    with each given result list (status, error, multiset of targets): the serial
    run and every in-flight lane's last step. Test infrastructure, after the timed
    region. Returns (bindings checked, mismatches summed over the lists)."""
    import random
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from karmada_amd import api
    n = min(n_check, u.n_bindings)
    if n <= 0:
        return 0, 0
    idx = sorted(random.Random(seed).sample(range(u.n_bindings), n))
    arr = (api.kp_binding * n)(*[u.bindings[i] for i in idx])
    want = O.schedule_c(u.clusters, u.n_clusters, arr, n, opts, O.FAST, min(16, cpu_threads()))
    bad = sum(1 for res in results for k, i in enumerate(idx) if res[i] != want[k])
    return n, bad


def launch_ranks(n):
    """`bench.py --gpus N` without WORLD_SIZE: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them,
    rendezvous on 127.0.0.1) and exit with the first failing rank's code. This parent
    never touches the GPU: each rank selects its own device (LOCAL_RANK)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in procs:  # a rank failed: the others would wait at a collective
                    q.terminate()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--clusters", type=int, default=None)
    ap.add_argument("--bindings", type=int, default=None, help="bindings per GPU")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", type=int, default=1000,
                    help="bindings of the timed batch re-checked against the oracle after timing (0: off)")
    ap.add_argument("--e2e-reps", type=int, default=5, help="timed pack+upload+schedule repetitions (0: off)")
    ap.add_argument("--e2e-churn", type=float, default=0.1,
                    help="share of bindings at a new generation per end-to-end cycle (the rest reuse their records)")
    ap.add_argument("--lib", default=None, help="engine library (default karmada_amd/libkp.so)")
    ap.add_argument("--per-lane", type=int, default=None,
                    help="batches per in-flight lane (2: the lane submits its next batch before collecting "
                         "the last, kp_schedule_batch_submit/_collect; default 1)")
    # (6: the driver's exact command on two boxes, 5 runs each, means 74.9 / 74.2 M/s at 4 lanes,
    # 80.1 / 85.3 at 6, 86.0 at 8 with a wider spread; profiles/r06_ab/inflight_*.json)
    ap.add_argument("--inflight", type=int, default=6,
                    help="batches in flight per GPU: engines (own HIP streams) driven by as many host threads, "
                         "so one batch's result copy-back and host steps overlap another's kernels")
    args = ap.parse_args()
    if args.steps < 1:
        sys.exit("bench.py: --steps must be >= 1 (the timed window ends at the K-th completion)")

    # One HIP stream per engine when several batches are in flight: the lanes' streams then
    # fit HIP's default 4 hardware queues instead of sharing them in order (same-box A/B at 4
    # queues, profiles/r06_streams_ab.jsonl: 3 streams x 4 lanes 64.4-66.5 M/s, 1 x 4
    # 72.3-80.0 M/s; DESIGN.md §5 "Round 6"). KP_STREAMS set in the environment wins.
    if args.inflight > 1:
        os.environ.setdefault("KP_STREAMS", "1")
        # The lanes' host waits sleep instead of polling (hipEventBlockingSync), leaving the
        # box's CPU quota to the lanes with host work (same box, driver's command, four runs
        # each: 93.0-98.8 vs 76.2-95.3 M/s, profiles/r06_ab/sync_*.json)
        os.environ.setdefault("KP_SYNC_BLOCK", "1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    from karmada_amd import api, synth
    from karmada_amd.dist import Csr
    from karmada_amd.engine import Batch, Engine, Snapshot

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # KP_DIST_FORCE=1 runs the collective path (snapshot broadcast, CSR all-gather)
    # even at world size 1, so RCCL is exercised on a one-GPU box
    if world > 1 or os.environ.get("KP_DIST_FORCE"):
        import torch
        import torch.distributed as dist
        # one rank per GPU over RCCL ("nccl"); KP_DIST_BACKEND=gloo rehearses the
        # same path with host tensors (ranks may then share a GPU)
        backend = os.environ.get("KP_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            # gloo: host tensors; ranks may share a GPU, or run the CPU build (--lib
            # karmada_amd/libkp_cpusim.so) with no GPU at all
            local = local % max(1, torch.cuda.device_count())
            if torch.cuda.device_count() > 0:
                torch.cuda.set_device(local)
            dist.init_process_group(backend=backend)
        tdev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    cfg = args.config
    C_def, B_def = synth.CONFIGS[cfg]
    C_ = args.clusters or C_def
    B = args.bindings or B_def
    seed = args.seed if args.seed is not None else cfg
    total = B * world  # B bindings per GPU on average (weak scaling)
    t0 = time.perf_counter()
    if world > 1:
        # cost-balanced contiguous shards of the whole universe (SURVEY §8(e) cost
        # model C + Rep_b * log2 F_b, F_b bounded by C before filtering)
        from karmada_amd.dist import binding_costs, shard_range_weighted
        costs = binding_costs(synth.replicas(cfg, seed, C_, 0, total), C_)
        lo, hi = shard_range_weighted(costs, world, rank)
    else:
        lo, hi = 0, B
    u = synth.Universe(cfg, seed, C_, lo, hi)
    B_rank = hi - lo
    gen_s = time.perf_counter() - t0
    opts = api.options()
    eng = Engine(local, lib_path=os.path.join(ROOT, args.lib)) if args.lib else Engine(local)
    t0 = time.perf_counter()
    if dist is None:
        snap = Snapshot.from_structs(eng, u.clusters, u.n_clusters, u.names, opts)
    else:  # rank 0 packs once; the packed bytes go to every rank over RCCL (dist.py)
        from karmada_amd.dist import broadcast_snapshot
        snap = Snapshot.from_structs(eng, u.clusters, u.n_clusters, u.names, opts) if rank == 0 else None
        snap = broadcast_snapshot(eng, snap, u.names)
    snap_s = time.perf_counter() - t0
    snap_bytes = len(snap.to_bytes())
    t0 = time.perf_counter()
    batch = Batch(snap, structs=u.binding_slice(0, u.n_bindings))
    pack_s = time.perf_counter() - t0

    def barrier_sync():
        if dist is not None:
            import torch
            dist.barrier()
            if torch.cuda.device_count() > 0:
                torch.cuda.synchronize()

    # in-flight batches: engine k schedules the same packed bindings (its own snapshot
    # replica and batch); steps are split over them, each step = one whole batch
    import threading
    # per_lane 2: each lane alternates two batches of the same bindings, submitting the next
    # before collecting the last (kp_schedule_batch_submit / _collect), so its engine's
    # stream stays queued while the host reads a batch back
    # (default 1: two per lane measured slower, 58.3-69.8 vs 67.7-85.6 M/s on one box,
    # profiles/r06_ab/perlane_*.json: more batches' kernels overlap on the GPU)
    per_lane = args.per_lane if args.per_lane is not None else 1
    per_lane = max(1, min(2, per_lane))
    lanes = [(eng, snap, batch, Batch(snap, structs=u.binding_slice(0, u.n_bindings)) if per_lane > 1 else None)]
    for _ in range(1, max(1, args.inflight)):
        e2 = Engine(local, lib_path=os.path.join(ROOT, args.lib)) if args.lib else Engine(local)
        s2 = Snapshot.from_bytes(e2, snap.to_bytes(), u.names)
        lanes.append((e2, s2, Batch(s2, structs=u.binding_slice(0, u.n_bindings)),
                      Batch(s2, structs=u.binding_slice(0, u.n_bindings)) if per_lane > 1 else None))
    st_all = []
    results = [None] * len(lanes)
    # completions counted over all lanes: the first n_warm are the warm-up (every lane
    # issues `warmup` of them on average), the next K are timed; a lane stops issuing
    # once the K-th timed step has completed
    n_warm = args.warmup * len(lanes)
    lock = threading.Lock()
    clock = {"done": 0, "t0": None, "t1": None, "stamps": []}
    if n_warm == 0:
        clock["t0"] = "at start"

    def drive(k):
        e_k, _, b_k, b_k2 = lanes[k]
        st = []
        pair = [b_k, b_k2] if b_k2 is not None else None
        i = 0
        if pair:
            pair[0].submit()
        while True:
            with lock:
                if clock["done"] >= n_warm + args.steps:
                    break
            if pair:
                pair[(i + 1) % 2].submit()  # the next batch queued behind this one
                r = pair[i % 2].collect()
                i += 1
            else:
                r = b_k.schedule_raw()
            with lock:
                now = time.perf_counter()  # (stamped in completion order, under the lock)
                clock["done"] += 1
                d = clock["done"]
                clock["stamps"].append((now, k))
                if d == n_warm:
                    clock["t0"] = now
                elif d == n_warm + args.steps:
                    clock["t1"] = now
                timed = n_warm < d <= n_warm + args.steps
            results[k] = r
            if timed:
                st.append(e_k.stage_times())
        if pair:  # the batch still in flight (after the window; its results stay unread)
            pair[i % 2].collect()
        with lock:
            st_all.extend(st)

    # The lanes' batches were just packed on every CPU the process may use: under a cgroup
    # CPU quota (16 CPUs on the GPU boxes) that burst can exhaust the current quota period,
    # and the lane threads would then be throttled inside the short timed window. Idle for a
    # few periods first (setup, outside the timed region).
    if len(lanes) > 1:
        time.sleep(float(os.environ.get("KP_BENCH_SETTLE_S", "0.3")))
    barrier_sync()
    t_start = time.perf_counter()
    if clock["t0"] == "at start":
        clock["t0"] = t_start
    if len(lanes) == 1:
        drive(0)
    else:
        th = [threading.Thread(target=drive, args=(k,)) for k in range(len(lanes))]
        for x in th:
            x.start()
        for x in th:
            x.join()
    barrier_sync()
    lanes_wall = time.perf_counter() - t_start
    elapsed = clock["t1"] - clock["t0"]
    rank_ms = 1e3 * elapsed / args.steps
    # every lane's last result (engine-owned until that engine's next call), copied
    # now: the in-flight lanes are parity-checked too, not only the serial run below
    lane_csr = [Csr.from_results(x) for x in results if x is not None]
    # one batch at a time (no overlap), for reference: a short serial run on engine 0
    serial_ms = None
    if len(lanes) > 1:
        n_ser = max(1, min(args.steps, 50))
        barrier_sync()
        t1 = time.perf_counter()
        st_ser = []
        for _ in range(n_ser):
            r = batch.schedule_raw()
            st_ser.append(eng.stage_times())
        barrier_sync()
        serial_ms = 1e3 * (time.perf_counter() - t1) / n_ser
        # copied before the profiled runs below reuse the engine's result buffers
        csr = Csr.from_results(r)
        # then every kernel of the step timed by its own HIP event pair (on the stream it
        # runs on), one batch at a time, for the per-kernel ranking and the roofline
        eng.set_profile(True)
        kt_runs = []
        for _ in range(n_ser):
            batch.schedule_raw()
            kt_runs.append(eng.kernel_times())
        eng.set_profile(False)
        st_all = st_ser  # per-stage HIP event times without another batch's kernels beside them
        if dist is not None:
            import torch
            t = torch.tensor([serial_ms], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            serial_ms = float(t.item())
    # ---- after the timed region ----
    if len(lanes) == 1:
        csr = Csr.from_results(results[0])  # before the profiled runs reuse the buffers
        eng.set_profile(True)
        kt_runs = []
        for _ in range(max(1, min(args.steps, 50))):
            batch.schedule_raw()
            kt_runs.append(eng.kernel_times())
        eng.set_profile(False)
    res = csr.to_python()
    n_ok = int((csr.status == 0).sum())
    n_targets_rank = n_targets = csr.n_targets
    per_rank_ms = [round(rank_ms, 3)]
    if dist is not None:
        import torch
        from karmada_amd.dist import gather_csr
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        pr = [torch.zeros(1, dtype=torch.float64, device=tdev) for _ in range(dist.get_world_size())]
        dist.all_gather(pr, torch.tensor([rank_ms], dtype=torch.float64, device=tdev))
        per_rank_ms = [round(float(x.item()), 3) for x in pr]
        whole = gather_csr(csr)  # two-phase CSR all-gather (counts, then padded arrays)
        n_ok = int((whole.status == 0).sum())
        n_targets = whole.n_targets
        # the parity check reads this rank's range of the GATHERED CSR (so the
        # collective's placement of every rank's block is checked too), not the local one
        res = whole.slice(lo, hi).to_python()

    # the oracle re-checks a sample of the serial run and of every in-flight lane's
    # last batch (lanes run concurrently on separate engines and streams)
    results_checked = [res] + [c.to_python() for c in lane_csr]
    n_chk, n_bad = parity_check(u, results_checked, opts, args.check, 1000 + rank) if args.check > 0 else (0, 0)
    n_lanes_chk = len(results_checked) if args.check > 0 else 0
    if dist is not None:
        t = torch.tensor([n_chk, n_bad], dtype=torch.int64, device=tdev)
        dist.all_reduce(t)
        n_chk, n_bad = int(t[0].item()), int(t[1].item())

    # end to end: binding packing + upload + schedule + results to host, per batch.
    # serial: one batch at a time; pipelined: two engines on this GPU, each packing
    # its next batch on the host while the other's batch runs on the device (a
    # scheduler draining its queue), timed over 2 x e2e_reps batches.
    for e_k, s_k, b_k, b_k2 in lanes[1:]:
        b_k.close()
        if b_k2 is not None:
            b_k2.close()
        s_k.close()
        e_k.close()
    if lanes[0][3] is not None:
        lanes[0][3].close()
    batch.close()
    e2e = e2e_pipe = e2e_reuse = None
    reuse_hits = 0.0
    if args.e2e_reps > 0:
        structs = u.binding_slice(0, u.n_bindings)
        ts = []
        for _ in range(args.e2e_reps):
            t1 = time.perf_counter()
            b2 = Batch(snap, structs=structs)
            b2.schedule_raw()
            ts.append(time.perf_counter() - t1)
            b2.close()
        e2e = sum(ts) / len(ts)
        import threading
        eng2 = Engine(local, lib_path=os.path.join(ROOT, args.lib)) if args.lib else Engine(local)
        snap2 = Snapshot.from_bytes(eng2, snap.to_bytes(), u.names)

        def drain(sn):
            for _ in range(args.e2e_reps):
                b3 = Batch(sn, structs=structs)
                b3.schedule_raw()
                b3.close()
        t1 = time.perf_counter()
        th = [threading.Thread(target=drain, args=(sn,)) for sn in (snap, snap2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        e2e_pipe = (time.perf_counter() - t1) / (2 * args.e2e_reps)
        # the same pipeline with packed records reused across cycles (kp_pack_cache, keyed by
        # (uid, metadata.generation)): each cycle re-schedules the batch with a different
        # `churn` share of its bindings at a new generation (re-packed), the rest unchanged
        # (their records copied); every lane's cache is warmed by one cycle first
        import numpy as np
        from karmada_amd.engine import PackCache
        n_b = u.n_bindings
        base_keys = api.binding_keys(structs[0], n_b, [1] * n_b)
        kdt = np.dtype({"names": ["ptr", "len", "gen"], "formats": ["<u8", "<u4", "<i8"], "offsets": [0, 8, 16],
                        "itemsize": C.sizeof(api.kp_binding_key)})

        def cycle_keys(c):  # generation 1 + (cycles in which the binding changed so far)
            ks = (api.kp_binding_key * n_b).from_buffer_copy(base_keys)
            g = np.frombuffer(ks, dtype=kdt)["gen"]
            idx = np.arange(n_b)
            for q in range(1, c + 1):
                g[(idx * 2654435761 + q * 40503) % 1000 < int(1000 * args.e2e_churn)] += 1
            return ks
        lanes_keys = [[cycle_keys(c) for c in range(args.e2e_reps + 1)] for _ in range(2)]
        caches = [PackCache(eng), PackCache(eng2)]
        for j, sn in enumerate((snap, snap2)):
            Batch(sn, structs=structs, cache=caches[j], keys=lanes_keys[j][0]).close()  # (warm)

        def drain_keyed(j, sn):
            for c in range(1, args.e2e_reps + 1):
                b3 = Batch(sn, structs=structs, cache=caches[j], keys=lanes_keys[j][c])
                b3.schedule_raw()
                b3.close()
        t1 = time.perf_counter()
        th = [threading.Thread(target=drain_keyed, args=(j, sn)) for j, sn in enumerate((snap, snap2))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        e2e_reuse = (time.perf_counter() - t1) / (2 * args.e2e_reps)
        reuse_hits = caches[0].stats()["last_hits"] / max(1, n_b)
        for c_ in caches:
            c_.close()
        snap2.close()
        eng2.close()
        if dist is not None:
            t = torch.tensor([e2e, e2e_pipe, e2e_reuse], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e2e, e2e_pipe, e2e_reuse = float(t[0].item()), float(t[1].item()), float(t[2].item())

    def avg(k):
        return sum(x[k] for x in st_all) / len(st_all)
    ms_per_step = 1e3 * elapsed / args.steps
    value = total / (elapsed / args.steps)  # every rank's bindings over the max-over-ranks time
    last = st_all[-1]
    pair_ms, sel_ms = avg("pair_kernel_ms"), avg("select_kernel_ms")
    sel_all_ms, filter_ms = avg("sel_all_kernel_ms"), avg("filter_kernel_ms")
    bits = last["bits"] == 1
    pair_b, sel_b = compulsory_bytes(B_rank, int(last["n_sel_all"]), C_, n_targets_rank, snap_bytes,
                                     int(last["n_classes"]) if bits else 0)
    top_ms = avg("top_kernel_ms")
    # every kernel of the step, ranked by its HIP-event time (averaged over the profiled
    # serial steps), with its compulsory bytes
    Cp = (C_ + 63) // 64 * 64
    n_cls = int(last["n_classes"]) if bits else 0
    kern = {}
    for run in kt_runs:
        for name, v in run.items():
            k = kern.setdefault(name, {"ms": 0.0, "launches": 0, "units": 0})
            k["ms"] += v["ms"] / len(kt_runs)
            k["launches"] = v["launches"]
            k["units"] = v["units"]
    kernels = []
    for name, v in kern.items():
        by = kernel_bytes(name, v["units"], Cp, n_cls, B_rank, n_targets_rank, snap_bytes, 0,
                          orders="k_class_order" in kern)
        kernels.append({"kernel": name, "ms": round(v["ms"], 4), "launches": v["launches"], "units": v["units"],
                        "bytes": round(by), "gbs": round(by / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None})
    kernels.sort(key=lambda x: -x["ms"])
    cands = [(k["kernel"], k["ms"], k["bytes"]) for k in kernels] or [("step", ms_per_step, pair_b + sel_b)]
    kname, kms, kbytes = max(cands, key=lambda x: x[1])
    klaunch = next((k["launches"] for k in kernels if k["kernel"] == kname), 1) or 1
    achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    profiled = (C_, B) == tuple(synth.CONFIGS[cfg])
    pmc = load_pmc(cfg, kname) if profiled else None

    # the PMC summary holds per-launch averages; the kernel's time and bytes here cover
    # all its launches in a step (k_select_top: two), so both sides are per step
    def pmc_frac(key, peak):
        if not pmc or not pmc.get(key) or kms <= 0:
            return None
        return round(pmc[key] * klaunch / (kms * 1e-3) / 1e9 / peak, 4)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": round(pmc["hbm_bytes"] * klaunch) if pmc and pmc.get("hbm_bytes") else None,
            # the same with FETCH_SIZE as counted (the x2 gfx950 correction holds for wide
            # coalesced reads only; this kernel's reads are mostly 8-64 B per lane)
            "traffic_fetch_raw": (round((pmc["fetch_bytes_x2"] / 2 + pmc["write_bytes"]) * klaunch)
                                  if pmc and pmc.get("fetch_bytes_x2") is not None and pmc.get("write_bytes") is not None
                                  else None),
            "kernel": kname, "kernel_ms": round(kms, 4), "algorithmic_bytes": round(kbytes),
            "dram_frac": pmc_frac("hbm_bytes", HBM_PEAK_GBS), "valu_frac": pmc_frac("valu_insts", VALU_PEAK_GINST)}
    step_bytes = pair_b + sel_b
    step_gbs = step_bytes / (ms_per_step * 1e-3) / 1e9
    line = {
        "metric": "ResourceBindings scheduled/sec at 100k bindings x 5k clusters",
        "value": round(value, 1),
        "unit": "ResourceBindings/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "inflight": len(lanes),
        "batches_per_lane": per_lane,
        # the hardware-queue count requested of the HIP runtime (GPU_MAX_HW_QUEUES; unset:
        # HIP's default 4) and the streams each engine drives
        "hip_hw_queues_requested": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
        "streams_per_engine": int(os.environ.get("KP_STREAMS", "3")),
        "host_wait": "blocking" if os.environ.get("KP_SYNC_BLOCK", "0") not in ("", "0") else "polling",
        # the timed window: from the (warmup x inflight)-th completed step to the K-th
        # completion after it, every lane mid-stream (module docstring)
        "timed_window": {"warmup_completions": n_warm, "timed_completions": args.steps,
                         # gaps between consecutive completions in the window (ms, lane): a
                         # stall shows as one long gap, a uniformly slow run as even ones
                         "gaps_ms": timed_gaps(clock, n_warm, args.steps),
                         "total_completions": clock["done"],
                         "lanes_wall_s": round(lanes_wall, 3)},
        # one batch at a time on one engine (nothing overlapped): ms per batch and the rate
        "serial_ms_per_step": round(serial_ms, 3) if serial_ms else round(ms_per_step, 3),
        "serial_value": round(total / (serial_ms * 1e-3), 1) if serial_ms else round(value, 1),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {"workload": f"config{cfg}: {B} bindings/GPU x {C_} clusters, seed {seed}, "
                               "resource-model grades, DynamicWeight/Aggregated" if cfg == 3 else
                   f"config{cfg}: {B} bindings/GPU x {C_} clusters, seed {seed}",
                   "bindings_per_gpu": B, "bindings_total": total, "clusters": C_,
                   "parallelism": f"binding-shard x{world}" + (" (cost-balanced, RCCL snapshot broadcast + "
                                                               "CSR all-gather)" if world > 1 else "")},
        "roofline": roof,
        # every kernel of one step (serial, profiled): HIP-event ms, launches, bindings (or
        # class rows) covered, compulsory bytes and the rate they imply, slowest first
        "kernels": kernels,
        # compulsory bytes of the whole step (every kernel) over the whole step's time
        "step_roofline": {"achieved": round(step_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(step_gbs / HBM_PEAK_GBS, 4), "bytes": round(step_bytes)},
        # filter stage: k_est_class + k_filter (bits mode) or the pair kernel
        "stages_ms": {"filter_stage": round(pair_ms, 3), "filter_kernel": round(filter_ms, 3),
                      "select_kernels": round(sel_ms, 3), "sel_all_kernel": round(sel_all_ms, 3),
                      "select_top_kernel": round(top_ms, 3), "select_cluster_kernel": round(avg("cluster_kernel_ms"), 3),
                      "host_region": round(avg("host_ms"), 3), "copy_back": round(avg("copy_ms"), 3),
                      "call_total": round(avg("total_ms"), 3)},
        "filter_mode": "bitset filter + estimator classes" if bits else "per-binding pair rows",
        "estimator_classes": int(last["n_classes"]) if bits else None,
        # bindings/s including host packing + upload, pipelined over two engines (every
        # binding packed anew), and one batch at a time (end_to_end_serial_ms per batch);
        # reuse: the same pipeline re-scheduling each batch with `churn` of its bindings at a
        # new generation and the rest's packed records copied from a kp_pack_cache
        "end_to_end_value": round(total / e2e_pipe, 1) if e2e_pipe else None,
        "end_to_end_ms": round(1e3 * e2e_pipe, 2) if e2e_pipe else None,
        "end_to_end_serial_ms": round(1e3 * e2e, 2) if e2e else None,
        "end_to_end_reuse": {"value": round(total / e2e_reuse, 1) if e2e_reuse else None,
                             "ms": round(1e3 * e2e_reuse, 2) if e2e_reuse else None,
                             "churn": args.e2e_churn, "records_reused": round(reuse_hits, 4)},
        "setup_s": {"generate": round(gen_s, 2), "snapshot_pack_upload": round(snap_s, 3),
                    "binding_pack_upload": round(pack_s, 3)},
        "per_rank_ms": per_rank_ms,
        "scheduled_ok": n_ok,
        "result_targets": n_targets,
        "slow_path_bindings": int(last["n_slow"]),
        # SEL_ALL DynamicWeight/Aggregated bindings scheduled over their deciding candidates
        # (k_select_top) and the ones it handed to the full-candidate kernel
        "select_top": {"bindings": int(last["n_top"]), "fallback": int(last["n_top_fallback"])},
        # cluster-spread bindings, and those selected over their estimator-class order
        "select_cluster": {"bindings": int(last["n_cluster"]), "class_order": int(last["n_cluster_order"])},
        "select_region": {"bindings": int(last["n_region"]), "class_order": int(last["n_region_order"])},
        # bindings of the timed batch (sampled over all ranks) re-checked against the oracle
        "parity_checked": n_chk,
        "parity_lanes": n_lanes_chk,  # result lists checked per rank: the serial run + each in-flight lane
        "parity_bad": n_bad,
        "parity_source": "all-gathered CSR (each rank's range) + every in-flight lane" if dist is not None else
                         "serial run + every in-flight lane",
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(u, opts, args.cpu_budget)
    if rank == 0:
        print(json.dumps(line), flush=True)
    snap.close()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
