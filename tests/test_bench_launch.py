"""bench.py's multi-GPU launch path on the CPU: `--gpus 2` without WORLD_SIZE starts
two rank processes itself (one per GPU on a GPU node; here gloo + the engine's CPU
build), cost-balanced shards of one universe, the snapshot broadcast and the
two-phase CSR all-gather. The gathered results must cover the same universe as a
one-rank run over all of its bindings."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "6", "--steps", "2", "--warmup", "1", "--check", "40", "--e2e-reps", "0", "--no-cpu",
        "--inflight", "2", "--lib", "karmada_amd/libkp_cpusim.so"]


def run(extra, env_extra=None):
    env = dict(os.environ, KP_DIST_BACKEND="gloo", KP_CPUSIM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS + extra, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    return p


def line(p):
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])


def test_bench_two_ranks_gloo():
    two = line(run(["--gpus", "2", "--bindings", "250"]))
    one = line(run(["--gpus", "1", "--bindings", "500"]))
    assert two["n_gpus"] == 2 and len(two["per_rank_ms"]) == 2
    assert two["config"]["bindings_total"] == 500 == one["config"]["bindings_total"]
    assert two["parity_bad"] == 0 and two["parity_checked"] == 80 and two["parity_lanes"] == 3
    # the all-gathered CSR covers the whole universe: same totals as one rank over all of it
    assert two["result_targets"] == one["result_targets"]
    assert two["scheduled_ok"] == one["scheduled_ok"]


def test_bench_four_ranks_gloo_config5_whole_csr():
    """Four rank processes over config 5's mix (SEL_ALL StaticWeight, Dynamic/Aggregated
    and spread constraints, interleaved), cost-balanced shards (dist.shard_range_weighted):
    every binding of the gathered CSR is re-checked against the oracle (--check covers each
    rank's whole shard), and the totals equal one rank over the same universe."""
    common = ["--config", "5", "--clusters", "300", "--check", "400", "--inflight", "1"]
    four = line(run(common + ["--gpus", "4", "--bindings", "100"], {"KP_CPUSIM_THREADS": "1"}))
    one = line(run(common + ["--gpus", "1", "--bindings", "400"]))
    assert four["n_gpus"] == 4 and len(four["per_rank_ms"]) == 4
    assert four["config"]["bindings_total"] == 400 == one["config"]["bindings_total"]
    # the shards are cut by cost, not by count, yet cover the universe: every binding checked once
    assert four["parity_checked"] == 400 and four["parity_bad"] == 0
    assert one["parity_checked"] == 400 and one["parity_bad"] == 0
    assert four["result_targets"] == one["result_targets"]
    assert four["scheduled_ok"] == one["scheduled_ok"]


def test_bench_gpus_must_match_world_size():
    p = run(["--gpus", "2", "--bindings", "50"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE" in (p.stderr + p.stdout)
