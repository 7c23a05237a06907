"""bench.py's collective path at world size 1 (KP_DIST_FORCE=1): the snapshot
broadcast (rank 0's packed bytes imported by kp_snapshot_import on every rank) and
the two-phase CSR all-gather, with the oracle re-checking the GATHERED CSR (each
rank's range of it) and every in-flight lane. On the GPU the backend is `nccl`
(RCCL over xGMI), on the CPU `gloo` with the engine's host build.

The bench runs as a fresh child process (subprocess.run): nothing here touches the
GPU before it starts. SURVEY §8(e); the reference's single worker is
pkg/scheduler/scheduler.go:327."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def run_world1(args, env_extra, timeout):
    env = dict(os.environ, KP_DIST_FORCE="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1"] + args, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout[-1500:], p.stderr[-3000:])
    return json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])


def test_world1_gloo_cpusim():
    line = run_world1(["--config", "6", "--bindings", "300", "--steps", "2", "--warmup", "1", "--check", "300",
                       "--no-cpu", "--e2e-reps", "0", "--inflight", "2", "--lib", "karmada_amd/libkp_cpusim.so"],
                      {"KP_DIST_BACKEND": "gloo", "KP_CPUSIM_THREADS": "2"}, 300)
    assert line["parity_source"].startswith("all-gathered CSR")
    assert line["parity_checked"] == 300 and line["parity_lanes"] == 3 and line["parity_bad"] == 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_world1_rccl_config5():
    """Config 5 (C = 10 000, the mix of configs 2-4) over RCCL at world size 1: the
    gathered CSR of 2 000 bindings equals the oracle's placements."""
    line = run_world1(["--config", "5", "--bindings", "2000", "--steps", "2", "--warmup", "1", "--check", "2000",
                       "--no-cpu", "--e2e-reps", "0", "--inflight", "2"], {"KP_DIST_BACKEND": "nccl"}, 600)
    assert line["parity_source"].startswith("all-gathered CSR")
    assert line["parity_checked"] == 2000 and line["parity_bad"] == 0
    assert line["result_targets"] > 0
