"""bench.py's multi-GPU entry point: `bench.py --gpus N` must run N ranks whether or not a
launcher started it, and refuse a launch whose WORLD_SIZE disagrees with --gpus (otherwise an
N-GPU job could report a 1-GPU number).  The unit of work the ranks split is the relay of
p2pnetwork/node.py:114-116 (config 2: 64 * (8 + 999 * 7) = 448,064 relays per broadcast run)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
C2_RELAYS = 64 * (8 + 999 * 7)


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    env.update(extra)
    return env


def _bench(args, env, timeout=600):
    p = subprocess.run([sys.executable, "-u", BENCH, *args], env=env, cwd=REPO, timeout=timeout,
                       capture_output=True, text=True)
    return p


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("world_env", ["1", "3"])
def test_world_size_must_match_gpus(world_env):
    """A launcher-set WORLD_SIZE that disagrees with --gpus stops the bench before it touches
    the GPU (no HIP call: this runs on the CPU-only container)."""
    p = _bench(["--gpus", "2", "--workload", "c2"],
               _env(WORLD_SIZE=world_env, RANK="0", LOCAL_RANK="0"), timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr and "--gpus 2" in p.stderr


def test_gpus_zero_rejected():
    p = _bench(["--gpus", "0"], _env(), timeout=120)
    assert p.returncode != 0


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` without a launcher: two ranks (gloo, both on cuda:0 of the one-GPU
    box) split config 2's 64 broadcasts; the JSON line reports n_gpus 2 and the 1-GPU run's
    relays."""
    common = ["--workload", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench(["--gpus", "1", *common], _env(), timeout=300)
    assert one.returncode == 0, one.stderr[-4000:]
    j1 = _json_line(one.stdout)
    assert j1["n_gpus"] == 1 and j1["relays_per_step"] == C2_RELAYS
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", *common], _env(), timeout=300)
    assert two.returncode == 0, two.stderr[-4000:]
    j2 = _json_line(two.stdout)
    assert j2["n_gpus"] == 2
    assert j2["relays_per_step"] == C2_RELAYS
    assert "x2" in j2["config"]["parallelism"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_c5_partitioned_8_ranks_gloo():
    """Config 5's vertex-partitioned job at 8 ranks (gloo, all on cuda:0 of the one-GPU box) at
    2M peers, W = 64, churn 0.05: the JSON line reports n_gpus 8 and the same relays per step as
    the unpartitioned 1-GPU run of the same size (records of 1 + 64 int64 through 8 list segments,
    interior peers overlapping the exchange)."""
    common = ["--workload", "c5", "--peers", "2000000", "--steps", "1", "--warmup", "0",
              "--no-cpu-baseline"]
    one = _bench(["--gpus", "1", *common], _env(), timeout=300)
    assert one.returncode == 0, one.stderr[-4000:]
    j1 = _json_line(one.stdout)
    eight = _bench(["--gpus", "8", "--dist-backend", "gloo", *common], _env(), timeout=600)
    assert eight.returncode == 0, eight.stderr[-4000:]
    j8 = _json_line(eight.stdout)
    assert j8["n_gpus"] == 8
    assert "vertex partition x8" in j8["config"]["parallelism"]
    assert j8["relays_per_step"] == j1["relays_per_step"]
    assert j8["config"]["rounds"] == j1["config"]["rounds"]
    assert 0.0 < j8["exchange_live_row_frac"] <= 1.0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_c4_vertex_split_4_ranks_gloo():
    """Config 4's gossip as a 1-D vertex partition (`--split vertex`) at 4 ranks (gloo, cuda:0)
    on a 1M-peer BA graph, W = 64: the ranks run the dense rounds in their partitioned form (E
    planes for local connections, ghost pushes exchanged) and the JSON line reports the 1-GPU
    run's relays and rounds."""
    common = ["--workload", "c4", "--peers", "1000000", "--steps", "1", "--warmup", "0",
              "--no-cpu-baseline"]
    one = _bench(["--gpus", "1", *common], _env(), timeout=300)
    assert one.returncode == 0, one.stderr[-4000:]
    j1 = _json_line(one.stdout)
    four = _bench(["--gpus", "4", "--split", "vertex", "--dist-backend", "gloo", *common], _env(),
                  timeout=600)
    assert four.returncode == 0, four.stderr[-4000:]
    j4 = _json_line(four.stdout)
    assert j4["n_gpus"] == 4
    assert "vertex partition x4" in j4["config"]["parallelism"]
    assert j4["relays_per_step"] == j1["relays_per_step"]
    assert j4["config"]["rounds"] == j1["config"]["rounds"]
    assert j4["kernel_ms_per_step"].get("gossip_fused", 0.0) > 0.0  # dense rounds on the ranks
