"""World-size-2 and -8 CPU (gloo) rehearsals of bench.py's multi-GPU plumbing: the
batch partitions by block id with no data-path collective; ranks only meet at
the barrier and the max-over-ranks of the timing."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

SCRIPT = r'''
import os, sys
sys.path.insert(0, os.environ["TFS_ROOT"])
import numpy as np
import bench
world, rank, local, dist = bench._dist_init()
assert world == int(os.environ["TFS_EXPECT_WORLD"]) and dist is not None
mine = bench.rank_blocks(1024 * world, world, rank)
assert len(mine) == 1024 and (mine % world == rank).all()
t = bench._max_over_ranks(dist, 1.0 + rank)
assert t == float(world), t
g = bench._gather_floats(dist, world, 10.0 + rank)  # per-rank kernel times of the roofline
assert g == [10.0 + r for r in range(world)], g
# per-rank rates of the N > 1 line (device-resident and end-to-end legs): rank r
# "takes" 1 + r seconds for 2 GiB, so rank world-1 is the slowest and named as such
pr = bench.per_rank(dist, world, 1.0 + rank, 2 * 2**30)
assert len(pr["values"]) == world and pr["values"][0] == 2.0 and abs(pr["min"] - 2.0 / world) < 1e-12, pr
assert pr["slowest_rank"] == world - 1 and pr["fastest_rank"] == 0 and pr["elapsed_s"][rank] == 1.0 + rank
assert abs(pr["min_over_max"] - 1.0 / world) < 1e-12
for k in ("values", "elapsed_s", "min", "max", "mean", "slowest_rank", "fastest_rank", "min_over_max"):
    assert k in pr, k
import torch
allb = [None] * world
dist.all_gather_object(allb, mine.tolist())
if rank == 0:
    flat = sorted(x for b in allb for x in b)
    assert flat == list(range(1024 * world))
    print("PARTITION_OK")
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_partition_and_timing(tmp_path, world):
    """world 8 rehearses the driver's 8-GPU node (configs[4]) with CPU ranks."""
    script = tmp_path / "w.py"
    script.write_text(SCRIPT)
    env = dict(os.environ, TFS_ROOT=ROOT, MASTER_ADDR="127.0.0.1", TFS_EXPECT_WORLD=str(world), OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % world,
                        "--master-addr", "127.0.0.1", "--master-port", str(29517 + world), str(script)],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "PARTITION_OK" in r.stdout


def test_zipf_sizes_match_config():
    sys.path.insert(0, ROOT)
    import bench
    blocks = bench.zipf_sizes(42, 3)
    for L in blocks:
        assert L.min() >= 4096 and L.max() < 256 * 4096
        assert int((L + 36).sum()) <= bench.BLOCK_DATA
    allL = np.concatenate(blocks)
    assert (allL // 4096 == 1).mean() > 0.1   # heavy head of the Zipf law


def test_bench_gpus_n_starts_its_own_ranks():
    """Plain `python3 bench.py --gpus N` (no launcher around it) starts N ranks
    itself through torch.distributed.run; --launch-check stops each rank after
    the rendezvous, so this runs on the CPU (the -m gpu twin runs the real line)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    # the JSON line is all there is on stdout (gloo's per-rank connection messages go to stderr)
    assert [ln for ln in r.stdout.splitlines() if ln.strip()] == lines, r.stdout
    chk = json.loads(lines[0])["launch_check"]
    assert chk["world"] == 3 and chk["gpus"] == 3
    assert sorted(x[0] for x in chk["ranks"]) == [0, 1, 2]
    assert sorted(x[1] for x in chk["ranks"]) == [0, 1, 2]
    assert len({x[2] for x in chk["ranks"]}) == 3 and os.getpid() not in {x[2] for x in chk["ranks"]}


@pytest.mark.parametrize("world,gpus", [(2, 1), (8, 4), (1, 2)])
def test_bench_refuses_world_size_mismatch(world, gpus):
    """A launcher that started another number of ranks than --gpus asks for is
    refused before any GPU work (the line would report the wrong N)."""
    env = dict(os.environ, WORLD_SIZE=str(world), RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=%d but --gpus %d" % (world, gpus) in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("local_world", [1, 2, 8])
def test_cpu_budget_split_by_local_world(monkeypatch, local_world):
    """Legs every local rank runs at once (the parity oracle) get quota / LOCAL_WORLD_SIZE
    CPUs, so N ranks never ask for N times the container's cpu.max quota; the
    baseline leg (other ranks waiting at a barrier) keeps the whole budget."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("LOCAL_WORLD_SIZE", str(local_world))
    whole = bench._cpu_budget()
    share = bench._cpu_budget(shared=True)
    assert whole >= 1 and 1 <= share <= whole
    if local_world == 1:
        assert share == whole
    else:
        assert share <= max(1, whole // local_world) or share == 1
