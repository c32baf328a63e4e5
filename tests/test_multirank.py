"""World-size-2 and -8 CPU (gloo) rehearsals of bench.py's multi-GPU plumbing: the
batch partitions by block id with no data-path collective; ranks only meet at
the barrier and the max-over-ranks of the timing."""
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
