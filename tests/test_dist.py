"""Multi-process path on CPU (gloo, world_size 2): trial sharding + histogram
all-reduce give a histogram bit-identical to one process running every trial.
The per-rank engine here is the CPU oracle (the GPU path is exercised by the
driver's multi-GPU bench with the same benor.parallel functions)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT
from benor.parallel import merge_histogram, strong_range, weak_range

N, F, K, SEED = 10, 4, 16, 0xBEEF


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    faulty = [i < F for i in range(N)]
    total = torch.zeros(oracle.hist_len(K), dtype=torch.int64)
    for step in range(3):
        if mode == "weak":
            b, n = weak_range(step, rank, world, 5000)
        else:
            b, n = strong_range(step * 12345, 12345, rank, world)
        h = oracle.run_trials(N, F, faulty, seed=SEED, trial_begin=b, trial_count=n, k_max=K, threads=1).hist
        t = torch.from_numpy(h.astype(np.int64))
        merge_histogram(t)
        total += t
    if rank == 0:
        out_q.put(total.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_two_rank_histogram_merge(mode):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    faulty = [i < F for i in range(N)]
    if mode == "weak":
        ref = oracle.run_trials(N, F, faulty, seed=SEED, trial_begin=0, trial_count=3 * world * 5000, k_max=K).hist
    else:
        ref = oracle.run_trials(N, F, faulty, seed=SEED, trial_begin=0, trial_count=3 * 12345, k_max=K).hist
    np.testing.assert_array_equal(got.astype(np.uint64), ref)


def test_ranges_partition():
    for world in (1, 2, 3, 8):
        shards = [strong_range(7, 1001, r, world) for r in range(world)]
        assert shards[0][0] == 7 and sum(n for _, n in shards) == 1001
        for (b0, n0), (b1, _) in zip(shards, shards[1:]):
            assert b0 + n0 == b1
        ws = sorted(weak_range(s, r, world, 10) for s in range(3) for r in range(world))
        assert [b for b, _ in ws] == list(range(0, 3 * world * 10, 10))
