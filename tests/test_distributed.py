"""N>1 path on CPU: two gloo ranks run bench.py's control plane (independent
per-rank stripe seeds and erasure masks, max-over-ranks timing, whole-job
throughput) -- no data-path collective exists to test."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import rs_oracle as O
    seed = bench.rank_seed_base(rank)
    data = O.stripe_data(3, 64, gpu=rank)
    assert np.array_equal(data, O.splitmix64_bytes(seed + 3, 640).reshape(10, 64))
    masks = bench.erasure_masks(16, rank)
    t = bench.reduce_max(1.0 + rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, (masks.tolist(), data[0, :8].tolist()))
    q.put((rank, t, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_control_plane():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, gathered in res:
        assert t == 2.0  # max over ranks
        (m0, d0), (m1, d1) = gathered
        assert m0 != m1 and d0 != d1  # independent stripe batches per rank
        for m in m0 + m1:
            assert bin(m & 0x3FFF).count("1") == 10  # exactly 4 erasures


def test_job_throughput():
    import bench
    # 2 ranks x 20 GiB per step x 3 steps in 1.5 s (max over ranks) = 80 GiB/s
    assert abs(bench.job_throughput(20 * 2**30, 3, 2, 1.5) - 80.0) < 1e-9
