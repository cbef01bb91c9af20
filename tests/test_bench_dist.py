"""The multi-GPU contract of bench.py, rehearsed on CPU with gloo at world
size 2 (replicas only: no data-path collective; the job time is the max over
ranks and the value counts every rank's frames)."""
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    elapsed = [1.5, 2.0][rank]  # rank 1 is the straggler
    el = bench.max_over_ranks(elapsed, world, device="cpu")
    q.put((rank, el, bench.replica_throughput(480, world, el)))
    dist.barrier()
    dist.destroy_process_group()


def test_replica_timing_world_size_2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]           # both ranks see the max time
    assert all(abs(r[2] - 480 * 2 / 2.0) < 1e-12 for r in res)  # frames of all ranks / max time


def test_single_rank_needs_no_collective():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.max_over_ranks(3.0, 1) == 3.0
    assert bench.replica_throughput(100, 1, 0.5) == 200.0
