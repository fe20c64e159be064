"""CPU: image sharding and the batch all-gather (idn.parallel) on world_size-2 gloo process groups.
The GPU run uses the same code over RCCL; images are independent, so the only collective is the
optional reassembly all-gather."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from idn import parallel


def test_shard_range_partitions():
    for n in range(0, 40):
        for world in (1, 2, 3, 8):
            rs = [parallel.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        parallel.shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, dtype, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, w, _, dev = parallel.init_from_env(backend="gloo")
        assert (r, w) == (rank, world) and dev.type == "cpu"
        lo, hi = parallel.shard_range(n_total, rank, world)
        full = torch.arange(n_total * 2 * 3 * 3).reshape(n_total, 2, 3, 3).to(dtype)
        local = full[lo:hi].clone()
        got = parallel.all_gather_batch(local, n_total)
        q.put((rank, bool(torch.equal(got, full)), None))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, False, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("n_total,dtype", [(4, torch.uint8), (5, torch.uint8), (3, torch.float64),
                                           (1, torch.uint8)])
def test_all_gather_batch_gloo_world2(n_total, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, dtype, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, err in res:
        assert ok, f"rank {rank}: {err}"


def test_all_gather_rejects_wrong_shard_size():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bad_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all("expected" in msg for _, msg in res), res


def _bad_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE="2", LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env(backend="gloo")
        parallel.all_gather_batch(torch.zeros(3, 2, 2, 3, dtype=torch.uint8), 4)
        q.put((rank, "no error"))
    except ValueError as e:
        q.put((rank, str(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


# ---- ShardedPreprocessor: plan assignment and image ids per rank (no GPU work) ---------------

def _plan_worker(rank, world, port, sizes, spec, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env(backend="gloo")
        sp = parallel.ShardedPreprocessor(spec, mode, seed=26)
        got = []
        for n_total in sizes:  # consecutive batches: every rank's rng must stay in step
            lo, hi, ids, mine, _ = sp.assign(n_total, (600, 1000))
            got.append((lo, hi, ids, mine))
        q.put((rank, got, None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, (7, 5)), (3, (7, 4)), (3, (2, 8))])
def test_sharded_preprocessor_assignment_matches_one_process(world, sizes):
    """Each rank's shard gets the plans (bloom circle draws included) and global image ids a
    single process would give those images, over two consecutive uneven batches."""
    import random
    from idn.pipeline import Preprocessor
    spec, mode = "noise_mix_var_low", "test_v0"
    ref_pre = Preprocessor(spec, mode, seed=26, rng=random.Random(26))
    ref = [ref_pre.plans(n, hw=(600, 1000)) for n in sizes]
    assert any(st.op == "bloom" and st.args for b in ref for p in b for st in p.steps), \
        "the seed must draw at least one bloom to exercise the circle draws"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, sizes, spec, mode, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, got, err in res:
        assert err is None, f"rank {rank}: {err}"
        for b, n_total in enumerate(sizes):
            lo, hi, ids, mine = got[b]
            assert (lo, hi) == parallel.shard_range(n_total, rank, world)
            assert ids == list(range(lo, hi))
            assert mine == ref[b][lo:hi]
