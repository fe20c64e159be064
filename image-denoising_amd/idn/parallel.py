"""Multi-GPU image sharding: one process per GPU, images are independent, so each
rank filters its own contiguous shard with no data-path collective.  Reassembling the filtered
batch on every rank (the blob the detector consumes) is one all-gather over RCCL/xGMI
(torch.distributed backend "nccl" is RCCL on ROCm); gloo works the same way on CPU tensors.

The reference runs one image at a time in a single process (lib/model/test.py:189,
lib/roi_data_layer/layer.py:74); there is no reference collective to mirror.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced shard [lo, hi) of n images for `rank` (first n % world ranks get +1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_counts(n: int, world: int) -> List[int]:
    return [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]


def init_from_env(backend: Optional[str] = None):
    """(rank, world, local_rank, device) from torchrun's env; initialises the process group
    (RCCL when GPUs are present, gloo otherwise) when WORLD_SIZE > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        be = backend or ("nccl" if gpu else "gloo")
        if be == "nccl":
            dist.init_process_group(be, device_id=dev)
        else:
            dist.init_process_group(be)
    return rank, world, local, dev


def all_gather_batch(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Reassemble the (n_total, ...) batch from every rank's contiguous shard `local`
    ((count_r, ...) with count_r = shard_counts(n_total, world)[rank]).  Uneven shards are
    padded to the largest shard for one all_gather_into_tensor, then compacted."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = shard_counts(n_total, world)
    if local.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank}: local shard has {local.shape[0]} images, "
                         f"expected {counts[rank]}")
    m = max(counts)
    item = tuple(local.shape[1:])
    if local.shape[0] == m:
        send = local.contiguous()
    else:
        send = torch.zeros((m, *item), dtype=local.dtype, device=local.device)
        send[: local.shape[0]] = local
    buf = torch.empty((world * m, *item), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and (local.device.type == "cuda"
                                                    or dist.get_backend(group) != "gloo"):
        dist.all_gather_into_tensor(buf, send, group=group)
    else:
        dist.all_gather(list(buf.chunk(world)), send, group=group)
    if all(c == m for c in counts):
        return buf
    return torch.cat([buf[r * m: r * m + counts[r]] for r in range(world)])


class ShardedPreprocessor:
    """Preprocessor over a global batch: this rank runs its shard, optionally all-gathers.

    Plans are resolved for the WHOLE batch from the shared seeded rng on every rank (cheap host
    work), bloom circle draws included (idn.noise_spec.plan(hw=...)), so a rank's images get the
    same recipes -- and every rank's rng advances identically, batch after batch -- as on one
    GPU; device noise is keyed by the global image id, so results do not depend on the world
    size."""

    def __init__(self, noise: str, mode: str = "canonical", seed: int = 3, rng=None,
                 group=None):
        from .pipeline import Preprocessor
        self.pre = Preprocessor(noise, mode, seed=seed, rng=rng, noise_rng="philox")
        self.group = group

    def assign(self, n_total: int, hw: Tuple[int, int], plans: Optional[Sequence] = None):
        """(lo, hi, global image ids, this shard's plans, all plans) for this rank; draws the
        whole batch's plans from the shared rng when `plans` is None."""
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        lo, hi = shard_range(n_total, rank, world)
        all_plans = list(plans) if plans is not None else self.pre.plans(n_total, hw=hw)
        if len(all_plans) != n_total:
            raise ValueError(f"{len(all_plans)} plans for a batch of {n_total}")
        return lo, hi, list(range(lo, hi)), all_plans[lo:hi], all_plans

    def __call__(self, shard: torch.Tensor, n_total: int, gather: bool = False,
                 plans: Optional[Sequence] = None):
        lo, hi, ids, mine, all_plans = self.assign(n_total, tuple(shard.shape[1:3]), plans)
        if shard.shape[0] != hi - lo:
            raise ValueError(f"shard of {shard.shape[0]} images, expected {hi - lo}")
        outs, _ = self.pre(shard, image_ids=ids, plans=mine)
        if not gather:
            return outs, all_plans
        if len({(o.dtype, tuple(o.shape)) for o in outs}) > 1:
            raise ValueError("gather needs one dtype/shape across the shard's outputs")
        if outs:
            local = torch.stack(outs)
        else:  # this rank owns no image: an empty shard of the batch's output dtype
            dt = torch.uint8 if all_plans[0].out_dtype == "u8" else torch.float64
            local = torch.empty((0, *shard.shape[1:]), dtype=dt, device=shard.device)
        return all_gather_batch(local, n_total, self.group), all_plans
