"""Multi-GPU sharding of independent blocks.

One process per GPU.  The blocks of a job are independent (fresh deflator
per 64 KiB block, deflator.c:455-504 reset semantics), so rank r owns the
contiguous block range `shard_range(nblocks, r, world)` and compresses it with
no data-path collective.  The only exchange is the gather that turns the
per-rank bitstreams into the job's single RFC 1951 stream on rank 0:

  1. all_gather of the per-block compressed sizes (the size index that lets
     inflate shard the same way, §8e step 1);
  2. an exclusive scan of the per-rank totals, on every rank (step 2);
  3. one grouped send/recv of the variable-length bitstreams into their final
     offsets on rank 0 (step 3).

Every block ends byte aligned (FLUSH terminator 00 00 FF FF, deflator.c
:610-654), so concatenation needs no bit shifting.  Only the last rank's last
block uses END; every other shard is deflated with lastflush = FLUSH, so the
gathered stream equals the reference's single-stream output byte for byte.

The functions take torch tensors and a process group, so the same code runs
over RCCL on device tensors (bench.py) and over gloo on CPU tensors
(tests/test_distributed.py).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

DEFLT_END = 1
DEFLT_FLUSH = 2


def shard_range(nblocks: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block range [b0, b1) of `rank`: GPU g takes blocks
    [g*B/W, (g+1)*B/W) (§8e partitioning)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return nblocks * rank // world, nblocks * (rank + 1) // world


def shard_lastflush(rank: int, world: int) -> int:
    """Flush mode of a shard's last block: END only for the job's last block."""
    return DEFLT_END if rank == world - 1 else DEFLT_FLUSH


def gather_sizes(csizes: torch.Tensor, group=None) -> List[torch.Tensor]:
    """all_gather of the per-block compressed sizes (int32, same block count
    on every rank, as weak-scaled shards are)."""
    world = dist.get_world_size(group)
    out = [torch.empty_like(csizes) for _ in range(world)]
    dist.all_gather(out, csizes, group=group)
    return out


def gather_streams(stream: torch.Tensor, nbytes, group=None,
                   recv: Optional[torch.Tensor] = None
                   ) -> Tuple[Optional[torch.Tensor], List[int]]:
    """Gather every rank's first `nbytes` of `stream` (uint8) to rank 0 in rank
    order.  `nbytes` is an int or a one-element int64 tensor on the stream's
    device (the engine's d_total: the count never visits the host before the
    all_gather).  Returns (gathered tensor on rank 0 / None elsewhere,
    per-rank byte counts).  `recv` may be a preallocated buffer on rank 0.

    The host learns the counts once, from the all-gathered totals (one
    synchronisation of the current stream, which need not be the stream the
    deflate and inflate kernels run on: bench.py issues the gather on a side
    stream so the local inflate runs on the GPU meanwhile)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = stream.device
    if isinstance(nbytes, torch.Tensor):
        mine = nbytes.reshape(1).to(device=dev, dtype=torch.int64)
    else:
        mine = torch.tensor([nbytes], dtype=torch.int64, device=dev)
    tots = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(tots, mine, group=group)
    sz = [int(x) for x in torch.cat(tots).tolist()]
    offs = [0]
    for s in sz:
        offs.append(offs[-1] + s)
    nccl = dist.get_backend(group) == "nccl"
    if rank == 0:
        if recv is None or recv.numel() < offs[-1]:
            recv = torch.empty(offs[-1], dtype=torch.uint8, device=dev)
        recv[:sz[0]].copy_(stream[:sz[0]])
        ops = [dist.P2POp(dist.irecv, recv[offs[r]:offs[r + 1]], r, group=group)
               for r in range(1, world) if sz[r]]
        if ops:
            if nccl:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            else:
                for w in [dist.irecv(o.tensor, o.peer, group=group) for o in ops]:
                    w.wait()
        return recv[:offs[-1]], sz
    if sz[rank]:
        if nccl:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, stream[:sz[rank]], 0,
                                                        group=group)]):
                w.wait()
        else:
            dist.send(stream[:sz[rank]].contiguous(), 0, group=group)
    return None, sz
