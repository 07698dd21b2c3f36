"""Pair sharding across ranks (one process per GPU) and the end-of-solve pose gather.

Frame pairs are independent units, so a batch is split into contiguous shards,
one per rank, with no collective on the data path; the only exchange is one
all-gather of the 12 pose floats (R row-major, t) per pair.  The
reference's batch-global min/max masks become per-shard, exactly as under its own
nn.DataParallel (train.py:295-298).
"""
import torch
import torch.distributed as dist


def shard_range(n_pairs, world, rank):
    """Contiguous [begin, end) of `n_pairs` for `rank` (sizes differ by at most one)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(n_pairs, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def pack_poses(R, t):
    """[B,3,3], [B,3(,1)] -> [B,12] fp32."""
    B = R.shape[0]
    return torch.cat((R.reshape(B, 9), t.reshape(B, 3)), 1).to(torch.float32).contiguous()


def unpack_poses(P):
    return P[:, :9].reshape(-1, 3, 3), P[:, 9:].reshape(-1, 3, 1)


def gather_poses(R, t, out=None, async_op=False):
    """All-gather every rank's [B,12] poses into [world*B, 12] (rank-major).

    Equal shard sizes on every rank (the bench's weak-scaling layout).  RCCL uses
    the single-buffer all_gather_into_tensor; other backends (gloo in the CPU
    tests) the list form.  The poses are packed into a fresh buffer first, so with
    async_op=True the caller may overwrite R / t at once (the next solve) while the
    gather runs on the collective stream; it returns (out, work) and `out` is valid
    after work.wait()."""
    P = pack_poses(R, t)
    world = dist.get_world_size()
    if out is None:
        out = torch.empty(world * P.shape[0], 12, dtype=P.dtype, device=P.device)
    if dist.get_backend() == "nccl":
        work = dist.all_gather_into_tensor(out, P, async_op=async_op)
    else:
        work = dist.all_gather(list(out.chunk(world, 0)), P, async_op=async_op)
    return (out, work) if async_op else out
