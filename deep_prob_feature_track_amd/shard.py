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


def stream_calls(steps, group):
    """Step counts of the calls that cover exactly `steps` global batches of a stream when a
    rank solves `group` consecutive global batches per call: full calls, then one short
    remainder call."""
    return [group] * (steps // group) + ([steps % group] if steps % group else [])


def stream_group(shard_pairs, batch, min_launch_pairs=64, max_batches=32):
    """Global batches per grouped call on a rank: enough consecutive global batches of the
    stream that one call holds >= min_launch_pairs pairs (each global batch's shard stays
    its own independent batches of `batch` pairs, DPFT_GROUP), at most max_batches
    independent batches per call.  With 64-pair global batches the N = 8 rank shard (8 pairs)
    is grouped 8 at a time -- the same 64-pair launch shape as N = 1."""
    per_step = max(1, shard_pairs // batch)
    q = max(1, -(-min_launch_pairs // shard_pairs))
    return max(1, min(q, max_batches // per_step))


def stream_pair_index(step, rank_pair, global_batch, world, rank):
    """Stream-wide index of pair `rank_pair` of `rank`'s shard in global batch `step`: the
    order rank 0 finds the all-gathered poses of a grouped call in is rank-major, then step,
    then shard position -- this maps a gathered row back to its pair."""
    begin, _ = shard_range(global_batch, world, rank)
    return step * global_batch + begin + rank_pair


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


def pack_results(R, t, jtj=None, status=None):
    """Per-pair result rows: [R(9), t(3)] + optionally JtJ(36) + a
    non-finite flag(1) -> [B, 12 | 48 | 13 | 49] fp32.  `status` is the solve's status
    word (one per batch): every pair row carries it."""
    B = R.shape[0]
    cols = [R.reshape(B, 9).to(torch.float32), t.reshape(B, 3).to(torch.float32)]
    if jtj is not None:
        cols.append(jtj.reshape(B, 36).to(torch.float32))
    if status is not None:
        cols.append(status.reshape(1, 1).to(torch.float32).expand(B, 1))
    return torch.cat(cols, 1).contiguous()


def unpack_results(P, with_jtj=False, with_status=False):
    """Inverse of pack_results: dict(R [N,3,3], t [N,3,1][, jtj [N,6,6]][, status [N]])."""
    out = dict(R=P[:, :9].reshape(-1, 3, 3), t=P[:, 9:12].reshape(-1, 3, 1))
    c = 12
    if with_jtj:
        out["jtj"] = P[:, c:c + 36].reshape(-1, 6, 6)
        c += 36
    if with_status:
        out["status"] = P[:, c].to(torch.int32)
    return out


def gather_results(R, t, jtj=None, status=None, n_pairs=None):
    """All-gather every rank's result rows into [n_pairs, F] in pair order, for shards
    of unequal size too (n_pairs not a multiple of the world size: shard_range's
    split).  Each rank pads its rows to ceil(n_pairs / world) for the single
    fixed-size collective and the padding is dropped after it.  n_pairs None: equal
    shards (world * B rows)."""
    return gather_rows(pack_results(R, t, jtj, status), n_pairs)


def gather_rows(P, n_pairs=None):
    """gather_results for any per-pair rows P [B, F] (fp32): this rank's shard_range
    shard of n_pairs, all ranks' rows in pair order on every rank."""
    world, rank = dist.get_world_size(), dist.get_rank()
    B, F = P.shape
    if n_pairs is None:
        n_pairs = world * B
    b, e = shard_range(n_pairs, world, rank)
    if e - b != B:
        raise ValueError(f"rank {rank} holds {B} pairs, its shard of {n_pairs} is {e - b}")
    cap = -(-n_pairs // world)
    if B < cap:
        P = torch.cat((P, P.new_zeros(cap - B, F)), 0)
    full = torch.empty(world * cap, F, dtype=P.dtype, device=P.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(full, P)
    else:
        dist.all_gather(list(full.chunk(world, 0)), P)
    rows = []
    for r in range(world):
        rb, re_ = shard_range(n_pairs, world, r)
        rows.append(full[r * cap:r * cap + (re_ - rb)])
    return torch.cat(rows, 0)

