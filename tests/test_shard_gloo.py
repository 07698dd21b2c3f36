"""Multi-process path on CPU: world_size-2 gloo run of the pair-sharded solve.

Each rank solves its contiguous shard of a 4-pair batch (the oracle stands in for
the GPU solver -- test infrastructure only) and all-gathers the poses with
`shard.gather_poses`, the same call bench.py makes over RCCL.  Rank 0 checks the
gathered tensor against per-shard solves done locally (shard semantics: the
batch-global truncated-sigma extrema are per shard, as under the reference's
nn.DataParallel).
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deep_prob_feature_track_amd import shard

PAIRS = [(0, 1), (1, 2), (2, 3), (3, 4)]


def test_shard_range_partitions():
    for n in (1, 4, 7, 64):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)


def test_pack_unpack_roundtrip():
    R = torch.randn(3, 3, 3)
    t = torch.randn(3, 3, 1)
    R2, t2 = shard.unpack_poses(shard.pack_poses(R, t))
    assert torch.equal(R2, R) and torch.equal(t2, t)


def _solve_pairs(pairs):
    import golden_io
    import recipe
    from oracle import ic_oracle as O
    case = recipe.make_case(pairs=pairs, C=8, levels=1, base_down=4)
    level = golden_io.levels_torch(case, torch.float32)[0]
    R0, t0 = golden_io.init_pose(case, torch.float32)
    K = torch.from_numpy(case["K"])
    with torch.no_grad():
        return O.solve_pyramid(R0, t0, [level], K, iters=3, remove_tru_sigma=True)


def _worker(rank, world, port, q, paths):
    import sys
    sys.path[:0] = paths
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        b, e = shard.shard_range(len(PAIRS), world, rank)
        R, t = _solve_pairs(PAIRS[b:e])
        out = shard.gather_poses(R, t)
        # bench.py's pipelined form: async gather, poses overwritten at once (next solve)
        out2, work = shard.gather_poses(R, t, async_op=True)
        R.zero_()
        t.zero_()
        work.wait()
        if rank == 0:
            q.put(out.numpy().copy())
            q.put(out2.numpy().copy())
    finally:
        dist.destroy_process_group()


def _free_port():
    """A fresh rendezvous file for init_method="file://..." (no TCP port to race for)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="dpft_gloo_")
    os.close(fd)
    os.unlink(path)
    return path


def test_two_rank_gloo_gather_matches_per_shard_solves():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    import sys
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, list(sys.path))) for r in range(world)]
    for p in procs:
        p.start()
    gathered = torch.from_numpy(q.get(timeout=120))
    gathered_async = torch.from_numpy(q.get(timeout=120))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = []
    for r in range(world):
        b, e = shard.shard_range(len(PAIRS), world, r)
        expect.append(shard.pack_poses(*_solve_pairs(PAIRS[b:e])))
    assert torch.equal(gathered, torch.cat(expect, 0))
    assert torch.equal(gathered_async, gathered)


def _worker_results(rank, world, port, q, n_pairs):
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        b, e = shard.shard_range(n_pairs, world, rank)
        idx = torch.arange(b, e, dtype=torch.float32).view(-1, 1, 1)
        R = idx + 0.01 * torch.arange(9, dtype=torch.float32).view(1, 3, 3)
        t = -idx.view(-1, 1, 1) * torch.ones(1, 3, 1)
        jtj = idx * torch.ones(1, 6, 6) + torch.eye(6)
        status = torch.tensor([rank], dtype=torch.int32)
        out = shard.gather_results(R, t, jtj=jtj, status=status, n_pairs=n_pairs)
        if rank == 0:
            q.put(out.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs", [4, 7])
def test_two_rank_gather_results_ragged_shards(n_pairs):
    """gather_results: poses + JtJ + status rows of unequal shards (7 pairs on 2 ranks:
    4 + 3) come back in pair order, padding dropped (SURVEY.md 8e's gathered record)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_results, args=(r, world, port, q, n_pairs)) for r in range(world)]
    for p in procs:
        p.start()
    out = torch.from_numpy(q.get(timeout=120))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = shard.unpack_results(out, with_jtj=True, with_status=True)
    assert out.shape == (n_pairs, 49)
    idx = torch.arange(n_pairs, dtype=torch.float32)
    assert torch.equal(res["R"][:, 0, 0], idx) and torch.equal(res["t"][:, 2, 0], -idx)
    assert torch.equal(res["jtj"][:, 0, 1], idx)
    spans = [shard.shard_range(n_pairs, world, r) for r in range(world)]
    owner = torch.cat([torch.full((e - b,), r, dtype=torch.int32) for r, (b, e) in enumerate(spans)])
    assert torch.equal(res["status"], owner)



def _worker_stream(rank, world, port, q, global_batch, batch, min_launch, steps):
    """bench.py's grouped stream on `world` gloo ranks: each rank solves its shard of Q
    consecutive global batches per call (shard.stream_group / stream_calls), the poses of a
    call are all-gathered asynchronously; a pose here encodes its stream pair (R = index,
    t = step) so rank 0 can check the coverage and the row order."""
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        b, e = shard.shard_range(global_batch, world, rank)
        n_r = e - b
        Q = shard.stream_group(n_r, batch, min_launch)
        rows, step0 = [], 0
        for qn in shard.stream_calls(steps, Q):
            idx = torch.tensor([float(shard.stream_pair_index(step0 + k, i, global_batch, world, rank))
                                for k in range(qn) for i in range(n_r)])
            R = idx.view(-1, 1, 1) * torch.ones(1, 3, 3)
            t = torch.tensor([float(step0 + k) for k in range(qn) for _ in range(n_r)]).view(-1, 1) * torch.ones(1, 3)
            out, work = shard.gather_poses(R, t, async_op=True)
            R.zero_()  # the next call overwrites the poses while the gather runs
            work.wait()
            rows.append(out.numpy().copy())
            step0 += qn
        if rank == 0:
            q.put((Q, rows))
    finally:
        dist.destroy_process_group()


def test_two_rank_grouped_stream_covers_every_pair_once():
    """The N > 1 bench step shape: 2 ranks, global batches of 4 pairs (2 per rank), grouped 3
    global batches per call (>= 6 pairs per call), 7 global batches (calls of 3, 3 and a
    remainder of 1): the gathered rows cover every stream pair exactly once, in the
    rank-major / step / shard order that shard.stream_pair_index names."""
    import numpy as np
    world, gb, batch, min_launch, steps = 2, 4, 2, 6, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_stream, args=(r, world, port, q, gb, batch, min_launch, steps))
             for r in range(world)]
    for p in procs:
        p.start()
    Q, rows = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert Q == 3 and [r.shape[0] for r in rows] == [12, 12, 4]
    seen = np.concatenate([r[:, 0] for r in rows])
    assert sorted(seen.astype(int).tolist()) == list(range(steps * gb))
    assert np.all(np.floor(seen / gb) == np.concatenate([r[:, 9] for r in rows]))  # pair i of step s: s*gb + ...
