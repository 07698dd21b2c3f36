"""Child of tests/test_rccl_gather.py: one rank under torch.distributed.run with the nccl
(= RCCL) backend on its GPU.  Solves a batch of pairs with the library, then runs the three
collectives bench.py / evaluate.py use -- shard.gather_poses (sync, and async with the poses
overwritten at once, as the bench's pipelined loop does) and shard.gather_rows with the result
rows of a ragged pair count -- and checks each gathered tensor bit for bit against the local
solve.  Writes a JSON verdict to $DPFT_RCCL_OUT; exit code 0 when every check passed.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl")
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "rank": dist.get_rank()}
    try:
        import golden_io
        import recipe
        from deep_prob_feature_track_amd import ic, shard
        pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (1, 0), (2, 1)]  # 7: a ragged count
        n = len(pairs)
        world, rank = dist.get_world_size(), dist.get_rank()
        b, e = shard.shard_range(n, world, rank)
        case = recipe.make_case(pairs=pairs[b:e], C=16, levels=2, base_down=2)
        lv = golden_io.levels_torch(case, torch.float32, dev)
        K = torch.from_numpy(case["K"]).to(dev)
        levels = [dict(x0=d["f0"], x1=d["f1"], invD0=d["invD0"], invD1=d["invD1"], sigma0=d["s0"], sigma1=d["s1"])
                  for d in lv]
        solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True)
        B = e - b
        R = torch.eye(3, device=dev).repeat(B, 1, 1).contiguous()
        t = torch.zeros(B, 3, device=dev)
        solver.run(R, t)
        torch.cuda.synchronize()
        ic.check_status(solver.status)
        local_rows = shard.pack_poses(R, t)
        g_sync = shard.gather_poses(R, t)
        R2, t2 = R.clone(), t.clone()
        g_async, work = shard.gather_poses(R2, t2, async_op=True)
        R2.zero_()  # the next solve overwrites the pose buffers at once
        t2.zero_()
        work.wait()
        rows = shard.gather_rows(shard.pack_results(R, t, status=solver.status), n_pairs=n)
        torch.cuda.synchronize()
        mine = slice(rank * B, (rank + 1) * B) if n % world == 0 else None
        out.update(
            pairs=n, shard=[b, e],
            sync_shape=list(g_sync.shape), async_shape=list(g_async.shape), rows_shape=list(rows.shape),
            sync_equal=bool(mine is None or torch.equal(g_sync[mine], local_rows)),
            async_equal=bool(torch.equal(g_async, g_sync)),
            rows_equal=bool(torch.equal(rows[b:e, :12], local_rows)),
            rows_status_zero=bool((rows[b:e, 12] == 0).all()),
            finite=bool(torch.isfinite(local_rows).all()),
            moved=bool((local_rows[:, 9:] != 0).any()))
        ok = all(out[k] for k in ("sync_equal", "async_equal", "rows_equal", "rows_status_zero", "finite", "moved"))
        ok = ok and out["rows_shape"] == [n, 13] and out["sync_shape"] == [world * B, 12]
        out["ok"] = bool(ok)
    finally:
        dist.destroy_process_group()
    with open(os.environ["DPFT_RCCL_OUT"], "w") as f:
        json.dump(out, f)
    return 0 if out.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
