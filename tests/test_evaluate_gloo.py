"""The sharded evaluation driver (deep_prob_feature_track_amd/evaluate.py) on CPU: two
gloo ranks, a ragged pair list (7 pairs: shards of 4 and 3, batches of 2), the oracle
standing in for the GPU tracker (test infrastructure only).  Rank 0 must end up with every
pair's row in pair order -- equal to each shard evaluated alone -- and write the
reference's pkl / CSV (evaluate.py:318-372)."""
import os
import pickle

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deep_prob_feature_track_amd import evaluate as E
from deep_prob_feature_track_amd import shard

PAIRS = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (0, 2), (1, 3)]


def _load(i0, i1):
    import recipe
    sel = PAIRS[i0:i1]
    b = len(sel)
    depth0 = torch.stack([torch.from_numpy(recipe.depth_m(i, 4))[None] for i, _ in sel])
    return {"pairs": sel, "depth0": depth0, "K": torch.from_numpy(np.tile(recipe.K_FULL[None] / 4, (b, 1))),
            "R_gt": torch.eye(3).repeat(b, 1, 1), "t_gt": torch.zeros(b, 3)}


def _solve(d):
    import golden_io
    import recipe
    from oracle import ic_oracle as O
    case = recipe.make_case(pairs=d["pairs"], C=8, levels=1, base_down=4)
    level = golden_io.levels_torch(case, torch.float32)[0]
    R0, t0 = golden_io.init_pose(case, torch.float32)
    with torch.no_grad():
        return O.solve_pyramid(R0, t0, [level], torch.from_numpy(case["K"]), iters=3, remove_tru_sigma=True)


def _worker(rank, world, port, q, paths, out_dir):
    import sys
    sys.path[:0] = paths
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        rows = E.evaluate_sharded(_load, _solve, len(PAIRS), batch=2)
        if rank == 0:
            names = [f"{i}->{j}" for i, j in PAIRS]
            from deep_prob_feature_track_amd import metrics
            metrics.write_results({"fr1_desk_keyframe_1": E.rows_to_outputs(rows, names)}, [1], "test",
                                  root=out_dir)
            q.put(rows.numpy().copy())
    finally:
        dist.destroy_process_group()


def _free_port():
    """A fresh rendezvous file for init_method="file://..." (no TCP port to race for)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="dpft_gloo_")
    os.close(fd)
    os.unlink(path)
    return path


def test_two_rank_sharded_evaluation_writes_reference_outputs(tmp_path):
    import sys
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, list(sys.path), str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    rows = torch.from_numpy(q.get(timeout=180))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rows.shape == (len(PAIRS), E.ROW)
    # shard semantics: rank r evaluated pairs shard_range(7, 2, r) in batches of 2 (same
    # thread count as the ranks: CPU reductions are ordered by it)
    old = torch.get_num_threads()
    torch.set_num_threads(2)
    try:
        expect = torch.cat([E.evaluate_shard(_load, _solve, *shard.shard_range(len(PAIRS), world, r), 2)
                            for r in range(world)])
    finally:
        torch.set_num_threads(old)
    assert torch.equal(rows, expect)
    base = tmp_path / "test_results" / "nolearning"
    info = pickle.load(open(base / "fr1_desk_keyframe_1.pkl", "rb"))  # written by this test's own rank 0
    assert info["names"] == [f"{i}->{j}" for i, j in PAIRS]
    np.testing.assert_array_equal(info["t_est"], rows[:, 9:12].numpy())
    np.testing.assert_array_equal(info["epes"], rows[:, 14].numpy())
    assert (base / "fr1_desk_keyframe_1.csv").exists()
    # the rows carry the errors evaluate.py computes: translation error = |t| against identity
    np.testing.assert_allclose(info["translation_error"], np.linalg.norm(info["t_est"], axis=1), rtol=1e-5)
