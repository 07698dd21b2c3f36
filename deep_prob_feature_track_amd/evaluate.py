"""Sharded evaluation driver over the drop-in tracker (one process per GPU).

The reference's evaluation (code/evaluate.py:123-374) loads batches of
`batch_per_gpu * device_count()` frame pairs (evaluate.py:237) but runs them on ONE device
(no DataParallel), records per batch R / t and the RPE / 3D-EPE errors against ground
truth (evaluate_trust_region, 142-226) and writes one pickle per (trajectory, keyframe) and a
summary CSV (318-372).  Here the pair list of an evaluation set is sharded contiguously over
the ranks (shard.shard_range); each rank runs the tracker on its shard in batches of
`batch` pairs (each batch one reference call: its own batch-global masks), computes its
pairs' errors, and ONE padded all-gather of the per-pair rows [R(9), t(3), angle, trans,
epe] (shard.gather_rows: RCCL over xGMI, gloo on CPU) brings every pair to every rank in
pair order; rank 0 writes the reference's pkl / CSV (metrics.write_results).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m deep_prob_feature_track_amd.evaluate --pairs 64 --batch 8 --out eval_out

The CLI evaluates the TUM fr1/desk example frames the reference ships (examples.py:
data/tum_fr1_desk_frames.npz; the datasets and checkpoints are absent): the ordered pairs
cycled to --pairs, the tracker with deterministic synthetic weights
(examples.synthetic_weights), ground truth = identity (no poses ship with the frames), so the
errors are the estimated motions' magnitudes.
"""
import argparse
import os

import numpy as np
import torch

from . import metrics, shard

ROW = 15  # R(9), t(3), angular error, translation error, 3D EPE


def evaluate_shard(load, solve, begin, end, batch):
    """Rows [end - begin, 15] of pairs [begin, end): load(i0, i1) -> dict(color0, color1,
    depth0, depth1, K, R_gt, t_gt[, obj_mask0, obj_mask1]) for pairs [i0, i1);
    solve(d) -> (R [b,3,3], t [b,3(,1)]).  Errors as evaluate.py:203-212 (RPE against
    ground truth; 3D EPE over pixels whose depth is not the batch min / max, inside obj_mask0)."""
    rows = []
    for i0 in range(begin, end, batch):
        d = load(i0, min(i0 + batch, end))
        R, t = solve(d)
        b = R.shape[0]
        rec = metrics.EvalRecorder()
        rec.add(R.detach().float().cpu(), t.detach().float().cpu().reshape(b, 3), d["R_gt"].float().cpu(),
                d["t_gt"].float().cpu().reshape(b, 3), d["depth0"].float().cpu(), d["K"].float().cpu(),
                obj_mask0=d["obj_mask0"].cpu() if d.get("obj_mask0") is not None else None)
        o = rec.outputs()
        rows.append(torch.cat([torch.from_numpy(o["R_est"]).reshape(b, 9), torch.from_numpy(o["t_est"]).reshape(b, 3),
                               torch.from_numpy(np.stack([o["angular_error"], o["translation_error"], o["epes"]], 1))],
                              1).float())
    return torch.cat(rows, 0) if rows else torch.zeros(0, ROW)


def evaluate_sharded(load, solve, n_pairs, batch, device=None):
    """Every rank: its shard's rows, then the all-gather -> [n_pairs, 15] rows in pair
    order (on every rank).  Without an initialised process group: one rank, no gather."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return evaluate_shard(load, solve, 0, n_pairs, batch)
    world, rank = torch.distributed.get_world_size(), torch.distributed.get_rank()
    b, e = shard.shard_range(n_pairs, world, rank)
    rows = evaluate_shard(load, solve, b, e, batch)
    if device is not None:
        rows = rows.to(device)
    return shard.gather_rows(rows.contiguous(), n_pairs).cpu()


def rows_to_outputs(rows, names):
    """[n, 15] rows -> evaluate_trust_region's `outputs` dict (evaluate.py:142-154)."""
    r = rows.numpy()
    return {"R_est": r[:, :9].reshape(-1, 3, 3), "t_est": r[:, 9:12], "angular_error": r[:, 12],
            "translation_error": r[:, 13], "epes": r[:, 14], "names": list(names)}


# ----------------------------------------------------------------------------- CLI
def _example_loader(n_pairs, H, W, device):
    """TUM fr1/desk example pairs (ordered pairs of the five frames, cycled), ground truth
    identity; color [3,H,W] in [0,1], depth in m clipped to [0.5, 5] (SimpleLoader.py:77-80)."""
    from . import examples as ex
    down = 640 // W
    pairs = [ex.ORDERED_PAIRS[k % len(ex.ORDERED_PAIRS)] for k in range(n_pairs)]

    def load(i0, i1):
        sel = pairs[i0:i1]
        b = len(sel)
        col = lambda i: torch.from_numpy(ex.color_float(i, down))
        dep = lambda i: torch.from_numpy(ex.depth_m(i, down))[None]
        K = torch.from_numpy(np.tile(ex.K_FULL[None] / down, (b, 1)))
        return {"color0": torch.stack([col(i) for i, _ in sel]).to(device),
                "color1": torch.stack([col(j) for _, j in sel]).to(device),
                "depth0": torch.stack([dep(i) for i, _ in sel]).to(device),
                "depth1": torch.stack([dep(j) for _, j in sel]).to(device),
                "K": K.to(device), "R_gt": torch.eye(3).repeat(b, 1, 1), "t_gt": torch.zeros(b, 3)}
    return pairs, load


def _tracker(C, device):
    """The drop-in LeastSquareTracking (ConvRGBD2 encoder, laplacian uncertainty, U_IC,
    remove_tru_sigma) with deterministic synthetic weights (examples.py)."""
    from .examples import load_synthetic_weights
    from .models.LeastSquareTracking import LeastSquareTracking, default_options
    net = LeastSquareTracking("ConvRGBD2", "laplacian", 3, "None", "Direct-Nodamping",
                              options=default_options(feature_channel=C, uncertainty_channel=1,
                                                      feature_extract="conv", remove_tru_sigma=True))
    return load_synthetic_weights(net).to(device).eval()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=64)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--width", type=int, default=640, choices=[640, 320, 160])
    p.add_argument("--channels", type=int, default=32)
    p.add_argument("--out", default="eval_out")
    p.add_argument("--eval-set", default="test")
    p.add_argument("--trajectory", default="fr1_desk_examples")
    p.add_argument("--keyframe", type=int, default=1)
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("the evaluation driver runs the HIP tracker: no device visible")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        torch.distributed.init_process_group("nccl")
    rank = torch.distributed.get_rank() if world > 1 else 0
    pairs, load = _example_loader(a.pairs, a.width * 3 // 4, a.width, device)
    net = _tracker(a.channels, device)

    def solve(d):
        with torch.no_grad():
            R, t = net.forward(d["color0"], d["color1"], d["depth0"], d["depth1"], d["K"])
        return R, t
    rows = evaluate_sharded(load, solve, a.pairs, a.batch, device=device if world > 1 else None)
    if rank == 0:
        names = [f"{i}->{j}" for i, j in pairs]
        key = f"{a.trajectory}_keyframe_{a.keyframe}"
        table = metrics.write_results({key: rows_to_outputs(rows, names)}, [a.keyframe], a.eval_set,
                                      root=a.out)
        print(table.to_string(), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
