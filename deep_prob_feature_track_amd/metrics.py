"""Pose-error metrics of the evaluation scripts ("3DPE vs ref", RPE).

The reference's criterions (code/models/criterions.py) live in models/criterions.py
(the drop-in `models.criterions` the reference's evaluate.py / convergence_basin.py
import); this module adds the bench / evaluation bookkeeping around them:
  EPE3D_loss            criterions.py:23-46   per-sample mean |flow_gt - flow_est|_2
                                              over pixels that are not NaN / invalid
  RPE                   criterions.py:49-57   (rotation angle, |t|) of a relative pose
  compute_RPE_loss      criterions.py:79-98   RPE of between(T_est -> T_gt)
  compute_RT_EPE_loss   criterions.py:101-136 3D end-point error of the back-projected
                                              frame-0 depth under T_est vs T_gt
Host-side PyTorch (runs on whichever device the tensors are on).
"""
from .models import geometry as geo
from .models.criterions import EPE3D_loss, RPE, compute_RPE_loss, compute_RT_EPE_loss  # noqa: F401


# ---------------------------------------------------------------- bench helpers
def back_project(depth, K):
    """[B,1,H,W] depth, [B,4] K -> [B,3,H*W] points."""
    B = depth.shape[0]
    return geo.batch_inverse_project(depth, K).view(B, 3, -1)


def epe3d_between(Ra, ta, Rb, tb, depth, K, invalid=None):
    """Per-pair mean 3D end-point error [B] between poses a and b (compute_RT_EPE_loss)."""
    return compute_RT_EPE_loss(Ra, ta, Rb, tb, depth, K, invalid=invalid)


def rpe(Ra, ta, Rb, tb):
    """(angle [B] rad, translation [B]) of the relative pose between a and b (compute_RPE_loss)."""
    return compute_RPE_loss(Ra, ta, Rb, tb)


# ---------------------------------------------------------------- evaluation bookkeeping
# evaluate.py's per-batch record (evaluate_trust_region, evaluate.py:195-224), the
# per-(trajectory, keyframe) summary and the frame-weighted means (test_TrustRegion,
# evaluate.py:318-372), and its two outputs: the per-frame `info` dict as
# <eval_set>_results/<checkpoint>/<trajectory>_keyframe_<k>.pkl and the summary CSV.

class EvalRecorder:
    """Accumulates evaluate_trust_region's `outputs` dict batch by batch."""

    def __init__(self):
        import numpy as np
        self._np = np
        self.parts = {k: [] for k in ("R_est", "t_est", "angular_error", "translation_error", "epes")}
        self.names = []

    def add(self, R, t, R_gt, t_gt, depth0, K, names=(), obj_mask0=None):
        """One batch: the solver's (R [B,3,3], t [B,3(,1)]) against ground truth; EPE3D
        over pixels whose depth is not the batch min / max (and inside obj_mask0), as
        evaluate.py:206-212."""
        B = R.shape[0]
        t = t.reshape(B, 3)
        t_gt = t_gt.reshape(B, 3)
        ang, trans = compute_RPE_loss(R, t, R_gt, t_gt)
        invalid = (depth0 == depth0.min()) | (depth0 == depth0.max())
        if obj_mask0 is not None:
            invalid = ~obj_mask0 | invalid
        epes = compute_RT_EPE_loss(R, t, R_gt, t_gt, depth0, K, invalid=invalid)
        for k, v in (("R_est", R), ("t_est", t), ("angular_error", ang), ("translation_error", trans),
                     ("epes", epes)):
            self.parts[k].append(v.detach().cpu().numpy())
        self.names += list(names)

    def outputs(self):
        np = self._np
        out = {k: (np.concatenate(v, 0) if v else np.zeros((0,))) for k, v in self.parts.items()}
        out["names"] = list(self.names)
        return out


def summarize(results, keyframes):
    """results: {'<trajectory>_keyframe_<k>': EvalRecorder.outputs()} -> pandas.DataFrame
    with one row per entry (3D EPE cm, axis error deg, trans error cm, total frames,
    keyframe, trajectory) followed by, per keyframe, the mean over trajectories and the
    frame-weighted mean (evaluate.py:318-370; DataFrame.append there = pd.concat here)."""
    import numpy as np
    import pandas as pd
    rows = {}
    for k, info in results.items():
        traj, kf = k.split("_keyframe_")
        rows[k] = pd.Series([info["epes"].mean(), info["angular_error"].mean(), info["translation_error"].mean(),
                             info["epes"].shape[0], int(kf), traj],
                            index=["3D EPE", "axis error", "trans error", "total frames", "keyframe", "trajectory"])
    out = pd.DataFrame(rows).T
    for c in ("3D EPE", "axis error", "trans error"):
        out[c] = out[c].astype(float)
    out["3D EPE"] *= 100
    out["axis error"] *= 180 / np.pi
    out["trans error"] *= 100
    stats = {}
    for kf in keyframes:
        sel = out[out["keyframe"] == kf]
        stats[f"mean values of trajectories keyframe {kf}"] = pd.Series(
            [sel["3D EPE"].mean(), sel["axis error"].mean(), sel["trans error"].mean(), kf],
            index=["3D EPE", "axis error", "trans error", "keyframe"])
        n = sel["total frames"].astype(float)
        total = n.sum()
        stats[f"mean values of frames keyframe {kf}"] = pd.Series(
            [(sel["3D EPE"] * n).sum() / total, (sel["axis error"] * n).sum() / total,
             (sel["trans error"] * n).sum() / total, kf],
            index=["3D EPE", "axis error", "trans error", "keyframe"])
    return pd.concat([out, pd.DataFrame(stats).T], sort=False)


def write_results(results, keyframes, eval_set, checkpoint_name="nolearning", root="."):
    """evaluate.py's outputs: one pickle of the per-frame dict per entry and the summary
    CSV, under <root>/<eval_set>_results/<checkpoint_name>/ (the CSV is named after the
    last entry, as evaluate.py:372 does).  Returns the summary DataFrame."""
    import os
    import pickle
    base = os.path.join(root, f"{eval_set}_results", checkpoint_name)
    os.makedirs(base, exist_ok=True)
    last = None
    for k, info in results.items():
        last = os.path.join(base, k)
        with open(last + ".pkl", "wb") as f:
            pickle.dump(info, f)
    table = summarize(results, keyframes)
    if last is not None:
        table.to_csv(f"{last}.csv")
    return table
