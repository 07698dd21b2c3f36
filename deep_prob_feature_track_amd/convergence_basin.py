"""Convergence-basin sweep of the learned tracker on the HIP solver.

Per batch, the same quantities as the reference's convergence_basin.py
(`evaluate_convergence_basin` 264-475 and `evaluate_2d_convergence_basin`
85-262, without the dataloader / tqdm loop): the optimised pose, the residual
landscape along each of the 6 pose axes around the ground truth (rotation as
static x-y-z Euler offsets, translation offsets), the losses at the identity,
predicted and optimised poses, and the RPE / 3D-EPE of the estimate.

The reference re-runs the encoder and one residual pass per perturbation
(`compute_residual`, LeastSquareTracking.py:605-651); here the pyramids are
computed once per batch and every perturbation of a level is evaluated in ONE
multi-pose residual launch (`dpft_ic_residual_poses`).  Each pose is still
evaluated as its own reference call over the batch (per-pose batch-global
truncated-sigma extrema), so the numbers are the reference's.

`convergence_counts` adds what the reference does not define:
the number of pairs whose optimised pose lies within rotation / translation
thresholds of the ground truth, with per-pair margins so a count can be
checked for stability under the fp32 noise floor.
"""
import numpy as np
import torch

from . import metrics
from .models import geometry as geo

ROTATION_AXES = ['yaw', 'pitch', 'roll']
TRANSLATION_AXES = ['tran-x', 'tran-y', 'tran-z']


def _euler_stack(R):
    return torch.stack(geo.batch_mat2euler(R), dim=1)


def _euler_to_R(angles):
    return geo.batch_euler2mat(angles[:, 0], angles[:, 1], angles[:, 2])


def axis_perturbations(R_gt, t_gt, rot_pert, trs_pert):
    """Poses [6*S,B] of the 1-D sweeps: rotation axis i offset by rot_pert[s]
    (translation at GT), then translation axis i offset by trs_pert[s]."""
    B = R_gt.shape[0]
    ang = _euler_stack(R_gt)
    Rs, ts = [], []
    for i in range(3):
        for e in rot_pert:
            a = ang.clone()
            a[:, i] = ang[:, i] + float(e)
            Rs.append(_euler_to_R(a))
            ts.append(t_gt.reshape(B, 3))
    for i in range(3):
        for e in trs_pert:
            tp = t_gt.reshape(B, 3).clone()
            tp[:, i] = tp[:, i] + float(e)
            Rs.append(R_gt)
            ts.append(tp)
    return torch.stack(Rs), torch.stack(ts)


def evaluate_convergence_basin(net, color0, color1, depth0, depth1, Rt, K, obj_mask0=None, obj_mask1=None,
                               level_i=None, trans_pert_range=(-0.1, 0.1), rot_pert_range=(-0.1, 0.1),
                               pert_samples=31, objectives=('EPE3D', 'RPE')):
    """One batch of convergence_basin.py:264-475.  Returns numpy arrays:
    R_est [B,3,3], t_est [B,3], R_gt [B,3] (Euler), t_gt [B,3],
    pose_per / avg_loss [6, S+3, B] (S sweep samples, then identity, predicted, optimised),
    coarse_pose_per / coarse_avg_loss [L-1, 6, S, B], epes, angular_error, translation_error [B]."""
    levels = [0] if level_i is None else list(level_i)
    S = pert_samples
    B = depth0.shape[0]
    R_gt, t_gt = Rt[:, :3, :3].contiguous(), Rt[:, :3, 3].contiguous()
    ang_gt = _euler_stack(R_gt)
    with torch.no_grad():
        R_est, t_est = net.forward(color0, color1, depth0, depth1, K, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        t_est = t_est.reshape(B, 3)
        prep = net.prepare(color0, color1, depth0, depth1, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        rot_pert = np.linspace(rot_pert_range[0], rot_pert_range[1], S)
        trs_pert = np.linspace(trans_pert_range[0], trans_pert_range[1], S)
        Rp, tp = axis_perturbations(R_gt, t_gt, rot_pert, trs_pert)
        out = {
            'R_est': R_est.cpu().numpy(), 't_est': t_est.cpu().numpy(),
            'R_gt': ang_gt.cpu().numpy(), 't_gt': t_gt.cpu().numpy(),
            'pose_per': np.zeros((6, S + 3, B)), 'avg_loss': np.zeros((6, S + 3, B)),
            'coarse_pose_per': np.zeros((max(len(levels) - 1, 0), 6, S, B)),
            'coarse_avg_loss': np.zeros((max(len(levels) - 1, 0), 6, S, B)),
        }
        grid = np.concatenate([np.tile(rot_pert, 3), np.tile(trs_pert, 3)]).reshape(6, S)
        for level in levels:
            loss = net.compute_residual_poses(prep, K, Rp, tp, level_i=level).view(6, S, B).cpu().numpy()
            if level == 0:
                out['avg_loss'][:, :S] = loss
                out['pose_per'][:, :S] = grid[:, :, None]
            else:
                out['coarse_avg_loss'][level - 1] = loss
                out['coarse_pose_per'][level - 1] = grid[:, :, None]

        # identity (per axis: that coordinate set to 0), predicted init, optimised -- level 0
        R_pred, t_pred = prep[-1]
        special_R, special_t = [], []
        for i in range(3):
            a = ang_gt.clone()
            a[:, i] = 0.0
            special_R.append(_euler_to_R(a))
            special_t.append(t_gt)
        for i in range(3):
            t0 = t_gt.clone()
            t0[:, i] = 0.0
            special_R.append(R_gt)
            special_t.append(t0)
        special_R += [R_pred.reshape(B, 3, 3), R_est]
        special_t += [t_pred.reshape(B, 3), t_est]
        loss = net.compute_residual_poses(prep, K, torch.stack(special_R), torch.stack(special_t), level_i=0)
        loss = loss.cpu().numpy()
        ang_pred = _euler_stack(R_pred.reshape(B, 3, 3))
        ang_est = _euler_stack(R_est)
        for i in range(6):
            out['avg_loss'][i, S] = loss[i]
            out['avg_loss'][i, S + 1] = loss[6]
            out['avg_loss'][i, S + 2] = loss[7]
            if i < 3:
                out['pose_per'][i, S] = (0.0 - ang_gt[:, i]).cpu().numpy()
                out['pose_per'][i, S + 1] = (ang_pred[:, i] - ang_gt[:, i]).cpu().numpy()
                out['pose_per'][i, S + 2] = (ang_est[:, i] - ang_gt[:, i]).cpu().numpy()
            else:
                j = i - 3
                out['pose_per'][i, S] = (0.0 - t_gt[:, j]).cpu().numpy()
                out['pose_per'][i, S + 1] = (t_pred.reshape(B, 3)[:, j] - t_gt[:, j]).cpu().numpy()
                out['pose_per'][i, S + 2] = (t_est[:, j] - t_gt[:, j]).cpu().numpy()

        if 'RPE' in objectives:
            ae, te = metrics.compute_RPE_loss(R_est, t_est, R_gt, t_gt)
            out['angular_error'], out['translation_error'] = ae.cpu().numpy(), te.cpu().numpy()
        if 'EPE3D' in objectives:
            invalid = (depth0 == depth0.min()) | (depth0 == depth0.max())
            if obj_mask0 is not None:
                invalid = ~obj_mask0 | invalid
            out['epes'] = metrics.compute_RT_EPE_loss(R_est, t_est, R_gt, t_gt, depth0, K, invalid=invalid).cpu().numpy()
    return out


def evaluate_2d_convergence_basin(net, color0, color1, depth0, depth1, Rt, K, obj_mask0=None, obj_mask1=None,
                                  level_i=None, trans_pert_range=(-0.1, 0.1), pert_samples=31):
    """One batch of convergence_basin.py:85-262: the x-y translation landscape
    avg_loss [L, S, S, B] around the ground truth (rotation and z frozen)."""
    levels = [0] if level_i is None else list(level_i)
    S = pert_samples
    B = depth0.shape[0]
    R_gt, t_gt = Rt[:, :3, :3].contiguous(), Rt[:, :3, 3].contiguous()
    trs = np.linspace(trans_pert_range[0], trans_pert_range[1], S)
    with torch.no_grad():
        prep = net.prepare(color0, color1, depth0, depth1, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        Rs, ts = [], []
        for ex in trs:
            for ey in trs:
                Rs.append(R_gt)
                ts.append(t_gt + torch.tensor([ex, ey, 0.0], dtype=t_gt.dtype, device=t_gt.device).view(1, 3))
        Rp, tp = torch.stack(Rs), torch.stack(ts)
        out = {'avg_loss': np.zeros((len(levels), S, S, B)),
               'pose_per_x': np.broadcast_to(trs[None, :, None, None], (len(levels), S, S, B)).copy(),
               'pose_per_y': np.broadcast_to(trs[None, None, :, None], (len(levels), S, S, B)).copy()}
        for li, level in enumerate(levels):
            out['avg_loss'][li] = net.compute_residual_poses(prep, K, Rp, tp, level_i=level).view(S, S, B).cpu().numpy()
    return out


def convergence_counts(R_est, t_est, R_gt, t_gt, rot_thresh=0.01, trans_thresh=0.01):
    """Pairs whose estimate is within `rot_thresh` rad and `trans_thresh` m of the
    ground truth (compute_RPE_loss errors), plus each pair's signed margins
    (threshold - error) so that a count can be checked for stability."""
    ae, te = metrics.compute_RPE_loss(R_est, t_est.reshape(-1, 3), R_gt, t_gt.reshape(-1, 3))
    ok = (ae < rot_thresh) & (te < trans_thresh)
    return int(ok.sum().item()), {'rot_margin': (rot_thresh - ae).cpu().numpy(),
                                  'trans_margin': (trans_thresh - te).cpu().numpy(),
                                  'converged': ok.cpu().numpy()}


# ---------------------------------------------------------------------------------------
# Solves from perturbed starts (cfg4: the large-baseline convergence-basin sweep)
#
# The reference's LeastSquareTracking.forward has no initial-pose argument; a solve from a
# given start is the per-level solver chain tr_update3 .. tr_update0 entered with that pose
# (LeastSquareTracking.py:349-445 after the init pose of 686-695), which is what
# ic.PyramidSolver runs.  Each start set (one start per pair) is solved as its own
# reference call over the batch -- its own batch-global truncated-sigma extrema -- and up
# to 32 start sets share every launch as independent batches (DPFT_GROUP).

def solve_from_starts(levels, K, R0, t0, iters=3, remove_tru_sigma=True, max_pairs=2048):
    """levels: per-level dicts of B pairs (x0, x1 NCHW or channel-quad packed, invD0, invD1,
    sigma0, sigma1[, obj_mask0, obj_mask1]), K [B,4] level-0 intrinsics; R0 [P,B,3,3],
    t0 [P,B,3(,1)] start poses -> (R [P,B,3,3], t [P,B,3]): start set p solved as one call
    over the B pairs.  Start sets go max_pairs // B at a time (at most 32) through one
    grouped PyramidSolver; a short last round is padded with copies of its first set."""
    from . import _native as N
    from . import ic
    P, B = R0.shape[:2]
    if B > max_pairs:
        raise ValueError(f"B={B} pairs exceed {max_pairs} per call")
    G = max(1, min(P, N.GROUP_MAX_BATCHES, max_pairs // B))
    rep = lambda v: v.repeat(G, *([1] * (v.dim() - 1))) if G > 1 else v
    lv = [{k: rep(v) for k, v in d.items()} for d in levels]
    solver = ic.PyramidSolver(lv, rep(K.reshape(B, 4)).contiguous(), iters=iters, remove_tru_sigma=remove_tru_sigma,
                              group=B if G > 1 else None)
    dev = levels[0]["x0"].device
    R0 = R0.to(device=dev, dtype=torch.float32).reshape(P, B, 3, 3)
    t0 = t0.to(device=dev, dtype=torch.float32).reshape(P, B, 3)
    R = torch.empty(G * B, 3, 3, device=dev)
    t = torch.empty(G * B, 3, device=dev)
    out_R, out_t = torch.empty(P, B, 3, 3, device=dev), torch.empty(P, B, 3, device=dev)
    for p0 in range(0, P, G):
        g = min(G, P - p0)
        idx = list(range(p0, p0 + g)) + [p0] * (G - g)
        R.copy_(R0[idx].reshape(G * B, 3, 3))
        t.copy_(t0[idx].reshape(G * B, 3))
        solver.run(R, t)
        out_R[p0:p0 + g] = R[:g * B].view(g, B, 3, 3)
        out_t[p0:p0 + g] = t[:g * B].view(g, B, 3)
    ic.check_status(solver.status)
    return out_R, out_t


def perturbed_starts(R_c, t_c, rot_pert, trs_pert):
    """Start poses [6 S, B] around the pose (R_c, t_c): the reference's 1-D sweep axes
    (convergence_basin.py:337-418: static x-y-z Euler offsets for rotation, offsets of one
    translation coordinate) applied as initial poses instead of residual evaluations."""
    return axis_perturbations(R_c, t_c.reshape(-1, 3), rot_pert, trs_pert)


def basin_counts(R_fin, t_fin, R_tgt, t_tgt, rot_thresh=0.01, trans_thresh=0.01):
    """Convergence of every start set: count [P] of pairs whose solve from that start lands
    within (rot_thresh rad, trans_thresh m) of the target pose (compute_RPE_loss errors),
    and the per-(start, pair) margins [P,B] (threshold - error; a count is stable under a
    pose noise eps when no |margin| is below it)."""
    P, B = R_fin.shape[:2]
    counts, rot_m, trs_m = [], [], []
    for p in range(P):
        n, m = convergence_counts(R_fin[p], t_fin[p], R_tgt, t_tgt, rot_thresh, trans_thresh)
        counts.append(n)
        rot_m.append(m["rot_margin"])
        trs_m.append(m["trans_margin"])
    return np.array(counts), {"rot_margin": np.stack(rot_m), "trans_margin": np.stack(trs_m)}
