"""Pose-error metrics of the evaluation scripts ("3DPE vs ref", RPE).

Restated from the reference's criterions (code/models/criterions.py), same names
and conventions, evaluation (non-training) branch:
  EPE3D_loss            criterions.py:23-46   per-sample mean |flow_gt - flow_est|_2
                                              over pixels that are not NaN / invalid
  RPE                   criterions.py:49-57   (rotation angle, |t|) of a relative pose
  compute_RPE_loss      criterions.py:79-98   RPE of between(T_est -> T_gt)
  compute_RT_EPE_loss   criterions.py:101-136 3D end-point error of the back-projected
                                              frame-0 depth under T_est vs T_gt
Host-side PyTorch (runs on whichever device the tensors are on).
"""
import torch

from .models import geometry as geo


def EPE3D_loss(input_flow, target_flow, invalid=None):
    epe_map = torch.norm(target_flow - input_flow, p=2, dim=1)
    B = epe_map.shape[0]
    bad = torch.isnan(target_flow).any(1)
    if invalid is not None:
        bad = bad | (invalid.view(bad.shape) > 0)
    out = []
    for i in range(B):
        e = epe_map[i][~bad[i]]
        out.append(e.mean() if e.numel() else torch.zeros((), dtype=input_flow.dtype, device=input_flow.device))
    return torch.stack(out)


def RPE(R, t):
    return geo.batch_mat2angle(R), torch.norm(t.reshape(t.shape[0], 3), p=2, dim=1)


def compute_RPE_loss(R_est, t_est, R_gt, t_gt):
    dR, dt = geo.batch_Rt_between(R_est, t_est, R_gt, t_gt)
    return RPE(dR, dt)


def compute_RT_EPE_loss(R_est, t_est, R_gt, t_gt, depth0, K, invalid=None):
    xyz = geo.batch_inverse_project(depth0, K)
    flow_gt = geo.batch_transform_xyz(xyz, R_gt, t_gt)
    flow_est = geo.batch_transform_xyz(xyz, R_est, t_est)
    return EPE3D_loss(flow_est, flow_gt, invalid=invalid)


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
