"""Pose-error criterions of the evaluation scripts: the drop-in `models.criterions`.

Restated from the reference's code/models/criterions.py, same names, arguments and
conventions, evaluation (non-training) branch -- the functions evaluate.py:203-212 and
convergence_basin.py call:
  EPE3D_loss            criterions.py:23-46   per-sample mean |flow_gt - flow_est|_2
                                              over pixels that are not NaN / invalid
  RPE                   criterions.py:49-57   (rotation angle, |t|) of a relative pose
  compute_RPE_loss      criterions.py:79-98   RPE of between(T_est -> T_gt)
  compute_RT_EPE_loss   criterions.py:101-136 3D end-point error of the back-projected
                                              frame-0 depth under T_est vs T_gt
The training losses with learned pose uncertainty (compute_RPE_uncertainty,
compute_RT_EPE_uncertainty_loss, criterions.py:60-77, 139-248) belong to train.py,
which this build does not support (no backward kernels).  Host-side PyTorch.
"""
import torch

from . import geometry as geo


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


