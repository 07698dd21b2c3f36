"""Pose-error metrics used to report "3DPE vs ref" (host-side, PyTorch).

Restated from the reference's criterions (code/models/criterions.py):
3D end-point error = mean over valid reference pixels of
|(R_a X + t_a) - (R_b X + t_b)|_2 with X the back-projected frame-0 depth
(`compute_RT_EPE_loss` + `EPE3D_loss`, criterions.py:23-46, 101-136), and the
relative pose error = (rotation angle, translation norm) of T_b^-1-between
(`compute_RPE_loss`, criterions.py:49-57, 79-98; geometry.py:125-144, 187-207).
"""
import torch


def back_project(depth, K):
    """[B,1,H,W] depth, [B,4] K -> [B,3,H*W] points (geometry.batch_inverse_project)."""
    B, _, H, W = depth.shape
    fx, fy, cx, cy = (K[:, i].view(B, 1) for i in range(4))
    u = torch.arange(W, dtype=depth.dtype, device=depth.device).repeat(H).view(1, -1)
    v = torch.arange(H, dtype=depth.dtype, device=depth.device).repeat_interleave(W).view(1, -1)
    z = depth.reshape(B, -1)
    return torch.stack(((u - cx) / fx * z, (v - cy) / fy * z, z), 1)


def epe3d_between(Ra, ta, Rb, tb, depth, K, invalid=None):
    """Per-pair mean 3D end-point error [B] between poses a and b."""
    B = Ra.shape[0]
    X = back_project(depth, K)
    pa = torch.bmm(Ra, X) + ta.reshape(B, 3, 1)
    pb = torch.bmm(Rb, X) + tb.reshape(B, 3, 1)
    err = (pa - pb).norm(dim=1)
    bad = torch.isnan(pb).any(1)
    if invalid is not None:
        bad = bad | invalid.reshape(B, -1)
    out = []
    for i in range(B):
        e = err[i][~bad[i]]
        out.append(e.mean() if e.numel() else torch.zeros((), dtype=err.dtype, device=err.device))
    return torch.stack(out)


def rpe(Ra, ta, Rb, tb):
    """(angle [B] rad, translation [B]) of the relative pose between a and b."""
    B = Ra.shape[0]
    dR = torch.bmm(Rb, Ra.transpose(1, 2))
    dt = tb.reshape(B, 3) - torch.bmm(dR, ta.reshape(B, 3, 1)).view(B, 3)
    tr = dR.diagonal(dim1=1, dim2=2).sum(1)
    eps = 1e-7
    ang = torch.acos(((tr - 1) / 2).clamp(-1 + eps, 1 - eps))
    return ang, dt.norm(dim=1)
