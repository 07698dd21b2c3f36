"""Host-side SE(3) helpers used around the solver (init-pose networks, callers).

The per-pixel geometry of the hot path (warp, occlusion, sampling, Jacobians)
lives in the HIP kernels; these are the small batched [B,3,3] helpers:
  batch_euler2mat   geometry.py:447-504 ('sxyz' axes, the only ones the tracker uses)
  pose_vec2mat      geometry.py:274-289 (keeps the reference's quirk: the rotation is
                    built from vec[:, 3:], the translation part -- Appendix C of SURVEY.md)
  batch_Rt_compose  geometry.py:105-123
  batch_inverse_Rt  geometry.py:87-103
  batch_Rt_between  geometry.py:125-144
"""
import torch


def batch_euler2mat(ai, aj, ak):
    """Rotation matrices [B,3,3] from static x-y-z Euler angles [B] each."""
    si, sj, sk = torch.sin(ai), torch.sin(aj), torch.sin(ak)
    ci, cj, ck = torch.cos(ai), torch.cos(aj), torch.cos(ak)
    cc, cs, sc, ss = ci * ck, ci * sk, si * ck, si * sk
    rows = (
        (cj * ck, sj * sc - cs, sj * cc + ss),
        (cj * sk, sj * ss + cc, sj * cs - sc),
        (-sj, cj * si, cj * ci),
    )
    return torch.stack([torch.stack(r, 1) for r in rows], 1)


def pose_vec2mat(vec, rotation_mode='euler'):
    """[B,6] -> (R [B,3,3], t [B,3]); rotation from vec[:, 3:] exactly as the reference."""
    if rotation_mode != 'euler':
        raise NotImplementedError("only euler pose vectors are used by the tracker")
    trs = vec[:, 3:]
    rot = batch_euler2mat(vec[:, 3], vec[:, 4], vec[:, 5])
    return rot, trs


def batch_Rt_compose(d_R, d_t, R0, t0):
    """(d_R R0, d_R t0 + d_t), translations [B,3]."""
    R1 = torch.bmm(d_R, R0)
    t1 = torch.bmm(d_R, t0.reshape(-1, 3, 1)) + d_t.reshape(-1, 3, 1)
    return R1, t1.view(-1, 3)


def batch_inverse_Rt(R, t):
    """Inverse transform (R^T, -R^T t), translation [B,3]."""
    Rt = R.transpose(1, 2)
    return Rt, -torch.bmm(Rt, t.reshape(-1, 3, 1)).view(-1, 3)


def batch_Rt_between(R0, t0, R1, t1):
    """Transform from T0 to T1: T1 T0^-1 = (R1 R0^T, t1 - R1 R0^T t0)."""
    dR = torch.bmm(R1, R0.transpose(1, 2))
    return dR, t1.reshape(-1, 3) - torch.bmm(dR, t0.reshape(-1, 3, 1)).view(-1, 3)


def batch_mat2euler(M):
    """Static x-y-z Euler angles (ax, ay, az) [B] each of rotations [B,3,3]
    (geometry.py:506-554, 'sxyz': i, j, k = 0, 1, 2, no repetition / parity / frame)."""
    cy = torch.sqrt(M[:, 0, 0] ** 2 + M[:, 1, 0] ** 2)
    degenerate = ~(cy > 1e-8)
    ax = torch.atan2(M[:, 2, 1], M[:, 2, 2])
    ay = torch.atan2(-M[:, 2, 0], cy)
    az = torch.atan2(M[:, 1, 0], M[:, 0, 0])
    if bool(degenerate.any()):
        ax = torch.where(degenerate, torch.atan2(-M[:, 1, 2], M[:, 1, 1]), ax)
        az = torch.where(degenerate, torch.zeros_like(az), az)
    return ax, ay, az


def batch_mat2angle(R):
    """Rotation angle [B] of rotations [B,3,3] (geometry.py:187-207)."""
    tr = torch.stack([torch.trace(R[i]) for i in range(R.shape[0])])  # the reference's per-matrix trace
    eps = 1e-7
    return torch.acos(((tr - 1) / 2).clamp(-1 + eps, 1 - eps))


def batch_inverse_project(depth, K):
    """[B,1,H,W] depth, [B,4] K -> [B,3,H,W] camera points (geometry.py:429-445)."""
    B, _, H, W = depth.shape
    fx, fy, cx, cy = (K[:, i].view(B, 1, 1, 1) for i in range(4))
    v, u = torch.meshgrid(torch.arange(H, dtype=depth.dtype, device=depth.device),
                          torch.arange(W, dtype=depth.dtype, device=depth.device), indexing='ij')
    x = (u.view(1, 1, H, W) - cx) / fx * depth
    y = (v.view(1, 1, H, W) - cy) / fy * depth
    return torch.cat((x, y, depth), 1)


def batch_transform_xyz(xyz, R, t):
    """R xyz + t for [B,3,H,W] points (geometry.py:376-399, without the Jacobian)."""
    B, _, H, W = xyz.shape
    return (torch.bmm(R, xyz.view(B, 3, -1)) + t.reshape(B, 3, 1)).view(B, 3, H, W)
