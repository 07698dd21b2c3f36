"""Host-side SE(3) helpers used around the solver (init-pose networks, callers).

The per-pixel geometry of the hot path (warp, occlusion, sampling, Jacobians)
lives in the HIP kernels; these are the small batched [B,3,3] helpers:
  batch_euler2mat   geometry.py:447-504 (every transforms3d axis convention)
  batch_mat2euler   geometry.py:506-554
  batch_create_transform  geometry.py:1139-1149 (kf_vo.py's 4x4 poses)
  pose_vec2mat      geometry.py:274-289 (keeps the reference's quirk: the rotation is
                    built from vec[:, 3:], the translation part -- Appendix C of SURVEY.md)
  batch_Rt_compose  geometry.py:105-123
  batch_inverse_Rt  geometry.py:87-103
  batch_Rt_between  geometry.py:125-144
"""
import numpy as np
import torch


# Euler axis conventions (transforms3d.euler, which geometry.py:447-554 follows): the 24
# axis strings -> (first axis, parity, repetition, frame); 's' = static, 'r' = rotating frame
_NEXT_AXIS = (1, 2, 0, 1)
_AXES2TUPLE = {
    'sxyz': (0, 0, 0, 0), 'sxyx': (0, 0, 1, 0), 'sxzy': (0, 1, 0, 0), 'sxzx': (0, 1, 1, 0),
    'syzx': (1, 0, 0, 0), 'syzy': (1, 0, 1, 0), 'syxz': (1, 1, 0, 0), 'syxy': (1, 1, 1, 0),
    'szxy': (2, 0, 0, 0), 'szxz': (2, 0, 1, 0), 'szyx': (2, 1, 0, 0), 'szyz': (2, 1, 1, 0),
    'rzyx': (0, 0, 0, 1), 'rxyx': (0, 0, 1, 1), 'ryzx': (0, 1, 0, 1), 'rxzx': (0, 1, 1, 1),
    'rxzy': (1, 0, 0, 1), 'ryzy': (1, 0, 1, 1), 'rzxy': (1, 1, 0, 1), 'ryxy': (1, 1, 1, 1),
    'ryxz': (2, 0, 0, 1), 'rzxz': (2, 0, 1, 1), 'rxyz': (2, 1, 0, 1), 'rzyz': (2, 1, 1, 1)}


def _axes(axes):
    """(i, j, k, parity, repetition, frame) of an axis string or tuple."""
    if isinstance(axes, str):
        if axes.lower() not in _AXES2TUPLE:
            raise KeyError(f"unknown Euler axes {axes!r}")
        first, parity, rep, frame = _AXES2TUPLE[axes.lower()]
    else:
        if tuple(axes) not in _AXES2TUPLE.values():
            raise KeyError(f"unknown Euler axes {axes!r}")
        first, parity, rep, frame = axes
    return first, _NEXT_AXIS[first + parity], _NEXT_AXIS[first - parity + 1], parity, rep, frame


def batch_euler2mat(ai, aj, ak, axes='sxyz'):
    """Rotation matrices [B,3,3] from Euler angles [B] each (geometry.py:447-504)."""
    i, j, k, parity, rep, frame = _axes(axes)
    if frame:
        ai, ak = ak, ai
    if parity:
        ai, aj, ak = -ai, -aj, -ak
    si, sj, sk = torch.sin(ai), torch.sin(aj), torch.sin(ak)
    ci, cj, ck = torch.cos(ai), torch.cos(aj), torch.cos(ak)
    cc, cs, sc, ss = ci * ck, ci * sk, si * ck, si * sk
    if rep:
        e = ((cj, sj * si, sj * ci), (sj * sk, -cj * ss + cc, -cj * cs - sc), (-sj * ck, cj * sc + cs, cj * cc - ss))
    else:
        e = ((cj * ck, sj * sc - cs, sj * cc + ss), (cj * sk, sj * ss + cc, sj * cs - sc), (-sj, cj * si, cj * ci))
    # e[a][b] is the entry at (axis a, axis b) of (i, j, k): place it at its matrix position
    ax = (i, j, k)
    M = [[None] * 3 for _ in range(3)]
    for a in range(3):
        for b in range(3):
            M[ax[a]][ax[b]] = e[a][b]
    return torch.stack([torch.stack(r, 1) for r in M], 1)


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


def batch_mat2euler(M, axes='sxyz'):
    """Euler angles (ax, ay, az) [B] each of rotations [B,3,3] (geometry.py:506-554); a
    degenerate matrix (|cos| or |sin| of the middle angle below 1e-8) takes the
    reference's gimbal-lock branch."""
    i, j, k, parity, rep, frame = _axes(axes)
    if rep:
        sy = torch.sqrt(M[:, i, j] ** 2 + M[:, i, k] ** 2)
        degenerate = ~(sy > 1e-8)
        ax = torch.atan2(M[:, i, j], M[:, i, k])
        ay = torch.atan2(sy, M[:, i, i])
        az = torch.atan2(M[:, j, i], -M[:, k, i])
    else:
        cy = torch.sqrt(M[:, i, i] ** 2 + M[:, j, i] ** 2)
        degenerate = ~(cy > 1e-8)
        ax = torch.atan2(M[:, k, j], M[:, k, k])
        ay = torch.atan2(-M[:, k, i], cy)
        az = torch.atan2(M[:, j, i], M[:, i, i])
    if bool(degenerate.any()):
        ax = torch.where(degenerate, torch.atan2(-M[:, j, k], M[:, j, j]), ax)
        az = torch.where(degenerate, torch.zeros_like(az), az)
    if parity:
        ax, ay, az = -ax, -ay, -az
    if frame:
        ax, az = az, ax
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


def batch_create_transform(trs, rot, debug=False):
    """4x4 homogeneous transform(s) from a translation and a rotation (geometry.py:1139-1149):
    numpy [3] + [3,3] -> [4,4]; torch [B,3] + [B,3,3] -> [B,4,4] on rot's device.  `debug` is
    accepted for signature parity and ignored, as there; the bottom row moves device only
    (its float32 zeros / ones promote with `top` in the concatenation, as there).  A torch
    translation of [B,3,1] -- what LeastSquareTracking.forward returns, and what kf_vo.py:173
    passes -- is taken as [B,3] (the reference's concatenation raises on it)."""
    if isinstance(trs, np.ndarray):
        top = np.hstack((rot, trs.reshape(3, 1)))
        return np.vstack((top, np.hstack((np.zeros([1, 3]), np.ones([1, 1])))))
    B = trs.shape[0]
    if trs.dim() == 3:
        trs = trs.reshape(B, 3)
    top = torch.cat((rot, trs.unsqueeze(2)), dim=2)
    bot = torch.cat((torch.zeros(B, 1, 3), torch.ones(B, 1, 1)), 2).to(top.device)
    return torch.cat((top, bot), dim=1)
