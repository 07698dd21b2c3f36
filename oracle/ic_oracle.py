"""CPU ORACLE for the trust-region inverse-compositional (U_IC) solver path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the
`deep_prob_feature_track_amd` package, `libdpft_ic.so`) may import, call or
link this module.  It is used as the checker by `tests/`, by
`__graft_entry__.smoke()` and as the `cpu_baseline` leg of `bench.py`.

This is a from-scratch restatement, on PyTorch-CPU tensors (fp32 or fp64), of
the reference's per-level solver `TrustRegionInverseWUncertainty`
(`code/models/algorithms.py:579-997`) and the helpers it calls.  Each function
cites the reference lines it follows.  It is pinned against the golden
fixtures produced by running the reference itself
(`tests/golden/gen_golden.py`, checked in `tests/test_oracle_golden.py`).

Tensor conventions (as in the reference): features / sigma [B,C,H,W],
inverse depth [B,1,H,W], K [B,4] = (fx, fy, cx, cy) already divided by 2^l,
pose = (R [B,3,3], t [B,3,1]).
"""
import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------- geometry
def pixel_rays(B, H, W, K):
    """x = (u - cx) / fx, y = (v - cy) / fy.  geometry.py:63-85 (meshgrid 37-61)."""
    fx, fy, cx, cy = (K[:, i].view(B, 1) for i in range(4))
    u = torch.arange(W, dtype=K.dtype).repeat(H).view(1, H * W)
    v = torch.arange(H, dtype=K.dtype).repeat_interleave(W).view(1, H * W)
    return ((u - cx) / fx).view(B, 1, H, W), ((v - cy) / fy).view(B, 1, H, W)


def warp_inverse_depth(x, y, invD0, R, t, K):
    """Rigid warp through inverse depth.  geometry.py:291-323.

    [X,Y,Z] = R [x,y,1]^T + t * invD0 ; u = X/Z fx + cx ; v = Y/Z fy + cy ; iz = invD0 / Z
    """
    B, _, H, W = x.shape
    ray = torch.cat((x, y, torch.ones_like(x)), 1).view(B, 3, H * W)
    P = torch.bmm(R, ray) + t.view(B, 3, 1) * invD0.view(B, 1, H * W)
    X, Y, Z = P[:, 0], P[:, 1], P[:, 2]
    u = (X / Z) * K[:, 0:1] + K[:, 2:3]
    v = (Y / Z) * K[:, 1:2] + K[:, 3:4]
    return u.view(B, 1, H, W), v.view(B, 1, H, W), invD0 / Z.view(B, 1, H, W)


def bilinear(F_, u, v):
    """Bilinear sample with border clamp, align_corners=True.  geometry.py:353-365."""
    B, C, H, W = F_.shape
    gu = u / ((W - 1) / 2) - 1
    gv = v / ((H - 1) / 2) - 1
    grid = torch.cat((gu.view(B, H, W, 1), gv.view(B, H, W, 1)), 3)
    return F.grid_sample(F_, grid, mode="bilinear", padding_mode="border", align_corners=True)


def occlusion(iz, invD1, u, v, thres=0.1):
    """z-buffer + in-view test; returns True where INVALID.  geometry.py:334-350."""
    _, _, H, W = iz.shape
    d1w = bilinear(invD1, u, v)
    ok = (iz > d1w - thres) & (u > 0) & (u < W) & (v > 0) & (v < H)
    return ~ok


def so3_exp(w):
    """Rodrigues, NaN at |w| = 0 like the reference.  geometry.py:146-185."""
    B = w.shape[0]
    th = w.norm(dim=1).view(B, 1)
    k = w / th
    z = torch.zeros(B, dtype=w.dtype)
    Kx = torch.stack((z, -k[:, 2], k[:, 1], k[:, 2], z, -k[:, 0], -k[:, 1], k[:, 0], z), 1).view(B, 3, 3)
    I = torch.eye(3, dtype=w.dtype).expand(B, 3, 3)
    return I + Kx * torch.sin(th).view(B, 1, 1) + torch.bmm(Kx, Kx) * (1 - torch.cos(th)).view(B, 1, 1)


# --------------------------------------------------------------------------- jacobians
def sobel(img, normalize=True):
    """3x3 Sobel (+-1, +-2) with replicate padding, unit-normalised.  algorithms.py:1844-1865."""
    B, C, H, W = img.shape
    kx = torch.tensor([[-1.0, 0.0, 1.0], [-2.0, 0.0, 2.0], [-1.0, 0.0, 1.0]], dtype=img.dtype)
    p = F.pad(img.reshape(B * C, 1, H, W), (1, 1, 1, 1), mode="replicate")
    gx = F.conv2d(p, kx.view(1, 1, 3, 3))
    gy = F.conv2d(p, kx.t().contiguous().view(1, 1, 3, 3))
    if normalize:
        mag = torch.sqrt(gx * gx + gy * gy + 1e-8)
        gx, gy = gx / mag, gy / mag
    return gx.view(B, C, H, W), gy.view(B, C, H, W)


def warp_jacobian(invD0, K, x, y):
    """d(u,v)/d xi at the origin, xi = [rot, trs].  algorithms.py:1884-1917."""
    B, _, H, W = invD0.shape
    x, y, d = x.reshape(B, -1, 1), y.reshape(B, -1, 1), invD0.reshape(B, -1, 1)
    o = torch.zeros_like(x)
    Jx = torch.cat((-x * y, 1 + x * x, -y, d, o, -d * x), 2) * K[:, 0].view(B, 1, 1)
    Jy = torch.cat((-1 - y * y, x * y, x, o, d, -d * y), 2) * K[:, 1].view(B, 1, 1)
    return Jx, Jy  # [B, HW, 6]


# --------------------------------------------------------------------------- residuals
def residuals(R, t, invD0, invD1, f0, f1, s0, s1, x, y, K, mask0=None, mask1=None, remove_tru_sigma=False):
    """Warped, uncertainty-normalised residuals and the invalid mask.

    algorithms.py:1992-2015 (compute_inverse_residuals) + 1960-1989 (compose_residuals).
    Returns (rw [B,C,H,W] with invalid pixels = 1e-6, r, sigma, invalid [B,1,H,W]).
    """
    B, C, H, W = f0.shape
    u, v, iz = warp_inverse_depth(x, y, invD0, R, t, K)
    invalid = occlusion(iz, invD1, u, v)
    if mask0 is not None:                                                  # 2000-2002
        invalid = invalid | ~mask0.view(B, 1, H, W)
    if mask1 is not None:                                                  # 2003-2008
        invalid = invalid | ~(bilinear(mask1.to(f0.dtype), u, v) > 0).view(B, 1, H, W)
    fr = bilinear(f1, u, v)
    sr = bilinear(s1, u, v)
    r = fr - f0
    sigma = torch.sqrt(sr * sr + s0 * s0)
    rw = r / sigma
    if remove_tru_sigma:                                                   # 1975-1980
        tru = (sr == sr.min()) | (sr == sr.max()) | (s0 == s0.min()) | (s0 == s0.max())
        invalid = invalid | tru[:, 0:1]
    rw = torch.where(invalid, torch.full_like(rw[:1], 1e-6), rw)          # 1982-1983
    return rw, r, sigma, invalid


def inverse_jacobian(r, sigma, s0, gf0, gs0, Jx, Jy):
    """Per-channel IC Jacobian, NOT masked.  algorithms.py:867-887 + 1867-1882.

    a = -gx/s - r s0 hx / s^3 ; J = -(a Jx + b Jy)  -> [B, C, HW, 6]
    """
    B, C, H, W = r.shape
    a = -gf0[0] / sigma - r * (s0 * gs0[0] / sigma ** 3)
    b = -gf0[1] / sigma - r * (s0 * gs0[1] / sigma ** 3)
    J = a.view(B, C, -1, 1) * Jx.view(B, 1, -1, 6) + b.view(B, C, -1, 1) * Jy.view(B, 1, -1, 6)
    return -J


def normal_equations(J, rw):
    """JtJ [B,6,6], JtR [B,6,1] summed over channels and pixels.  algorithms.py:812-834."""
    B = J.shape[0]
    Jf = J.reshape(B, -1, 6)
    return torch.bmm(Jf.transpose(1, 2), Jf), torch.bmm(Jf.transpose(1, 2), rw.reshape(B, -1, 1))


# --------------------------------------------------------------------------- IC tracker (no uncertainty)
def ic_residuals(R, t, invD0, invD1, f0, f1, x, y, K, mask0=None, mask1=None):
    """compute_warped_residual, algorithms.py:1919-1957: r = f1(warp) - f0, 1e-3 where
    occluded / masked.  Returns (r [B,C,H,W], occ [B,1,H,W])."""
    B, C, H, W = f0.shape
    u, v, iz = warp_inverse_depth(x, y, invD0, R, t, K)
    occ = occlusion(iz, invD1, u, v)
    if mask0 is not None:
        occ = occ | ~mask0.view(B, 1, H, W)
    if mask1 is not None:
        occ = occ | ~(bilinear(mask1.to(f0.dtype), u, v) > 0).view(B, 1, H, W)
    r = bilinear(f1, u, v) - f0
    return torch.where(occ.expand(B, C, H, W), torch.full_like(r, 1e-3), r), occ


def ic_jacobian(invD0, f0, x, y, K):
    """precompute_Jacobian, algorithms.py:103-121: J = gx Jx + gy Jy per channel
    (compute_jacobian_dIdp 1867-1882) -> [B, C*HW, 6]."""
    B, C, H, W = f0.shape
    gx, gy = sobel(f0)
    Jx, Jy = warp_jacobian(invD0, K, x, y)
    J = gx.view(B, C, -1, 1) * Jx.view(B, 1, -1, 6) + gy.view(B, C, -1, 1) * Jy.view(B, 1, -1, 6)
    return J.view(B, -1, 6)


def ic_normal_equations(J, r, weights=None):
    """JtWJ = J^T (w J) (algorithms.py:71-76), JtR = J^T (w r) (DirectSolverNet 1631-1632);
    weights [B,1,H,W] (one per pixel, C = 1) or None (unit)."""
    B = J.shape[0]
    w = torch.ones_like(r) if weights is None else weights.expand_as(r)
    wJ = w.reshape(B, -1, 1) * J
    return torch.bmm(J.transpose(1, 2), wJ), torch.bmm(J.transpose(1, 2), (w * r).reshape(B, -1, 1))


# --------------------------------------------------------------------------- ICP term
def vertex_map(depth, x, y):
    """[x,y,1] * depth.  geometry.py:1129-1136."""
    return torch.cat((x, y, torch.ones_like(x)), 1) * depth


def normal_map(V):
    """Normalised cross of unnormalised Sobel derivatives; zero where depth is the
    batch-global min or max.  algorithms.py:2148-2172."""
    B, C, H, W = V.shape
    dx, dy = sobel(V, normalize=False)
    n = torch.linalg.cross(dx.view(B, 3, -1).permute(0, 2, 1), dy.view(B, 3, -1).permute(0, 2, 1), dim=2)
    n = n.permute(0, 2, 1)
    n = n / (n.norm(dim=1, keepdim=True) + 1e-8)
    z = V[:, 2:3]
    bad = ((z == z.min()) | (z == z.max())).view(B, 1, -1)
    n = torch.where(bad.expand(B, 3, H * W), torch.zeros_like(n), n)
    return n.view(B, 3, H, W)


def icp_terms(V0, V1, N1, R, t, K, mask0=None, mask1=None):
    """Point-to-plane residual + Jacobian.  algorithms.py:916-997."""
    B, _, H, W = V0.shape
    P = torch.bmm(R, V0.view(B, 3, -1)) + t.view(B, 3, 1)
    u = (P[:, 0] / P[:, 2]) * K[:, 0:1] + K[:, 2:3]
    v = (P[:, 1] / P[:, 2]) * K[:, 1:2] + K[:, 3:4]
    inview = (u > 0) & (u < W - 1) & (v > 0) & (v < H - 1)
    uu, vv = u.view(B, 1, H, W), v.view(B, 1, H, W)
    V1w = bilinear(V1, uu, vv).view(B, 3, -1)
    N1w = bilinear(N1, uu, vv).view(B, 3, -1)
    diff = P - V1w
    occ = ~inview.view(B, 1, H, W) | (diff.view(B, 3, H, W).norm(dim=1, keepdim=True) > 0.1)
    if mask0 is not None:
        occ = occ | ~mask0.view(B, 1, H, W)
    if mask1 is not None:
        occ = occ | ~(bilinear(mask1.to(V0.dtype), uu, vv) > 0).view(B, 1, H, W)
    r = (N1w * diff).sum(1).view(B, 1, H, W)
    n = torch.bmm(N1w.permute(0, 2, 1), R)                              # [B, HW, 3]
    p = V0.view(B, 3, -1).permute(0, 2, 1)                              # [B, HW, 3]
    Jrot = torch.linalg.cross(n, p, dim=2)                              # n^T [p]_x  ==  n x p
    J = torch.cat((Jrot, -n), 2).view(B, 1, -1, 6)
    # stereo-model sigma, hard-coded TUM constants (975-997)
    z = V0[:, 2:3].reshape(B, 1, -1)
    sxy = z / 525.0 * 5.5
    sz = z * z * 0.4 / (525.0 * 1.2)
    cov = (n[:, :, 0:1].transpose(1, 2) * sxy) ** 2 + (n[:, :, 1:2].transpose(1, 2) * sxy) ** 2 \
        + (n[:, :, 2:3].transpose(1, 2) * sz) ** 2
    sig = torch.sqrt(cov + 1e-8).view(B, 1, H, W)
    r = r / (sig + 1e-8)
    J = -(J / (sig.view(B, 1, -1, 1) + 1e-8))
    r = torch.where(occ, torch.full_like(r, 1e-6), r)
    return r, J, occ


# --------------------------------------------------------------------------- solver
def damped_solve_update(JtJ, JtR, R, t):
    """H = JtJ + 1e-6 tr(JtJ) I ; xi = H^-1 JtR ; R <- R Exp(-w) ; t <- R (-Exp(-w) v) + t.

    algorithms.py:2094-2103 (lev_mar_H), 2017-2054 (least_square_solve,
    inverse_update_pose), geometry.py:105-123 (compose, argument order of 2053).
    """
    B = JtJ.shape[0]
    tr = torch.diagonal(JtJ, dim1=1, dim2=2).sum(1)
    H = JtJ + (tr * 1e-6).view(B, 1, 1) * torch.eye(6, dtype=JtJ.dtype)
    xi = torch.bmm(torch.linalg.inv(H), JtR)
    dR = so3_exp(-xi[:, :3].view(B, 3))
    dt = -torch.bmm(dR, xi[:, 3:])
    return torch.bmm(R, dR), torch.bmm(R, dt) + t.view(B, 3, 1), xi.view(B, 6)


def solve_level(R, t, f0, f1, s0, s1, invD0, invD1, K, iters=3, remove_tru_sigma=False,
                mask0=None, mask1=None, depth0=None, depth1=None, icp_scale=None, trace=None):
    """One pyramid level: exactly `iters` GN iterations, no early exit.

    algorithms.py:611-723.  s0/s1 may have 1 channel (broadcast to C, as the
    reference's `.repeat`, algorithms.py:1426-1427).  `icp_scale` not None
    enables the combined ICP term with constant weight (ScaleNet 'None' =
    0.01, algorithms.py:1535,1563-1567).
    """
    B, C, H, W = f0.shape
    s0 = s0.expand(B, C, H, W)
    s1 = s1.expand(B, C, H, W)
    x, y = pixel_rays(B, H, W, K)
    gf0 = sobel(f0)
    gs0 = sobel(s0)
    Jx, Jy = warp_jacobian(invD0, K, x, y)
    if icp_scale is not None:
        V0 = vertex_map(depth0, x, y)
        V1 = vertex_map(depth1, x, y)
        N1 = normal_map(V1)
    t = t.view(B, 3, 1)
    for _ in range(iters):
        rw, r, sigma, invalid = residuals(R, t, invD0, invD1, f0, f1, s0, s1, x, y, K,
                                          mask0, mask1, remove_tru_sigma)
        if torch.isnan(rw).any() or torch.isinf(rw).any():
            raise AssertionError("non-finite weighted residual")            # algorithms.py:1988
        J = inverse_jacobian(r, sigma, s0, gf0, gs0, Jx, Jy)
        JtJ, JtR = normal_equations(J, rw)
        if icp_scale is not None:
            ri, Ji, _ = icp_terms(V0, V1, N1, R, t, K, mask0, mask1)
            ri, Ji = icp_scale * ri, icp_scale * Ji
            JtJ = JtJ + torch.bmm(Ji.view(B, -1, 6).transpose(1, 2), Ji.view(B, -1, 6))
            JtR = JtR + torch.bmm(Ji.view(B, -1, 6).transpose(1, 2), ri.view(B, -1, 1))
        R, t, xi = damped_solve_update(JtJ, JtR, R, t)
        if trace is not None:
            trace.append(dict(JtJ=JtJ, JtR=JtR.view(B, 6), R=R, t=t.view(B, 3), xi=xi,
                              invalid=invalid.view(B, -1).sum(1)))
    return R, t.view(B, 3)


def residual_loss(R, t, f0, f1, s0, s1, invD0, invD1, K, remove_tru_sigma=False,
                  mask0=None, mask1=None, depth0=None, depth1=None, icp_scale=None):
    """Per-pair average loss at a fixed pose.  algorithms.py:725-786 + 2119-2137."""
    B, C, H, W = f0.shape
    s0 = s0.expand(B, C, H, W)
    s1 = s1.expand(B, C, H, W)
    x, y = pixel_rays(B, H, W, K)
    t = t.view(B, 3, 1)
    rw, _, _, invalid = residuals(R, t, invD0, invD1, f0, f1, s0, s1, x, y, K, mask0, mask1, remove_tru_sigma)
    terms = [rw]
    if icp_scale is not None:
        V0 = vertex_map(depth0, x, y)
        V1 = vertex_map(depth1, x, y)
        ri, _, occ_i = icp_terms(V0, V1, normal_map(V1), R, t, K)
        terms.append(icp_scale * ri)
        invalid = invalid | occ_i
    total = torch.zeros(B, 1, H, W, dtype=f0.dtype)
    for a in terms:
        total = total + (torch.where(invalid, torch.zeros_like(a), a) ** 2).sum(1, keepdim=True)
    nvalid = H * W - invalid.view(B, -1).sum(1)
    return total.view(B, -1).sum(1) / nvalid


def solve_pyramid(R, t, levels, K, iters=3, remove_tru_sigma=False, combine_icp=False, trace=None):
    """Coarse-to-fine driver over levels L-1 .. 0 with K / 2^l.  LeastSquareTracking.py:345-445.

    `levels[l]` is a dict with f0, f1, s0, s1, invD0, invD1 and optionally
    mask0, mask1, depth0, depth1.
    """
    for l in reversed(range(len(levels))):
        d = levels[l]
        R, t = solve_level(R, t, d["f0"], d["f1"], d["s0"], d["s1"], d["invD0"], d["invD1"], K / (2 ** l),
                           iters=iters, remove_tru_sigma=remove_tru_sigma,
                           mask0=d.get("mask0"), mask1=d.get("mask1"),
                           depth0=d.get("depth0"), depth1=d.get("depth1"),
                           icp_scale=0.01 if combine_icp else None, trace=trace)
    return R, t
