"""PyTorch path of the per-level solvers: CPU tensors and autograd (SURVEY.md 8(b) dispatch).

libdpft_ic.so serves device tensors at inference.  This module serves what the library
cannot: (1) CPU tensors -- the reference's callers run on the host when no GPU is present
(train_utils.check_cuda leaves the batch on the CPU, run_example.py:102-103); (2) calls with
gradients -- grad enabled and an input that requires grad (the reference's training path,
autograd through the unrolled solver; the library has no backward kernels).  It is never a
fallback for device tensors at inference: those run on the library or raise.

The math restates the reference's per-level solvers in torch ops, on the caller's device and
dtype, differentiable end to end:
  U_IC (TrustRegionInverseWUncertainty, algorithms.py:611-786): warp (geometry.py:291-323),
  occlusion / masks / truncated sigma (1960-2015), the inverse-compositional Jacobian
  (867-887) in the regrouped form the fused kernel uses -- per pixel the channel sums
  Saa, Sab, Sbb, Sar, Sbr, so J [B,C,HW,6] is never formed (SURVEY.md 8(a) kernel spec) --,
  the ICP term (916-997, 2148-2172), lev_mar_H + inverse_update_pose (2017-2103), and the
  residual loss (725-786, 2119-2137);
  IC (TrustRegionBase, algorithms.py:23-139): the template Jacobian (103-121), the warped
  residual (1919-1957), M-estimator weights, 'Direct-Nodamping' and the 'Direct-ResVol'
  residual volume (1583-1691).
The 6x6 systems are solved in fp64 (as the library does; the reference inverts in fp32 on
the host, 2077-2091).  Pinned against the reference's own goldens by tests/test_torch_path.py.
"""
import torch
import torch.nn.functional as func

from . import geometry


def needs_torch_path(*tensors):
    """the PyTorch path takes CPU tensors, and calls with grad enabled where an
    input requires grad; device tensors at inference go to libdpft_ic.so."""
    ts = [t for t in tensors if isinstance(t, torch.Tensor)]
    on_dev = [t.is_cuda for t in ts]
    if any(on_dev) and not all(on_dev):
        raise ValueError("the solver's tensors span devices (%s); move them to one device first"
                         % ", ".join(sorted({str(t.device) for t in ts})))
    if not on_dev[0]:
        return True
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


def nchw(x):
    """Features as [B,C,H,W] (a channel-quad packed [B,C/4,H,W,4] map is unpacked)."""
    if x.dim() == 5:
        B, Q, H, W, _ = x.shape
        return x.permute(0, 1, 4, 2, 3).reshape(B, 4 * Q, H, W)
    return x


# ------------------------------------------------------------------ geometry
def pixel_grid(B, H, W, K):
    """Normalised pixel coordinates (x - cx) / fx, (y - cy) / fy, [B,1,H,W] each
    (generate_xy_grid, geometry.py:63-85)."""
    xs = torch.arange(W, device=K.device, dtype=K.dtype).view(1, 1, 1, W)
    ys = torch.arange(H, device=K.device, dtype=K.dtype).view(1, 1, H, 1)
    fx, fy, cx, cy = (K[:, i].reshape(B, 1, 1, 1) for i in range(4))
    return ((xs - cx) / fx).expand(B, 1, H, W), ((ys - cy) / fy).expand(B, 1, H, W)


def warp(px, py, invD0, R, t, K):
    """u, v, inverse depth of the warped template pixels (batch_warp_inverse_depth,
    geometry.py:291-323): X = R [x, y, 1] + t invD0."""
    B, _, H, W = px.shape
    ray = torch.cat((px, py, torch.ones_like(px)), 1).reshape(B, 3, H * W)
    P = torch.bmm(R, ray) + t.reshape(B, 3, 1) * invD0.reshape(B, 1, H * W)
    Z = P[:, 2]
    u = (P[:, 0] / Z) * K[:, 0:1] + K[:, 2:3]
    v = (P[:, 1] / Z) * K[:, 1:2] + K[:, 3:4]
    return u.view(B, 1, H, W), v.view(B, 1, H, W), (invD0.reshape(B, H * W) / Z).view(B, 1, H, W)


def sample(F, u, v):
    """Bilinear lookup at pixel coordinates, border clamp, align_corners (warp_features,
    geometry.py:353-365)."""
    B, C, H, W = F.shape
    grid = torch.stack((u.reshape(B, H, W) / ((W - 1) / 2) - 1, v.reshape(B, H, W) / ((H - 1) / 2) - 1), 3)
    return func.grid_sample(F, grid, mode='bilinear', padding_mode='border', align_corners=True)


def sobel(f, unit=True):
    """3x3 Sobel (+-1, +-2, replicate padding), unit-normalised g / sqrt(gx^2 + gy^2 + 1e-8)
    (feature_gradient, algorithms.py:1844-1865)."""
    B, C, H, W = f.shape
    k = torch.tensor([[-1.0, 0.0, 1.0], [-2.0, 0.0, 2.0], [-1.0, 0.0, 1.0]], dtype=f.dtype, device=f.device)
    p = func.pad(f.reshape(B * C, 1, H, W), (1, 1, 1, 1), mode='replicate')
    gx = func.conv2d(p, k.view(1, 1, 3, 3)).view(B, C, H, W)
    gy = func.conv2d(p, k.t().reshape(1, 1, 3, 3)).view(B, C, H, W)
    if unit:
        n = torch.sqrt(gx * gx + gy * gy + 1e-8)
        gx, gy = gx / n, gy / n
    return gx, gy


def warp_jacobian(px, py, invD0, K):
    """d(u, v) / d xi at the origin, xi = [rotation, translation], [B,HW,6] each
    (compute_jacobian_warping, algorithms.py:1884-1917)."""
    B = px.shape[0]
    x, y, d = px.reshape(B, -1, 1), py.reshape(B, -1, 1), invD0.reshape(B, -1, 1)
    o = torch.zeros_like(x)
    Jx = torch.cat((-x * y, 1 + x * x, -y, d, o, -d * x), 2) * K[:, 0].view(B, 1, 1)
    Jy = torch.cat((-1 - y * y, x * y, x, o, d, -d * y), 2) * K[:, 1].view(B, 1, 1)
    return Jx, Jy


def _check_finite(x, what):
    if not torch.isfinite(x).all():
        raise AssertionError(f"non-finite {what} (reference: assert check_nan(...) == 0)")


# ------------------------------------------------------------------ pose update
def damped_update(JtJ, JtR, pose, diag_add=None):
    """H = JtJ + diag(diag_add) + 1e-6 tr(JtJ) I ; xi = H^-1 JtR (fp64) ; R <- R Exp(-w),
    t <- R (-Exp(-w) v) + t (lev_mar_H 2094-2103, inverse_update_pose 2017-2054, the
    Direct-ResVol Hessian 1683-1691).  JtJ [B,6,6], JtR [B,6(,1)], diag_add [B,6] or None."""
    R, t = pose
    B = JtJ.shape[0]
    J64 = JtJ.double()
    eye = torch.eye(6, dtype=torch.float64, device=JtJ.device)
    H = J64 + (torch.diagonal(J64, dim1=1, dim2=2).sum(1) * 1e-6).view(B, 1, 1) * eye
    if diag_add is not None:
        H = H + torch.diag_embed(diag_add.double())
    xi = torch.linalg.solve(H, JtR.double().reshape(B, 6, 1)).view(B, 6)
    w = -xi[:, :3]
    th = torch.sqrt((w * w).sum(1, keepdim=True))
    k = w / th  # Rodrigues; NaN at |w| = 0 as in batch_twist2Mat (geometry.py:163-185)
    z = torch.zeros_like(k[:, 0])
    Kx = torch.stack((z, -k[:, 2], k[:, 1], k[:, 2], z, -k[:, 0], -k[:, 1], k[:, 0], z), 1).view(B, 3, 3)
    dR = torch.eye(3, dtype=torch.float64, device=JtJ.device) + torch.sin(th).view(B, 1, 1) * Kx \
        + (1 - torch.cos(th)).view(B, 1, 1) * torch.bmm(Kx, Kx)
    dt = -torch.bmm(dR, xi[:, 3:].reshape(B, 3, 1))
    R1, t1 = geometry.batch_Rt_compose(R.double(), t.double().reshape(B, 3, 1), dR, dt)
    return [R1.to(R.dtype), t1.to(t.dtype).view(B, 3)]  # t [B,3]: batch_Rt_compose's t1.view(-1,3) (geometry.py:122)


# ------------------------------------------------------------------ U_IC
class UICLevel:
    """One U_IC level's pose-independent terms (precompute_jacobian_components,
    algorithms.py:848-865, + the ICP vertex / normal maps, 628-635)."""

    def __init__(self, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0=None, depth1=None, obj_mask0=None,
                 obj_mask1=None, remove_tru_sigma=False, icp_scale=None):
        x0, x1 = nchw(x0), nchw(x1)
        B, C, H, W = x0.shape
        self.B, self.C, self.H, self.W = B, C, H, W
        self.x0, self.x1, self.invD0, self.invD1, self.K = x0, x1, invD0, invD1, K.reshape(B, 4)
        self.s0, self.s1 = sigma0.expand(B, -1, H, W), sigma1.expand(B, -1, H, W)
        self.m0, self.m1 = obj_mask0, obj_mask1
        self.tru = remove_tru_sigma
        self.px, self.py = pixel_grid(B, H, W, self.K)
        self.gx, self.gy = sobel(x0)
        # sigma0's gradient: one plane when sigma is a channel broadcast of one (Cs = 1)
        s0 = self.s0[:, :1] if self.s0.shape[1] == 1 or self.s0.stride(1) == 0 else self.s0
        self.hx, self.hy = sobel(s0)
        self.Jx, self.Jy = warp_jacobian(self.px, self.py, invD0, self.K)
        self.icp_scale = icp_scale
        if icp_scale is not None:
            self.V0 = torch.cat((self.px, self.py, torch.ones_like(self.px)), 1) * depth0
            V1 = torch.cat((self.px, self.py, torch.ones_like(self.px)), 1) * depth1
            dx, dy = sobel(V1, unit=False)
            n = torch.linalg.cross(dx, dy, dim=1)
            n = n / (torch.linalg.norm(n, dim=1, keepdim=True) + 1e-8)
            z = V1[:, 2:3]
            self.N1 = torch.where((z == z.min()) | (z == z.max()), torch.zeros_like(n), n)
            self.V1 = V1

    def residuals(self, pose):
        """(rw [B,C,H,W] with 1e-6 on invalid pixels, r, sigma, invalid [B,1,H,W])
        (compute_inverse_residuals 1992-2015, compose_residuals 1960-1989)."""
        R, t = pose
        B, C, H, W = self.B, self.C, self.H, self.W
        u, v, iz = warp(self.px, self.py, self.invD0, R, t, self.K)
        d1w = sample(self.invD1, u, v)
        invalid = ~((iz > d1w - 0.1) & (u > 0) & (u < W) & (v > 0) & (v < H))
        if self.m0 is not None:
            invalid = invalid | ~self.m0.reshape(B, 1, H, W).bool()
        if self.m1 is not None:
            invalid = invalid | ~(sample(self.m1.reshape(B, 1, H, W).to(self.x0.dtype), u, v) > 0)
        fr = sample(self.x1, u, v)
        sr = sample(self.s1, u, v)
        r = fr - self.x0
        s0 = self.s0
        sigma = torch.sqrt(sr * sr + s0 * s0)
        rw = r / sigma
        if self.tru:  # batch-global extrema of sigma_r and sigma0 (algorithms.py:1975-1980)
            m = (sr == sr.min()) | (sr == sr.max()) | (s0 == s0.min()) | (s0 == s0.max())
            invalid = invalid | m[:, 0:1]
        rw = torch.where(invalid, torch.full_like(rw, 1e-6), rw)
        _check_finite(rw, "weighted residual")
        return rw, r, sigma, invalid

    def normal_equations(self, pose):
        """JtJ [B,6,6], JtR [B,6,1], #invalid [B] at `pose`: per pixel a_c = -gx/s -
        r s0 hx / s^3 (b_c likewise), J_c = -(a_c Jx + b_c Jy) is never formed --
        sum_c J_c J_c^T = Saa JxJx^T + Sab (JxJy^T + JyJx^T) + Sbb JyJy^T and
        sum_c J_c rw_c = -(Sar Jx + Sbr Jy) (compose_inverse_jacobians 867-887, compute_jtj /
        compute_jtr 812-834); + the weighted ICP term (668-689)."""
        B = self.B
        rw, r, sigma, invalid = self.residuals(pose)
        k = r * self.s0 / sigma ** 3
        a = -(self.gx / sigma + k * self.hx)
        b = -(self.gy / sigma + k * self.hy)
        _check_finite(a, "Jacobian")
        _check_finite(b, "Jacobian")
        S = lambda p, q: (p * q).sum(1).reshape(B, 1, -1)  # noqa: E731
        Saa, Sab, Sbb, Sar, Sbr = S(a, a), S(a, b), S(b, b), S(a, rw), S(b, rw)
        Jx, Jy = self.Jx.transpose(1, 2), self.Jy.transpose(1, 2)  # [B,6,HW]
        JtJ = torch.bmm(Saa * Jx, self.Jx) + torch.bmm(Sbb * Jy, self.Jy)
        cross = torch.bmm(Sab * Jx, self.Jy)
        JtJ = JtJ + cross + cross.transpose(1, 2)
        JtR = -(torch.bmm(Jx, Sar.transpose(1, 2)) + torch.bmm(Jy, Sbr.transpose(1, 2)))
        if self.icp_scale is not None:
            ri, Ji, _ = self.icp_terms(pose)
            Ji = self.icp_scale * Ji.reshape(B, -1, 6)
            JtJ = JtJ + torch.bmm(Ji.transpose(1, 2), Ji)
            JtR = JtR + torch.bmm(Ji.transpose(1, 2), (self.icp_scale * ri).reshape(B, -1, 1))
        return JtJ, JtR, invalid.reshape(B, -1).sum(1)

    def icp_terms(self, pose, masks=True):
        """Point-to-plane residual r [B,1,H,W], Jacobian J [B,HW,6] (both divided by the
        stereo-model sigma, J negated, r = 1e-6 where occluded) and the occlusion map
        (compute_ICP_residuals_jacobian 916-973, compute_icp_sigma 975-997).  The object
        masks join the occlusion in the solve (670-675), not in forward_residuals (765)."""
        R, t = pose
        B, H, W = self.B, self.H, self.W
        P = torch.bmm(R, self.V0.reshape(B, 3, -1)) + t.reshape(B, 3, 1)
        u = (P[:, 0] / P[:, 2]) * self.K[:, 0:1] + self.K[:, 2:3]
        v = (P[:, 1] / P[:, 2]) * self.K[:, 1:2] + self.K[:, 3:4]
        inview = (u > 0) & (u < W - 1) & (v > 0) & (v < H - 1)
        uu, vv = u.view(B, 1, H, W), v.view(B, 1, H, W)
        V1w = sample(self.V1, uu, vv).reshape(B, 3, -1)
        N1w = sample(self.N1, uu, vv).reshape(B, 3, -1)
        diff = P - V1w
        occ = ~inview.view(B, 1, H, W) | (torch.linalg.norm(diff, dim=1).view(B, 1, H, W) > 0.1)
        if masks and self.m0 is not None:
            occ = occ | ~self.m0.reshape(B, 1, H, W).bool()
        if masks and self.m1 is not None:
            occ = occ | ~(sample(self.m1.reshape(B, 1, H, W).to(self.x0.dtype), uu, vv) > 0)
        r = (N1w * diff).sum(1).view(B, 1, H, W)
        n = torch.bmm(N1w.transpose(1, 2), R)                       # n^T R, [B,HW,3]
        J = torch.cat((torch.linalg.cross(n, self.V0.reshape(B, 3, -1).transpose(1, 2), dim=2), -n), 2)
        z = self.V0[:, 2].reshape(B, -1, 1)
        sxy, sz = z / 525.0 * 5.5, z * z * 0.4 / (525.0 * 1.2)
        sig = torch.sqrt((n[:, :, 0:1] * sxy) ** 2 + (n[:, :, 1:2] * sxy) ** 2 + (n[:, :, 2:3] * sz) ** 2 + 1e-8)
        r = r / (sig.view(B, 1, H, W) + 1e-8)
        J = -(J / (sig + 1e-8))
        return torch.where(occ, torch.full_like(r, 1e-6), r), J, occ

    def loss(self, pose):
        """forward_residuals' per-pair loss [B] (algorithms.py:725-786, compute_avg_loss
        2119-2137): sum over valid pixels of the squared weighted residuals (+ the weighted ICP
        residual, its occlusion joining the invalid set) / #valid."""
        B, H, W = self.B, self.H, self.W
        rw, _, _, invalid = self.residuals(pose)
        terms = [rw]
        if self.icp_scale is not None:
            ri, _, occ = self.icp_terms(pose, masks=False)
            terms.append(self.icp_scale * ri)
            invalid = invalid | occ
        total = sum((torch.where(invalid, torch.zeros_like(a), a) ** 2).reshape(B, -1).sum(1) for a in terms)
        return total / (H * W - invalid.reshape(B, -1).sum(1)).to(total.dtype)


def uic_solve(pose, level, iters, want_jtj=False):
    """`iters` Gauss-Newton steps (algorithms.py:646-710: no early exit) -> (pose, JtJ of the
    last step or None)."""
    JtJ = None
    for _ in range(iters):
        JtJ, JtR, _ = level.normal_equations(pose)
        pose = damped_update(JtJ, JtR, pose)
    return pose, (JtJ if want_jtj else None)


# ------------------------------------------------------------------ IC (TrustRegionBase)
def ic_residual(pose, x0, x1, invD0, invD1, K, px, py, obj_mask0=None, obj_mask1=None):
    """r = f1(warp) - f0 with 1e-3 where occluded / masked, occ [B,1,H,W]
    (compute_warped_residual, algorithms.py:1919-1957)."""
    R, t = pose
    B, C, H, W = x0.shape
    u, v, iz = warp(px, py, invD0, R, t, K)
    occ = ~((iz > sample(invD1, u, v) - 0.1) & (u > 0) & (u < W) & (v > 0) & (v < H))
    if obj_mask0 is not None:
        occ = occ | ~obj_mask0.reshape(B, 1, H, W).bool()
    if obj_mask1 is not None:
        occ = occ | ~(sample(obj_mask1.reshape(B, 1, H, W).to(x0.dtype), u, v) > 0)
    r = sample(x1, u, v) - x0
    return torch.where(occ.expand(B, C, H, W), torch.full_like(r, 1e-3), r), occ


def ic_template_jacobian(invD0, x0, px, py, K):
    """J = gx Jx + gy Jy per channel and pixel, [B,C*HW,6] (precompute_Jacobian 103-121,
    compute_jacobian_dIdp 1867-1882)."""
    B, C, H, W = x0.shape
    gx, gy = sobel(x0)
    Jx, Jy = warp_jacobian(px, py, invD0, K)
    return (gx.reshape(B, C, -1, 1) * Jx.view(B, 1, -1, 6) + gy.reshape(B, C, -1, 1) * Jy.view(B, 1, -1, 6)).view(B, -1, 6)


def ic_forward(tracker, pose, x0, x1, invD0, invD1, K, wPrior=None, obj_mask0=None, obj_mask1=None):
    """TrustRegionBase.forward (algorithms.py:44-101) -> (pose, weights)."""
    x0, x1 = nchw(x0), nchw(x1)
    B, C, H, W = x0.shape
    K = K.reshape(B, 4)
    px, py = pixel_grid(B, H, W, K)
    J = ic_template_jacobian(invD0, x0, px, py, K)
    res, _ = ic_residual(pose, x0, x1, invD0, invD1, K, px, py, obj_mask0, obj_mask1)
    weights = tracker.mEstimator(res, x0, x1, wPrior)
    Jt = J.transpose(1, 2)
    JtWJ = torch.bmm(Jt, weights.reshape(B, -1, 1) * J)
    for _ in range(tracker.max_iterations):
        JtR = torch.bmm(Jt, (weights * res).reshape(B, -1, 1))
        solver = tracker.directSolver
        if getattr(solver, 'type', 0) == solver.SOLVER_RESIDUAL_VOLUME:
            diag = torch.diagonal(JtWJ, dim1=1, dim2=2)
            lambdas = torch.logspace(-5, 5, solver.samples, dtype=JtWJ.dtype, device=JtWJ.device)
            vols = []
            for s in range(solver.samples):  # the residual volume (1662-1680)
                pose_s = damped_update(JtWJ, JtR, pose, lambdas[s] * diag)
                res_s, _ = ic_residual(pose_s, x0, x1, invD0, invD1, K, px, py, obj_mask1=obj_mask1)
                vols.append(torch.bmm(Jt, (weights * res_s).reshape(B, -1, 1)))
            damp = solver.net(torch.cat((torch.cat(vols, dim=2).reshape(B, -1), JtWJ.reshape(B, -1)), dim=1))
            pose = damped_update(JtWJ, JtR, pose, damp.reshape(B, 6))
        else:
            pose = damped_update(JtWJ, JtR, pose)
        res, _ = ic_residual(pose, x0, x1, invD0, invD1, K, px, py, obj_mask1=obj_mask1)
    return pose, weights


def ic_loss(tracker, pose, x0, x1, invD0, invD1, K, wPrior=None, obj_mask0=None, obj_mask1=None):
    """TrustRegionBase.forward_residuals (algorithms.py:125-139): compute_avg_loss of the
    weighted residuals over the non-occluded pixels."""
    x0, x1 = nchw(x0), nchw(x1)
    B, C, H, W = x0.shape
    K = K.reshape(B, 4)
    px, py = pixel_grid(B, H, W, K)
    res, occ = ic_residual(pose, x0, x1, invD0, invD1, K, px, py, obj_mask0, obj_mask1)
    wr = tracker.mEstimator(res, x0, x1, wPrior) * res
    wr = torch.where(occ.expand_as(wr), torch.zeros_like(wr), wr)
    return (wr ** 2).reshape(B, -1).sum(1) / (H * W - occ.reshape(B, -1).sum(1)).to(wr.dtype)
