"""Modules of the tracker: the HIP-backed U_IC solver and the host-side networks.

`TrustRegionInverseWUncertainty` is the drop-in for the reference's class of the
same name (code/models/algorithms.py:579-997): same constructor, same
`forward` / `forward_residuals` signatures and return values.  Device tensors at
inference run every level through libdpft_ic.so (deep_prob_feature_track_amd.ic), which
fails loudly when it is missing; CPU tensors and calls with gradients (grad enabled and an
input that requires grad: the reference's training path) take the PyTorch path of
torch_solver.py (SURVEY.md 8(b)'s dispatch rule).  Configurations neither implements
raise NotImplementedError.

The networks around it (feature encoder, pose initialisers, estimator
networks of the IC tracker) are PyTorch modules whose parameter names match the
reference's state_dict keys, so the reference's checkpoints load unchanged:
  ImagePyramids 1201-1219, FeaturePyramid 1221-1430, DeepRobustEstimator
  1432-1499 (applied by the IC tracker), ScaleNet 1501-1581, DirectSolverNet
  1583-1692 ('Direct-ResVol' for the IC tracker; the U_IC path never calls it,
  algorithms.py:691), PoseNetFeat / PoseNet / SFMPoseNet 1694-1832,
  deep_damping_regressor 1834-1842.
"""
import torch
import torch.nn as nn
import torch.nn.functional as func

from .. import ic
from .. import torch_ops  # noqa: F401  (registers the dpft:: ops torch.compile traces)
from . import geometry
from . import torch_solver as TS
from .submodules import convLayer as conv
from .submodules import convLayer1d as conv1d
from .submodules import fcLayer, initialize_weights


# ------------------------------------------------------------------ pyramids
class ImagePyramids(nn.Module):
    """Average / max pooling by 2^s for every scale s; bool maps pool as float and
    come back as `> 0` (algorithms.py:1201-1219)."""

    def __init__(self, scales, pool='avg'):
        super().__init__()
        if pool not in ('avg', 'max'):
            raise NotImplementedError(pool)
        make = nn.AvgPool2d if pool == 'avg' else nn.MaxPool2d
        self.multiscales = [make(1 << s, 1 << s) for s in scales]

    def forward(self, x):
        if x.dtype == torch.bool:
            xf = x.to(torch.float32)
            return [f(xf).to(torch.bool) for f in self.multiscales]
        return [f(x) for f in self.multiscales]


# ------------------------------------------------------------------ encoder
_UNCERTAINTY_ACTIVATIONS = {
    'gaussian': lambda s: torch.exp(0.5 * torch.clamp(s, min=-6, max=6)),
    'laplacian': lambda s: torch.exp(torch.clamp(s, min=-3, max=3)),
    'sigmoid': torch.sigmoid,
    'old_gaussian': lambda s: torch.exp(0.5 * torch.clamp(s, min=1e-3, max=1e3)),
    'old_laplacian': lambda s: torch.exp(torch.clamp(s, min=1e-3, max=1e3)),
}


class FeaturePyramid(nn.Module):
    """Four-scale feature + uncertainty encoder (algorithms.py:1221-1430).

    Returns (features [4], sigmas [4], backbone maps [4]); a 1-channel uncertainty
    is repeated to the feature channels as in the reference (1426-1427), as a
    channel-broadcast view (same shape and values, no copy) that the solver wrapper
    recognises and hands to the kernel as one plane (Cs = 1: 2 sigma planes of reads
    per pixel instead of 2C)."""

    def __init__(self, D, w_uncertainty='None', feature_channel=1, feature_extract='conv', uncertainty_channel=1):
        super().__init__()
        assert uncertainty_channel == feature_channel or uncertainty_channel == 1
        self.w_uncertainty = w_uncertainty != 'None'
        self.uncertainty_type = w_uncertainty
        self.output_C = feature_channel
        self.uncertainty_C = uncertainty_channel
        self.feature_extract = feature_extract
        self.f_channels = [32, 64, 96, 128]
        # backbone: per scale (in, mid, out) with dilations 1, 2, 2
        stages = [(D, 16, 32, 32), (32, 32, 64, 64), (64, 64, 96, 96), (96, 96, 128, 128)]
        for s, (cin, c1, c2, cout) in enumerate(stages):
            net = nn.Sequential(conv(True, cin, c1, 3), conv(True, c1, c2, 3, dilation=2),
                                conv(True, c2, cout, 3, dilation=2))
            setattr(self, f'net{s}', net)
            initialize_weights(net)

        if feature_extract not in ('average', 'skip'):
            if feature_extract == 'prob_fuse':
                self.output_C = 16
            if feature_extract in ('conv', 'prob_fuse'):
                heads = [conv(True, c, self.output_C, kernel_size=1) for c in self.f_channels]
            elif feature_extract == '1by1':
                heads = [nn.Conv2d(c, self.output_C, kernel_size=(1, 1)) for c in self.f_channels]
            else:
                raise NotImplementedError("not supported feature extraction option")
            for s, h in enumerate(heads):
                setattr(self, f'f_conv{s}', h)
            initialize_weights(heads)

        if self.w_uncertainty and self.uncertainty_type != 'identity':
            if self.uncertainty_type == 'feature':
                heads = [conv(True, c, self.output_C, 1) for c in self.f_channels]
            elif self.uncertainty_type in _UNCERTAINTY_ACTIVATIONS:
                heads = [nn.Sequential(conv(True, c, 16, kernel_size=1), nn.Conv2d(16, self.uncertainty_C, kernel_size=1))
                         for c in self.f_channels]
            else:
                raise NotImplementedError(self.uncertainty_type)
            for s, h in enumerate(heads):
                setattr(self, f'sigma_conv{s}', h)
            initialize_weights(heads)

        self.downsample = nn.AvgPool2d(kernel_size=2)

    def _prob_fuse(self, x, head):
        f, p = head(x).chunk(2, dim=1)
        return torch.sum(f * torch.sigmoid(p), dim=1, keepdim=True)

    def forward(self, x, packed=False):
        """packed=True (the drop-in's solve path): the 'conv' feature heads write their
        output straight in the solver's channel-quad layout [B,C/4,H,W,4] (their batchnorm +
        ELU epilogue stores it, ConvBlock.forward_packed) where the layout applies (eval
        mode on the device, channels_last maps, C % 4 == 0); otherwise, and for every other
        output, the reference's [B,C,H,W]."""
        maps = []
        for s in range(4):
            x = getattr(self, f'net{s}')(x if s == 0 else self.downsample(x))
            maps.append(x)

        if packed and self.feature_extract == 'conv':
            f = [getattr(self, f'f_conv{s}').forward_packed(m) for s, m in enumerate(maps)]
        elif self.feature_extract == 'skip':
            f = list(maps)
        elif self.feature_extract == 'average':
            f = [m.sum(dim=1, keepdim=True) / m.shape[1] for m in maps]
        elif self.feature_extract == 'prob_fuse':
            f = [self._prob_fuse(m, getattr(self, f'f_conv{s}')) for s, m in enumerate(maps)]
        elif self.feature_extract in ('conv', '1by1'):
            f = [getattr(self, f'f_conv{s}')(m) for s, m in enumerate(maps)]
        else:
            raise NotImplementedError()

        if not self.w_uncertainty:
            return f, [None] * 4, maps
        if self.uncertainty_type == 'identity':
            return f, [torch.ones_like(fi) for fi in f], maps
        sigma = [getattr(self, f'sigma_conv{s}')(m) for s, m in enumerate(maps)]
        if self.uncertainty_type != 'feature':
            sigma = [_UNCERTAINTY_ACTIVATIONS[self.uncertainty_type](si) for si in sigma]
        if self.uncertainty_C == 1 and self.output_C != 1:
            sigma = [si.expand(-1, self.output_C, -1, -1) for si in sigma]
        return f, sigma, maps


# ------------------------------------------------------------------ estimators
def _weight_net(D, final):
    net = nn.Sequential(conv(True, D, 16, 3, dilation=1), conv(True, 16, 32, 3, dilation=2),
                        conv(True, 32, 64, 3, dilation=4), *final)
    initialize_weights(net)
    return net


class DeepRobustEstimator(nn.Module):
    """M-estimator (algorithms.py:1432-1499): 'None' (unit weights) or the
    convolutional 'MultiScale2w' on [|r|, x0, x1, bilinear-upsampled prior weights]
    (1467-1477; 4 input channels, so 1-channel features).  The IC tracker applies it;
    the U_IC solver never does (commented out in the reference, 638-641)."""

    def __init__(self, estimator_type):
        super().__init__()
        if estimator_type == 'MultiScale2w':
            self.D = 4
            self.net = _weight_net(4, [conv(True, 64, 1, 3, dilation=1), nn.Sigmoid()])
        elif estimator_type == 'None':
            self.D = -1
            self.net = None
        else:
            raise NotImplementedError()

    def forward(self, residual, x0, x1, ws=None):
        if self.D < 0:
            return torch.ones_like(residual)
        H, W = residual.shape[-2:]
        wl = func.interpolate(ws, (H, W), mode='bilinear', align_corners=True)
        return self.net(torch.cat((residual.abs(), x0, x1, wl), dim=1))


class ScaleNet(nn.Module):
    """ICP / feature balance (algorithms.py:1501-1581).  'None' is the constant
    `scale` (0.01) the fused ICP kernel applies; the learned scalers need the
    residual maps the kernel never materialises and are not offered."""

    _DIMS = {'oneResidual': 1, 'twoResidual': 2, 'MultiScale2w': 3, 'expMultiScale': 3, 'None': -1}

    def __init__(self, estimator_type, scale=None):
        super().__init__()
        if estimator_type not in self._DIMS:
            raise NotImplementedError()
        self.estimator_type = estimator_type
        self.D = self._DIMS[estimator_type]
        self.net = _weight_net(self.D, [conv(True, 64, 16, 3, dilation=1), nn.Conv2d(16, 1, kernel_size=1, padding=0)]) \
            if self.D > 0 else None
        self.scale = 0.01 if scale is None else scale

    def forward(self, residual, another_residual=None, ws=None):
        if self.D > 0:
            raise NotImplementedError("learned ICP scalers are not supported by the fused HIP solver")
        return torch.ones_like(residual) * self.scale


def deep_damping_regressor(D):
    """MLP D -> 128 -> 256 -> 6 with ReLUs (algorithms.py:1834-1842)."""
    return nn.Sequential(fcLayer(D, 128), fcLayer(128, 256), fcLayer(256, 6))


def _twist2mat(w):
    """Exp of so(3) vectors [B,3] by Rodrigues (geometry.py:163-185); NaN at |w| = 0 as there."""
    th = torch.sqrt((w * w).sum(1, keepdim=True))
    k = w / th
    K = torch.zeros(w.shape[0], 3, 3, dtype=w.dtype, device=w.device)
    K[:, 0, 1], K[:, 0, 2] = -k[:, 2], k[:, 1]
    K[:, 1, 0], K[:, 1, 2] = k[:, 2], -k[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -k[:, 1], k[:, 0]
    s, c = torch.sin(th).view(-1, 1, 1), torch.cos(th).view(-1, 1, 1)
    I = torch.eye(3, dtype=w.dtype, device=w.device).expand_as(K)
    return I + s * K + (1 - c) * torch.bmm(K, K)


def inverse_update_pose(H, JtR, pose):
    """xi = H^-1 JtR, R <- R Exp(-w), t <- R (-Exp(-w) v) + t (algorithms.py:2017-2054),
    batched on the device in fp64 (the reference inverts on the host CPU in fp32, 2077-2091).
    `solve_ex`: no host read of the factorisation status (a singular H gives inf / NaN
    poses, as the reference's inverse does)."""
    R, t = pose
    B = H.shape[0]
    xi = torch.linalg.solve_ex(H.double(), JtR.double().reshape(B, 6, 1))[0].view(B, 6)
    dR = _twist2mat(-xi[:, :3])
    dt = -torch.bmm(dR, xi[:, 3:].reshape(B, 3, 1))
    R1, t1 = geometry.batch_Rt_compose(R.double(), t.double(), dR, dt)
    return [R1.to(R.dtype), t1.to(t.dtype).view(B, 3)]  # t [B,3] as batch_Rt_compose returns it (geometry.py:122)


class DirectSolverNet(nn.Module):
    """Damping module (algorithms.py:1583-1692).  The U_IC solver does not call it (it
    always uses lev_mar_H, algorithms.py:836-846); the IC tracker (TrustRegionBase) runs
    'Direct-Nodamping' inside the fused HIP iteration and 'Direct-ResVol' through
    `resvol_step`: the residual volume's ten J^T W r samples come from the HIP kernel
    (DPFT_ITER_NO_UPDATE), the damping MLP and the 6x6 solves from PyTorch."""

    SOLVER_NO_DAMPING = 0
    SOLVER_RESIDUAL_VOLUME = 1

    def __init__(self, solver_type, samples=10, direction='inverse'):
        super().__init__()
        self.direction = direction
        if solver_type == 'Direct-Nodamping':
            self.net = None
            self.type = self.SOLVER_NO_DAMPING
        elif solver_type == 'Direct-ResVol':
            self.samples = samples
            self._lambdas = None  # logspace(-5, 5, samples) on the device, made once
            self.net = deep_damping_regressor(D=6 * 6 + 6 * samples)
            self.type = self.SOLVER_RESIDUAL_VOLUME
            initialize_weights(self.net)
        else:
            raise NotImplementedError()

    def forward(self, *args, **kwargs):
        raise NotImplementedError("DirectSolverNet is driven by TrustRegionBase (resvol_step); not on the U_IC path")

    def replicate(self, level_args, weights, obj_mask1):
        """The level's inputs repeated `samples` times along the batch (trial s of pair b
        at s * B + b), made once per level call: the ten residual-volume samples of every
        iteration then run as ONE no-update launch over samples x pairs.  The IC tracker
        has no batch-global term (no truncated sigma), so each (trial, pair) row is
        solved exactly as alone."""
        S = self.samples
        x0, x1, invD0, invD1, K = level_args
        rep = lambda a: None if a is None else a.repeat(S, *([1] * (a.dim() - 1)))  # noqa: E731
        return rep(x0), rep(x1), rep(invD0), rep(invD1), rep(K), rep(weights), rep(obj_mask1)

    def resvol_step(self, pose, level_args, weights, obj_mask0, obj_mask1, first, replicated=None):
        """One Gauss-Newton step with the learned residual-volume damping
        (__regularize_residual_volume, algorithms.py:1644-1691, then inverse_update_pose):
        JtWJ, JtWr at `pose` (obj_mask0 only on a level's first step, 72-73 / 77-78), ten
        trial poses under damping lambda_s diag(JtWJ) + 1e-6 tr(JtWJ) I with lambda_s in
        logspace(-5, 5), the J^T W r of each trial (masks of frame 1 only, 1683), the MLP
        on [JtR_1 .. JtR_10, JtWJ] -> per-axis damping, and the damped update."""
        x0, x1, invD0, invD1, K = level_args
        B = x0.shape[0]
        R, t, JtJ, JtR, _ = ic.iterate(pose, x0, x1, invD0, invD1, K, None, None, first=first, update=False,
                                       no_uncertainty=True, weights=weights, obj_mask0=obj_mask0,
                                       obj_mask1=obj_mask1)
        pose = [R, t]
        S = self.samples
        if self._lambdas is None or self._lambdas.device != JtJ.device:
            self._lambdas = torch.logspace(-5, 5, S, dtype=torch.float32, device=JtJ.device).view(S, 1, 1)
        # the S trial poses (JtJ + lambda_s diag(JtJ) + 1e-6 tr I) in one launch, their
        # J^T W r through one LevelCall, the learned damping's update in one more launch
        R_s, t_s = ic.damped_update(JtJ, JtR, self._lambdas * torch.diagonal(JtJ, dim1=1, dim2=2), pose)
        if replicated is not None:
            xs0, xs1, ds0, ds1, Ks, ws, ms1 = replicated
            _, _, _, JtR_s, _ = ic.iterate((R_s.view(S * B, 3, 3), t_s.view(S * B, 3, 1)), xs0, xs1, ds0, ds1, Ks,
                                           None, None, first=False, update=False, no_uncertainty=True, weights=ws,
                                           obj_mask1=ms1)
            JtR_s = JtR_s.view(S, B, 6)
        else:
            _, JtR_s = ic.iterate_poses(R_s, t_s, x0, x1, invD0, invD1, K, None, None,
                                        no_uncertainty=True, weights=weights, obj_mask1=obj_mask1)
        JtR_flat = JtR_s.permute(1, 2, 0).reshape(B, -1)  # [B, 6, S]: as the reference's cat(dim=2)
        damp = self.net(torch.cat((JtR_flat, JtJ.view(B, -1)), dim=1))
        R1, t1 = ic.damped_update(JtJ, JtR, damp.view(1, B, 6), pose)
        return [R1[0], t1[0].view(B, 3)]


# ------------------------------------------------------------------ init-pose networks
class PoseNetFeat(nn.Module):
    """algorithms.py:1694-1720."""

    def __init__(self):
        super().__init__()
        self.final_C = 1024
        self.sep_cov = nn.Sequential(conv(True, 128, 128, kernel_size=3, stride=2),
                                     conv(True, 128, 128, kernel_size=3, stride=2))
        self.conv1 = conv1d(True, 128, 256, 1)
        self.conv2 = conv1d(True, 256, 512, 1)
        self.conv3 = conv1d(True, 512, self.final_C, 1)
        initialize_weights((self.sep_cov, self.conv1, self.conv2, self.conv3))

    def forward(self, feat_map):
        B, C = feat_map.shape[:2]
        emb1 = self.conv1(self.sep_cov(feat_map).view(B, C, -1))
        emb2 = self.conv2(emb1)
        final = self.conv3(emb2)
        N = final.shape[-1]
        pooled = func.avg_pool1d(final, N).view(B, self.final_C, 1).repeat(1, 1, N)
        return emb1, emb2, pooled


def _pose_head(cin, cout):
    return nn.Sequential(conv1d(True, cin, 640, 1), conv1d(True, 640, 256, 1), conv1d(True, 256, 128, 1),
                         nn.Conv1d(128, cout, kernel_size=1, padding=0))


class PoseNet(nn.Module):
    """Dense init-pose regressor (algorithms.py:1722-1768)."""

    def __init__(self, scale_motion=0.01, multi_hypo='None', res_input=False):
        super().__init__()
        self.feat_net = PoseNetFeat()
        self.input_C = 3584
        self.scale_motion = scale_motion
        self.net_r = _pose_head(self.input_C, 3)
        self.net_t = _pose_head(self.input_C, 3)
        self.net_c = _pose_head(self.input_C, 1)
        initialize_weights((self.net_r, self.net_t, self.net_c))

    def forward(self, x0, x1):
        a = self.feat_net(x0)
        b = self.feat_net(x1)
        feat = torch.cat([a[0], b[0], a[1], b[1], a[2], b[2]], dim=1)
        conf = func.softmax(self.net_c(feat), dim=-1)
        rot = self.scale_motion * torch.sum(self.net_r(feat) * conf, dim=-1)
        trs = self.scale_motion * torch.sum(self.net_t(feat) * conf, dim=-1)
        return geometry.batch_euler2mat(rot[:, 0], rot[:, 1], rot[:, 2]), trs


class SFMPoseNet(nn.Module):
    """Init-pose regressor on the coarsest backbone maps (algorithms.py:1770-1832)."""

    def __init__(self, scale_motion=0.01, multi_hypo='None', res_input=False):
        super().__init__()
        self.batchnorm = True
        self.res_input = res_input
        planes = [384, 256, 256] if res_input else [256, 256, 256]
        self.scale_motion = scale_motion
        self.multi_hypo = multi_hypo
        self.hypo_num = 16 if multi_hypo != 'None' else 1
        self.net = nn.Sequential(conv(True, planes[0], planes[1], kernel_size=3, dilation=2),
                                 conv(True, planes[1], planes[2], kernel_size=3, dilation=2))
        if multi_hypo == 'None':
            self.final_layer = nn.Conv2d(planes[2], 6, kernel_size=1, padding=0)
        elif multi_hypo in ('average', 'prob_fuse'):
            per = 6 if multi_hypo == 'average' else 7
            self.final_layer = nn.Sequential(conv1d(True, planes[2], 128, 1),
                                             nn.Conv1d(128, self.hypo_num * per, kernel_size=1, padding=0))
        else:
            raise NotImplementedError(multi_hypo)
        initialize_weights(self.net, self.final_layer)

    def forward(self, x0, x1):
        inp = torch.cat((x0, x1, x0 - x1) if self.res_input else (x0, x1), dim=1)
        B = inp.shape[0]
        h = self.net(inp)
        if self.multi_hypo == 'None':
            pose = self.final_layer(h).mean(dim=3).mean(dim=2)
        else:
            h = self.final_layer(h.view(B, h.shape[1], -1)).mean(dim=-1)
            if self.multi_hypo == 'average':
                pose = h.view(B, 6, -1).mean(dim=-1)
            else:
                poses, conf = h.view(B, -1, 7).split((6, 1), dim=-1)
                pose = torch.sum(poses * func.softmax(conf, dim=1), dim=1)
        return geometry.pose_vec2mat(self.scale_motion * pose.view(B, 6), rotation_mode='euler')


# ------------------------------------------------------------------ the HIP-backed solvers
class TrustRegionBase(nn.Module):
    """Inverse-compositional Gauss-Newton WITHOUT uncertainty -- the 'IC' tracker
    (algorithms.py:23-139), on libdpft_ic.so (flag DPFT_NO_UNCERTAINTY).

    forward -> (pose [R, t], weights): the constant J^T W J of the template
    (precompute_Jacobian 103-121, identical in every iteration, so the fused kernel
    simply recomputes it), JtR of the residual at the current pose with occluded
    residuals 1e-3 (compute_warped_residual 1919-1957), and the damped inverse update.
    M-estimator (66-68): 'None' = unit weights; 'MultiScale2w' = the convolutional
    estimator on [|r|, x0, x1, upsampled wPrior] of the first residual (the HIP
    residual map, dpft_ic_residual_map), whose per-pixel weights the fused kernel then
    applies to J^T W J and J^T W r in every iteration.  Solver: 'Direct-Nodamping'
    (lev_mar_H, solved in-kernel) or 'Direct-ResVol' (DirectSolverNet.resvol_step).  As
    in the reference, only the first residual sees obj_mask0 (the loop re-evaluates with
    obj_mask1 alone, 77-78)."""

    def __init__(self, max_iter=3, mEst_func=None, solver_func=None, timers=None):
        super().__init__()
        self.max_iterations = max_iter
        self.mEstimator = mEst_func
        self.directSolver = solver_func
        self.timers = timers


    def _learned_weights(self):
        return self.mEstimator is not None and getattr(self.mEstimator, 'D', -1) > 0

    def precompute_Jacobian(self, invD, x, px, py, K):
        """Template image Jacobian J = gx Jx + gy Jy per channel and pixel (algorithms.py:
        103-121) -> [B, C*HW, 6], materialised by the HIP inverse-Jacobian kernel with sigma
        = 1 and a zero residual (its a = -gx / sigma, J = -(a Jx + b Jy)).  The fused
        iteration never builds it."""
        B, C, H, W = x.shape
        if TS.needs_torch_path(x, invD):  # CPU tensors / gradients
            return TS.ic_template_jacobian(invD, x, px.expand(B, -1, -1, -1), py.expand(B, -1, -1, -1), K.reshape(B, 4))
        g = ic.feature_gradient(x)
        Jx_p, Jy_p = ic.warp_jacobian(invD, K, px, py)
        one = torch.ones((1, 1, 1, 1), dtype=torch.float32, device=x.device).expand(B, C, H, W)
        zero = torch.zeros((1, 1, 1, 1), dtype=torch.float32, device=x.device)
        J = ic.inverse_jacobian(zero.expand(B, C, H, W), one, one[:, :1].expand(B, C, H, W),
                                g, zero.expand(B, 1, 2, H, W), Jx_p, Jy_p)
        return J.view(B, C * H * W, 6)

    def GN_solver(self, JtJ, JtR, pose0):
        """lev_mar_H + inverse_update_pose (algorithms.py:105-107, 2094-2103, 2017-2054) in
        one launch (dpft_ic_damped_update); the PyTorch path for CPU tensors / gradients."""
        B = JtJ.shape[0]
        if TS.needs_torch_path(JtJ, JtR, *pose0):
            return TS.damped_update(JtJ, JtR, pose0)
        R, t = ic.damped_update(JtJ, JtR.reshape(B, 6), None, pose0)
        return [R[0], t[0].view(B, 3)]  # inverse_update_pose's t [B,3] (geometry.py:122)

    def _weights(self, pose, x0, x1, invD0, invD1, K, wPrior, obj_mask0, obj_mask1):
        """(weights [B,1,H,W] of the learned estimator, residual map, occlusion) or Nones."""
        if not self._learned_weights():
            return None, None, None
        if wPrior is None:
            raise ValueError("a learned M-estimator needs the weight prior wPrior (LeastSquareTracking.py:346)")
        res, occ = ic.residual_map(pose, x0, x1, invD0, invD1, K, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        return self.mEstimator(res, x0, x1, wPrior), res, occ

    def forward(self, pose, x0, x1, invD0, invD1, K, wPrior=None, vis_res=False, obj_mask0=None, obj_mask1=None):
        if TS.needs_torch_path(x0, x1, invD0, invD1, *pose):  # CPU tensors / gradients
            return TS.ic_forward(self, pose, x0, x1, invD0, invD1, K, wPrior, obj_mask0, obj_mask1)
        B, C, H, W = x0.shape
        resvol = getattr(self.directSolver, 'type', 0) == DirectSolverNet.SOLVER_RESIDUAL_VOLUME
        with torch.no_grad():
            w, _, _ = self._weights(pose, x0, x1, invD0, invD1, K, wPrior, obj_mask0, obj_mask1)
            # one launch over (trial, pair) rows while they fit a call (ic.MAX_PAIRS_PER_CALL);
            # larger batches take iterate_poses (one no-update call per trial)
            rep = None
            if resvol and self.directSolver.samples * B <= ic.MAX_PAIRS_PER_CALL:
                rep = self.directSolver.replicate((x0, x1, invD0, invD1, K), w, obj_mask1)
            for it in range(self.max_iterations):
                m0 = obj_mask0 if it == 0 else None
                if resvol:
                    pose = self.directSolver.resvol_step(pose, (x0, x1, invD0, invD1, K), w, m0, obj_mask1,
                                                         replicated=rep,
                                                         first=(it == 0))
                else:
                    R, t, _, _, _ = ic.iterate(pose, x0, x1, invD0, invD1, K, None, None, first=(it == 0),
                                               no_uncertainty=True, weights=w, obj_mask0=m0, obj_mask1=obj_mask1)
                    pose = [R, t.view(B, 3)]  # the updated t is [B,3] (batch_Rt_compose, geometry.py:122)
        weights = w if w is not None else torch.ones((1, 1, 1, 1), dtype=x0.dtype, device=x0.device).expand(B, C, H, W)
        return pose, weights

    def forward_residuals(self, pose, x0, x1, invD0, invD1, K, wPrior=None, vis_res=False, obj_mask0=None,
                          obj_mask1=None):
        """loss [B] (algorithms.py:125-139): the unit-weight loss in one HIP launch, or
        with a learned estimator compute_avg_loss([weights * r], occ) (2119-2137) on the
        HIP residual map."""
        if TS.needs_torch_path(x0, x1, invD0, invD1, *pose):  # CPU tensors / gradients
            return TS.ic_loss(self, pose, x0, x1, invD0, invD1, K, wPrior, obj_mask0, obj_mask1)
        with torch.no_grad():
            if not self._learned_weights():
                return ic.residual_level(pose, x0, x1, invD0, invD1, K, None, None, no_uncertainty=True,
                                         obj_mask0=obj_mask0, obj_mask1=obj_mask1)
            w, res, occ = self._weights(pose, x0, x1, invD0, invD1, K, wPrior, obj_mask0, obj_mask1)
            H, W = res.shape[-2:]
            wr = torch.where(occ, torch.zeros_like(res), w * res)
            return (wr ** 2).sum(dim=(1, 2, 3)) / (H * W - occ.sum(dim=(1, 2, 3)))


class TrustRegionInverseWUncertainty(nn.Module):
    """Inverse-compositional, uncertainty-weighted Gauss-Newton with Levenberg
    damping (algorithms.py:579-997), one level per call, on libdpft_ic.so.

    forward  -> (pose [R, t], weights[, JtWJ])   algorithms.py:611-723
    forward_residuals -> loss [B]                algorithms.py:725-786
    `weights` is the reference's all-ones [B,C,H,W] map (a broadcast view, no
    memory) or, with combine_icp, the constant ICP scale [B,1,H,W].
    """

    def __init__(self, max_iter=3, mEst_func=None, solver_func=None, timers=None, uncer_prop=False,
                 combine_icp=False, scale_func=None, remove_tru_sigma=False):
        super().__init__()
        # a [1] int32 device word set by LeastSquareTracking.forward for one pyramid
        # solve: the levels OR their non-finite flag into it and the driver checks it once
        # (one host read per forward instead of one per level); None = check every call
        self._deferred_status = None
        self.max_iterations = max_iter
        self.mEstimator = mEst_func
        self.directSolver = solver_func
        self.timers = timers
        self.uncer_prop = uncer_prop
        self.combine_icp = combine_icp
        self.scale_func = scale_func
        self.remove_tru_sigma = remove_tru_sigma

    def _check_path(self, x0):
        if self.combine_icp and self.scale_func is not None and getattr(self.scale_func, 'D', -1) > 0:
            raise NotImplementedError("learned ICP scalers are not supported by the fused HIP solver")

    def _torch_level(self, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1):
        """The level for the PyTorch path (CPU tensors / gradients, torch_solver.py)."""
        if self.combine_icp:
            assert depth0 is not None and depth1 is not None
        return TS.UICLevel(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1,
                           remove_tru_sigma=bool(self.remove_tru_sigma),
                           icp_scale=self._icp_scale() if self.combine_icp else None)

    def _icp_scale(self):
        return float(self.scale_func.scale) if self.scale_func is not None else 0.01

    def _common(self, x0, depth0, depth1, obj_mask0, obj_mask1):
        kw = dict(remove_tru_sigma=bool(self.remove_tru_sigma), obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        if self.combine_icp:
            assert depth0 is not None and depth1 is not None
            kw.update(combine_icp=True, depth0=depth0, depth1=depth1, icp_weight=self._icp_scale())
        return kw

    def forward(self, pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, wPrior=None,
                depth0=None, depth1=None, vis_res=True, obj_mask0=None, obj_mask1=None):
        out = self.solve(pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1)
        if self._deferred_status is None and out[3] is not None:
            ic.check_status(out[3])
        return out[:3] if self.uncer_prop else out[:2]

    def solve(self, pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0=None, depth1=None, obj_mask0=None,
              obj_mask1=None):
        """-> (pose [R, t], weights, JtWJ or None, status [1] int32 device word): forward
        without the host check.  Traced by torch.compile it is one dpft::ic_solve_level op
        (torch_ops.py); eager, the same library call through ctypes.  CPU tensors and calls
        with gradients take the PyTorch path (status None: it raises AssertionError itself on
        a non-finite residual or Jacobian, as the reference's asserts do)."""
        assert sigma0 is not None and sigma1 is not None
        self._check_path(x0)
        B, C, H, W = ic.feature_shape(x0)  # NCHW, or the channel-quad layout of a packed encoder
        if TS.needs_torch_path(x0, x1, invD0, invD1, sigma0, sigma1, *pose10):
            lv = self._torch_level(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1)
            pose, jtj = TS.uic_solve(pose10, lv, self.max_iterations, want_jtj=self.uncer_prop)
            if self.combine_icp:
                weights = torch.full((1, 1, 1, 1), self._icp_scale(), dtype=x0.dtype, device=x0.device).expand(B, 1, H, W)
            else:
                weights = torch.ones((1, 1, 1, 1), dtype=x0.dtype, device=x0.device).expand(B, C, H, W)
            return pose, weights, jtj, None
        kw = self._common(x0, depth0, depth1, obj_mask0, obj_mask1)
        with torch.no_grad():
            if torch.compiler.is_compiling():
                R, t, jtj, status = torch.ops.dpft.ic_solve_level(
                    pose10[0], pose10[1], x0, x1, invD0, invD1, K, sigma0, sigma1, kw.get("depth0"),
                    kw.get("depth1"), obj_mask0, obj_mask1, self.max_iterations, bool(self.remove_tru_sigma),
                    bool(self.combine_icp), float(kw.get("icp_weight", 0.01)), False, bool(self.uncer_prop))
                out = (R, t, jtj if self.uncer_prop else None)
            else:
                status = self._deferred_status
                if status is None:
                    status = torch.zeros(1, dtype=torch.int32, device=x0.device)
                out = ic.solve_level(pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, iters=self.max_iterations,
                                     return_jtj=self.uncer_prop, check=False, status=status, **kw)
        # an updated translation is [B,3], as the reference's batch_Rt_compose returns it
        # (geometry.py:122); with no iteration the initial pose passes through unchanged
        pose = [out[0], out[1].view(B, 3)] if self.max_iterations > 0 else list(pose10)
        if self.combine_icp:
            weights = torch.full((1, 1, 1, 1), self._icp_scale(), dtype=x0.dtype, device=x0.device).expand(B, 1, H, W)
        else:
            weights = torch.ones((1, 1, 1, 1), dtype=x0.dtype, device=x0.device).expand(B, C, H, W)
        return pose, weights, (out[2] if self.uncer_prop else None), status

    # ---- the reference solver's Jacobian API (algorithms.py:812-887), materialised by HIP
    # kernels for callers that inspect J; forward never builds J (it stays in registers)
    def precompute_jacobian_components(self, invD0, f0, sigma0, px, py, K, grad_interp=False, crd0=None):
        """(grad_f0 [B,C,2,H,W], grad_sigma0, Jx_p [B,HW,6], Jy_p) -- algorithms.py:848-865."""
        if grad_interp:
            raise NotImplementedError("bilinear-interpolation gradients (grad_interp) belong to the forward "
                                      "direction; the inverse path linearises at the origin")
        if TS.needs_torch_path(f0, sigma0, invD0):  # CPU tensors / gradients
            B = f0.shape[0]
            Jx_p, Jy_p = TS.warp_jacobian(px.expand(B, -1, -1, -1), py.expand(B, -1, -1, -1), invD0, K.reshape(B, 4))
            return torch.stack(TS.sobel(f0), 2), torch.stack(TS.sobel(sigma0), 2), Jx_p, Jy_p
        grad_f0 = ic.feature_gradient(f0)
        if sigma0.shape[1] != 1 and sigma0.stride(1) == 0:  # channel broadcast: one plane's gradient
            grad_sigma0 = ic.feature_gradient(sigma0[:, :1]).expand(-1, sigma0.shape[1], -1, -1, -1)
        else:
            grad_sigma0 = ic.feature_gradient(sigma0)
        Jx_p, Jy_p = ic.warp_jacobian(invD0, K, px, py)
        return grad_f0, grad_sigma0, Jx_p, Jy_p

    def compose_inverse_jacobians(self, res, sigma, sigma0, grad_f0, grad_sigma0, Jx_p, Jy_p):
        """(J [B,C,HW,6], J_res_trs [B,C,3,H,W], J_res_rot) -- algorithms.py:867-887; the
        two parts are of -J, the chained derivative before the reference's sign flip."""
        B, C, H, W = sigma0.shape
        if TS.needs_torch_path(res, sigma, sigma0, grad_f0):  # CPU tensors / gradients
            k = res * sigma0 / sigma ** 3
            a = -(grad_f0[:, :, 0] / sigma + k * grad_sigma0[:, :, 0])
            b = -(grad_f0[:, :, 1] / sigma + k * grad_sigma0[:, :, 1])
            J = -(a.reshape(B, C, -1, 1) * Jx_p.view(B, 1, -1, 6) + b.reshape(B, C, -1, 1) * Jy_p.view(B, 1, -1, 6))
        else:
            J = ic.inverse_jacobian(res, sigma, sigma0, grad_f0, grad_sigma0, Jx_p, Jy_p)
        J_res_rot, J_res_trs = (-J).view(B, C, H, W, 6).split(3, dim=-1)
        if not torch.isfinite(J).all():
            raise AssertionError("non-finite Jacobian (reference: assert check_nan(J_res_p) == 0)")
        return J, J_res_trs.permute(0, 1, 4, 2, 3), J_res_rot.permute(0, 1, 4, 2, 3)

    def GN_solver(self, JtJ, JtR, pose0, direction='inverse'):
        """lev_mar_H + inverse_update_pose (algorithms.py:836-846, 2094-2103, 2017-2054):
        H = JtJ + 1e-6 tr(JtJ) I solved in fp64 and the inverse-compositional update, in
        one launch (dpft_ic_damped_update)."""
        if direction != 'inverse':
            raise NotImplementedError("the forward-compositional update belongs to the U_FC tracker")
        B = JtJ.shape[0]
        if TS.needs_torch_path(JtJ, JtR, *pose0):
            return TS.damped_update(JtJ, JtR, pose0)
        R, t = ic.damped_update(JtJ, JtR.reshape(B, 6), None, pose0)
        return [R[0], t[0].view(B, 3)]  # inverse_update_pose's t [B,3] (geometry.py:122)

    def compute_jtj(self, jac):
        """J [B,C,HW,6] -> JtJ [B,6,6] (algorithms.py:812-820)."""
        if TS.needs_torch_path(jac):
            Jf = jac.reshape(jac.shape[0], -1, 6)
            return torch.bmm(Jf.transpose(1, 2), Jf)
        return ic.normal_equations(jac)[0]

    def compute_jtr(self, jac, res):
        """J [B,C,HW,6], res [B,C,H,W] -> JtR [B,6,1] (algorithms.py:822-834)."""
        if TS.needs_torch_path(jac, res):
            Jf = jac.reshape(jac.shape[0], -1, 6)
            return torch.bmm(Jf.transpose(1, 2), res.reshape(jac.shape[0], -1, 1))
        return ic.normal_equations(jac, res)[1]

    def forward_residuals(self, pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, wPrior=None,
                          depth0=None, depth1=None, vis_res=True, obj_mask0=None, obj_mask1=None):
        assert sigma0 is not None and sigma1 is not None
        self._check_path(x0)
        if TS.needs_torch_path(x0, x1, invD0, invD1, sigma0, sigma1, *pose10):
            lv = self._torch_level(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1)
            return lv.loss(pose10)
        kw = self._common(x0, depth0, depth1, obj_mask0, obj_mask1)
        with torch.no_grad():
            if torch.compiler.is_compiling():
                return torch.ops.dpft.ic_residual_level(
                    pose10[0], pose10[1], x0, x1, invD0, invD1, K, sigma0, sigma1, kw.get("depth0"), kw.get("depth1"),
                    obj_mask0, obj_mask1, bool(self.remove_tru_sigma), bool(self.combine_icp),
                    float(kw.get("icp_weight", 0.01)), False)
            return ic.residual_level(pose10, x0, x1, invD0, invD1, K, sigma0, sigma1, **kw)
