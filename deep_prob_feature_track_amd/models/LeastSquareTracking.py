"""Drop-in `LeastSquareTracking` (reference: code/models/LeastSquareTracking.py).

Same constructor arguments and `options` attributes (LeastSquareTracking.py:
38-103), same attributes (`tr_update0..3`, `track_type`, `scales`, `encoder`,
`pose_predictor`, ...), same state_dict keys, same `forward` /
`compute_residual` signatures and return values.  The coarse-to-fine solve runs
on libdpft_ic.so through `TrustRegionInverseWUncertainty`; the encoder and
init-pose networks run as PyTorch modules on the same device.

Supported: track_type 'U_IC' (uncertainty_type != 'None', direction 'inverse')
and 'IC' (uncertainty_type 'None': TrustRegionBase with M-estimator 'None' or
'MultiScale2w' and solver 'Direct-Nodamping' or 'Direct-ResVol', the weight prior
chained across levels as LeastSquareTracking.py:346-445 does) with encoders RGB /
ConvRGBD / ConvRGBD2, identity or
learned init pose, remove_tru_sigma, combine_ICP, uncer_prop (returns JtWJ) and
object masks.  Device tensors at inference run the solver levels on libdpft_ic.so;
CPU tensors and training mode run them on the PyTorch path (torch_solver.py, SURVEY.md
8(b)): a host without a GPU runs the reference's callers unchanged, and training-mode
forward returns the per-level poses stacked (LeastSquareTracking.py:568-575) with
gradients through the encoder and the unrolled solver (the reference's own training path
fails on torch 2.x, algorithms.py:874-875).  The reference's U_FC / ICP-only trackers raise
NotImplementedError.  Visualisation / logging arguments are accepted and ignored (they
only draw with cv2 / tensorboard).
"""
import contextlib
import types

import torch
import torch.nn as nn

from .algorithms import (DeepRobustEstimator, DirectSolverNet, FeaturePyramid, ImagePyramids, PoseNet, ScaleNet,
                         SFMPoseNet, TrustRegionBase, TrustRegionInverseWUncertainty)
from .submodules import color_normalize
from . import torch_solver as TS
from .. import ic
from .. import torch_ops  # noqa: F401  (registers the dpft:: ops torch.compile traces)

# options attributes the reference constructor reads, with config.py's defaults
DEFAULT_OPTIONS = dict(vis_feat=False, train_uncer_prop=False, combine_ICP=False, feature_extract='average',
                       feature_channel=1, uncertainty_channel=1, scaler='None', remove_tru_sigma=False,
                       init_pose='identity', train_init_pose=False, scale_init_pose=0.01, multi_hypo='None',
                       res_input=False, checkpoint='')


def default_options(**overrides):
    """A namespace with every `options` attribute the constructor reads."""
    d = dict(DEFAULT_OPTIONS)
    d.update(overrides)
    return types.SimpleNamespace(**d)


class LeastSquareTracking(nn.Module):
    NONE = -1
    RGB = 0
    CONV_RGBD = 1
    CONV_RGBD2 = 2

    def __init__(self, encoder_name, uncertainty_type, max_iter_per_pyr, mEst_type, solver_type, tr_samples=10,
                 direction='inverse', options=None, vis_res=False, add_init_noise=False, no_weight_sharing=False,
                 init_pose_type=None, feature_channel=None, uncertainty_channel=None, remove_tru_sigma=None,
                 feature_extract=None, combine_ICP=None, scaler=None, scale_scaler=None, timers=None):
        super().__init__()
        if options is None:
            options = default_options()
        self.scales = [0, 1, 2, 3]
        self.construct_image_pyramids = ImagePyramids(self.scales, pool='avg')
        self.construct_depth_pyramids = ImagePyramids(self.scales, pool='max')
        self.timers = timers
        self.direction = direction
        self.mEst_type = mEst_type
        self.vis_res = vis_res
        self.add_init_noise = add_init_noise

        pick = lambda arg, name: getattr(options, name) if arg is None else arg  # noqa: E731
        self.vis_feat_uncer = options.vis_feat
        self.uncer_prop = options.train_uncer_prop
        self.combine_icp = pick(combine_ICP, 'combine_ICP')
        feature_extract = pick(feature_extract, 'feature_extract')
        self.uncertainty_type = uncertainty_type
        feature_channel = pick(feature_channel, 'feature_channel')
        uncertainty_channel = pick(uncertainty_channel, 'uncertainty_channel')
        scale_type = pick(scaler, 'scaler')
        remove_tru_sigma = pick(remove_tru_sigma, 'remove_tru_sigma')
        init_pose_type = pick(init_pose_type, 'init_pose')
        self.predict_init_pose = init_pose_type != 'identity'
        self.train_init_pose = options.train_init_pose
        self.checkpoint = options.checkpoint

        # ---- feature encoder (LeastSquareTracking.py:105-139)
        if encoder_name in ('RGB', 'ICP'):
            self.encoder = None
            self.encoder_type = self.RGB
        elif encoder_name in ('ConvRGBD', 'ConvRGBD2'):
            self.encoder_type = self.CONV_RGBD if encoder_name == 'ConvRGBD' else self.CONV_RGBD2
            self.encoder = FeaturePyramid(D=4 if encoder_name == 'ConvRGBD' else 8, w_uncertainty=uncertainty_type,
                                          feature_channel=feature_channel, feature_extract=feature_extract,
                                          uncertainty_channel=uncertainty_channel)
        else:
            raise NotImplementedError()
        self._encoder_nhwc = False  # weights moved to channels_last at the first GPU encode

        # ---- per-level helper modules, shared unless no_weight_sharing (143-197)
        def per_level(attr, make):
            if no_weight_sharing:
                mods = [make() for _ in range(4)]
                for i, m in enumerate(mods):
                    setattr(self, f'{attr}{i}', m)
                return mods
            m = make()
            setattr(self, attr, m)
            return [m] * 4

        scaler_funcs = per_level('scaler_func', lambda: ScaleNet(scale_type, scale=scale_scaler))
        mEst_funcs = per_level('mEst_func', lambda: DeepRobustEstimator(mEst_type))
        solver_funcs = per_level('solver_func', lambda: DirectSolverNet(solver_type, samples=tr_samples,
                                                                        direction=direction))

        # ---- trust-region solver per level (203-291)
        if uncertainty_type == 'ICP':
            self.track_type = 'ICP'
        elif uncertainty_type == 'None' and direction == 'inverse':
            self.track_type = 'IC'
        elif uncertainty_type != 'None' and direction == 'forward':
            self.track_type = 'U_FC'
        elif uncertainty_type != 'None' and direction == 'inverse':
            self.track_type = 'U_IC'
        else:
            raise NotImplementedError("Not supported tracking method, check again about the configs of "
                                      "uncertainty and direction.")
        if self.track_type not in ('U_IC', 'IC'):
            raise NotImplementedError(f"track type {self.track_type}: this build implements the U_IC and IC solvers")
        for i in range(4):
            if self.track_type == 'IC':
                solver = TrustRegionBase(max_iter_per_pyr, mEst_func=mEst_funcs[i], solver_func=solver_funcs[i],
                                         timers=timers)
            else:
                solver = TrustRegionInverseWUncertainty(
                    max_iter_per_pyr, mEst_func=mEst_funcs[i], solver_func=solver_funcs[i], timers=timers,
                    combine_icp=self.combine_icp, scale_func=scaler_funcs[i], uncer_prop=options.train_uncer_prop,
                    remove_tru_sigma=remove_tru_sigma)
            setattr(self, f'tr_update{i}', solver)

        # ---- init-pose network (295-309)
        if self.predict_init_pose:
            nets = {'sfm_net': SFMPoseNet, 'dense_net': PoseNet}
            if init_pose_type not in nets:
                raise NotImplementedError('unsupported pose predictor network')
            self.pose_predictor = nets[init_pose_type](scale_motion=options.scale_init_pose,
                                                       multi_hypo=options.multi_hypo, res_input=options.res_input)

    # ------------------------------------------------------------------ API
    def forward(self, img0, img1, depth0, depth1, K, init_only=False, logger=None, iteration=0, vis=False,
                obj_mask0=None, obj_mask1=None, index=None):
        """Coarse-to-fine tracking (LeastSquareTracking.py:311-577); returns [R [B,3,3], t [B,3]]
        (t as the reference's batch_Rt_compose leaves it, geometry.py:122), or in training mode
        the per-level poses stacked, (R [B,L,3,3], t [B,L,3][, JtWJ [B,L,6,6]]) with L = 4 (5 with
        a trained init pose, its pose first), levels 3 .. 0."""
        (I0, I1, x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, poseI) = self._preprocess(
            img0, img1, depth0, depth1, poseI=None, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        if self.training:
            return self._forward_train(x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, poseI, K)
        pose = poseI
        # the weight prior of level 3 (LeastSquareTracking.py:346); each level's returned
        # weights are the next level's prior (375-445) -- read by the IC tracker's learned
        # M-estimator, unused by the U_IC solver (its estimator call is commented out)
        wPrior = torch.ones_like(inv_d0[3]) * 0.001
        # U_IC: the four levels share one status word, read once after the finest level
        # (the reference asserts per iteration; either way a non-finite Jacobian or
        # residual raises AssertionError out of forward and no pose is returned)
        compiling = torch.compiler.is_compiling()
        status = None
        if self.track_type != 'IC' and not compiling and not TS.needs_torch_path(x0[0]):
            status = torch.zeros(1, dtype=torch.int32, device=x0[0].device)
        try:
            for l in (3, 2, 1, 0):
                tr = getattr(self, f'tr_update{l}')
                Kl = K / float(1 << l)
                if self.track_type == 'IC':
                    out = tr(pose, x0[l], x1[l], inv_d0[l], inv_d1[l], Kl, wPrior, vis_res=False,
                             obj_mask0=m0[l], obj_mask1=m1[l])
                    wPrior = out[1]
                elif compiling:  # traced: dpft::ic_solve_level ops, the levels' status words OR-ed
                    out = tr.solve(pose, x0[l], x1[l], inv_d0[l], inv_d1[l], Kl, sigma0[l], sigma1[l], dpt0[l],
                                   dpt1[l], m0[l], m1[l])
                    status = out[3] if status is None else torch.bitwise_or(status, out[3])
                else:
                    tr._deferred_status = status
                    out = tr(pose, x0[l], x1[l], inv_d0[l], inv_d1[l], Kl, sigma0=sigma0[l], sigma1=sigma1[l],
                             wPrior=None, vis_res=False, depth0=dpt0[l], depth1=dpt1[l], obj_mask0=m0[l],
                             obj_mask1=m1[l])
                pose = out[0]
        finally:
            if not compiling:
                for l in (3, 2, 1, 0):
                    getattr(self, f'tr_update{l}')._deferred_status = None
        self.last_status = status
        if compiling:
            # traced (torch.compile): no host read inside the graph -- the caller checks
            # `model.last_status` (ic.check_status), as after a HIP-graph replay
            return pose
        # under HIP-graph capture the host read is deferred to the caller (check
        # `model.last_status` after a replay, e.g. ic.check_status): forward is then
        # capturable whole -- encoder, pyramids and the four levels in one graph
        if status is not None and not torch.cuda.is_current_stream_capturing():
            ic.check_status(status)
        return pose

    def _forward_train(self, x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, poseI, K):
        """Training-mode forward (LeastSquareTracking.py:333-445, 568-575) on the PyTorch path:
        every level's pose (and JtWJ with uncer_prop) collected, gradients kept."""
        poses, sig = [[], []], []
        B = poseI[0].shape[0]
        if self.predict_init_pose and self.train_init_pose:
            poses[0].append(poseI[0])
            poses[1].append(poseI[1].reshape(B, 3))  # the predictors' translation is [B,3]
            if self.uncer_prop:
                sig.append(torch.eye(6, dtype=poseI[0].dtype, device=poseI[0].device).repeat(poseI[0].shape[0], 1, 1))
        pose = poseI
        wPrior = torch.ones_like(inv_d0[3]) * 0.001
        for l in (3, 2, 1, 0):
            tr = getattr(self, f'tr_update{l}')
            Kl = K / float(1 << l)
            if self.track_type == 'IC':
                out = TS.ic_forward(tr, pose, x0[l], x1[l], inv_d0[l], inv_d1[l], Kl, wPrior, m0[l], m1[l])
                wPrior = out[1]
            else:
                lv = tr._torch_level(x0[l], x1[l], inv_d0[l], inv_d1[l], Kl, sigma0[l], sigma1[l], dpt0[l], dpt1[l],
                                     m0[l], m1[l])
                out = TS.uic_solve(pose, lv, tr.max_iterations, want_jtj=self.uncer_prop)
                if self.uncer_prop:
                    sig.append(out[1])
            pose = out[0]
            poses[0].append(pose[0])
            poses[1].append(pose[1].reshape(B, 3))  # [B,3] after an update (geometry.py:122)
        if self.uncer_prop and len(sig) != len(poses[0]):
            raise NotImplementedError("uncer_prop needs the U_IC solver's JtWJ output (the IC tracker returns "
                                      "none, algorithms.py:101)")
        pyr_R, pyr_t = torch.stack(poses[0], dim=1), torch.stack(poses[1], dim=1)
        return (pyr_R, pyr_t, torch.stack(sig, dim=1)) if self.uncer_prop else (pyr_R, pyr_t)

    def compute_residual(self, img0, img1, depth0, depth1, K, poseI=None, level_i=0, logger=None, vis=False,
                         obj_mask0=None, obj_mask1=None):
        """Residual-only loss at `level_i` for pose `poseI` (LeastSquareTracking.py:605-651)."""
        (I0, I1, x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, poseI) = self._preprocess(
            img0, img1, depth0, depth1, poseI=poseI, obj_mask0=obj_mask0, obj_mask1=obj_mask1)
        i = level_i
        if self.track_type == 'IC':  # the IC branch's prior is all ones (LeastSquareTracking.py:641)
            loss = self.tr_update0.forward_residuals(poseI, x0[i], x1[i], inv_d0[i], inv_d1[i], K / float(1 << i),
                                                     torch.ones_like(inv_d0[i]), vis_res=False, obj_mask0=m0[i],
                                                     obj_mask1=m1[i])
        else:
            loss = self.tr_update0.forward_residuals(
                poseI, x0[i], x1[i], inv_d0[i], inv_d1[i], K / float(1 << i), sigma0=sigma0[i], sigma1=sigma1[i],
                wPrior=None, vis_res=False, depth0=dpt0[i], depth1=dpt1[i], obj_mask0=m0[i], obj_mask1=m1[i])
        return poseI, loss

    def prepare(self, img0, img1, depth0, depth1, obj_mask0=None, obj_mask1=None):
        """The preprocessed pyramids (`_preprocess` output) for reuse across many
        residual evaluations -- the convergence-basin sweep computes them once
        instead of once per pose (LeastSquareTracking.py:620)."""
        return self._preprocess(img0, img1, depth0, depth1, poseI=None, obj_mask0=obj_mask0, obj_mask1=obj_mask1)

    def compute_residual_poses(self, prepared, K, R, t, level_i=0):
        """Losses [P,B] of P poses per pair at `level_i` in one launch: pose p is
        what compute_residual(..., poseI=[R[p], t[p]], level_i) returns for the batch."""
        (I0, I1, x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, _) = prepared
        i = level_i
        tr = self.tr_update0
        if TS.needs_torch_path(x0[i]):  # CPU tensors: one residual evaluation per pose
            Ki = K / float(1 << i)
            if self.track_type == 'IC':
                return torch.stack([tr.forward_residuals([R[p], t[p].reshape(-1, 3, 1)], x0[i], x1[i], inv_d0[i],
                                                         inv_d1[i], Ki, torch.ones_like(inv_d0[i]), obj_mask0=m0[i],
                                                         obj_mask1=m1[i]) for p in range(R.shape[0])])
            return torch.stack([tr.forward_residuals([R[p], t[p].reshape(-1, 3, 1)], x0[i], x1[i], inv_d0[i], inv_d1[i],
                                                     Ki, sigma0[i], sigma1[i], depth0=dpt0[i], depth1=dpt1[i],
                                                     obj_mask0=m0[i], obj_mask1=m1[i]) for p in range(R.shape[0])])
        if self.track_type == 'IC':
            if tr._learned_weights():
                raise NotImplementedError("the multi-pose residual sweep uses unit weights; with a learned "
                                          "M-estimator call compute_residual per pose")
            kw = dict(no_uncertainty=True, obj_mask0=m0[i], obj_mask1=m1[i])
        else:
            kw = tr._common(x0[i], dpt0[i], dpt1[i], m0[i], m1[i])
        with torch.no_grad():
            return ic.residual_poses(R, t, x0[i], x1[i], inv_d0[i], inv_d1[i], K / float(1 << i),
                                     sigma0[i], sigma1[i], **kw)

    # ------------------------------------------------------------------ internals
    def _encode(self, img0, invD0, img1, invD1):
        if self.encoder_type == self.RGB:
            B, _, H, W = img0.shape
            grey = (img0[:, 0] * 0.299 + img0[:, 1] * 0.587 + img0[:, 2] * 0.114).view(B, 1, H, W)
            x = self.construct_image_pyramids(grey)
            return x, [torch.ones_like(a) for a in x], x
        if self.encoder_type == self.CONV_RGBD:
            x = torch.cat((img0, invD0), dim=1)
        else:
            x = torch.cat((img0, invD0, img1, invD1), dim=1)
        if x.is_cuda:
            # On the GPU the encoder runs in channels_last memory format: MIOpen's NHWC
            # convolutions skip the NCHW<->NHWC transposes around every layer (13.2 ->
            # 11.1 ms for both frames of 8 pairs at 640x480, C = 32), and the feature heads'
            # epilogue writes the solver's channel-quad layout (_packed_features) -- the same
            # values, laid out differently
            if not self._encoder_nhwc:
                self.encoder.to(memory_format=torch.channels_last)
                self._encoder_nhwc = True
            x = x.contiguous(memory_format=torch.channels_last)
        return self.encoder(x, packed=self._packed_features(x))

    def _packed_features(self, x):
        """The U_IC solve reads the channel-quad layout; its feature heads then write it
        directly (FeaturePyramid(packed=True): the batchnorm + ELU epilogue of each f_conv
        head stores [B,C/4,H,W,4], dpft_bn_elu_pack) instead of NCHW features that every
        level call would relayout (ic.LevelCall).  Needs one uncertainty plane (Cs = 1) and
        C % 4 == 0; the features feed only the solver here (the init-pose networks read the
        backbone maps)."""
        e = self.encoder
        return (x.is_cuda and self.track_type == 'U_IC' and e.feature_extract == 'conv' and e.output_C % 4 == 0
                and e.w_uncertainty and e.uncertainty_type not in ('identity', 'feature') and e.uncertainty_C == 1
                and not self.training and not torch.is_grad_enabled())

    @staticmethod
    def _inverse_depth(depth):
        """clamp(1/depth, 0, 10) with the batch-global min and max zeroed (653-661)."""
        invD = torch.clamp(1.0 / depth, 0, 10)
        invD[invD == invD.min()] = 0
        invD[invD == invD.max()] = 0
        return invD

    def _preprocess(self, img0, img1, depth0, depth1, poseI=None, obj_mask0=None, obj_mask1=None):
        """LeastSquareTracking.py:653-699."""
        if depth0.is_cuda:  # fused device pre-pass (dpft_preprocess_depth), bit-identical to the torch ops
            L = len(self.scales)
            if torch.compiler.is_compiling():  # traced: the dpft::preprocess_depth op
                o0 = torch.ops.dpft.preprocess_depth(depth0, L, bool(self.combine_icp))
                o1 = torch.ops.dpft.preprocess_depth(depth1, L, bool(self.combine_icp))
                inv_d0, inv_d1 = o0[:L], o1[:L]
                dp0, dp1 = (o0[L:], o1[L:]) if self.combine_icp else (None, None)
            else:
                inv_d0, dp0 = ic.preprocess_depth(depth0, L, depth_pyramid=self.combine_icp)
                inv_d1, dp1 = ic.preprocess_depth(depth1, L, depth_pyramid=self.combine_icp)
            invD0, invD1 = inv_d0[0], inv_d1[0]
        else:
            invD0 = self._inverse_depth(depth0)
            invD1 = self._inverse_depth(depth1)
            inv_d0 = self.construct_depth_pyramids(invD0)
            inv_d1 = self.construct_depth_pyramids(invD1)
            dp0 = dp1 = None
        I0 = color_normalize(img0)
        I1 = color_normalize(img1)
        with (contextlib.nullcontext() if self.training else torch.no_grad()):  # training: through the encoder
            x0, sigma0, orig_x0 = self._encode(I0, invD0, I1, invD1)
            x1, sigma1, orig_x1 = self._encode(I1, invD1, I0, invD0)
        if self.combine_icp:
            dpt0 = dp0 if dp0 is not None else self.construct_depth_pyramids(depth0)
            dpt1 = dp1 if dp1 is not None else self.construct_depth_pyramids(depth1)
        else:
            dpt0 = dpt1 = [None] * len(self.scales)
        m0 = self.construct_image_pyramids(obj_mask0) if obj_mask0 is not None else [None] * len(self.scales)
        m1 = self.construct_image_pyramids(obj_mask1) if obj_mask1 is not None else [None] * len(self.scales)
        if poseI is None:
            if self.predict_init_pose:
                with (contextlib.nullcontext() if self.training and self.train_init_pose else torch.no_grad()):
                    R0, t0 = self.pose_predictor(orig_x0[3], orig_x1[3])
            else:
                B = invD0.shape[0]
                # made on the device (the reference builds them on the host and copies,
                # 693-695: a synchronous copy that stalls the host behind the encoder)
                R0 = torch.eye(3, dtype=I0.dtype, device=I0.device).expand(B, 3, 3)
                t0 = torch.zeros(B, 3, 1, dtype=I0.dtype, device=I0.device)
            poseI = [R0, t0]
        return (I0, I1, x0, x1, sigma0, sigma1, dpt0, dpt1, inv_d0, inv_d1, m0, m1, poseI)
