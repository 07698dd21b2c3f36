"""torch.library custom ops over libdpft_ic.so: the drop-in's device calls as `dpft::*` ops.

Each op is a thin functional wrapper of an `ic` entry point (the same C ABI call with the
same arguments), registered with a fake (meta) kernel so that torch.compile / dynamo traces
the drop-in forward as one graph instead of breaking at every ctypes call:

  dpft::ic_solve_level      TrustRegionInverseWUncertainty.forward (algorithms.py:611-723)
                            -> (R [B,3,3], t [B,3,1], JtJ [B,6,6] or [0,6,6], status [1] int32)
  dpft::ic_residual_level   forward_residuals (algorithms.py:725-786) -> loss [B]
  dpft::preprocess_depth    _preprocess's depth part (LeastSquareTracking.py:653-676)
                            -> [invD_0 .. invD_{L-1}] (+ [depth_0 .. depth_{L-1}])
  dpft::pack_features       NCHW / channels_last -> channel-quad layout [B,C/4,H,W,4]
  dpft::bn_elu_             the encoder blocks' eval-mode batchnorm + ELU, in place
  dpft::bn_elu_pack         the feature heads' batchnorm + ELU written to the channel-quad layout

The ops never synchronise: a non-finite Jacobian / residual is reported in the returned
status word, which the caller checks once (the reference's `assert check_nan(...) == 0`,
algorithms.py:886, 1988).  The drop-in (models/) calls them while torch.compile traces it
(`torch.compiler.is_compiling()`); eager calls take the direct ctypes path, which makes the
same library calls without the dispatcher's per-op cost.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import ic


def _level_call(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1, iters,
                remove_tru_sigma, combine_icp, icp_weight, no_uncertainty, status=None):
    return ic.LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=iters, remove_tru_sigma=remove_tru_sigma,
                        obj_mask0=obj_mask0, obj_mask1=obj_mask1, depth0=depth0, depth1=depth1,
                        combine_icp=combine_icp, icp_weight=icp_weight, status=status,
                        no_uncertainty=no_uncertainty, private_workspace=True)


@torch.library.custom_op("dpft::ic_solve_level", mutates_args=())
def ic_solve_level(R: Tensor, t: Tensor, x0: Tensor, x1: Tensor, invD0: Tensor, invD1: Tensor, K: Tensor,
                   sigma0: Optional[Tensor], sigma1: Optional[Tensor], depth0: Optional[Tensor],
                   depth1: Optional[Tensor], obj_mask0: Optional[Tensor], obj_mask1: Optional[Tensor], iters: int,
                   remove_tru_sigma: bool, combine_icp: bool, icp_weight: float, no_uncertainty: bool,
                   return_jtj: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    import ctypes
    status = torch.zeros(1, dtype=torch.int32, device=x0.device)
    c = _level_call(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1, iters,
                    remove_tru_sigma, combine_icp, icp_weight, no_uncertainty, status)
    Ro, to = c.pose_buffers((R, t))
    jtj = torch.empty((c.B if return_jtj else 0), 6, 6, dtype=torch.float32, device=x0.device)
    rc = ic.N.lib().dpft_ic_solve_level(ctypes.byref(c.desc), ctypes.byref(c.tens), ic._ptr(Ro), ic._ptr(to),
                                        ic._ptr(jtj) if return_jtj else None, None, ic._ptr(c.ws), c.ws_bytes,
                                        ic._stream(c.device))
    ic.N.check(rc, "dpft_ic_solve_level")
    return Ro, to.view(c.B, 3, 1), jtj, status


@ic_solve_level.register_fake
def _(R, t, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1, iters,
      remove_tru_sigma, combine_icp, icp_weight, no_uncertainty, return_jtj):
    B = R.shape[0]
    f32 = dict(dtype=torch.float32, device=R.device)  # the real op always returns fp32 (pose_buffers)
    return (torch.empty(B, 3, 3, **f32), torch.empty(B, 3, 1, **f32), torch.empty(B if return_jtj else 0, 6, 6, **f32),
            torch.empty(1, dtype=torch.int32, device=R.device))


@torch.library.custom_op("dpft::ic_residual_level", mutates_args=())
def ic_residual_level(R: Tensor, t: Tensor, x0: Tensor, x1: Tensor, invD0: Tensor, invD1: Tensor, K: Tensor,
                      sigma0: Optional[Tensor], sigma1: Optional[Tensor], depth0: Optional[Tensor],
                      depth1: Optional[Tensor], obj_mask0: Optional[Tensor], obj_mask1: Optional[Tensor],
                      remove_tru_sigma: bool, combine_icp: bool, icp_weight: float,
                      no_uncertainty: bool) -> Tensor:
    import ctypes
    c = _level_call(x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1, 1,
                    remove_tru_sigma, combine_icp, icp_weight, no_uncertainty)
    Rb, tb = c.pose_buffers((R, t))
    loss = torch.empty(c.B, dtype=torch.float32, device=c.device)
    rc = ic.N.lib().dpft_ic_residual_level(ctypes.byref(c.desc), ctypes.byref(c.tens), ic._ptr(Rb), ic._ptr(tb),
                                           ic._ptr(loss), ic._ptr(c.ws), c.ws_bytes, ic._stream(c.device))
    ic.N.check(rc, "dpft_ic_residual_level")
    return loss


@ic_residual_level.register_fake
def _(R, t, x0, x1, invD0, invD1, K, sigma0, sigma1, depth0, depth1, obj_mask0, obj_mask1, remove_tru_sigma,
      combine_icp, icp_weight, no_uncertainty):
    return R.new_empty(R.shape[0])


@torch.library.custom_op("dpft::preprocess_depth", mutates_args=())
def preprocess_depth(depth: Tensor, levels: int, depth_pyramid: bool) -> List[Tensor]:
    ws = torch.zeros(int(ic.N.lib().dpft_preprocess_workspace_size()), dtype=torch.uint8, device=depth.device)
    inv, dep = ic.preprocess_depth(depth, levels, depth_pyramid=depth_pyramid, workspace=ws)
    return inv + (dep if dep is not None else [])


@preprocess_depth.register_fake
def _(depth, levels, depth_pyramid):
    B, _, H, W = depth.shape
    out = [depth.new_empty(B, 1, H >> l, W >> l) for l in range(levels)]
    return out + ([depth.new_empty(B, 1, H >> l, W >> l) for l in range(levels)] if depth_pyramid else [])


@torch.library.custom_op("dpft::pack_features", mutates_args=())
def pack_features(x: Tensor) -> Tensor:
    return ic.pack_features(x)


@pack_features.register_fake
def _(x):
    B, C, H, W = x.shape
    return x.new_empty(B, C // 4, H, W, 4)


@torch.library.custom_op("dpft::bn_elu_", mutates_args=("x",))
def bn_elu_(x: Tensor, chan: Tensor) -> None:
    """x = elu(x * chan[:C] + chan[C:]) in place; x fp32, channels_last with C % 4 == 0 or
    NCHW contiguous with H W % 4 == 0 (ic.bn_elu_ decides; the caller checks first)."""
    B, C, H, W = x.shape
    nhwc = ic.channels_last(x)
    if x.data_ptr() % 16:  # (the kernel's 16-byte accesses; conv outputs are allocator-aligned)
        ic.bn_elu_unaligned_(x, chan)  # the same torch formula the eager path takes here
        return
    rc = ic.N.lib().dpft_bn_elu(ic._ptr(x), ic._ptr(chan), x.numel(), C, 1 if nhwc else H * W, 1 if nhwc else 0,
                                ic._stream(x.device))
    ic.N.check(rc, "dpft_bn_elu")


@bn_elu_.register_fake
def _(x, chan):
    return None


@torch.library.custom_op("dpft::bn_elu_pack", mutates_args=())
def bn_elu_pack(x: Tensor, chan: Tensor) -> Tensor:
    """ELU(x a + b) of a channels_last map, out of place in the channel-quad layout
    [B,C/4,H,W,4] (dpft_bn_elu_pack; ic.bn_elu_pack_applies decides)."""
    B, C, H, W = x.shape
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.channels_last)
    out = torch.empty(B, C // 4, H, W, 4, dtype=torch.float32, device=x.device)
    rc = ic.N.lib().dpft_bn_elu_pack(ic._ptr(x), ic._ptr(chan), ic._ptr(out), B, C, H, W, ic._stream(x.device))
    ic.N.check(rc, "dpft_bn_elu_pack")
    return out


@bn_elu_pack.register_fake
def _(x, chan):
    B, C, H, W = x.shape
    return x.new_empty(B, C // 4, H, W, 4)


def bn_elu_applies(x, bn):
    """The layouts dpft_bn_elu takes (traceable: shapes, strides, dtype only)."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or bn.running_mean is None:
        return False
    B, C, H, W = x.shape
    if C != bn.num_features:
        return False
    if ic.channels_last(x):
        return C % 4 == 0
    return x.is_contiguous() and (H * W) % 4 == 0


def bn_coeffs(bn):
    """[a | b] of an eval-mode BatchNorm2d as torch ops (what ic._bn_coeffs caches in eager,
    the same operations in the same order: the same bits)."""
    a = 1.0 / torch.sqrt(bn.running_var.float() + bn.eps)
    if bn.affine:
        a = a * bn.weight.float()
    b = -bn.running_mean.float() * a
    if bn.affine:
        b = b + bn.bias.float()
    return torch.cat((a, b)).contiguous()

