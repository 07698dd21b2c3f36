"""Torch-facing entry points of the HIP solver (device tensors in, device tensors out).

These are thin marshalling functions over libdpft_ic.so: they validate shapes,
pick the uncertainty layout (Cs = 1 when sigma is a broadcast view or has one
channel, Cs = C otherwise), hand raw device pointers and the caller's current
HIP stream to the C ABI and never synchronise -- except `check_status`, which
reads the device status word once (the reference asserts finiteness with a
host sync every iteration, algorithms.py:886, 1988).

Reference counterparts: `TrustRegionInverseWUncertainty.forward` /
`forward_residuals` (code/models/algorithms.py:611-786).
"""
import ctypes
import os

import torch

from . import _native as N

MAX_PAIRS_PER_CALL = 2048  # pairs per library call (kMaxPairs: one completion counter each)

_ws_cache = {}
_ws_retired = []


def _eager_only(fn):
    """ctypes calls are opaque to dynamo: under torch.compile these run eagerly (a graph
    break) -- the drop-in's traced path uses the dpft:: ops of torch_ops.py instead."""
    return torch.compiler.disable(fn, recursive=True)


def _workspace(device, nbytes):
    """The per-(device, stream) workspace of the one-call entry points: one per stream
    because concurrent launches must not share completion counters (dpft_ic.h).  A
    buffer outgrown by a larger call is kept alive, not freed: a HIP graph captured
    with it still replays into it."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None:
            _ws_retired.append(buf)
        # zero-filled once: the library's completion counters live in it (dpft_ic.h)
        buf = torch.zeros(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _sigma_planes(sigma, B, C, H, W):
    """Return (tensor, Cs).  A channel-broadcast view ([B,1,H,W] expanded, stride 0)
    or a single-channel tensor is passed with Cs=1 -- the reference's `.repeat`
    (algorithms.py:1426-1427) carries no extra information."""
    if sigma.dim() != 4 or sigma.shape[0] != B or sigma.shape[2:] != (H, W):
        raise ValueError(f"sigma shape {tuple(sigma.shape)} incompatible with features [{B},{C},{H},{W}]")
    if sigma.shape[1] == 1:
        return sigma.contiguous(), 1
    if sigma.shape[1] != C:
        raise ValueError(f"sigma has {sigma.shape[1]} channels, expected 1 or {C}")
    if sigma.stride(1) == 0:
        return sigma[:, :1].contiguous(), 1
    return sigma.contiguous(), C


@_eager_only
def pack_features(x):
    """Feature map [B,C,H,W] -> channel-quad layout [B,C/4,H,W,4] (dpft_pack_features).

    The packed tensor holds the same values; the solver reads 4 channels of a pixel /
    bilinear tap with one coalesced 16-byte load (DPFT_FEATURES_C4).  Every solver
    entry point accepts either form for x0 / x1."""
    if not x.is_cuda:
        raise RuntimeError("pack_features needs a device tensor; there is no CPU fallback")
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] % 4 != 0:
        raise ValueError(f"need fp32 [B,C,H,W] with C % 4 == 0, got {x.dtype} {tuple(x.shape)}")
    B, C, H, W = x.shape
    out = torch.empty(B, C // 4, H, W, 4, dtype=torch.float32, device=x.device)
    if channels_last(x):  # NHWC storage: one relayout pass (dpft_pack_features_nhwc)
        if x.data_ptr() % 16:
            x = x.contiguous(memory_format=torch.channels_last)
        rc = N.lib().dpft_pack_features_nhwc(_ptr(x), _ptr(out), B, C, H, W, _stream(x.device))
        N.check(rc, "dpft_pack_features_nhwc")
        return out
    x = x.contiguous()
    rc = N.lib().dpft_pack_features(_ptr(x), _ptr(out), B, C, H, W, _stream(x.device))
    N.check(rc, "dpft_pack_features")
    return out


def _bn_coeffs(bn, device):
    """[a | b] (2C fp32 on `device`) of an eval-mode BatchNorm2d: a = w / sqrt(var + eps),
    b = bias - mean * a.  Cached on the module until its statistics or affine parameters
    change (in-place updates such as load_state_dict bump the tensor versions)."""
    ts = [bn.running_mean, bn.running_var] + ([bn.weight, bn.bias] if bn.affine else [])
    key = (device,) + tuple(t._version for t in ts) + tuple(t.data_ptr() for t in ts)
    hit = getattr(bn, "_dpft_coeffs", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        a = 1.0 / torch.sqrt(bn.running_var.float() + bn.eps)
        if bn.affine:
            a = a * bn.weight.float()
        b = -bn.running_mean.float() * a
        if bn.affine:
            b = b + bn.bias.float()
        chan = torch.cat((a, b)).to(device=device, dtype=torch.float32).contiguous()
    bn._dpft_coeffs = (key, chan)
    return chan


@_eager_only
def bn_elu_(x, bn):
    """In place x = ELU(bn(x)) for an eval-mode BatchNorm2d with running statistics
    (the reference's convLayer epilogue, submodules.py:25-39) in one pass
    (dpft_bn_elu).  Returns False, x untouched, when x's layout does not fit the kernel
    (the caller then runs the two torch modules)."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or bn.running_mean is None:
        return False
    B, C, H, W = x.shape
    if channels_last(x):
        nhwc, inner, ok = 1, 1, C % 4 == 0
    elif x.is_contiguous():
        nhwc, inner, ok = 0, H * W, (H * W) % 4 == 0
    else:
        return False
    if not ok or C != bn.num_features:
        return False
    chan = _bn_coeffs(bn, x.device)
    if x.data_ptr() % 16:  # the kernel's 16-byte accesses (conv outputs are allocator-aligned)
        bn_elu_unaligned_(x, chan)
        return True
    rc = N.lib().dpft_bn_elu(_ptr(x), _ptr(chan), x.numel(), C, inner, nhwc, _stream(x.device))
    N.check(rc, "dpft_bn_elu")
    return True


def bn_elu_pack_applies(x, bn):
    """The conv outputs dpft_bn_elu_pack takes: an fp32 channels_last map with C % 4 == 0 on
    the device, an eval-mode BatchNorm2d with running statistics (traceable: shapes,
    strides, dtype only; alignment is checked at the call)."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and bn.running_mean is not None
            and x.shape[1] == bn.num_features and x.shape[1] % 4 == 0 and channels_last(x))


@_eager_only
def bn_elu_pack(x, bn):
    """ELU(bn(x)) of a channels_last conv output, written to the channel-quad layout
    [B,C/4,H,W,4] the solver reads (dpft_bn_elu_pack): the feature heads' epilogue
    (algorithms.py:1273-1277) and the relayout in one pass.  The values are those of
    bn_elu_ + pack_features."""
    B, C, H, W = x.shape
    chan = _bn_coeffs(bn, x.device)
    if x.data_ptr() % 16:
        x = x.contiguous(memory_format=torch.channels_last).clone(memory_format=torch.channels_last)
    out = torch.empty(B, C // 4, H, W, 4, dtype=torch.float32, device=x.device)
    rc = N.lib().dpft_bn_elu_pack(_ptr(x), _ptr(chan), _ptr(out), B, C, H, W, _stream(x.device))
    N.check(rc, "dpft_bn_elu_pack")
    return out


def bn_elu_unaligned_(x, chan):
    """x = ELU(x a + b) in place by torch ops, for a map the kernel cannot take (not 16-byte
    aligned): the formula of dpft_bn_elu, shared by the eager path and the dpft::bn_elu_ op so
    that compiled and eager forwards agree."""
    C = x.shape[1]
    a, b = chan[:C].view(1, C, 1, 1), chan[C:].view(1, C, 1, 1)
    x.copy_(torch.nn.functional.elu(x * a + b))


def channels_last(x):
    """True for a 4-D map stored channels_last (NHWC) rather than NCHW -- the encoder's
    output when it runs in torch.channels_last memory format."""
    return x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)


def unpack_features(xp):
    """Inverse of pack_features (a torch view + copy; tests / inspection only)."""
    B, Q, H, W, _ = xp.shape
    return xp.permute(0, 1, 4, 2, 3).reshape(B, 4 * Q, H, W).contiguous()


def packable(x, sigma=None, no_uncertainty=False):
    """True when `x` [B,C,H,W] may run in the channel-quad layout: C % 4 == 0 and
    one sigma plane (a [B,1,H,W] map or its channel broadcast) or no uncertainty."""
    if x.dim() != 4 or x.shape[1] % 4 != 0 or not x.is_cuda:
        return False
    if no_uncertainty:
        return True
    return sigma is not None and sigma.dim() == 4 and (sigma.shape[1] == 1 or sigma.stride(1) == 0)


def feature_shape(x):
    """(B, C, H, W) of a feature map in either layout."""
    if x.dim() == 5:
        B, Q, H, W, four = x.shape
        if four != 4:
            raise ValueError(f"packed features must be [B,C/4,H,W,4], got {tuple(x.shape)}")
        return B, 4 * Q, H, W
    return tuple(x.shape)


class LevelCall:
    """Validated, pointer-ready arguments of one pyramid level.

    x0 / x1 are [B,C,H,W] (NCHW or channels_last) or channel-quad packed
    [B,C/4,H,W,4]; eligible inputs are packed here (once for all iterations) when
    pack=True or when they are stored channels_last.
    schedule (None = "auto", "march", "split") forces the channel-quad
    reduce kernel (include/dpft_ic.h, DPFT_SCHED_*); it changes only the order in
    which the per-pixel sums are added."""

    def __init__(self, x0, x1, invD0, invD1, K, sigma0, sigma1, iters=3, remove_tru_sigma=False,
                 obj_mask0=None, obj_mask1=None, depth0=None, depth1=None, combine_icp=False,
                 icp_weight=0.01, status=None, no_uncertainty=False, pack=False, schedule=None, weights=None,
                 group=None, private_workspace=False):
        if not x0.is_cuda:
            raise RuntimeError("the HIP solver needs device tensors (got CPU); there is no CPU fallback")
        for name, t in (("x0", x0), ("x1", x1), ("invD0", invD0), ("invD1", invD1), ("K", K)):
            if t.dtype != torch.float32:
                raise TypeError(f"{name} must be float32 (got {t.dtype})")
            if t.device != x0.device:
                raise ValueError(f"{name} is on {t.device}, expected {x0.device}")
        if x1.shape != x0.shape:
            raise ValueError(f"x1 {tuple(x1.shape)} != x0 {tuple(x0.shape)}")
        # channels_last maps need a relayout pass either way: make it the one to the
        # channel-quad layout (the faster solve) whenever the level is packable
        if packable(x0, sigma0, no_uncertainty) and (pack or channels_last(x0) or channels_last(x1)):
            x0, x1 = pack_features(x0), pack_features(x1)
        c4 = x0.dim() == 5
        B, C, H, W = feature_shape(x0)
        for name, t in (("invD0", invD0), ("invD1", invD1)):
            if tuple(t.shape) != (B, 1, H, W):
                raise ValueError(f"{name} shape {tuple(t.shape)} != {(B, 1, H, W)}")
        self.device = x0.device
        self.x0, self.x1 = x0.contiguous(), x1.contiguous()
        if no_uncertainty:  # IC tracker (TrustRegionBase): sigma = 1, no sigma planes
            self.s0 = self.s1 = None
            cs0 = 1
        else:
            self.s0, cs0 = _sigma_planes(sigma0, B, C, H, W)
            self.s1, cs1 = _sigma_planes(sigma1, B, C, H, W)
            if cs0 != cs1:  # mixed layouts: full planes for both
                self.s0, self.s1, cs0 = (sigma0.expand(B, C, H, W).contiguous(),
                                         sigma1.expand(B, C, H, W).contiguous(), C)
        self.invD0, self.invD1 = invD0.contiguous(), invD1.contiguous()
        self.K = K.reshape(B, 4).contiguous()
        self.m0 = obj_mask0.reshape(B, 1, H, W).to(torch.uint8).contiguous() if obj_mask0 is not None else None
        self.m1 = obj_mask1.reshape(B, 1, H, W).to(torch.uint8).contiguous() if obj_mask1 is not None else None
        flags = N.REMOVE_TRU_SIGMA if remove_tru_sigma else 0
        if c4:
            if cs0 != 1 and not no_uncertainty:
                raise ValueError("packed features need a single sigma plane ([B,1,H,W] or its broadcast)")
            flags |= N.FEATURES_C4
        if no_uncertainty:
            flags |= N.NO_UNCERTAINTY
        if schedule is not None:  # channel-quad reduce kernel override (tests / tuning)
            if schedule not in N.SCHEDULES:
                raise ValueError(f"schedule must be one of {sorted(N.SCHEDULES)} (got {schedule!r})")
            flags |= N.SCHEDULES[schedule]
        if combine_icp:
            if depth0 is None or depth1 is None:
                raise ValueError("combine_icp needs depth0 and depth1")
            flags |= N.COMBINE_ICP
        if weights is not None:  # IC tracker's M-estimator weights, one per pixel
            if not no_uncertainty:
                raise ValueError("per-pixel weights belong to the IC tracker (no_uncertainty=True)")
            if weights.numel() != B * H * W:
                raise ValueError(f"weights must hold one value per pixel [B,1,H,W] (got {tuple(weights.shape)})")
            weights = weights.reshape(B, 1, H, W).to(torch.float32).contiguous()
        self.w = weights
        self.d0 = depth0.contiguous() if depth0 is not None else None
        self.d1 = depth1.contiguous() if depth1 is not None else None
        self.status = status if status is not None else torch.zeros(1, dtype=torch.int32, device=self.device)
        if group is not None and group < B:  # independent batches of `group` pairs (DPFT_GROUP)
            if group < 1 or B % group or B // group > N.GROUP_MAX_BATCHES:
                raise ValueError(f"group={group}: B={B} must be a multiple, at most {N.GROUP_MAX_BATCHES} batches")
            flags |= group << N.GROUP_SHIFT
        self.desc = N.LevelDesc(B, C, cs0, H, W, iters, flags, icp_weight)
        self.tens = N.LevelTensors(_ptr(self.x0), _ptr(self.x1), _ptr(self.s0), _ptr(self.s1), _ptr(self.invD0),
                                   _ptr(self.invD1), _ptr(self.d0), _ptr(self.d1), _ptr(self.m0), _ptr(self.m1),
                                   _ptr(self.K), _ptr(self.status), _ptr(self.w))
        self.B = B
        nbytes = N.lib().dpft_workspace_size(ctypes.byref(self.desc))
        if nbytes == 0:
            N.check(-1, "dpft_workspace_size")
        self.ws_bytes = nbytes
        # private_workspace: a zero-filled buffer of this call's own (the dpft:: ops: a
        # buffer cached across calls would outlive a torch.compile CUDA-graph capture)
        if private_workspace:  # only the control words (completion counters) must start at zero
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self.ws[:min(nbytes, N.CTRL_BYTES)].zero_()
        else:
            self.ws = _workspace(self.device, nbytes)

    def pose_buffers(self, pose):
        R, t = pose
        R = R.to(torch.float32).reshape(self.B, 3, 3).contiguous().clone()
        t = t.to(torch.float32).reshape(self.B, 3).contiguous().clone()
        return R, t


@_eager_only
def check_status(status):
    """Mirror of `assert check_nan(...) == 0` (algorithms.py:886, 1988): one host read."""
    if int(status.item()) & N.STATUS_NONFINITE:
        raise AssertionError("non-finite Jacobian / residual in the IC solver (reference: check_nan assert)")


@_eager_only
def solve_level(pose, x0, x1, invD0, invD1, K, sigma0, sigma1, iters=3, return_jtj=False, check=True, **kw):
    """`iters` Gauss-Newton steps at one level; returns (R [B,3,3], t [B,3,1][, JtJ [B,6,6]]).
    pack=True (keyword) packs eligible NCHW features first (pays off from 2 iterations)."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=iters, **kw)
    R, t = c.pose_buffers(pose)
    jtj = torch.empty(c.B, 6, 6, dtype=torch.float32, device=c.device) if return_jtj else None
    rc = N.lib().dpft_ic_solve_level(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), _ptr(jtj),
                                     None, _ptr(c.ws), c.ws_bytes, _stream(c.device))
    N.check(rc, "dpft_ic_solve_level")
    if check:
        check_status(c.status)
    out = (R, t.view(c.B, 3, 1))
    return out + (jtj,) if return_jtj else out


@_eager_only
def iterate(pose, x0, x1, invD0, invD1, K, sigma0, sigma1, first=True, reverse=False, update=True, **kw):
    """One iteration; returns (R, t [B,3,1], JtJ [B,6,6], JtR [B,6], invalid [B]) -- test / trace API.
    reverse=True: the marching order of the solve's odd iterations (DPFT_ITER_REVERSE).
    update=False: the normal equations at `pose` only, R / t returned unchanged
    (DPFT_ITER_NO_UPDATE, the residual-volume samples of 'Direct-ResVol')."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=1, **kw)
    R, t = c.pose_buffers(pose)
    jtj = torch.empty(c.B, 6, 6, dtype=torch.float32, device=c.device)
    jtr = torch.empty(c.B, 6, dtype=torch.float32, device=c.device)
    inv = torch.empty(c.B, dtype=torch.int32, device=c.device)
    rc = N.lib().dpft_ic_iterate(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), _ptr(jtj), _ptr(jtr),
                                 _ptr(inv), (N.ITER_FIRST if first else 0) | (N.ITER_REVERSE if reverse else 0) |
                                 (0 if update else N.ITER_NO_UPDATE), _ptr(c.ws), c.ws_bytes, _stream(c.device))
    N.check(rc, "dpft_ic_iterate")
    return R, t.view(c.B, 3, 1), jtj, jtr, inv


@_eager_only
def iterate_poses(R, t, x0, x1, invD0, invD1, K, sigma0, sigma1, **kw):
    """J^T J and J^T R at S poses per pair, no update: R [S,B,3,3], t [S,B,3(,1)] ->
    (JtJ [S,B,6,6], JtR [S,B,6]).  One validated LevelCall (workspace, pointers) for all
    S, then S dpft_ic_iterate calls with DPFT_ITER_NO_UPDATE on the current stream --
    the residual-volume samples of 'Direct-ResVol' (algorithms.py:1668-1685)."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=1, **kw)
    S = R.shape[0]
    R = R.to(torch.float32).reshape(S, c.B, 3, 3).contiguous()
    t = t.to(torch.float32).reshape(S, c.B, 3).contiguous()
    jtj = torch.empty(S, c.B, 6, 6, dtype=torch.float32, device=c.device)
    jtr = torch.empty(S, c.B, 6, dtype=torch.float32, device=c.device)
    st = _stream(c.device)
    for s in range(S):
        rc = N.lib().dpft_ic_iterate(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R[s]), _ptr(t[s]),
                                     _ptr(jtj[s]), _ptr(jtr[s]), None, N.ITER_NO_UPDATE, _ptr(c.ws), c.ws_bytes, st)
        N.check(rc, "dpft_ic_iterate")
    return jtj, jtr


# ------------------------------------------------------------------ Jacobian API (materialised)
def _dev_f32(name, t):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: the HIP kernels need device tensors (got CPU); there is no CPU fallback")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


@_eager_only
def feature_gradient(f):
    """Unit-normalised Sobel (feature_gradient, algorithms.py:1844-1865): f [B,C,H,W] ->
    [B,C,2,H,W], (x, y) stacked on dim 2 as precompute_jacobian_components stacks them."""
    f = _dev_f32("f", f)
    B, C, H, W = f.shape
    g = torch.empty(B, C, 2, H, W, dtype=torch.float32, device=f.device)
    N.check(N.lib().dpft_feature_gradient(_ptr(f), _ptr(g), B, C, H, W, _stream(f.device)), "dpft_feature_gradient")
    return g


@_eager_only
def warp_jacobian(invD0, K, px, py):
    """compute_jacobian_warping at the origin (algorithms.py:1884-1917) -> Jx, Jy [B,HW,6]."""
    invD0 = _dev_f32("invD0", invD0)
    B, _, H, W = invD0.shape
    K = _dev_f32("K", K.reshape(B, 4))
    px = _dev_f32("px", px.expand(B, 1, H, W))
    py = _dev_f32("py", py.expand(B, 1, H, W))
    Jx = torch.empty(B, H * W, 6, dtype=torch.float32, device=invD0.device)
    Jy = torch.empty_like(Jx)
    N.check(N.lib().dpft_warp_jacobian(_ptr(invD0), _ptr(K), _ptr(px), _ptr(py), _ptr(Jx), _ptr(Jy), B, H, W,
                                       _stream(invD0.device)), "dpft_warp_jacobian")
    return Jx, Jy


@_eager_only
def inverse_jacobian(res, sigma, sigma0, grad_f0, grad_sigma0, Jx, Jy):
    """compose_inverse_jacobians' J (algorithms.py:867-887): [B,C,HW,6], not masked.
    sigma0 / grad_sigma0 may carry one channel or C (a channel broadcast is read once)."""
    B, C, H, W = res.shape
    res, sigma = _dev_f32("res", res), _dev_f32("sigma", sigma.expand(B, C, H, W))
    s0, gs0 = sigma0, grad_sigma0
    if s0.shape[1] != 1 and s0.stride(1) == 0:
        s0, gs0 = s0[:, :1], gs0[:, :1]
    Cs = s0.shape[1]
    s0, gs0 = _dev_f32("sigma0", s0), _dev_f32("grad_sigma0", gs0)
    gf0 = _dev_f32("grad_f0", grad_f0)
    Jx, Jy = _dev_f32("Jx", Jx), _dev_f32("Jy", Jy)
    J = torch.empty(B, C, H * W, 6, dtype=torch.float32, device=res.device)
    N.check(N.lib().dpft_inverse_jacobian(_ptr(res), _ptr(sigma), _ptr(s0), _ptr(gf0), _ptr(gs0), _ptr(Jx), _ptr(Jy),
                                          _ptr(J), B, C, Cs, H, W, _stream(res.device)), "dpft_inverse_jacobian")
    return J


@_eager_only
def normal_equations(J, r=None):
    """compute_jtj / compute_jtr (algorithms.py:812-834): J [B,...,6] (rows = every
    channel and pixel), r [B,...] -> (JtJ [B,6,6], JtR [B,6,1] or None); fixed-order fp64."""
    J = _dev_f32("J", J)
    B = J.shape[0]
    n = J.numel() // (6 * B)
    if r is not None:
        r = _dev_f32("r", r)
        if r.numel() != B * n:
            raise ValueError(f"r has {r.numel()} values, J has {B * n} rows")
    L = N.lib()
    nbytes = L.dpft_normal_equations_workspace_size(B)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=J.device)
    jtj = torch.empty(B, 6, 6, dtype=torch.float32, device=J.device)
    jtr = torch.empty(B, 6, 1, dtype=torch.float32, device=J.device) if r is not None else None
    N.check(L.dpft_normal_equations(_ptr(J), _ptr(r), n, B, _ptr(jtj), _ptr(jtr), _ptr(ws), nbytes,
                                    _stream(J.device)), "dpft_normal_equations")
    return jtj, jtr


@_eager_only
def damped_update(JtJ, JtR, diag_add, pose):
    """S damped inverse-compositional updates per pair in one launch (dpft_ic_damped_update):
    JtJ [B,6,6], JtR [B,6], diag_add [S,B,6] or None (S = 1), pose ([B,3,3], [B,3(,1)])
    -> (R [S,B,3,3], t [S,B,3,1])."""
    R, t = pose
    dev = JtJ.device
    B = JtJ.shape[0]
    jtj = JtJ.to(torch.float32).reshape(B, 36).contiguous()
    jtr = JtR.to(torch.float32).reshape(B, 6).contiguous()
    R = R.to(torch.float32).reshape(B, 9).contiguous()
    t = t.to(torch.float32).reshape(B, 3).contiguous()
    if diag_add is not None:
        diag_add = diag_add.to(torch.float32).reshape(-1, B, 6).contiguous()
    S = diag_add.shape[0] if diag_add is not None else 1
    R_out = torch.empty(S, B, 3, 3, dtype=torch.float32, device=dev)
    t_out = torch.empty(S, B, 3, 1, dtype=torch.float32, device=dev)
    rc = N.lib().dpft_ic_damped_update(_ptr(jtj), _ptr(jtr), _ptr(diag_add), S, B, _ptr(R), _ptr(t), _ptr(R_out),
                                       _ptr(t_out), _stream(dev))
    N.check(rc, "dpft_ic_damped_update")
    return R_out, t_out


@_eager_only
def residual_map(pose, x0, x1, invD0, invD1, K, **kw):
    """IC tracker residuals at `pose` (compute_warped_residual, algorithms.py:1919-1957):
    (r [B,C,H,W] with 1e-3 on occluded / masked pixels, occ [B,1,H,W] bool)."""
    kw = dict(kw, no_uncertainty=True)
    c = LevelCall(x0, x1, invD0, invD1, K, None, None, iters=1, **kw)
    R, t = c.pose_buffers(pose)
    B, C, H, W = feature_shape(c.x0)
    out = torch.empty(B, C, H, W, dtype=torch.float32, device=c.device)
    occ = torch.empty(B, 1, H, W, dtype=torch.uint8, device=c.device)
    rc = N.lib().dpft_ic_residual_map(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), _ptr(out),
                                      _ptr(occ), _ptr(c.ws), c.ws_bytes, _stream(c.device))
    N.check(rc, "dpft_ic_residual_map")
    return out, occ.bool()


@_eager_only
def residual_level(pose, x0, x1, invD0, invD1, K, sigma0, sigma1, **kw):
    """forward_residuals: per-pair average loss [B] at a fixed pose."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=1, **kw)
    R, t = c.pose_buffers(pose)
    loss = torch.empty(c.B, dtype=torch.float32, device=c.device)
    rc = N.lib().dpft_ic_residual_level(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), _ptr(loss),
                                        _ptr(c.ws), c.ws_bytes, _stream(c.device))
    N.check(rc, "dpft_ic_residual_level")
    return loss


@_eager_only
def residual_poses(R, t, x0, x1, invD0, invD1, K, sigma0, sigma1, **kw):
    """forward_residuals for P poses per pair in one launch: R [P,B,3,3], t [P,B,3(,1)] -> loss [P,B].

    Each pose index is evaluated as one reference call over the batch (its own
    batch-global truncated-sigma extrema)."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=1, **kw)
    P = R.shape[0]
    if R.shape[1] != c.B or t.shape[:2] != (P, c.B):
        raise ValueError(f"poses R {tuple(R.shape)}, t {tuple(t.shape)} do not match B={c.B}")
    Rb = R.to(torch.float32).reshape(P, c.B, 9).contiguous()
    tb = t.to(torch.float32).reshape(P, c.B, 3).contiguous()
    loss = torch.empty(P, c.B, dtype=torch.float32, device=c.device)
    L = N.lib()
    nbytes = L.dpft_residual_poses_workspace_size(ctypes.byref(c.desc), P)
    if nbytes == 0:
        N.check(-1, "dpft_residual_poses_workspace_size")
    ws = _workspace(c.device, nbytes)
    rc = L.dpft_ic_residual_poses(ctypes.byref(c.desc), ctypes.byref(c.tens), P, _ptr(Rb), _ptr(tb), _ptr(loss),
                                  _ptr(ws), nbytes, _stream(c.device))
    N.check(rc, "dpft_ic_residual_poses")
    return loss


@_eager_only
def preprocess_depth(depth, levels=4, depth_pyramid=False, workspace=None):
    """LeastSquareTracking._preprocess on the device: invD = clamp(1/depth, 0, 10) with the
    batch-global min then max zeroed, and MaxPool(2^l) pyramids of invD (and of depth).
    depth [B,1,H,W] fp32 on a HIP device -> ([invD_l], [depth_l] or None)."""
    if not depth.is_cuda:
        raise RuntimeError("preprocess_depth needs a device tensor; there is no CPU fallback")
    if depth.dtype != torch.float32 or depth.dim() != 4 or depth.shape[1] != 1:
        raise ValueError(f"depth must be fp32 [B,1,H,W], got {depth.dtype} {tuple(depth.shape)}")
    d = depth.contiguous()
    B, _, H, W = d.shape
    inv = [torch.empty(B, 1, H >> l, W >> l, dtype=torch.float32, device=d.device) for l in range(levels)]
    dep = [torch.empty_like(t) for t in inv] if depth_pyramid else None
    arr = (ctypes.c_void_p * levels)(*[t.data_ptr() for t in inv])
    darr = (ctypes.c_void_p * levels)(*[t.data_ptr() for t in dep]) if dep else None
    L = N.lib()
    nbytes = L.dpft_preprocess_workspace_size()
    ws = workspace if workspace is not None else _workspace(d.device, nbytes)
    rc = L.dpft_preprocess_depth(_ptr(d), B, H, W, levels, arr, darr, _ptr(ws), nbytes, _stream(d.device))
    N.check(rc, "dpft_preprocess_depth")
    return inv, dep


@_eager_only
def debug_pixels(pose, x0, x1, invD0, invD1, K, sigma0, sigma1, **kw):
    """Per-pixel dump [B,5,H,W] (u, v, sigma_r ch0, sigma0 ch0, occlusion|mask invalid) -- tests only."""
    c = LevelCall(x0, x1, invD0, invD1, K, sigma0, sigma1, iters=1, **kw)
    R, t = c.pose_buffers(pose)
    _, _, H, W = feature_shape(x0)
    out = torch.empty(c.B, 5, H, W, dtype=torch.float32, device=c.device)
    rc = N.lib().dpft_ic_debug_pixels(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), _ptr(out),
                                      _ptr(c.ws), c.ws_bytes, _stream(c.device))
    N.check(rc, "dpft_ic_debug_pixels")
    return out


class PyramidSolver:
    """Coarse-to-fine solve over prepared levels with fixed device buffers.

    Mirrors `LeastSquareTracking.forward`'s level loop (LeastSquareTracking.py:349-445):
    levels L-1 .. 0, K / 2^l, pose chained, `iters` steps per level.  All levels share
    one workspace and one status word, and `run()` only enqueues kernels on the
    current stream with fixed pointers, so it can be captured once into a HIP graph
    and replayed.  `levels[l]` = dict(x0, x1, invD0, invD1, sigma0, sigma1[, obj_mask0,
    obj_mask1, depth0, depth1]); K is the level-0 intrinsics [B,4].
    """

    def __init__(self, levels, K, iters=3, remove_tru_sigma=False, combine_icp=False, icp_weight=0.01,
                 schedule=None, group=None):
        """group: pairs per independent batch (DPFT_GROUP).  The B pairs are then B / group
        consecutive batches, each solved exactly as its own call -- its own batch-global
        truncated-sigma extrema -- in launches that cover all of them (fewer, larger
        launches); None = one batch."""
        dev = levels[0]["x0"].device
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.calls = []
        for l, d in enumerate(levels):
            self.calls.append(LevelCall(d["x0"], d["x1"], d["invD0"], d["invD1"], (K / (2 ** l)).contiguous(),
                                        d["sigma0"], d["sigma1"], iters=iters, remove_tru_sigma=remove_tru_sigma,
                                        obj_mask0=d.get("obj_mask0"), obj_mask1=d.get("obj_mask1"),
                                        depth0=d.get("depth0"), depth1=d.get("depth1"), combine_icp=combine_icp,
                                        icp_weight=icp_weight, status=self.status, schedule=schedule))
        # One pose-independent pre-pass for every level's sigma0 extrema (truncated
        # sigma): each level keeps them in its own workspace slot and skips the
        # per-level min/max launch (dpft_sigma_extrema_levels, DPFT_EXTREMA_READY).
        # (combine_icp: each level's first iteration still takes its depth1 extrema and
        # builds frame 1's normal map -- per independent batch with `group`.)
        B = self.calls[0].B
        if group is not None and group < B:
            if group < 1 or B % group or B // group > N.GROUP_MAX_BATCHES or group >= 4096:
                raise ValueError(f"group={group}: B={B} must be a multiple, at most {N.GROUP_MAX_BATCHES} batches")
            for c in self.calls:
                c.desc.flags |= group << N.GROUP_SHIFT
        self.group = group if group is not None and group < B else B
        self.remove_tru_sigma = bool(remove_tru_sigma)
        self.combine_icp = bool(combine_icp)
        self.extrema_prepass = bool(remove_tru_sigma) and len(self.calls) <= 4
        if self.extrema_prepass:
            for l, c in enumerate(self.calls):
                c.desc.flags |= ((l + 1) << N.EXT_SLOT_SHIFT) | N.EXTREMA_READY
            self._descs = (N.LevelDesc * len(self.calls))(*[c.desc for c in self.calls])
            self._tens = (N.LevelTensors * len(self.calls))(*[c.tens for c in self.calls])
        nbytes = max(c.ws_bytes for c in self.calls)
        self.ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)  # private: safe to capture; zeroed (counters)
        self.ws_bytes = nbytes
        self.device = dev
        self.B = self.calls[0].B

    def prepare_extrema(self):
        """The sigma0 extrema of every level in one launch (run() does this first)."""
        if self.extrema_prepass:
            rc = N.lib().dpft_sigma_extrema_levels(self._descs, self._tens, len(self.calls), _ptr(self.ws),
                                                   self.ws_bytes, _stream(self.device))
            N.check(rc, "dpft_sigma_extrema_levels")

    def run(self, R, t, per_level=None):
        """In place: R [B,3,3], t [B,3] fp32 contiguous device buffers.

        One dpft_ic_solve_pyramid call (the sigma0 extrema pre-pass, then every level),
        or with per_level=True the same launches from one dpft_ic_solve_level call per
        level (tests check the two are bit-identical)."""
        if per_level is None:  # A/B knob for tuning runs only
            per_level = os.environ.get("DPFT_PER_LEVEL", "0") == "1"
        L = N.lib()
        st = _stream(self.device)
        # (truncated sigma without the one-launch extrema pre-pass -- more than 4 levels --
        # keeps the per-level minmax passes)
        if not per_level and (self.extrema_prepass or not self.remove_tru_sigma):
            n = len(self.calls)
            descs = (N.LevelDesc * n)(*[c.desc for c in reversed(self.calls)])
            tens = (N.LevelTensors * n)(*[c.tens for c in reversed(self.calls)])
            rc = L.dpft_ic_solve_pyramid(descs, tens, n, _ptr(R), _ptr(t), _ptr(self.ws), self.ws_bytes, st)
            N.check(rc, "dpft_ic_solve_pyramid")
            return
        self.prepare_extrema()
        for c in reversed(self.calls):
            rc = L.dpft_ic_solve_level(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), None, None,
                                       _ptr(self.ws), self.ws_bytes, st)
            N.check(rc, "dpft_ic_solve_level")

    def iterate(self, level, R, t, first=False, reverse=False):
        """One full iteration (fused reduce + in-kernel finalize) of `level`, in place.

        With first=False it reuses the sigma0 extrema the last pass over this level left
        in the workspace; reverse=True walks the level in the order the solve uses on odd
        iterations (DPFT_ITER_REVERSE).  bench.py times the dominant kernel this way."""
        c = self.calls[level]
        flags = (1 if first else 0) | (2 if reverse else 0)
        rc = N.lib().dpft_ic_iterate(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t), None, None, None,
                                     flags, _ptr(self.ws), self.ws_bytes, _stream(self.device))
        N.check(rc, "dpft_ic_iterate")

    def reduce_only(self, level, R, t):
        """Launch only the fused residual/Jacobian/JtJ kernel of `level` (roofline timing)."""
        c = self.calls[level]
        rc = N.lib().dpft_ic_reduce_only(ctypes.byref(c.desc), ctypes.byref(c.tens), _ptr(R), _ptr(t),
                                         _ptr(self.ws), self.ws_bytes, _stream(self.device))
        N.check(rc, "dpft_ic_reduce_only")

    def algorithmic_bytes(self, level):
        """HBM bytes one reduce launch must read: P (2C + 2Cs + 2) fp32, + 2 fp32 (depth0,
        depth1) with combine_icp (272 / 280 B per pixel at C = 32, Cs = 1)."""
        d = self.calls[level].desc
        return d.B * d.H * d.W * 4 * (2 * d.C + 2 * d.Cs + 2 + (2 if self.combine_icp else 0))
