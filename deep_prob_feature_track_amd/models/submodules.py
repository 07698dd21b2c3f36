"""Network building blocks of the tracker's host-side modules.

Restates the reference's code/models/submodules.py (color_normalize 20-23,
convLayer 25-39, convLayer1d 41-55, fcLayer 57-61, initialize_weights 63-78)
so that modules built from them carry the reference's state_dict keys:
a block is nn.Sequential(conv[, batchnorm], ELU) -> keys `<name>.0.weight`,
`<name>.1.running_mean`, ...
"""
import torch
import torch.nn as nn
from torch.nn import init

from .. import ic
from .. import torch_ops  # noqa: F401  (registers the dpft:: ops torch.compile traces)

_RGB_MEAN = (0.4914, 0.4822, 0.4465)
_RGB_STD = (0.2023, 0.1994, 0.2010)


_NORM_CONSTS = {}


def color_normalize(color):
    """Per-channel (x - mean) / std of an RGB batch [B,3,H,W] (submodules.py:20-23).
    The constants are copied to the device once per (device, dtype): a host-to-device
    copy per call would also make forward impossible to capture in a HIP graph."""
    key = (color.device, color.dtype)
    if key not in _NORM_CONSTS:
        _NORM_CONSTS[key] = (torch.tensor(_RGB_MEAN, dtype=color.dtype, device=color.device).view(1, 3, 1, 1),
                             torch.tensor(_RGB_STD, dtype=color.dtype, device=color.device).view(1, 3, 1, 1))
    mean, std = _NORM_CONSTS[key]
    return (color - mean) / std


def _padding(kernel_size, dilation):
    # the reference's "same" padding formula (kept literally: it is not k//2*d for every d)
    return (kernel_size - 1) // 2 + dilation - 1


class ConvBlock(nn.Sequential):
    """conv [-> batchnorm] -> ELU, an nn.Sequential (the reference's state_dict keys).
    In eval mode on the GPU, outside autograd, the batchnorm and the ELU of a 2-D block
    run as one in-place pass over the conv output (`ic.bn_elu_`, dpft_bn_elu) instead of
    two elementwise kernels; otherwise, or for a layout the kernel does not take, the
    modules run in turn."""

    def _fusable(self, x):
        return (len(self) == 3 and isinstance(self[1], nn.BatchNorm2d) and isinstance(self[2], nn.ELU)
                and self[2].alpha == 1.0 and not self.training and x.is_cuda and not torch.is_grad_enabled())

    def forward_packed(self, x):
        """The block's output in the solver's channel-quad layout [B,C/4,H,W,4] when the
        epilogue can write it (dpft_bn_elu_pack: the batchnorm + ELU of a channels_last
        conv output stored out of place, no separate relayout pass); otherwise forward(x),
        [B,C,H,W].  Same values either way."""
        if self._fusable(x):
            y = self[0](x)
            if ic.bn_elu_pack_applies(y, self[1]):
                if torch.compiler.is_compiling():
                    return torch.ops.dpft.bn_elu_pack(y, torch_ops.bn_coeffs(self[1]))
                return ic.bn_elu_pack(y, self[1])
            return self._epilogue(y)
        return self.forward(x)

    def _epilogue(self, y):
        if torch.compiler.is_compiling():  # traced: the dpft::bn_elu_ op (torch_ops.py)
            if torch_ops.bn_elu_applies(y, self[1]):
                torch.ops.dpft.bn_elu_(y, torch_ops.bn_coeffs(self[1]))
                return y
        elif ic.bn_elu_(y, self[1]):
            return y
        return self[2](self[1](y))

    def forward(self, x):
        if self._fusable(x):
            return self._epilogue(self[0](x))
        return super().forward(x)


def _block(conv_cls, bn_cls, batch_norm, cin, cout, kernel_size, stride, dilation, bias):
    layers = [conv_cls(cin, cout, kernel_size=kernel_size, stride=stride,
                       padding=_padding(kernel_size, dilation), dilation=dilation,
                       bias=bias if batch_norm else True)]
    if batch_norm:
        layers.append(bn_cls(cout))
    layers.append(nn.ELU(inplace=True))
    return ConvBlock(*layers)


def convLayer(batchNorm, in_planes, out_planes, kernel_size=3, stride=1, dilation=1, bias=False):
    """Conv2d [+ BatchNorm2d] + ELU."""
    return _block(nn.Conv2d, nn.BatchNorm2d, batchNorm, in_planes, out_planes, kernel_size, stride, dilation, bias)


def convLayer1d(batchNorm, in_planes, out_planes, kernel_size=3, stride=1, dilation=1, bias=False):
    """Conv1d [+ BatchNorm1d] + ELU."""
    return _block(nn.Conv1d, nn.BatchNorm1d, batchNorm, in_planes, out_planes, kernel_size, stride, dilation, bias)


def fcLayer(in_planes, out_planes, bias=True):
    """Linear + ReLU."""
    return nn.Sequential(nn.Linear(in_planes, out_planes, bias), nn.ReLU(inplace=True))


def initialize_weights(modules, method='xavier'):
    """Xavier / Kaiming-uniform init of the Conv2d / ConvTranspose2d among `modules`
    (their direct iteration, as the reference does), zero biases."""
    for m in modules:
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            if m.bias is not None:
                m.bias.data.zero_()
            if method == 'xavier':
                init.xavier_uniform_(m.weight)
            elif method == 'kaiming':
                init.kaiming_uniform_(m.weight)
