"""Encoder block epilogue (dpft_bn_elu) and the channels_last encoder on a real MI355X
(`-m gpu`): the fused in-place batchnorm + ELU pass against the torch modules it
replaces (reference submodules.py:25-39, convLayer), in both memory formats."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _block(cin, cout, k, dil, dev, seed):
    from deep_prob_feature_track_amd.models.submodules import convLayer
    torch.manual_seed(seed)
    blk = convLayer(True, cin, cout, k, dilation=dil)
    bn = blk[1]
    with torch.no_grad():  # non-trivial running statistics and affine terms
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.2, 3.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    return blk.to(dev).eval()


@pytest.mark.parametrize("cin,cout,k,dil,H,W", [(8, 16, 3, 1, 48, 64), (16, 32, 3, 2, 30, 40), (32, 32, 1, 1, 7, 9),
                                                (3, 6, 3, 1, 10, 10)])
@pytest.mark.parametrize("nhwc", [False, True])
def test_bn_elu_matches_torch_modules(cin, cout, k, dil, H, W, nhwc):
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    blk = _block(cin, cout, k, dil, dev, seed=cin + cout + H)
    x = torch.randn(2, cin, H, W, device=dev)
    if nhwc:
        blk = blk.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        conv = blk[0](x)
        ref = nn.functional.elu(nn.functional.batch_norm(conv, blk[1].running_mean, blk[1].running_var,
                                                         blk[1].weight, blk[1].bias, False, 0.0, blk[1].eps))
        y = conv.clone()
        fused = ic.bn_elu_(y, blk[1])
        out = blk(x)  # ConvBlock.forward: fused where the layout allows, the modules otherwise
    # (H W % 4 != 0 in NCHW, C % 4 != 0 in NHWC: the kernel declines and the modules run)
    assert fused == ((cout % 4 == 0) if nhwc else ((H * W) % 4 == 0))
    if fused:
        torch.testing.assert_close(y, ref, rtol=2e-6, atol=2e-6)
    torch.testing.assert_close(out, ref, rtol=2e-6, atol=2e-6)
    assert out.is_contiguous(memory_format=torch.channels_last if nhwc else torch.contiguous_format)


def test_bn_coefficients_follow_state_dict_loads():
    """The cached [a | b] coefficients are rebuilt after load_state_dict changes the
    statistics (tensor versions move)."""
    dev = _dev()
    blk = _block(8, 16, 3, 1, dev, seed=3)
    x = torch.randn(1, 8, 16, 16, device=dev)
    with torch.no_grad():
        y0 = blk(x)
        sd = {k: v.clone() for k, v in blk.state_dict().items()}
        sd["1.running_var"] = sd["1.running_var"] * 4.0
        blk.load_state_dict(sd)
        y1 = blk(x)
        conv = blk[0](x)
        ref = nn.functional.elu(nn.functional.batch_norm(conv, blk[1].running_mean, blk[1].running_var,
                                                         blk[1].weight, blk[1].bias, False, 0.0, blk[1].eps))
    assert not torch.allclose(y0, y1)
    torch.testing.assert_close(y1, ref, rtol=2e-6, atol=2e-6)


def test_channels_last_encoder_matches_nchw():
    """The drop-in's channels_last encoder gives the NCHW encoder's features (MIOpen's
    NHWC convolutions sum in another order: fp32 rounding only)."""
    from deep_prob_feature_track_amd.models.algorithms import FeaturePyramid
    dev = _dev()
    torch.manual_seed(0)
    enc = FeaturePyramid(D=8, w_uncertainty="laplacian", feature_channel=8, feature_extract="conv",
                         uncertainty_channel=1).to(dev).eval()
    x = torch.randn(2, 8, 60, 80, device=dev)
    with torch.no_grad():
        f_a, s_a, _ = enc(x)
        enc.to(memory_format=torch.channels_last)
        f_b, s_b, _ = enc(x.contiguous(memory_format=torch.channels_last))
    for a, b in zip(f_a + s_a, f_b + s_b):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * a.abs().max().item())


@pytest.mark.parametrize("cout,H,W", [(32, 48, 64), (8, 15, 20), (16, 7, 9)])
def test_bn_elu_pack_equals_bn_elu_then_pack(cout, H, W):
    """The feature heads' epilogue written to the channel-quad layout (dpft_bn_elu_pack) is
    bit for bit the in-place epilogue followed by the relayout (dpft_bn_elu +
    dpft_pack_features_nhwc), and ConvBlock.forward_packed returns it."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    blk = _block(24, cout, 1, 1, dev, seed=cout + H).to(memory_format=torch.channels_last)
    x = torch.randn(3, 24, H, W, device=dev).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        conv = blk[0](x)
        y = conv.clone()
        assert ic.bn_elu_(y, blk[1])
        ref = ic.pack_features(y)
        got = ic.bn_elu_pack(conv, blk[1])
        via_block = blk.forward_packed(x)
    assert got.shape == (3, cout // 4, H, W, 4)
    assert torch.equal(got, ref) and torch.equal(via_block, ref)
    assert torch.equal(ic.unpack_features(got), y.contiguous())


def test_epilogue_channel_loads_aligned_and_unaligned_agree():
    """dpft_bn_elu / dpft_bn_elu_pack load the batchnorm scale / shift of a channel quad as
    two 16-byte words when the coefficient array is 16-byte aligned, else as eight floats:
    both paths give the same bits (the same fused multiply-add and ELU per channel)."""
    from deep_prob_feature_track_amd import _native as N, ic
    dev = _dev()
    torch.manual_seed(3)
    B, C, H, W = 2, 16, 24, 40
    conv = torch.randn(B, C, H, W, device=dev).contiguous(memory_format=torch.channels_last)
    coeffs = torch.cat((torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3))
    store = torch.zeros(2 * C + 4, device=dev)
    store[1:1 + 2 * C] = coeffs
    aligned, unaligned = coeffs.contiguous(), store[1:1 + 2 * C]
    assert aligned.data_ptr() % 16 == 0 and unaligned.data_ptr() % 16 != 0
    L = N.lib()
    outs = []
    for chan in (aligned, unaligned):
        packed = torch.empty(B, C // 4, H, W, 4, device=dev)
        N.check(L.dpft_bn_elu_pack(ic._ptr(conv), ic._ptr(chan), ic._ptr(packed), B, C, H, W, ic._stream(dev)),
                "dpft_bn_elu_pack")
        inplace = conv.clone(memory_format=torch.channels_last)
        N.check(L.dpft_bn_elu(ic._ptr(inplace), ic._ptr(chan), inplace.numel(), C, 1, 1, ic._stream(dev)),
                "dpft_bn_elu")
        outs.append((packed, inplace))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(ic.pack_features(outs[0][1]), outs[0][0])
    ref = torch.nn.functional.elu(conv * coeffs[:C].view(1, C, 1, 1) + coeffs[C:].view(1, C, 1, 1))
    torch.testing.assert_close(outs[0][1], ref, rtol=1e-6, atol=1e-6)


def test_dropin_encoder_writes_packed_features():
    """LeastSquareTracking's feature heads write the solver's channel-quad layout (no
    relayout pass in the forward): the packed features are bit for bit the heads' conv
    outputs through the in-place epilogue and the relayout (captured by hooks on the heads'
    convolutions -- MIOpen's convolution algorithms are not bitwise reproducible from one
    call to the next, so two forwards are not compared), and the forward solves on them: the same
    prepared features give the same poses twice, and within 1e-5 of the NCHW path's."""
    from deep_prob_feature_track_amd import ic
    from deep_prob_feature_track_amd.examples import K_FULL, color_float, depth_m, load_synthetic_weights
    from deep_prob_feature_track_amd.models.LeastSquareTracking import LeastSquareTracking, default_options
    dev = _dev()
    net = LeastSquareTracking("ConvRGBD2", "laplacian", 3, "None", "Direct-Nodamping",
                              options=default_options(feature_channel=16, uncertainty_channel=1,
                                                      feature_extract="conv", remove_tru_sigma=True))
    net = load_synthetic_weights(net).to(dev).eval()
    pairs = [(0, 1), (2, 4)]
    img0 = torch.stack([torch.from_numpy(color_float(i, 2)) for i, _ in pairs]).to(dev)
    img1 = torch.stack([torch.from_numpy(color_float(j, 2)) for _, j in pairs]).to(dev)
    d0 = torch.stack([torch.from_numpy(depth_m(i, 2))[None] for i, _ in pairs]).to(dev)
    d1 = torch.stack([torch.from_numpy(depth_m(j, 2))[None] for _, j in pairs]).to(dev)
    K = torch.from_numpy(K_FULL / 2).repeat(len(pairs), 1).to(dev)
    with torch.no_grad():
        net(img0, img1, d0, d1, K)  # channels_last conversion, MIOpen warm-up
        convs = []
        hooks = [getattr(net.encoder, f"f_conv{l}")[0].register_forward_hook(
            lambda m, i, o: convs.append(o.clone())) for l in range(4)]
        prep = net.prepare(img0, img1, d0, d1)
        for h in hooks:
            h.remove()
        R, t = net(img0, img1, d0, d1, K)
    assert len(convs) == 8  # 4 heads x 2 frames (the two-view encoder runs per frame)
    for l in range(4):
        for f, x in enumerate((prep[2][l], prep[3][l])):
            assert x.dim() == 5, f"level {l} frame {f}: not packed"
            y = convs[f * 4 + l]
            assert ic.channels_last(y)
            assert ic.bn_elu_(y, getattr(net.encoder, f"f_conv{l}")[1])
            assert torch.equal(x, ic.pack_features(y)), f"level {l} frame {f}"
    assert torch.isfinite(R).all() and torch.isfinite(t).all()
    # the poses: forward on the prepared (packed) features is deterministic, and equals the
    # forward on the same features unpacked to NCHW (the NCHW tile path) within 1e-5
    prep = tuple(prep)
    unpacked = list(prep)
    for i in (2, 3):
        unpacked[i] = [ic.unpack_features(x) for x in prep[i]]
    poses = []
    with torch.no_grad():
        for P in (prep, prep, tuple(unpacked)):
            net._preprocess = lambda *a, _P=P, **k: _P
            poses.append(net(img0, img1, d0, d1, K))
    del net._preprocess
    assert torch.equal(poses[0][0], poses[1][0]) and torch.equal(poses[0][1], poses[1][1])
    assert (poses[0][0] - poses[2][0]).abs().max().item() < 1e-5
    assert (poses[0][1] - poses[2][1]).abs().max().item() < 1e-5
