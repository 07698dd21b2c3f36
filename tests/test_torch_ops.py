"""torch.library custom ops (deep_prob_feature_track_amd/torch_ops.py) over the C ABI.

CPU: the dpft:: ops are registered with their schemas and their fake kernels propagate
shapes (fake CUDA tensors need no device).  GPU (`-m gpu`): each op makes the same library
call as the direct path (bit-identical outputs); the drop-in forward traces under
torch.compile with no graph break (U_IC) and the compiled forward (backend "aot_eager": the
traced graph run without code generation, and "cudagraphs") gives the eager poses within the
se(3) tolerance (the traced encoder's decomposed kernels round differently).
"""
import numpy as np
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import recipe
import gen_model_golden as G
from deep_prob_feature_track_amd import torch_ops  # noqa: F401  (registers dpft::*)

OPS = ["ic_solve_level", "ic_residual_level", "preprocess_depth", "pack_features", "bn_elu_"]


def test_ops_registered_with_schemas():
    for name in OPS:
        op = getattr(torch.ops.dpft, name)
        schema = str(op.default._schema)
        assert schema.startswith(f"dpft::{name}("), schema
    assert "!) x" in str(torch.ops.dpft.bn_elu_.default._schema)  # mutates its input (alias annotation)


def test_fake_kernels_propagate_shapes():
    with FakeTensorMode():
        B, C, H, W = 2, 32, 48, 64
        x = torch.empty(B, C, H, W, device="cuda")
        d = torch.empty(B, 1, H, W, device="cuda")
        K = torch.empty(B, 4, device="cuda")
        R, t = torch.empty(B, 3, 3, device="cuda"), torch.empty(B, 3, 1, device="cuda")
        o = torch.ops.dpft.ic_solve_level(R, t, x, x, d, d, K, d, d, None, None, None, None, 3, True, False, 0.01,
                                          False, True)
        assert [tuple(v.shape) for v in o] == [(B, 3, 3), (B, 3, 1), (B, 6, 6), (1,)] and o[3].dtype == torch.int32
        o = torch.ops.dpft.ic_solve_level(R, t, x, x, d, d, K, d, d, None, None, None, None, 3, True, False, 0.01,
                                          False, False)
        assert tuple(o[2].shape) == (0, 6, 6)
        assert tuple(torch.ops.dpft.ic_residual_level(R, t, x, x, d, d, K, d, d, None, None, None, None, True,
                                                      False, 0.01, False).shape) == (B,)
        p = torch.ops.dpft.preprocess_depth(d, 4, True)
        assert [tuple(v.shape) for v in p] == [(B, 1, H >> l, W >> l) for l in range(4)] * 2
        assert tuple(torch.ops.dpft.pack_features(x).shape) == (B, C // 4, H, W, 4)


def _model(name, device):
    from deep_prob_feature_track_amd.models.LeastSquareTracking import LeastSquareTracking, default_options
    spec = G.MODEL_CASES[name]
    m = LeastSquareTracking(spec["encoder"], spec["uncertainty"], 3, spec.get("mest", "None"),
                            spec.get("solver", "Direct-Nodamping"), options=default_options(**spec["opts"]),
                            **spec.get("ctor", {}))
    m.load_state_dict({k: torch.from_numpy(recipe.synthetic_weights(k, v.shape)) for k, v in m.state_dict().items()})
    inp = G.model_inputs(spec["pairs"], spec["masks"])
    return m.to(device).eval(), {k: torch.from_numpy(v).to(device) for k, v in inp.items()}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.mark.gpu
def test_ops_equal_direct_calls():
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(3)
    B, C, H, W = 2, 32, 40, 70
    f0 = torch.rand(B, C, H, W, generator=g)
    f1 = torch.roll(f0, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0, s1 = 0.5 + torch.rand(B, 1, H, W, generator=g), 0.5 + torch.rand(B, 1, H, W, generator=g)
    depth = 0.5 + 3 * torch.rand(B, 1, H, W, generator=g)
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    f0, f1, s0, s1, depth, K = [v.to(dev) for v in (f0, f1, s0, s1, depth, K)]
    inv, _ = ic.preprocess_depth(depth, 1)
    d0 = d1 = inv[0]
    pose = (torch.eye(3, device=dev).repeat(B, 1, 1), torch.zeros(B, 3, 1, device=dev))
    a = ic.solve_level(pose, f0, f1, d0, d1, K, s0, s1, iters=3, remove_tru_sigma=True, return_jtj=True)
    b = torch.ops.dpft.ic_solve_level(pose[0], pose[1], f0, f1, d0, d1, K, s0, s1, None, None, None, None, 3, True,
                                      False, 0.01, False, True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]) and int(b[3].item()) == 0
    la = ic.residual_level(pose, f0, f1, d0, d1, K, s0, s1, remove_tru_sigma=True)
    lb = torch.ops.dpft.ic_residual_level(pose[0], pose[1], f0, f1, d0, d1, K, s0, s1, None, None, None, None, True,
                                          False, 0.01, False)
    assert torch.equal(la, lb)
    pa = ic.preprocess_depth(depth, 3, depth_pyramid=True)
    pb = torch.ops.dpft.preprocess_depth(depth, 3, True)
    assert all(torch.equal(x, y) for x, y in zip(pa[0] + pa[1], pb))
    assert torch.equal(ic.pack_features(f0), torch.ops.dpft.pack_features(f0))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["convrgbd2_c8", "convrgbd2_c8_icp", "convrgbd_c8_ic_masks"])
def test_dropin_traces_without_graph_breaks_and_matches_eager(name):
    dev = _dev()
    m, T = _model(name, dev)
    args = (T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"])
    kw = dict(obj_mask0=T.get("mask0"), obj_mask1=T.get("mask1"))
    with torch.no_grad():
        Re, te = m(*args, **kw)  # eager (also converts the encoder to channels_last once)
        torch._dynamo.reset()
        if G.MODEL_CASES[name]["uncertainty"] != "None":  # the U_IC tracker: one graph
            ex = torch._dynamo.explain(m)(*args, **kw)
            assert ex.graph_break_count == 0, ex.break_reasons
        for backend in ("aot_eager", "cudagraphs"):
            torch._dynamo.reset()
            mc = torch.compile(m, backend=backend)
            for _ in range(3):  # cudagraphs: warm-up, record, replay
                Rc, tc = mc(*args, **kw)
            torch.cuda.synchronize()
            # the traced encoder may run other (decomposed) kernels than eager: features can
            # differ in the last bits, the poses by the se(3) tolerance at most
            d = max((Rc - Re).abs().max().item(), (tc - te).abs().max().item())
            assert d <= 1e-4, f"{backend}: compiled vs eager {d:.2e}"
            if m.last_status is not None:
                from deep_prob_feature_track_amd import ic
                ic.check_status(m.last_status)
    np.testing.assert_equal(Re.cpu().numpy().shape[1:], (3, 3))


@pytest.mark.gpu
def test_compiled_forward_reports_nonfinite_in_last_status():
    """Under torch.compile the drop-in cannot raise inside the graph (no host read there):
    a non-finite Jacobian / residual is reported in `model.last_status`, a device tensor the
    caller checks with ic.check_status -- as eager forward's
    AssertionError (the reference's `assert check_nan(...) == 0`, algorithms.py:886, 1988)."""
    from deep_prob_feature_track_amd import _native as Nn
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    m, T = _model("convrgbd2_c8", dev)
    img0 = T["img0"].clone()
    img0[:, :, 5:9, 7:11] = float("nan")
    args = (img0, T["img1"], T["depth0"], T["depth1"], T["K"])
    with torch.no_grad():
        with pytest.raises(AssertionError):
            m(*args)
        torch._dynamo.reset()
        mc = torch.compile(m, backend="aot_eager")
        mc(*args)
    torch.cuda.synchronize()
    st = m.last_status
    assert isinstance(st, torch.Tensor) and st.is_cuda, type(st)
    assert int(st.cpu()[0]) & Nn.STATUS_NONFINITE
    with pytest.raises(AssertionError):
        ic.check_status(st)
