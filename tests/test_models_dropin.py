"""Drop-in `models.LeastSquareTracking` against the reference's own module outputs.

Fixtures: tests/golden/gen_model_golden.py ran the REFERENCE LeastSquareTracking
(CPU fp32, deterministic synthetic weights from recipe.synthetic_weights) and
stored its state_dict keys / shapes, forward() poses and compute_residual()
losses.  Here the build's mirror is constructed with the same arguments, loaded
with the same weights, and run on the GPU (encoder in PyTorch, solver in HIP).
"""
import json
import os

import numpy as np
import pytest
import torch

import recipe
import gen_model_golden as G
from deep_prob_feature_track_amd.models.LeastSquareTracking import LeastSquareTracking, default_options

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEYS = json.load(open(os.path.join(HERE, "model_keys.json")))


def build(spec, mest=None, solver=None, no_weight_sharing=False):
    return LeastSquareTracking(spec["encoder"], spec["uncertainty"], 3, mest or spec.get("mest", "None"),
                               solver or spec.get("solver", "Direct-Nodamping"),
                               options=default_options(**spec["opts"]), no_weight_sharing=no_weight_sharing,
                               **spec.get("ctor", {}))


@pytest.mark.parametrize("name", sorted(G.KEY_VARIANTS))
def test_state_dict_surface_variants(name):
    spec = G.KEY_VARIANTS[name]
    m = build(spec, spec["mest"], spec["solver"], spec["no_weight_sharing"])
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert got == KEYS[name]


@pytest.mark.parametrize("name", sorted(G.MODEL_CASES))
def test_state_dict_surface_cases(name):
    m = build(G.MODEL_CASES[name])
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert got == KEYS[name]
    z = np.load(os.path.join(HERE, f"model_{name}.npz"), allow_pickle=False)
    assert list(z["keys"]) == [k for k, _ in got]


def test_unsupported_tracker_types_raise():
    spec = G.MODEL_CASES["convrgbd2_c8"]
    m = LeastSquareTracking(spec["encoder"], "None", 3, "None", "Direct-Nodamping",
                            options=default_options(**spec["opts"]))  # IC tracker: supported
    assert m.track_type == "IC"
    with pytest.raises(NotImplementedError):
        LeastSquareTracking(spec["encoder"], "laplacian", 3, "None", "Direct-Nodamping", direction="forward",
                            options=default_options(**spec["opts"]))  # U_FC tracker


def _loaded(name, device):
    spec = G.MODEL_CASES[name]
    m = build(spec)
    m.load_state_dict({k: torch.from_numpy(recipe.synthetic_weights(k, v.shape)) for k, v in m.state_dict().items()})
    m.eval()
    inp = G.model_inputs(spec["pairs"], spec["masks"])
    T = {k: torch.from_numpy(v).to(device) for k, v in inp.items()}
    return m.to(device), T


@pytest.mark.gpu
def test_mixed_device_inputs_raise_a_clear_error():
    """The dispatch rule looks at every tensor: features on the GPU with a pose on the host
    (or the reverse) raise ValueError up front instead of going to either path by argument
    order."""
    from deep_prob_feature_track_amd.models import torch_solver as TS
    from deep_prob_feature_track_amd.models.algorithms import TrustRegionInverseWUncertainty
    x = torch.zeros(1, 4, 8, 8, device="cuda")
    assert not TS.needs_torch_path(x, x)
    for args in ((x, torch.zeros(1, 3)), (torch.zeros(1, 3), x)):
        with pytest.raises(ValueError, match="span devices"):
            TS.needs_torch_path(*args)
    d = torch.ones(1, 1, 8, 8, device="cuda")
    K = torch.tensor([[8.0, 8.0, 4.0, 4.0]], device="cuda")
    with pytest.raises(ValueError, match="span devices"):
        TrustRegionInverseWUncertainty(3).forward([torch.eye(3).view(1, 3, 3), torch.zeros(1, 3, 1)], x, x, d, d, K,
                                                  d, d)


def test_device_solver_without_library_fails_loudly(monkeypatch):
    """Device tensors at inference never fall back to the PyTorch path: with the library
    unloadable the HIP solver raises (the CPU / gradient path is tests/test_torch_path.py)."""
    from deep_prob_feature_track_amd import _native
    from deep_prob_feature_track_amd.models import torch_solver as TS
    x = torch.zeros(1, 4, 8, 8)
    assert TS.needs_torch_path(x)  # CPU tensors: the PyTorch path
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libdpft_ic.so")
    monkeypatch.setattr(_native, "_lib", None)
    with pytest.raises((OSError, RuntimeError)):
        _native.lib()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(G.MODEL_CASES))
def test_forward_and_residual_match_reference(name):
    m, T = _loaded(name, "cuda")
    z = np.load(os.path.join(HERE, f"model_{name}.npz"), allow_pickle=False)
    kw = dict(obj_mask0=T.get("mask0"), obj_mask1=T.get("mask1"))
    with torch.no_grad():
        R, t = m(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"], **kw)
        B = R.shape[0]
        # se(3) tolerance of the contract: 1e-4; the encoder runs on MIOpen here
        # and on the CPU in the reference, so features differ in the last bits.
        assert np.abs(R.cpu().numpy() - z["R"]).max() < 1e-4
        assert tuple(t.shape) == z["t"].shape  # the reference's [B,3] translation (geometry.py:122)
        assert np.abs(t.cpu().numpy() - z["t"]).max() < 1e-4
        Rr = torch.from_numpy(z["R"]).cuda()
        tr = torch.from_numpy(z["t"]).cuda()
        _, loss = m.compute_residual(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"], poseI=[Rr, tr],
                                     level_i=0, **kw)
        np.testing.assert_allclose(loss.cpu().numpy(), z["res_pose_loss"], rtol=1e-4)
        ident = [torch.eye(3, device="cuda").expand(B, 3, 3).contiguous(), torch.zeros(B, 3, 1, device="cuda")]
        _, loss2 = m.compute_residual(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"], poseI=ident,
                                      level_i=2, **kw)
        np.testing.assert_allclose(loss2.cpu().numpy(), z["res_init_loss"], rtol=1e-4)


@pytest.mark.gpu
def test_forward_nonfinite_raises_assertion_and_module_recovers():
    """A NaN input pixel makes the Jacobian / residual non-finite: forward raises
    AssertionError like the reference's `assert check_nan(...) == 0` (algorithms.py:886,
    1988) -- the four levels share one status word read once per forward -- and the
    module then solves finite inputs exactly as before (no stale status)."""
    m, T = _loaded("convrgbd2_c8", "cuda")
    with torch.no_grad():
        R0, t0 = m(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"])
        bad = T["img0"].clone()
        bad[:, :, 40:44, 60:64] = float("nan")
        with pytest.raises(AssertionError):
            m(bad, T["img1"], T["depth0"], T["depth1"], T["K"])
        assert all(getattr(m, f"tr_update{l}")._deferred_status is None for l in range(4))
        R1, t1 = m(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"])
    # the encoder (MIOpen) is not bit-reproducible from call to call; the solver is
    assert (R0 - R1).abs().max().item() < 1e-5 and (t0 - t1).abs().max().item() < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["convrgbd2_c8", "convrgbd2_c8_icp", "rgb_identity_masks", "convrgbd_c8_ic_masks"])
def test_convergence_basin_landscape_matches_reference(name):
    """The multi-pose residual sweep equals the reference's one-compute_residual-per-pose
    loop (convergence_basin.py:340-369, 405-426) at levels 0 and 1."""
    from deep_prob_feature_track_amd import convergence_basin as CB
    m, T = _loaded(name, "cuda")
    z = np.load(os.path.join(HERE, f"model_{name}.npz"), allow_pickle=False)
    R_gt = torch.from_numpy(z["R"]).cuda()
    B = R_gt.shape[0]
    t_gt = torch.from_numpy(z["t"]).cuda().view(B, 3)
    offs = list(z["basin_offsets"])
    kw = dict(obj_mask0=T.get("mask0"), obj_mask1=T.get("mask1"))
    prep = m.prepare(T["img0"], T["img1"], T["depth0"], T["depth1"], **kw)
    Rp, tp = CB.axis_perturbations(R_gt, t_gt, offs, offs)
    for li, level in enumerate((0, 1)):
        got = m.compute_residual_poses(prep, T["K"], Rp, tp, level_i=level).view(6, len(offs), B).cpu().numpy()
        np.testing.assert_allclose(got, z["basin_loss"][li], rtol=1e-3)


@pytest.mark.gpu
def test_convergence_basin_driver_outputs():
    from deep_prob_feature_track_amd import convergence_basin as CB
    m, T = _loaded("convrgbd2_c8", "cuda")
    z = np.load(os.path.join(HERE, "model_convrgbd2_c8.npz"), allow_pickle=False)
    B = z["R"].shape[0]
    Rt = torch.eye(4).repeat(B, 1, 1).cuda()
    Rt[:, :3, :3] = torch.from_numpy(z["R"]).cuda()
    Rt[:, :3, 3] = torch.from_numpy(z["t"]).cuda().view(B, 3)
    S = 5
    out = CB.evaluate_convergence_basin(m, T["img0"], T["img1"], T["depth0"], T["depth1"], Rt, T["K"],
                                        level_i=[0, 1], pert_samples=S)
    assert out["avg_loss"].shape == (6, S + 3, B) and out["coarse_avg_loss"].shape == (1, 6, S, B)
    # the zero offset of every axis is the ground truth itself (= the reference's forward pose)
    for i in range(6):
        np.testing.assert_allclose(out["avg_loss"][i, S // 2], z["res_pose_loss"], rtol=1e-3)
    # the optimised pose (our forward) sits at the bottom of the basin as the reference's does
    np.testing.assert_allclose(out["avg_loss"][0, S + 2], z["res_pose_loss"], rtol=1e-3)
    assert np.all(out["angular_error"] < 1e-3) and np.all(out["translation_error"] < 1e-3)
    n, margins = CB.convergence_counts(torch.from_numpy(out["R_est"]), torch.from_numpy(out["t_est"]),
                                       torch.from_numpy(z["R"]), torch.from_numpy(z["t"]).view(B, 3))
    assert n == B and np.all(margins["rot_margin"] > 0)
    d2 = CB.evaluate_2d_convergence_basin(m, T["img0"], T["img1"], T["depth0"], T["depth1"], Rt, T["K"],
                                          pert_samples=3)
    np.testing.assert_allclose(d2["avg_loss"][0, 1, 1], z["res_pose_loss"], rtol=1e-3)


@pytest.mark.gpu
def test_forward_captured_in_a_hip_graph():
    """The whole drop-in forward (encoder, pyramids, four solver levels) captured into one
    HIP graph and replayed on new input contents equals eager forward calls; the
    non-finite status word is left in `last_status` for the caller."""
    from deep_prob_feature_track_amd import ic
    m, T = _loaded("convrgbd2_c8", "cuda")
    z = np.load(os.path.join(HERE, "model_convrgbd2_c8.npz"), allow_pickle=False)
    static = {k: T[k].clone() for k in ("img0", "img1", "depth0", "depth1", "K")}
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(**{k: static[k] for k in static})
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            R_g, t_g = m(static["img0"], static["img1"], static["depth0"], static["depth1"], static["K"])
        status = m.last_status
        g.replay()
        torch.cuda.synchronize()
        ic.check_status(status)
        assert np.abs(R_g.cpu().numpy() - z["R"]).max() < 1e-4
        R_e, t_e = m(T["img0"], T["img1"], T["depth0"], T["depth1"], T["K"])
        assert (R_g - R_e).abs().max().item() < 1e-5 and (t_g - t_e).abs().max().item() < 1e-5
        # new contents in the static inputs: the replay tracks the swapped pairs
        static["img0"].copy_(T["img1"])
        static["img1"].copy_(T["img0"])
        static["depth0"].copy_(T["depth1"])
        static["depth1"].copy_(T["depth0"])
        g.replay()
        torch.cuda.synchronize()
        R_s, t_s = m(T["img1"], T["img0"], T["depth1"], T["depth0"], T["K"])
        assert (R_g - R_s).abs().max().item() < 1e-5 and (t_g - t_s).abs().max().item() < 1e-5


@pytest.mark.gpu
def test_resvol_batch_beyond_one_call_of_trials():
    """'Direct-ResVol' with B = 208 pairs: the ten trials x 208 pairs exceed one library call
    (2048 pairs), so the trials run one no-update call each (ic.iterate_poses) instead of the
    replicated launch -- same poses: every replica of the fixture's pairs lands on the
    reference's (B > 204 used to fail with DPFT_E_INVALID)."""
    name = "rgb_ic_mest2w_resvol"
    m, T = _loaded(name, "cuda")
    z = np.load(os.path.join(HERE, f"model_{name}.npz"), allow_pickle=False)
    b = T["img0"].shape[0]
    reps = -(-208 // b)
    big = {k: v.repeat(reps, *([1] * (v.dim() - 1))) for k, v in T.items()}
    with torch.no_grad():
        R, t = m(big["img0"], big["img1"], big["depth0"], big["depth1"], big["K"], obj_mask0=big.get("mask0"),
                 obj_mask1=big.get("mask1"))
    assert R.shape[0] == b * reps >= 208
    assert np.abs(R.cpu().numpy() - np.tile(z["R"], (reps, 1, 1))).max() < 1e-4
    assert np.abs(t.cpu().numpy().reshape(-1, 3) - np.tile(z["t"].reshape(b, 3), (reps, 1))).max() < 1e-4
