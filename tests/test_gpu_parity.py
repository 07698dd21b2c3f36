"""HIP solver parity on a real MI355X (run with `-m gpu`).

Every case compares libdpft_ic.so, called through the C ABI (ctypes), with
  (a) the golden vectors produced by the reference itself (fp32 and fp64 runs),
  (b) the CPU oracle on the same inputs.
Tolerance (BASELINE.json north star): 1e-4 on every R and t entry (se(3)), per
iteration and at the end; iteration counts are exact (3 per level, no early
exit).  The reference's own fp32 noise floor is up to 9.7e-5 at 640x480 C=32
(SURVEY.md App. B), so the fp64 golden run is the sharper check.
"""
import numpy as np
import pytest
import torch

import golden_io
import recipe

pytestmark = pytest.mark.gpu

SE3_TOL = 1e-4


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _run_hip_trace(name, dev):
    from deep_prob_feature_track_amd import ic
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R, t = golden_io.init_pose(case, torch.float32, dev)
    t = t.view(-1, 3, 1)
    K = torch.from_numpy(case["K"]).to(dev)
    trace = []
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    for l in reversed(range(case["levels"])):
        d = lv[l]
        for it in range(3):
            R, t, jtj, jtr, inv = ic.iterate(
                (R, t), d["f0"], d["f1"], d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=(it == 0),
                remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                combine_icp=bool(z["opt_combine_icp"]), status=status)
            trace.append(dict(R=R.cpu().numpy(), t=t.view(-1, 3).cpu().numpy(), jtj=jtj.cpu().numpy(),
                              jtr=jtr.cpu().numpy(), invalid=inv.cpu().numpy()))
    ic.check_status(status)
    return case, z, trace


FEATURE_CASES = ["cfg1_160x120_c8", "cfg1b_160x120_c8_f04", "batch4_160x120_c8", "masks_160x120_c8",
                 "cfg2_640x480_c32", "icp_160x120_c8"]


@pytest.mark.parametrize("name", FEATURE_CASES)
def test_hip_matches_reference_golden(name):
    dev = _dev()
    case, z, trace = _run_hip_trace(name, dev)
    assert len(trace) == 3 * case["levels"]
    for prec in ("f32", "f64"):
        if f"{prec}_R" not in z:
            continue
        for i, tr in enumerate(trace):
            dR = np.abs(tr["R"] - z[f"{prec}_R"][i]).max()
            dt = np.abs(tr["t"] - z[f"{prec}_t"][i]).max()
            assert dR <= SE3_TOL and dt <= SE3_TOL, f"{name} vs {prec} iter {i}: |dR|={dR:.2e} |dt|={dt:.2e}"
    # first iteration: identical start pose and identical fp32 semantics -> the
    # invalid set (occlusion, masks, truncated sigma) is the reference's bit for
    # bit and the normal equations agree to accumulation-order rounding.
    rel = np.abs(trace[0]["jtj"] - z["f32_jtj"][0]).max() / np.abs(z["f32_jtj"][0]).max()
    assert rel < 1e-5, f"JtJ rel err {rel:.2e}"
    relr = np.abs(trace[0]["jtr"] - z["f32_jtr"][0]).max() / np.abs(z["f32_jtr"][0]).max()
    assert relr < 1e-4, f"JtR rel err {relr:.2e}"
    assert (trace[0]["invalid"] == z["f32_invalid"][0]).all(), (trace[0]["invalid"], z["f32_invalid"][0])


@pytest.mark.parametrize("name", ["cfg1_160x120_c8", "batch4_160x120_c8", "masks_160x120_c8", "icp_160x120_c8"])
def test_hip_residual_loss(name):
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R, t = golden_io.init_pose(case, torch.float32, dev)
    L = case["levels"]
    d = lv[L - 1]
    K = torch.from_numpy(case["K"]).to(dev) / 2 ** (L - 1)
    loss = ic.residual_level((R, t), d["f0"], d["f1"], d["invD0"], d["invD1"], K, d["s0"], d["s1"],
                             remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                             obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                             combine_icp=bool(z["opt_combine_icp"]))
    np.testing.assert_allclose(loss.cpu().numpy(), z["f32_loss_start"][0], rtol=2e-5)


def _random_case(B, C, Cs, H, W, seed, masks=False):
    g = torch.Generator().manual_seed(seed)
    f0 = torch.rand(B, C, H, W, generator=g)
    # a smooth shifted copy so the solve has signal
    f1 = torch.roll(f0, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0 = 0.5 + torch.rand(B, Cs, H, W, generator=g)
    s1 = 0.5 + torch.rand(B, Cs, H, W, generator=g)
    invD0 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    invD1 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    m0 = (torch.rand(B, 1, H, W, generator=g) > 0.2) if masks else None
    m1 = (torch.rand(B, 1, H, W, generator=g) > 0.2) if masks else None
    return f0, f1, s0, s1, invD0, invD1, K, m0, m1


@pytest.mark.parametrize("B,C,Cs,H,W,tru,masks", [
    (1, 8, 1, 120, 160, True, False),
    (2, 5, 1, 37, 70, True, True),      # ragged tiles, generic channel count
    (3, 8, 8, 48, 64, True, False),     # per-channel uncertainty (Cs = C)
    (2, 32, 1, 60, 80, False, False),
    (1, 3, 3, 17, 129, False, True),
])
def test_hip_matches_oracle_random(B, C, Cs, H, W, tru, masks):
    """HIP vs the fp32 CPU oracle on seeded random inputs, several shapes.

    Same precision on both sides: the invalid set (u > 0 at column 0, z-test,
    masks) is decided by the same fp32 bits, so iteration 0 must agree exactly
    on it; an fp64 oracle would legitimately flip border pixels here."""
    from deep_prob_feature_track_amd import ic
    from oracle import ic_oracle as O
    dev = _dev()
    f0, f1, s0, s1, invD0, invD1, K, m0, m1 = _random_case(B, C, Cs, H, W, seed=B * 1000 + C * 10 + W, masks=masks)
    R = torch.eye(3).repeat(B, 1, 1)
    t = torch.zeros(B, 3, 1)
    tr_o, tr_64 = [], []
    O.solve_level(R, t, f0, f1, s0, s1, invD0, invD1, K, iters=3, remove_tru_sigma=tru, mask0=m0, mask1=m1,
                  trace=tr_o)
    dd = lambda a: a.double() if a is not None and a.dtype == torch.float32 else a
    O.solve_level(dd(R), dd(t), dd(f0), dd(f1), dd(s0), dd(s1), dd(invD0), dd(invD1), dd(K), iters=1,
                  remove_tru_sigma=tru, mask0=m0, mask1=m1, trace=tr_64)
    cu = lambda a: a.to(dev) if a is not None else None
    Rg, tg = R.to(dev), t.to(dev)
    for it in range(3):
        Rg, tg, jtj, jtr, inv = ic.iterate((Rg, tg), cu(f0), cu(f1), cu(invD0), cu(invD1), cu(K), cu(s0), cu(s1),
                                           first=(it == 0), remove_tru_sigma=tru, obj_mask0=cu(m0),
                                           obj_mask1=cu(m1))
        ref = tr_o[it]
        if it == 0:
            # J is unmasked, so JtJ does not see the precision-dependent invalid set
            rel = (jtj.cpu().double() - tr_64[0]["JtJ"]).abs().max() / tr_64[0]["JtJ"].abs().max()
            assert rel < 1e-5, f"JtJ rel {rel:.2e}"
            relr = (jtr.cpu() - ref["JtR"]).abs().max() / ref["JtR"].abs().max()
            assert relr < 1e-4, f"JtR rel {relr:.2e}"
            assert torch.equal(inv.cpu().long(), ref["invalid"].long())
        dR = (Rg.cpu() - ref["R"]).abs().max().item()
        dt = (tg.view(B, 3).cpu() - ref["t"]).abs().max().item()
        assert dR <= SE3_TOL and dt <= SE3_TOL, f"iter {it}: |dR|={dR:.2e} |dt|={dt:.2e}"


@pytest.mark.parametrize("name", ["cfg1_160x120_c8", "masks_160x120_c8", "batch4_160x120_c8", "cfg2_640x480_c32"])
def test_invalid_mask_bit_exact(name):
    """u, v, sigma_r and the occlusion / mask set equal the reference's fp32 CPU
    arithmetic bit for bit at the start pose (tests/ref_arith.py emulates it
    host-independently; pinned against torch by tests/test_ref_arith.py)."""
    import ref_arith as A
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load(name)
    L = case["levels"]
    lvg = golden_io.levels_torch(case, torch.float32, dev)[L - 1]
    R, t = golden_io.init_pose(case, torch.float32)
    K = torch.from_numpy(case["K"]) / 2 ** (L - 1)
    dbg = ic.debug_pixels((R.to(dev), t.to(dev)), lvg["f0"], lvg["f1"], lvg["invD0"], lvg["invD1"], K.to(dev),
                          lvg["s0"], lvg["s1"], obj_mask0=lvg.get("mask0"), obj_mask1=lvg.get("mask1")).cpu().numpy()
    lv = L - 1
    for b in range(case["B"]):
        H, W = case[f"invD0_{lv}"].shape[2:]
        u, v, iz, _, _ = A.warp(H, W, case[f"invD0_{lv}"][b, 0], case["R_init"][b], case["t_init"][b], K[b].numpy())
        occ = A.occlusion(u, v, iz, case[f"invD1_{lv}"][b, 0])
        if f"mask0_{lv}" in case:
            occ = occ | ~case[f"mask0_{lv}"][b, 0]
        if f"mask1_{lv}" in case:
            occ = occ | ~(A.sample(case[f"mask1_{lv}"][b].astype(np.float32), u, v)[0] > 0)
        assert np.array_equal(dbg[b, 0], u) and np.array_equal(dbg[b, 1], v)
        assert np.array_equal(dbg[b, 2], A.sample(case[f"s1_{lv}"][b], u, v)[0])
        assert np.array_equal(dbg[b, 4].astype(bool), occ)


def test_solve_level_equals_iterate():
    """dpft_ic_solve_level (3 fused iterations) == 3 x dpft_ic_iterate, bit for bit."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    f0, f1, s0, s1, invD0, invD1, K, _, _ = [a.to(dev) if a is not None else None
                                             for a in _random_case(2, 8, 1, 60, 80, seed=7)]
    pose = (torch.eye(3, device=dev).repeat(2, 1, 1), torch.zeros(2, 3, 1, device=dev))
    R1, t1 = ic.solve_level(pose, f0, f1, invD0, invD1, K, s0, s1, iters=3, remove_tru_sigma=True)
    R2, t2 = pose
    for it in range(3):
        R2, t2, _, _, _ = ic.iterate((R2, t2), f0, f1, invD0, invD1, K, s0, s1, first=(it == 0),
                                     remove_tru_sigma=True)
    assert torch.equal(R1, R2) and torch.equal(t1, t2)


def test_deterministic_repeat():
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    f0, f1, s0, s1, invD0, invD1, K, _, _ = [a.to(dev) if a is not None else None
                                             for a in _random_case(4, 32, 1, 120, 160, seed=3)]
    pose = (torch.eye(3, device=dev).repeat(4, 1, 1), torch.zeros(4, 3, 1, device=dev))
    outs = [ic.solve_level(pose, f0, f1, invD0, invD1, K, s0, s1, iters=3, remove_tru_sigma=True) for _ in range(3)]
    for R, t in outs[1:]:
        assert torch.equal(R, outs[0][0]) and torch.equal(t, outs[0][1])


def test_nonfinite_raises_assertion():
    """sigma == 0 everywhere -> division by zero -> AssertionError like check_nan (algorithms.py:1988)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    f0, f1, s0, s1, invD0, invD1, K, _, _ = [a.to(dev) if a is not None else None
                                             for a in _random_case(1, 8, 1, 32, 64, seed=1)]
    z = torch.zeros_like(s0)
    pose = (torch.eye(3, device=dev)[None], torch.zeros(1, 3, 1, device=dev))
    with pytest.raises(AssertionError):
        ic.solve_level(pose, f0, f1, invD0, invD1, K, z, z, iters=1)


@pytest.mark.parametrize("B,C,Cs,H,W,tru,masks", [
    (2, 8, 1, 60, 80, True, False),
    (1, 16, 1, 48, 64, False, True),
    (2, 5, 5, 37, 70, True, True),      # generic C, per-channel sigma
])
def test_hip_icp_matches_oracle_random(B, C, Cs, H, W, tru, masks):
    """combine_ICP (algorithms.py:668-689, 916-997) vs the fp32 oracle on smooth random scenes."""
    import torch.nn.functional as F
    from deep_prob_feature_track_amd import ic
    from oracle import ic_oracle as O
    dev = _dev()
    f0, f1, s0, s1, _, _, K, m0, m1 = _random_case(B, C, Cs, H, W, seed=B * 7 + C * 3 + W, masks=masks)
    g = torch.Generator().manual_seed(W + H)
    smooth = lambda: F.interpolate(torch.rand(B, 1, 6, 8, generator=g), size=(H, W), mode="bilinear",  # noqa: E731
                                   align_corners=True)
    depth0 = 1.0 + 2.0 * smooth()
    depth1 = depth0 + 0.01 * smooth()
    invD0, invD1 = 1.0 / depth0, 1.0 / depth1
    R = torch.eye(3).repeat(B, 1, 1)
    t = torch.zeros(B, 3, 1)
    tr_o = []
    O.solve_level(R, t, f0, f1, s0, s1, invD0, invD1, K, iters=3, remove_tru_sigma=tru, mask0=m0, mask1=m1,
                  depth0=depth0, depth1=depth1, icp_scale=0.01, trace=tr_o)
    cu = lambda a: a.to(dev) if a is not None else None  # noqa: E731
    Rg, tg = R.to(dev), t.to(dev)
    for it in range(3):
        Rg, tg, jtj, jtr, inv = ic.iterate((Rg, tg), cu(f0), cu(f1), cu(invD0), cu(invD1), cu(K), cu(s0), cu(s1),
                                           first=(it == 0), remove_tru_sigma=tru, obj_mask0=cu(m0),
                                           obj_mask1=cu(m1), depth0=cu(depth0), depth1=cu(depth1),
                                           combine_icp=True, icp_weight=0.01)
        ref = tr_o[it]
        if it == 0:
            rel = (jtj.cpu() - ref["JtJ"]).abs().max() / ref["JtJ"].abs().max()
            assert rel < 1e-4, f"JtJ rel {rel:.2e}"
        dR = (Rg.cpu() - ref["R"]).abs().max().item()
        dt = (tg.view(B, 3).cpu() - ref["t"]).abs().max().item()
        assert dR <= SE3_TOL and dt <= SE3_TOL, f"iter {it}: |dR|={dR:.2e} |dt|={dt:.2e}"


@pytest.mark.parametrize("B,H,W,levels,extreme", [(2, 120, 160, 4, False), (3, 37, 70, 3, True), (1, 8, 8, 4, True)])
def test_preprocess_depth_bit_exact(B, H, W, levels, extreme):
    """dpft_preprocess_depth == the reference's torch ops (LeastSquareTracking.py:656-661, ImagePyramids max)."""
    import torch.nn.functional as F
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(B * 100 + H)
    depth = 0.3 + 6.0 * torch.rand(B, 1, H, W, generator=g)
    if extreme:
        depth[0, 0, 0, :3] = 0.0          # 1/0 -> inf -> clamped to 10 (the max)
        depth[-1, 0, -1, -2:] = 200.0     # tiny inverse depth (the min)
    ref = torch.clamp(1.0 / depth, 0, 10)
    ref[ref == ref.min()] = 0
    ref[ref == ref.max()] = 0
    inv, dep = ic.preprocess_depth(depth.to(dev), levels, depth_pyramid=True)
    for l in range(levels):
        k = 1 << l
        want = F.max_pool2d(ref, k, k) if k > 1 else ref
        wantd = F.max_pool2d(depth, k, k) if k > 1 else depth
        assert torch.equal(inv[l].cpu(), want), f"invD level {l}"
        assert torch.equal(dep[l].cpu(), wantd), f"depth level {l}"


@pytest.mark.parametrize("B,C,H,W,masks,packed", [(2, 1, 37, 70, True, False), (1, 8, 60, 80, False, True),
                                                  (3, 3, 17, 129, True, False)])
def test_ic_residual_map_and_weighted_normal_equations(B, C, H, W, masks, packed):
    """The IC tracker's residual map (dpft_ic_residual_map) and, with per-pixel M-estimator
    weights, its normal equations (dpft_ic_iterate with DPFT_ITER_NO_UPDATE) against the
    CPU oracle's compute_warped_residual / J^T W J / J^T W r (algorithms.py:71-76,
    103-121, 1631-1632, 1919-1957); then one weighted update equals the oracle's damped
    solve of the same normal equations."""
    from deep_prob_feature_track_amd import ic
    from oracle import ic_oracle as O
    dev = _dev()
    f0, f1, _, _, invD0, invD1, K, m0, m1 = _random_case(B, C, 1, H, W, seed=7 * B + C + W, masks=masks)
    g = torch.Generator().manual_seed(3 + C)
    w = torch.rand(B, 1, H, W, generator=g)
    R = torch.eye(3).repeat(B, 1, 1)
    R[:, 0, 1], R[:, 1, 0] = 0.01, -0.01
    t = torch.full((B, 3, 1), 0.002)
    x, y = O.pixel_rays(B, H, W, K)
    r_o, occ_o = O.ic_residuals(R, t, invD0, invD1, f0, f1, x, y, K, mask0=m0, mask1=m1)
    J = O.ic_jacobian(invD0, f0, x, y, K)
    cu = lambda a: a.to(dev) if a is not None else None
    x0, x1 = (ic.pack_features(cu(f0)), ic.pack_features(cu(f1))) if packed else (cu(f0), cu(f1))
    r_g, occ_g = ic.residual_map((cu(R), cu(t)), x0, x1, cu(invD0), cu(invD1), cu(K), obj_mask0=cu(m0),
                                 obj_mask1=cu(m1))
    assert torch.equal(occ_g.cpu(), occ_o)
    # a few ulps: the CPU grid sampler's multi-channel path does not always round as the
    # single-channel fma chain the kernel reproduces (2 of 38400 values at C = 8)
    torch.testing.assert_close(r_g.cpu(), r_o, rtol=0, atol=1e-5)
    for weights in (None, w):
        JtJ_o, JtR_o = O.ic_normal_equations(J.double(), r_o.double(), None if weights is None else weights.double())
        Rg, tg, jtj, jtr, inv = ic.iterate((cu(R), cu(t)), x0, x1, cu(invD0), cu(invD1), cu(K), None, None,
                                           update=False, no_uncertainty=True, weights=cu(weights),
                                           obj_mask0=cu(m0), obj_mask1=cu(m1))
        assert torch.equal(Rg.cpu(), R) and torch.equal(tg.cpu(), t)  # NO_UPDATE leaves the pose
        assert int(inv.sum()) == int(occ_o.sum())
        rel = (jtj.cpu().double() - JtJ_o).abs().max() / JtJ_o.abs().max()
        relr = (jtr.cpu().double() - JtR_o.view(B, 6)).abs().max() / JtR_o.abs().max()
        assert rel < 1e-5 and relr < 1e-4, f"weights={weights is not None}: JtJ rel {rel:.2e}, JtR rel {relr:.2e}"
    # the weighted update: the kernel's damped solve of its own normal equations
    R1, t1, jtj, jtr, _ = ic.iterate((cu(R), cu(t)), x0, x1, cu(invD0), cu(invD1), cu(K), None, None,
                                     no_uncertainty=True, weights=cu(w), obj_mask0=cu(m0), obj_mask1=cu(m1))
    Ro, to, _ = O.damped_solve_update(jtj.cpu().double(), jtr.cpu().double().view(B, 6, 1), R.double(), t.double())
    assert (R1.cpu().double() - Ro).abs().max() < 1e-5 and (t1.cpu().double().view(B, 3) - to.view(B, 3)).abs().max() < 1e-5


def test_damped_update_matches_fp64_reference_update():
    """dpft_ic_damped_update (the ResVol trial poses and the learned-damping step in one
    launch) against the fp64 PyTorch restatement of inverse_update_pose (algorithms.py:
    2017-2054) with H = JtJ + diag(d) + 1e-6 tr(JtJ) I (1664-1691)."""
    from deep_prob_feature_track_amd import ic
    from deep_prob_feature_track_amd.models.algorithms import inverse_update_pose
    dev = _dev()
    g = torch.Generator().manual_seed(3)
    S, B = 10, 5
    A = torch.randn(B, 6, 40, generator=g, dtype=torch.float64)
    JtJ = (A @ A.transpose(1, 2)).float()
    JtR = (0.05 * torch.randn(B, 6, generator=g, dtype=torch.float64)).float()
    ang = 0.3 * torch.randn(B, 3, generator=g, dtype=torch.float64)
    from deep_prob_feature_track_amd.models.algorithms import _twist2mat
    R = _twist2mat(ang).float()
    t = torch.randn(B, 3, 1, generator=g).float()
    lam = torch.logspace(-5, 5, S, dtype=torch.float32).view(S, 1, 1)
    diag = lam * torch.diagonal(JtJ, dim1=1, dim2=2).unsqueeze(0)
    Rs, ts = ic.damped_update(JtJ.to(dev), JtR.to(dev), diag.to(dev), [R.to(dev), t.to(dev)])
    eye = torch.eye(6, dtype=torch.float64)
    for s in range(S):
        H = (JtJ.double() + torch.diag_embed(diag[s].double()) +
             1e-6 * torch.diagonal(JtJ.double(), dim1=1, dim2=2).sum(1).view(B, 1, 1) * eye)
        Rr, tr = inverse_update_pose(H, JtR.double(), [R.double(), t.double()])
        assert (Rs[s].cpu().double() - Rr).abs().max().item() < 2e-6
        assert (ts[s].cpu().double().view(B, 3) - tr).abs().max().item() < 2e-6
    # S = 1 without extra damping: lev_mar_H's matrix
    R1, t1 = ic.damped_update(JtJ.to(dev), JtR.to(dev), None, [R.to(dev), t.to(dev)])
    H = JtJ.double() + 1e-6 * torch.diagonal(JtJ.double(), dim1=1, dim2=2).sum(1).view(B, 1, 1) * eye
    Rr, tr = inverse_update_pose(H, JtR.double(), [R.double(), t.double()])
    assert (R1[0].cpu().double() - Rr).abs().max().item() < 2e-6 and (t1[0].cpu().double().view(B, 3) - tr).abs().max() < 2e-6


def test_iterate_poses_equals_per_pose_iterate():
    """ic.iterate_poses (one LevelCall, S no-update iterations) against S separate
    ic.iterate(update=False) calls: the same launches, bit for bit."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg1_160x120_c8")
    lv = golden_io.levels_torch(case, torch.float32, dev)[0]
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    S = 4
    B = R0.shape[0]
    Rs = torch.stack([R0.reshape(B, 3, 3)] * S).contiguous()
    ts = torch.stack([t0.reshape(B, 3) + 0.01 * s for s in range(S)]).contiguous()
    w = torch.rand(B, 1, *lv["f0"].shape[2:], device=dev) + 0.5
    kw = dict(no_uncertainty=True, weights=w)
    jtj, jtr = ic.iterate_poses(Rs, ts, lv["f0"], lv["f1"], lv["invD0"], lv["invD1"], K, None, None, **kw)
    for s in range(S):
        _, _, jtj1, jtr1, _ = ic.iterate((Rs[s], ts[s].view(B, 3, 1)), lv["f0"], lv["f1"], lv["invD0"], lv["invD1"], K,
                                         None, None, first=False, update=False, **kw)
        assert torch.equal(jtj[s], jtj1) and torch.equal(jtr[s], jtr1)


def test_jacobian_api_matches_oracle_and_fused_kernel():
    """The reference solver's Jacobian API on the module (precompute_jacobian_components,
    compose_inverse_jacobians, compute_jtj, compute_jtr; algorithms.py:812-887),
    materialised by HIP kernels, against the oracle's restatement of each step at the
    golden case's initial pose, and its J^T J / J^T r against the fused kernel's."""
    from oracle import ic_oracle as O
    from deep_prob_feature_track_amd import ic
    from deep_prob_feature_track_amd.models.algorithms import TrustRegionInverseWUncertainty
    dev = _dev()
    case, z = golden_io.load("cfg1_160x120_c8")
    lv = golden_io.levels_torch(case, torch.float32, "cpu")[0]
    R0, t0 = golden_io.init_pose(case, torch.float32, "cpu")
    K = torch.from_numpy(case["K"])
    B, C, H, W = lv["f0"].shape
    x, y = O.pixel_rays(B, H, W, K)
    s0C, s1C = lv["s0"].expand(B, C, H, W), lv["s1"].expand(B, C, H, W)
    # the oracle in fp64 on the same (fp32-valued) inputs: the normal equations sum ~1e6
    # products, where an fp32 bmm drifts by a few 1e-5 of its result
    dd = lambda a: a.double()
    rw, r, sigma, invalid = O.residuals(dd(R0), dd(t0), dd(lv["invD0"]), dd(lv["invD1"]), dd(lv["f0"]), dd(lv["f1"]),
                                        dd(s0C), dd(s1C), dd(x), dd(y), dd(K))
    gx, gy = O.sobel(dd(lv["f0"]))
    hx, hy = O.sobel(dd(s0C))
    Jx, Jy = O.warp_jacobian(dd(lv["invD0"]), dd(K), dd(x), dd(y))
    J_ref = O.inverse_jacobian(r, sigma, dd(s0C), (gx, gy), (hx, hy), Jx, Jy)
    JtJ_ref, JtR_ref = O.normal_equations(J_ref, rw)
    gx, gy, hx, hy, Jx, Jy, J_ref = (a.float() for a in (gx, gy, hx, hy, Jx, Jy, J_ref))
    r, sigma, rw, JtJ_ref, JtR_ref = (a.float() for a in (r, sigma, rw, JtJ_ref, JtR_ref))

    tr = TrustRegionInverseWUncertainty()
    g = lambda a: a.to(dev)
    gf0, gs0, Jxh, Jyh = tr.precompute_jacobian_components(g(lv["invD0"]), g(lv["f0"]), g(s0C), g(x), g(y), g(K))
    assert gf0.shape == (B, C, 2, H, W) and gs0.shape == (B, C, 2, H, W) and Jxh.shape == (B, H * W, 6)
    # unit-normalised gradients: where the raw Sobel of a flat patch is rounding noise
    # (|dx|, |dy| ~ 1e-7, normalised by sqrt(1e-8)) its value depends on the summation
    # order (conv2d's vs this kernel's): one ulp of sigma ~ 1 (1.2e-7) becomes 1.2e-3
    torch.testing.assert_close(gf0.cpu(), torch.stack((gx, gy), 2), rtol=0, atol=5e-4)
    torch.testing.assert_close(gs0.cpu(), torch.stack((hx, hy), 2), rtol=0, atol=3e-3)
    torch.testing.assert_close(Jxh.cpu(), Jx, rtol=1e-6, atol=1e-4)
    torch.testing.assert_close(Jyh.cpu(), Jy, rtol=1e-6, atol=1e-4)
    J, J_trs, J_rot = tr.compose_inverse_jacobians(g(r), g(sigma), g(s0C), gf0, gs0, Jxh, Jyh)
    assert J.shape == (B, C, H * W, 6) and J_trs.shape == (B, C, 3, H, W) and J_rot.shape == (B, C, 3, H, W)
    # J inherits the gradient's order-dependent noise at flat patches (bounded by
    # 1.2e-3 |Jx| / sigma on the unit-gradient scale): every element within 2e-3 of max|J|,
    # and all but <= 0.05 % of them within 1e-5 of it
    Jmax = J_ref.abs().max().item()
    d = (J.cpu() - J_ref).abs()
    assert d.max().item() <= 2e-3 * Jmax
    assert (d > 1e-5 * Jmax).float().mean().item() <= 5e-4
    d_rot = (J_rot.cpu() - (-J_ref).view(B, C, H, W, 6)[..., :3].permute(0, 1, 4, 2, 3)).abs()
    assert d_rot.max().item() <= 2e-3 * Jmax
    JtJ = tr.compute_jtj(J)
    JtR = tr.compute_jtr(J, g(rw))
    torch.testing.assert_close(JtJ.cpu(), JtJ_ref, rtol=1e-5, atol=1e-6 * JtJ_ref.abs().max().item())
    torch.testing.assert_close(JtR.cpu(), JtR_ref, rtol=1e-4, atol=1e-5 * JtR_ref.abs().max().item())
    # the fused kernel's normal equations at the same pose (never materialising J); its
    # invalid set is the fp32 one (bit-exact vs the reference's CPU arithmetic), so J^T r
    # is compared with the fp32 oracle residual (an fp64 warp flips a few boundary pixels)
    rw32 = O.residuals(R0, t0, lv["invD0"], lv["invD1"], lv["f0"], lv["f1"], s0C, s1C, x, y, K)[0]
    JtR = tr.compute_jtr(J, g(rw32))
    _, _, JtJ_f, JtR_f, _ = ic.iterate((g(R0), g(t0)), g(lv["f0"]), g(lv["f1"]), g(lv["invD0"]), g(lv["invD1"]), g(K),
                                       g(lv["s0"]), g(lv["s1"]), first=True, update=False)
    torch.testing.assert_close(JtJ_f.cpu(), JtJ.cpu(), rtol=1e-5, atol=1e-6 * JtJ_ref.abs().max().item())
    torch.testing.assert_close(JtR_f.cpu(), JtR.cpu().view(B, 6), rtol=1e-4, atol=1e-5 * JtR_ref.abs().max().item())


def test_gn_solver_and_ic_precompute_jacobian_match_oracle():
    """GN_solver (lev_mar_H + inverse_update_pose) of both solver modules and the IC
    tracker's precompute_Jacobian (algorithms.py:103-121, 836-846) against the fp64 oracle."""
    from oracle import ic_oracle as O
    from deep_prob_feature_track_amd.models.algorithms import TrustRegionBase, TrustRegionInverseWUncertainty
    dev = _dev()
    case, z = golden_io.load("cfg1_160x120_c8")
    lv = golden_io.levels_torch(case, torch.float32, "cpu")[0]
    R0, t0 = golden_io.init_pose(case, torch.float32, "cpu")
    K = torch.from_numpy(case["K"])
    B, C, H, W = lv["f0"].shape
    x, y = O.pixel_rays(B, H, W, K)
    dd = lambda a: a.double()
    J_ref = O.ic_jacobian(dd(lv["invD0"]), dd(lv["f0"]), dd(x), dd(y), dd(K)).float()
    g = lambda a: a.to(dev)
    J = TrustRegionBase().precompute_Jacobian(g(lv["invD0"]), g(lv["f0"]), g(x), g(y), g(K))
    assert J.shape == (B, C * H * W, 6)
    Jmax = J_ref.abs().max().item()
    d = (J.cpu() - J_ref).abs()   # gradient noise at flat patches, as in the Jacobian API test
    assert d.max().item() <= 2e-3 * Jmax and (d > 1e-5 * Jmax).float().mean().item() <= 5e-4
    gen = torch.Generator().manual_seed(5)
    A = torch.randn(B, 6, 30, generator=gen, dtype=torch.float64)
    JtJ = A @ A.transpose(1, 2)
    JtR = 0.01 * torch.randn(B, 6, 1, generator=gen, dtype=torch.float64)
    R_ref, t_ref, _ = O.damped_solve_update(JtJ, JtR, dd(R0), dd(t0).view(B, 3, 1))
    for mod in (TrustRegionInverseWUncertainty(), TrustRegionBase()):
        R, t = mod.GN_solver(g(JtJ.float()), g(JtR.float()), [g(R0), g(t0)])
        assert t.shape == (B, 3)  # inverse_update_pose's translation layout (geometry.py:122)
        assert (R.cpu().double() - R_ref).abs().max().item() < 2e-6
        assert (t.cpu().double().view(B, 3, 1) - t_ref).abs().max().item() < 2e-6
