"""Channel-quad feature layout (DPFT_FEATURES_C4) on a real MI355X (`-m gpu`).

The packed layout changes only where the values live, not what is computed:
every Gauss-Newton iteration of the C4 reduce kernel must give the pose, the
normal equations and the invalid count of the NCHW kernel (same per-pixel
arithmetic, channels summed in the same order), and both must match the
reference's golden vectors within the se(3) tolerance.
"""
import numpy as np
import pytest
import torch

import golden_io

pytestmark = pytest.mark.gpu

SE3_TOL = 1e-4


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _trace(name, dev, pack):
    from deep_prob_feature_track_amd import ic
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R, t = golden_io.init_pose(case, torch.float32, dev)
    t = t.view(-1, 3, 1)
    K = torch.from_numpy(case["K"]).to(dev)
    out = []
    for l in reversed(range(case["levels"])):
        d = lv[l]
        f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
        for it in range(3):
            R, t, jtj, jtr, inv = ic.iterate(
                (R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=(it == 0),
                remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                combine_icp=bool(z["opt_combine_icp"]))
            out.append(dict(R=R.cpu().numpy(), t=t.view(-1, 3).cpu().numpy(), jtj=jtj.cpu().numpy(),
                            jtr=jtr.cpu().numpy(), invalid=inv.cpu().numpy()))
    return case, z, out


@pytest.mark.parametrize("B,C,H,W", [(2, 8, 37, 70), (1, 32, 120, 160), (3, 4, 5, 3), (2, 16, 6, 10), (8, 32, 60, 80)])
def test_pack_round_trip_bit_exact(B, C, H, W):
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    x = torch.randn(B, C, H, W, device=dev)
    p = ic.pack_features(x)
    assert p.shape == (B, C // 4, H, W, 4)
    ref = x.view(B, C // 4, 4, H, W).permute(0, 1, 3, 4, 2)
    assert torch.equal(p, ref)
    assert torch.equal(ic.unpack_features(p), x)


@pytest.mark.parametrize("B,C,H,W", [(2, 8, 37, 70), (1, 32, 120, 160), (3, 4, 5, 3), (2, 16, 6, 10), (8, 32, 60, 80)])
def test_pack_channels_last_bit_exact(B, C, H, W):
    """A channels_last map packs (dpft_pack_features_nhwc) to the same bytes as its
    NCHW copy, and a solve handed the channels_last maps runs the channel-quad path on
    them: the same poses, bit for bit, as one handed the packed maps."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    x = torch.randn(B, C, H, W, device=dev)
    xl = x.contiguous(memory_format=torch.channels_last)
    assert ic.channels_last(xl) and not ic.channels_last(x)
    assert torch.equal(ic.pack_features(xl), ic.pack_features(x))
    if H < 16:
        return
    f1 = torch.roll(x, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.randn(B, C, H, W, device=dev)
    s0 = 0.5 + torch.rand(B, 1, H, W, device=dev)
    s1 = 0.5 + torch.rand(B, 1, H, W, device=dev)
    d0 = 0.2 + torch.rand(B, 1, H, W, device=dev)
    d1 = 0.2 + torch.rand(B, 1, H, W, device=dev)
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]], device=dev).repeat(B, 1)
    pose = (torch.eye(3, device=dev).repeat(B, 1, 1), torch.zeros(B, 3, 1, device=dev))
    sig0, sig1 = s0.expand(B, C, H, W), s1.expand(B, C, H, W)
    ra = ic.solve_level(pose, ic.pack_features(x), ic.pack_features(f1), d0, d1, K, sig0, sig1, iters=3,
                        remove_tru_sigma=True)
    rb = ic.solve_level(pose, xl, f1.contiguous(memory_format=torch.channels_last), d0, d1, K, sig0, sig1,
                        iters=3, remove_tru_sigma=True)
    assert torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1])


@pytest.mark.parametrize("name", ["cfg1_160x120_c8", "batch4_160x120_c8", "masks_160x120_c8",
                                  "cfg2_640x480_c32", "icp_160x120_c8"])
def test_c4_equals_nchw_and_golden(name):
    dev = _dev()
    case, z, a = _trace(name, dev, pack=False)
    _, _, b = _trace(name, dev, pack=True)
    # Chained traces: poses drift apart by summation-order noise (the channel sums are
    # regrouped, see ic_reduce_kernel's Q); both stay on the reference's trajectory.
    for i, (x, y) in enumerate(zip(a, b)):
        for prec in ("f32", "f64"):  # the contract: the reference's own trajectory within 1e-4
            if f"{prec}_R" in z:
                assert np.abs(y["R"] - z[f"{prec}_R"][i]).max() <= SE3_TOL, f"iter {i} vs {prec}"
                assert np.abs(y["t"] - z[f"{prec}_t"][i]).max() <= SE3_TOL, f"iter {i} vs {prec}"
        # between the layouts: summation-order noise (the reference's own fp32 run sits up
        # to 9.7e-5 from its fp64 run at 640x480)
        dR, dt = np.abs(x["R"] - y["R"]).max(), np.abs(x["t"] - y["t"]).max()
        assert dR < 5e-5 and dt < 5e-5, f"iter {i}: |dR| {dR:.2e} |dt| {dt:.2e}"
    assert (a[0]["invalid"] == b[0]["invalid"]).all()


@pytest.mark.parametrize("name", ["cfg1_160x120_c8", "batch4_160x120_c8", "masks_160x120_c8",
                                  "cfg2_640x480_c32", "icp_160x120_c8"])
def test_c4_iteration_from_reference_pose(name):
    """Every iteration re-started from the reference's own pose of the previous
    iteration: both layouts give the reference's invalid count exactly and the same
    normal equations (a chained trace cannot show this: the invalid count of these
    cases moves by up to 3 % under 1e-5 pose noise)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    i = 0
    for l in reversed(range(case["levels"])):
        d = lv[l]
        packed = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"]))
        for it in range(3):
            R = torch.from_numpy(z["f32_R"][i - 1]).to(dev) if i else R0
            t = (torch.from_numpy(z["f32_t"][i - 1]).to(dev) if i else t0).reshape(-1, 3, 1)
            out = []
            for f0, f1 in ((d["f0"], d["f1"]), packed):
                o = ic.iterate((R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                               remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                               obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                               combine_icp=bool(z["opt_combine_icp"]))
                out.append([x.cpu().numpy() for x in o])
            (Ra, ta, ja, ra, na), (Rb, tb, jb, rb, nb) = out
            assert (na == nb).all() and (nb == z["f32_invalid"][i]).all(), f"iter {i}: {na} {nb} {z['f32_invalid'][i]}"
            assert np.abs(ja - jb).max() / np.abs(ja).max() < 1e-6, f"iter {i}"
            assert np.abs(ra - rb).max() / np.abs(ra).max() < 1e-4, f"iter {i}"
            i += 1


@pytest.mark.parametrize("no_unc", [False, True])
def test_c4_random_ragged_solve_and_residual(no_unc):
    """Ragged tiles, C = 12 (a non-specialised channel count), masks, IC and U_IC."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(7)
    B, C, H, W = 2, 12, 37, 70
    f0 = torch.rand(B, C, H, W, generator=g)
    f1 = torch.roll(f0, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    s1 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    d0 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    d1 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    m1 = torch.rand(B, 1, H, W, generator=g) > 0.2
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    T = [v.to(dev) for v in (f0, f1, s0, s1, d0, d1, m1, K)]
    f0, f1, s0, s1, d0, d1, m1, K = T
    pose = (torch.eye(3, device=dev).repeat(B, 1, 1), torch.zeros(B, 3, 1, device=dev))
    kw = dict(no_uncertainty=True) if no_unc else dict(remove_tru_sigma=True)
    sa, sb = (None, None) if no_unc else (s0, s1)
    ra = ic.solve_level(pose, f0, f1, d0, d1, K, sa, sb, iters=3, obj_mask1=m1, **kw)
    rb = ic.solve_level(pose, f0, f1, d0, d1, K, sa, sb, iters=3, obj_mask1=m1, pack=True, **kw)
    assert (ra[0] - rb[0]).abs().max().item() < 1e-5 and (ra[1] - rb[1]).abs().max().item() < 1e-5
    la = ic.residual_level(pose, f0, f1, d0, d1, K, sa, sb, obj_mask1=m1, **kw)
    lb = ic.residual_level(pose, ic.pack_features(f0), ic.pack_features(f1), d0, d1, K, sa, sb, obj_mask1=m1, **kw)
    torch.testing.assert_close(la, lb, rtol=1e-6, atol=0)


def test_c4_rejects_per_channel_sigma():
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    B, C, H, W = 1, 8, 16, 16
    x = ic.pack_features(torch.rand(B, C, H, W, device=dev))
    s = torch.rand(B, C, H, W, device=dev) + 0.5
    d = torch.rand(B, 1, H, W, device=dev) + 0.2
    K = torch.tensor([[12.0, 12.0, 7.5, 7.5]], device=dev)
    pose = (torch.eye(3, device=dev)[None], torch.zeros(1, 3, 1, device=dev))
    with pytest.raises(ValueError, match="single sigma plane"):
        ic.solve_level(pose, x, x, d, d, K, s, s)


SCHEDULES = ["march", "march-reverse", "split"]


def _sched_kw(schedule):
    """test schedule name -> ic.iterate keywords ("march-reverse": the odd-iteration order)"""
    if schedule == "march-reverse":
        return dict(schedule="march", reverse=True)
    return dict(schedule=schedule)


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_c4_schedules_from_reference_pose(schedule):
    """cfg2 (C = 32, 4 levels): every reduce schedule, re-started from the reference's
    pose of the previous iteration, gives the reference's invalid count exactly and the
    NCHW kernel's normal equations (summation-order noise only)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    i = 0
    for l in reversed(range(case["levels"])):
        d = lv[l]
        packed = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"]))
        for it in range(3):
            R = torch.from_numpy(z["f32_R"][i - 1]).to(dev) if i else R0
            t = (torch.from_numpy(z["f32_t"][i - 1]).to(dev) if i else t0).reshape(-1, 3, 1)
            out = []
            for (f0, f1), kw in (((d["f0"], d["f1"]), {}), (packed, _sched_kw(schedule))):
                o = ic.iterate((R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                               remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), **kw)
                out.append([x.cpu().numpy() for x in o])
            (Ra, ta, ja, ra, na), (Rb, tb, jb, rb, nb) = out
            assert (na == nb).all() and (nb == z["f32_invalid"][i]).all(), f"iter {i}: {na} {nb}"
            assert np.abs(ja - jb).max() / np.abs(ja).max() < 1e-6, f"iter {i}"
            assert np.abs(ra - rb).max() / np.abs(ra).max() < 1e-4, f"iter {i}"
            for prec in ("f32", "f64"):
                assert np.abs(Rb - z[f"{prec}_R"][i]).max() <= SE3_TOL, f"iter {i} vs {prec}"
                assert np.abs(tb.reshape(-1, 3) - z[f"{prec}_t"][i]).max() <= SE3_TOL, f"iter {i} vs {prec}"
            i += 1


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("C,H,W,no_unc,masks", [(32, 37, 70, False, True), (16, 61, 129, True, False),
                                                 (32, 3, 2, False, False), (16, 130, 63, False, True)])
def test_c4_schedules_random(schedule, C, H, W, no_unc, masks):
    """Ragged strips (W not a multiple of 62), tiny levels (H = 3, W = 2), masks, IC and
    U_IC with truncated sigma: each schedule against the NCHW kernel."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(C * 1000 + H)
    B = 3
    f0 = torch.rand(B, C, H, W, generator=g)
    f1 = torch.roll(f0, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    s1 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    d0 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    d1 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    m0 = torch.rand(B, 1, H, W, generator=g) > 0.1
    m1 = torch.rand(B, 1, H, W, generator=g) > 0.2
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    f0, f1, s0, s1, d0, d1, m0, m1, K = [v.to(dev) for v in (f0, f1, s0, s1, d0, d1, m0, m1, K)]
    R = torch.eye(3, device=dev).repeat(B, 1, 1)
    R[:, 0, 1], R[:, 1, 0] = 0.01, -0.01
    t = torch.full((B, 3, 1), 0.003, device=dev)
    kw = dict(no_uncertainty=True) if no_unc else dict(remove_tru_sigma=True)
    if masks:
        kw.update(obj_mask0=m0, obj_mask1=m1)
    sa, sb = (None, None) if no_unc else (s0, s1)
    a = ic.iterate((R, t), f0, f1, d0, d1, K, sa, sb, first=True, **kw)
    b = ic.iterate((R, t), ic.pack_features(f0), ic.pack_features(f1), d0, d1, K, sa, sb, first=True,
                   **_sched_kw(schedule), **kw)
    assert torch.equal(a[4], b[4])  # invalid counts
    torch.testing.assert_close(b[2], a[2], rtol=2e-6, atol=1e-6 * a[2].abs().max().item())
    torch.testing.assert_close(b[3], a[3], rtol=1e-4, atol=1e-5 * a[3].abs().max().item())
    torch.testing.assert_close(b[0], a[0], rtol=0, atol=2e-5)
    torch.testing.assert_close(b[1], a[1], rtol=0, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("reverse", [False, True])
@pytest.mark.parametrize("C,H,W,masks", [(32, 45, 131, True), (16, 64, 70, False), (32, 120, 160, False),
                                         (16, 6, 2050, False)])
def test_c4_combine_icp_march(C, H, W, masks, reverse):
    """combine_ICP (MODE 1) on the channel-quad marching path (C = 16 / 32: the ring, the
    tap cache and the per-pixel ICP term of ic_reduce_kernel<..., true>), forward and
    reverse marching order, against the NCHW kernel on the same inputs.  The sizes reach every
    pixel loop of the ICP records pass: masks; no masks with the coordinate table and IEEE tap
    divisions (64 x 70: not a verified divisor size); with the constant-divisor taps (120 x 160);
    without the table (W + H > kIcpTab, 6 x 2050)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(C * 7 + H)
    B = 2
    f0 = torch.rand(B, C, H, W, generator=g)
    f1 = torch.roll(f0, shifts=(1, 1), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    s1 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    dep0 = (1.5 + 0.3 * torch.sin(xx / 7.0) + 0.2 * torch.cos(yy / 5.0)).expand(B, 1, H, W).contiguous()
    dep1 = torch.roll(dep0, shifts=(1, 1), dims=(2, 3)) + 0.001 * torch.rand(B, 1, H, W, generator=g)
    d0, d1 = 1.0 / dep0, 1.0 / dep1
    m0 = torch.rand(B, 1, H, W, generator=g) > 0.1
    m1 = torch.rand(B, 1, H, W, generator=g) > 0.2
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    f0, f1, s0, s1, d0, d1, dep0, dep1, m0, m1, K = [
        v.to(dev) for v in (f0, f1, s0, s1, d0, d1, dep0, dep1, m0, m1, K)]
    R = torch.eye(3, device=dev).repeat(B, 1, 1)
    R[:, 0, 1], R[:, 1, 0] = 0.01, -0.01
    t = torch.full((B, 3, 1), 0.003, device=dev)
    kw = dict(remove_tru_sigma=True, combine_icp=True, depth0=dep0, depth1=dep1, icp_weight=0.01)
    if masks:
        kw.update(obj_mask0=m0, obj_mask1=m1)
    a = ic.iterate((R, t), f0, f1, d0, d1, K, s0, s1, first=True, reverse=reverse, **kw)
    b = ic.iterate((R, t), ic.pack_features(f0), ic.pack_features(f1), d0, d1, K, s0, s1, first=True,
                   reverse=reverse, schedule="march", **kw)
    assert torch.equal(a[4], b[4])  # invalid counts
    torch.testing.assert_close(b[2], a[2], rtol=2e-6, atol=1e-6 * a[2].abs().max().item())
    torch.testing.assert_close(b[3], a[3], rtol=1e-4, atol=1e-5 * a[3].abs().max().item())
    torch.testing.assert_close(b[0], a[0], rtol=0, atol=2e-5)
    torch.testing.assert_close(b[1], a[1], rtol=0, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
def test_pyramid_solver_extrema_prepass_bit_identical(packed):
    """PyramidSolver's one-launch sigma0 extrema pre-pass (per-level workspace slots,
    DPFT_EXTREMA_READY) against the per-level path (dpft_ic_solve_level computing the
    extrema itself): the extrema are exact min / max, so the poses are bit-identical."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    pk = (lambda x: ic.pack_features(x)) if packed else (lambda x: x)
    levels = [dict(x0=pk(d["f0"]), x1=pk(d["f1"]), invD0=d["invD0"], invD1=d["invD1"], sigma0=d["s0"],
                   sigma1=d["s1"]) for d in lv]
    solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True)
    assert solver.extrema_prepass
    R, t = R0.clone().contiguous(), t0.reshape(-1, 3).clone().contiguous()
    solver.run(R, t, per_level=True)
    Rs, ts = R0.clone(), t0.reshape(-1, 3, 1).clone()
    for l in reversed(range(len(levels))):
        d = levels[l]
        Rs, ts = ic.solve_level((Rs, ts), d["x0"], d["x1"], d["invD0"], d["invD1"], K / 2 ** l, d["sigma0"],
                                d["sigma1"], iters=3, remove_tru_sigma=True)
    torch.cuda.synchronize()
    assert torch.equal(R, Rs) and torch.equal(t, ts.reshape(-1, 3))
    for prec in ("f32", "f64"):
        assert np.abs(R.cpu().numpy() - z[f"{prec}_R"][-1]).max() <= SE3_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("no_unc", [False, True])
@pytest.mark.parametrize("B", [1, 8, 64])
def test_pyramid_entry_point(B, no_unc):
    """dpft_ic_solve_pyramid (the level loop of LeastSquareTracking.forward in one C call)
    against one dpft_ic_solve_level call per level: the same launches, bit for bit, and
    on the golden case the reference's own poses.  B = 8: the bench's batch, B = 64: the
    cfg3 batch on one GPU (the golden pair replicated: the batch-global extrema equal the
    pair's own, so every pair must land on the reference's B = 1 poses); B = 1."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    rep = lambda x: x.repeat(B, *([1] * (x.dim() - 1)))
    levels = [dict(x0=rep(ic.pack_features(d["f0"])), x1=rep(ic.pack_features(d["f1"])), invD0=rep(d["invD0"]),
                   invD1=rep(d["invD1"]), sigma0=rep(d["s0"]), sigma1=rep(d["s1"])) for d in lv]
    solver = ic.PyramidSolver(levels, rep(K), iters=3, remove_tru_sigma=not no_unc)
    if no_unc:
        for c in solver.calls:
            c.desc.flags |= ic.N.NO_UNCERTAINTY
    outs = []
    for per_level in (False, True):
        R, t = rep(R0).contiguous(), rep(t0.reshape(-1, 3)).contiguous()
        solver.run(R, t, per_level=per_level)
        torch.cuda.synchronize()
        ic.check_status(solver.status)
        outs.append((R.cpu().numpy(), t.cpu().numpy()))
    (Ra, ta), (Rb, tb) = outs
    assert np.array_equal(Ra, Rb) and np.array_equal(ta, tb)
    if not no_unc:
        for prec in ("f32", "f64"):
            assert np.abs(Ra - z[f"{prec}_R"][-1]).max() <= SE3_TOL
            assert np.abs(ta - z[f"{prec}_t"][-1]).max() <= SE3_TOL


@pytest.mark.gpu
def test_pyramid_solver_iterate_uses_ready_extrema():
    """bench.py times PyramidSolver.iterate(first=True) after run(): with
    DPFT_EXTREMA_READY it reads the level's slot filled by the pre-pass, and must match a
    standalone iteration that computes the extrema itself, bit for bit."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    levels = [dict(x0=ic.pack_features(d["f0"]), x1=ic.pack_features(d["f1"]), invD0=d["invD0"], invD1=d["invD1"],
                   sigma0=d["s0"], sigma1=d["s1"]) for d in lv]
    solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True)
    R, t = R0.clone().contiguous(), t0.reshape(-1, 3).clone().contiguous()
    solver.run(R, t)
    Ra, ta = R.clone(), t.clone()
    solver.iterate(0, Ra, ta, first=True)
    d = levels[0]
    Rb, tb, _, _, _ = ic.iterate((R.clone(), t.reshape(-1, 3, 1).clone()), d["x0"], d["x1"], d["invD0"], d["invD1"], K,
                                 d["sigma0"], d["sigma1"], first=True, remove_tru_sigma=True)
    torch.cuda.synchronize()
    assert torch.equal(Ra, Rb) and torch.equal(ta, tb.reshape(-1, 3))


@pytest.mark.gpu
def test_inflight_solves_bit_identical():
    """bench.py --inflight: independent batches solved concurrently on separate streams,
    each with its own PyramidSolver (workspace) and pose buffers, give exactly the poses
    each gives alone (no shared state but the read-only inputs)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    B, S = 8, 3
    rep = lambda x: x.repeat(B, *([1] * (x.dim() - 1)))
    levels = [dict(x0=rep(ic.pack_features(d["f0"])), x1=rep(ic.pack_features(d["f1"])), invD0=rep(d["invD0"]),
                   invD1=rep(d["invD1"]), sigma0=rep(d["s0"]), sigma1=rep(d["s1"])) for d in lv]
    # slot j starts from its own initial translations: distinct solves over shared inputs
    inits = []
    for j in range(S):
        t = rep(t0.reshape(-1, 3)).clone()
        t += 1e-3 * (j + 1) * torch.arange(B, device=dev, dtype=torch.float32).view(B, 1) / B
        inits.append((rep(R0).contiguous(), t.contiguous()))
    solvers = [ic.PyramidSolver(levels, rep(K), iters=3, remove_tru_sigma=True) for _ in range(S)]
    alone = []
    for j in range(S):
        R, t = inits[j][0].clone(), inits[j][1].clone()
        solvers[j].run(R, t)
        torch.cuda.synchronize()
        alone.append((R, t))
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    poses = [(inits[j][0].clone(), inits[j][1].clone()) for j in range(S)]
    torch.cuda.synchronize()
    for _ in range(4):
        for j in range(S):
            with torch.cuda.stream(streams[j]):
                poses[j][0].copy_(inits[j][0])
                poses[j][1].copy_(inits[j][1])
                solvers[j].run(*poses[j])
        torch.cuda.synchronize()
        for j in range(S):
            ic.check_status(solvers[j].status)
            assert torch.equal(poses[j][0], alone[j][0]) and torch.equal(poses[j][1], alone[j][1])
    assert not torch.equal(alone[0][1], alone[1][1])


def _grouped_case(dev, G=4, B=8):
    """G batches of B copies of the golden cfg2 pair; batch g's sigma0 / sigma1 scaled by
    1 + g / 4 (so every batch has its own sigma extrema) and each pair started from its
    own initial translation."""
    from deep_prob_feature_track_amd import ic
    case, z = golden_io.load("cfg2_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    n = G * B
    rep = lambda x: x.repeat(n, *([1] * (x.dim() - 1)))
    scale = (1.0 + torch.arange(G, device=dev, dtype=torch.float32) / 4).repeat_interleave(B).view(n, 1, 1, 1)
    levels = [dict(x0=rep(ic.pack_features(d["f0"])), x1=rep(ic.pack_features(d["f1"])), invD0=rep(d["invD0"]),
                   invD1=rep(d["invD1"]), sigma0=(rep(d["s0"]) * scale).contiguous(),
                   sigma1=(rep(d["s1"]) * scale).contiguous()) for d in lv]
    t = rep(t0.reshape(-1, 3)).clone()
    t[:, 0] += 2e-3 * (torch.arange(n, device=dev, dtype=torch.float32) % B) / B
    return z, levels, rep(K), rep(R0).contiguous(), t.contiguous()


def _invalid_counts(solver, level, R, t):
    """#invalid pixels per pair of one no-update iteration of `level` (exact integers)."""
    import ctypes
    from deep_prob_feature_track_amd import ic
    c = solver.calls[level]
    inv = torch.zeros(c.B, dtype=torch.int32, device=R.device)
    Rc, tc = R.contiguous().clone(), t.contiguous().clone()  # kept alive across the launch
    solver.prepare_extrema()
    rc = ic.N.lib().dpft_ic_iterate(ctypes.byref(c.desc), ctypes.byref(c.tens), ic._ptr(Rc), ic._ptr(tc), None,
                                    None, ic._ptr(inv), 1 | 4, ic._ptr(solver.ws), solver.ws_bytes,
                                    ic._stream(R.device))
    ic.N.check(rc, "dpft_ic_iterate")
    torch.cuda.synchronize()
    return inv.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("G", [4, 16])
def test_grouped_batches_solve_as_separate_calls(G):
    """DPFT_GROUP (bench.py --groups): G independent 8-pair batches in every launch (16 is
    the bench's operating point: 4 workgroups = 16 waves per pair, fewer than two per
    level-0 strip, so the marching bands are not a (row band x strip) grid).  Each
    batch is solved as a call of its own -- its own truncated-sigma extrema: the invalid
    pixel counts equal those of separate 8-pair calls exactly (and differ from one
    32-pair batch, whose extrema span all four), the poses within the fp32 summation
    noise (the launch splits each pair into fewer workgroup records), and batch 0 (the
    golden pair, unscaled) lands on the reference's poses."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    B = 8
    z, levels, K, R0, t0 = _grouped_case(dev, G, B)
    grouped = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True, group=B)
    assert grouped.group == B
    R, t = R0.clone(), t0.clone()
    grouped.run(R, t)
    torch.cuda.synchronize()
    ic.check_status(grouped.status)
    sl = lambda g: slice(g * B, (g + 1) * B)
    for g in range(G):
        lv_g = [{k: v[sl(g)] for k, v in d.items()} for d in levels]
        alone = ic.PyramidSolver(lv_g, K[sl(g)].contiguous(), iters=3, remove_tru_sigma=True)
        Ra, ta = R0[sl(g)].clone(), t0[sl(g)].clone()
        alone.run(Ra, ta)
        torch.cuda.synchronize()
        # (another fp32 summation grouping: measured up to 2.6e-5 on t; the reference's own
        # fp32 noise floor at 640x480 is 9.7e-5)
        torch.testing.assert_close(R[sl(g)], Ra, rtol=0, atol=5e-5)
        torch.testing.assert_close(t[sl(g)], ta, rtol=0, atol=5e-5)
        for level in (0, 1, 2):  # marching (level 1: the grid + pool split against the 8-pair grid) and split
            assert np.array_equal(_invalid_counts(grouped, level, R, t)[sl(g)],
                                  _invalid_counts(alone, level, R[sl(g)], t[sl(g)]))
    one_batch = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True)
    assert not np.array_equal(_invalid_counts(one_batch, 0, R, t), _invalid_counts(grouped, 0, R, t))
    for prec in ("f32", "f64"):
        assert np.abs(R[sl(0)].cpu().numpy()[:1] - z[f"{prec}_R"][-1]).max() <= SE3_TOL


@pytest.mark.gpu
def test_grouped_solve_deterministic_and_graph_capturable():
    """The grouped solve replayed from one HIP graph equals the eager solve bit for bit
    (fixed-order reductions, per-batch completion counters left at zero)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    z, levels, K, R0, t0 = _grouped_case(dev, 2, 8)
    solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True, group=8)
    R, t = R0.clone(), t0.clone()
    solver.run(R, t)
    torch.cuda.synchronize()
    Re, te = R.clone(), t.clone()
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        R.copy_(R0)
        t.copy_(t0)
        solver.run(R, t)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        R.copy_(R0)
        t.copy_(t0)
        solver.run(R, t)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(R, Re) and torch.equal(t, te)


@pytest.mark.gpu
def test_nchw_solve_packs_on_entry_bit_identical():
    """A solve handed the reference's NCHW features (C % 16 == 0, one sigma plane) packs them
    once on entry into the workspace and runs the channel-quad kernels (dpft_ic_solve_level /
    dpft_ic_solve_pyramid, packs_on_entry): the cfg3 batch at 640x480, C = 32 -- the pyramid
    entry point, the per-level entry point and the drop-in solver module's forward
    (algorithms.py:611-723) chained over the levels -- gives the poses of the pre-packed solve
    bit for bit, and those lie on the reference's run of the batch."""
    from deep_prob_feature_track_amd import ic
    from deep_prob_feature_track_amd.models.algorithms import TrustRegionInverseWUncertainty
    dev = _dev()
    name = "cfg3_b8_640x480_c32"
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    B, C, H, W = lv[0]["f0"].shape
    assert C % 16 == 0

    def levels(pack):
        return [dict(x0=ic.pack_features(d["f0"]) if pack else d["f0"], x1=ic.pack_features(d["f1"]) if pack else d["f1"],
                     invD0=d["invD0"], invD1=d["invD1"], sigma0=d["s0"], sigma1=d["s1"]) for d in lv]
    outs = {}
    for pack in (True, False):
        solver = ic.PyramidSolver(levels(pack), K, iters=3, remove_tru_sigma=True)
        for per_level in (False, True):
            R, t = R0.clone().contiguous(), t0.reshape(B, 3).clone().contiguous()
            solver.run(R, t, per_level=per_level)
            torch.cuda.synchronize()
            ic.check_status(solver.status)
            outs[(pack, per_level)] = (R, t)
    for key in outs:
        assert torch.equal(outs[key][0], outs[(True, False)][0]) and torch.equal(outs[key][1], outs[(True, False)][1]), key
    # the module, level by level (LeastSquareTracking.forward's loop) on NCHW and packed features
    tr = TrustRegionInverseWUncertainty(3, remove_tru_sigma=True)
    mods = {}
    for pack in (True, False):
        pose = [R0.clone(), t0.reshape(B, 3, 1).clone()]
        with torch.no_grad():
            for l, d in reversed(list(enumerate(levels(pack)))):
                pose = tr(pose, d["x0"], d["x1"], d["invD0"], d["invD1"], K / 2 ** l, d["sigma0"].expand(B, C, -1, -1),
                          d["sigma1"].expand(B, C, -1, -1), vis_res=False)[0]
        mods[pack] = pose
    assert torch.equal(mods[True][0], mods[False][0]) and torch.equal(mods[True][1], mods[False][1])
    assert mods[False][1].shape == (B, 3)
    dev_pose = golden_io.pose_deviation(mods[False][0], mods[False][1], z, "f32")
    floor = golden_io.noise_floor(z)
    bound = np.maximum(SE3_TOL, 1.5 * floor[-1]) if floor is not None else SE3_TOL
    assert (dev_pose <= bound).all(), (dev_pose, bound)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ragged", "misaligned"])
def test_nchw_entry_pack_fallback_bit_identical(case):
    """The entry pack's general kernel (pack_c4_pair_kernel: H W not a multiple of 4, or feature
    pointers not 16-byte aligned -- a view at a one-float offset) gives the poses of the
    caller-packed solve bit for bit (C = 16, so the NCHW solve packs on entry)."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    g = torch.Generator().manual_seed(11)
    B, C, (H, W) = 3, 16, ((37, 70) if case == "ragged" else (40, 64))
    f0 = torch.rand(B, C, H, W, generator=g)
    f1 = torch.roll(f0, shifts=(1, 2), dims=(2, 3)) + 0.01 * torch.rand(B, C, H, W, generator=g)
    s0 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    s1 = 0.5 + torch.rand(B, 1, H, W, generator=g)
    d0 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    d1 = 0.2 + torch.rand(B, 1, H, W, generator=g)
    K = torch.tensor([[W * 0.8, W * 0.8, (W - 1) / 2, (H - 1) / 2]]).repeat(B, 1)
    f0, f1, s0, s1, d0, d1, K = (v.to(dev) for v in (f0, f1, s0, s1, d0, d1, K))
    if case == "misaligned":  # the same values at a 4-byte offset from a 16-byte boundary
        f0 = torch.cat([torch.zeros(1, device=dev), f0.reshape(-1)])[1:].view(B, C, H, W)
        f1 = torch.cat([torch.zeros(1, device=dev), f1.reshape(-1)])[1:].view(B, C, H, W)
        assert f0.data_ptr() % 16 and f1.data_ptr() % 16
    pose = (torch.eye(3, device=dev).repeat(B, 1, 1), torch.zeros(B, 3, 1, device=dev))
    ra = ic.solve_level(pose, f0, f1, d0, d1, K, s0, s1, iters=3, remove_tru_sigma=True)
    rb = ic.solve_level(pose, f0, f1, d0, d1, K, s0, s1, iters=3, remove_tru_sigma=True, pack=True)
    torch.cuda.synchronize()
    assert torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1])
