"""BASELINE.json configurations 3, 4 and 5 on a real MI355X (`-m gpu`), against fixtures the
reference itself produced (tests/golden/gen_golden.py).

* cfg5 -- joint feature-metric + ICP (combine_ICP, weight 0.01) at 640x480, C = 32, 4 levels:
  the whole solve, every iteration restarted from the reference's pose, and independent
  batches in one call (DPFT_GROUP: per-batch depth1 extrema for the normal map).
* cfg3 -- the bench's first batch: 8 distinct ordered pairs at 640x480, C = 32, so the
  batch-global truncated-sigma extrema (algorithms.py:1975-1980) span different pairs; one
  call and the grouped launch of the bench (every batch solved as its own call).
* cfg4 -- object masks, 4 levels at 160x120, C = 8, large-baseline starts applied as the
  solver-level initial pose (three start sets + the identity start), and the B = 256 sweep
  of convergence_basin.solve_from_starts against the oracle and against separate calls.

Tolerances: se(3) 1e-4 against the fp32 and fp64 reference runs (BASELINE.json); invalid-
pixel counts exact when an iteration starts from the reference's own pose.
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


def _solver_levels(case, dev, pack):
    """Per-level PyramidSolver dicts of a recipe case (features packed to channel quads when
    `pack`)."""
    from deep_prob_feature_track_amd import ic
    out = []
    for d in golden_io.levels_torch(case, torch.float32, dev):
        e = dict(x0=ic.pack_features(d["f0"]) if pack else d["f0"], x1=ic.pack_features(d["f1"]) if pack else d["f1"],
                 invD0=d["invD0"], invD1=d["invD1"], sigma0=d["s0"], sigma1=d["s1"])
        for k in ("depth0", "depth1"):
            if k in d:
                e[k] = d[k]
        if "mask0" in d:
            e["obj_mask0"], e["obj_mask1"] = d["mask0"], d["mask1"]
        out.append(e)
    return out


def _assert_on_reference(R, t, z, i=-1, tol=SE3_TOL, what="", precs=("f32", "f64")):
    R = R.cpu().numpy().reshape(-1, 3, 3)
    t = t.cpu().numpy().reshape(-1, 3)
    for prec in precs:
        if f"{prec}_R" in z:
            dR = np.abs(R - z[f"{prec}_R"][i]).max()
            dt = np.abs(t - z[f"{prec}_t"][i]).max()
            assert dR <= tol and dt <= tol, f"{what} vs {prec} reference: |dR| {dR:.2e} |dt| {dt:.2e}"


def _chained_poses(name, dev, pack=True):
    """Every iteration of the GPU's own chained solve of a fixture: one dpft_ic_iterate per
    iteration from the GPU's previous pose (odd iterations of a level reversed: the schedule
    of dpft_ic_solve_level) -> (R [iters,B,3,3], t [iters,B,3]) numpy."""
    from deep_prob_feature_track_amd import ic
    case, z = golden_io.load(name, check_digests=False)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R, t = golden_io.init_pose(case, torch.float32, dev)
    t = t.reshape(-1, 3, 1)
    K = torch.from_numpy(case["K"]).to(dev)
    Rs, ts = [], []
    for l in reversed(range(case["levels"])):
        d = lv[l]
        f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
        for it in range(3):
            R, t, _, _, _ = ic.iterate(
                (R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                reverse=(it & 1) == 1, remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                combine_icp=bool(z["opt_combine_icp"]))
            Rs.append(R.cpu().numpy())
            ts.append(t.reshape(-1, 3).cpu().numpy())
    return np.stack(Rs), np.stack(ts)


FLOOR_FACTOR = golden_io.FLOOR_FACTOR  # the frozen rule's constants (golden_io, tests/test_parity_rule.py)


def _assert_within_reference_envelope(R, t, z, what="", i=-1):
    """A chained pose (iteration i; R [B,3,3], t [B,3]) against the reference's fp32 and
    fp64 runs, PER PAIR, by the frozen rule (golden_io.envelope): within 1e-4 or,
    where the reference's own trajectory of that pair moves by more than that when only rounding
    changes (golden_io.noise_floor: 33 runs, every update moved by the GPU's one-step deviation,
    and a one-thread run), within 1.5x that pair's own floor; at most as many pairs beyond that
    as ONE of the reference's own runs shows against the others' floors, capped at 4, each within
    twice its own bound; no more pairs beyond 1e-4 than any rounding-only run moves that far.
    Against the fp64 run each pair's bound is its fp32 bound plus the reference's own
    fp32-vs-fp64 distance of that pair (the triangle inequality through the fp32 run).
    Returns (deviation vs fp32 [B], floor [B])."""
    dev = golden_io.pose_deviation(R, t, z, "f32", i)
    msgs, bound, floor, over_pair = golden_io.envelope(dev, z, i)
    assert not msgs, f"{what}: " + "; ".join(msgs)
    allowed = golden_io.allowance(z, i)
    detail = {int(b): (f"{dev[b]:.2e}", f"floor {floor[b]:.2e}") for b in over_pair[:20]}
    n_over = int((dev > SE3_TOL).sum())
    n_ref = golden_io.noise_counts_beyond(z, SE3_TOL, i)
    if "f64_R" in z:
        d3264 = np.maximum(np.abs(z["f32_R"][i] - z["f64_R"][i]).max(axis=(1, 2)),
                           np.abs(z["f32_t"][i] - z["f64_t"][i]).max(axis=1))
        dev64 = golden_io.pose_deviation(R, t, z, "f64", i)
        b64 = bound + d3264  # the pair's fp32 bound plus the reference's own fp32-to-fp64 distance
        bad = np.flatnonzero(dev64 > b64)
        assert bad.size == 0, (f"{what} iter {i}: vs fp64 beyond the bound: "
                               + str({int(b): (f"{dev64[b]:.2e}", f"bound {b64[b]:.2e}") for b in bad[:20]}))
        over = np.flatnonzero(np.maximum(dev, dev64) > SE3_TOL)
    else:
        over = np.flatnonzero(dev > SE3_TOL)
    if over_pair.size:
        print(f"{what} iter {i}: {over_pair.size} pair(s) beyond their own bound (the rule admits {allowed}), "
              f"within {golden_io.EXCEEDANCE_SCALE} x their own bound: {detail}")
    if i in (-1, z["f32_R"].shape[0] - 1):
        print(f"{what}: {dev.size - over.size} of {dev.size} pairs within 1e-4 of both reference runs; max vs fp32 "
              f"{dev.max():.2e}" + (f", vs fp64 {dev64.max():.2e}" if "f64_R" in z else "")
              + f"; batch-max floor {floor.max():.2e} (diagnostic)")
        print(f"  vs the fp32 run alone: {int((dev <= SE3_TOL).sum())} of {dev.size} within 1e-4 ({n_over} beyond; "
              f"the reference's rounding-only runs: max {int(n_ref.max())}), {int((dev <= floor).sum())} within "
              f"their floor" + (f"; vs the fp64 run: {int((dev64 <= SE3_TOL).sum())} within 1e-4, "
                                 f"{int((dev64 <= d3264 + SE3_TOL).sum())} within the reference's own fp32-fp64 "
                                 f"distance + 1e-4" if "f64_R" in z else ""))
        if over.size:
            print("  beyond 1e-4 (pair: vs fp32 / vs fp64 / own noise floor / reference fp32-fp64):",
                  {int(b): (f"{dev[b]:.2e}", f"{dev64[b]:.2e}" if "f64_R" in z else "-", f"{floor[b]:.2e}",
                            f"{d3264[b]:.2e}" if "f64_R" in z else "-") for b in over[:40]})
    return dev, floor


def _assert_chain_within_envelope(name, dev, what=None):
    """Every iteration of the GPU's chained solve (_chained_poses) within its pairs' bounds."""
    _, z = golden_io.load(name, check_digests=False)
    Rs, ts = _chained_poses(name, dev)
    for i in range(Rs.shape[0]):
        _assert_within_reference_envelope(Rs[i], ts[i], z, what=what or name, i=i)
    return Rs, ts


def _restart_iterations(name, dev, pack, **extra):
    """Every iteration from the reference's pose of the previous one: exact invalid counts,
    normal equations and the updated pose to rounding."""
    from deep_prob_feature_track_amd import ic
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    L, i = case["levels"], 0
    for l in reversed(range(L)):
        d = lv[l]
        f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
        for it in range(3):
            R = torch.from_numpy(z["f32_R"][i - 1]).to(dev) if i else R0
            t = (torch.from_numpy(z["f32_t"][i - 1]).to(dev) if i else t0).reshape(-1, 3, 1)
            Rn, tn, jtj, jtr, inv = ic.iterate(
                (R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                reverse=(it & 1) == 1, remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                combine_icp=bool(z["opt_combine_icp"]), **extra)
            inv = inv.cpu().numpy()
            assert np.array_equal(inv, z["f32_invalid"][i]), f"{name} iter {i}: {inv} vs {z['f32_invalid'][i]}"
            ref_j, ref_r = z["f32_jtj"][i], z["f32_jtr"][i]
            assert np.abs(jtj.cpu().numpy() - ref_j).max() / np.abs(ref_j).max() < 1e-5, f"iter {i} JtJ"
            assert np.abs(jtr.cpu().numpy() - ref_r).max() / np.abs(ref_r).max() < 1e-4, f"iter {i} JtR"
            # one step from the fp32 run's pose: against that run's next pose
            _assert_on_reference(Rn, tn, z, i, tol=2e-5, what=f"{name} iter {i} (one step)", precs=("f32",))
            i += 1


# ------------------------------------------------------------------------------ cfg5
@pytest.mark.parametrize("pack", [True, False])
def test_cfg5_icp_full_size_solve(pack):
    """combine_ICP at 640x480, C = 32: the 4-level solve (one dpft_ic_solve_pyramid call:
    the sigma0 extrema pre-pass, each level's depth1 extrema and normal map) lands on the
    reference's fp32 and fp64 poses, and equals the per-level calls bit for bit."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("icp_640x480_c32")
    solver = ic.PyramidSolver(_solver_levels(case, dev, pack), torch.from_numpy(case["K"]).to(dev), iters=3,
                              remove_tru_sigma=True, combine_icp=True)
    assert solver.extrema_prepass
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    outs = []
    for per_level in (False, True):
        R, t = R0.clone().contiguous(), t0.reshape(-1, 3).clone().contiguous()
        solver.run(R, t, per_level=per_level)
        torch.cuda.synchronize()
        ic.check_status(solver.status)
        outs.append((R, t))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    _assert_on_reference(*outs[0], z, what="cfg5 final")
    # the epe between the two reference precisions bounds what 1e-4 means here
    assert np.abs(z["f32_t"][-1] - z["f64_t"][-1]).max() < SE3_TOL


@pytest.mark.parametrize("pack", [True, False])
def test_cfg5_icp_iterations_from_reference_pose(pack):
    _restart_iterations("icp_640x480_c32", _dev(), pack)


def test_cfg5_grouped_icp_batches_solve_as_separate_calls():
    """Independent batches with combine_ICP in one call: batch g's depths scaled by
    1 + g / 8 (inverse depths by its inverse), so each batch has its own depth1 extrema
    and the normal map must zero its own (algorithms.py:2168 over the batch one reference
    call holds).  Grouped = separate calls: JtJ of a no-update iteration at every level
    (the ICP term included) and the solved poses."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("icp_640x480_c32")
    G, B = 4, 2
    n = G * B
    base = _solver_levels(case, dev, True)
    scale = (1.0 + torch.arange(G, device=dev, dtype=torch.float32) / 8).repeat_interleave(B).view(n, 1, 1, 1)
    rep = lambda x: x.repeat(n, *([1] * (x.dim() - 1)))
    levels = []
    for d in base:
        e = {k: rep(v) for k, v in d.items()}
        for k in ("depth0", "depth1"):
            e[k] = (e[k] * scale).contiguous()
        for k in ("invD0", "invD1"):
            e[k] = (e[k] / scale).contiguous()
        levels.append(e)
    K = rep(torch.from_numpy(case["K"]).to(dev))
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    R0, t0 = rep(R0).contiguous(), rep(t0.reshape(-1, 3)).clone()
    t0[:, 1] += 1e-3 * (torch.arange(n, device=dev, dtype=torch.float32) % B)
    grouped = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True, combine_icp=True, group=B)
    Rg, tg = R0.clone(), t0.clone()
    grouped.run(Rg, tg)
    torch.cuda.synchronize()
    ic.check_status(grouped.status)
    sl = lambda g: slice(g * B, (g + 1) * B)
    for g in range(G):
        lv_g = [{k: v[sl(g)] for k, v in d.items()} for d in levels]
        alone = ic.PyramidSolver(lv_g, K[sl(g)].contiguous(), iters=3, remove_tru_sigma=True, combine_icp=True)
        Ra, ta = R0[sl(g)].clone(), t0[sl(g)].clone()
        alone.run(Ra, ta)
        torch.cuda.synchronize()
        torch.testing.assert_close(Rg[sl(g)], Ra, rtol=0, atol=5e-5)
        torch.testing.assert_close(tg[sl(g)], ta, rtol=0, atol=5e-5)
        for l in range(len(levels)):  # normal equations at the same pose, ICP term included
            dg, da = levels[l], lv_g[l]
            kw = dict(first=True, update=False, remove_tru_sigma=True, combine_icp=True)
            pose = (Ra, ta.view(-1, 3, 1))
            a = ic.iterate(pose, da["x0"], da["x1"], da["invD0"], da["invD1"], K[sl(g)] / 2 ** l, da["sigma0"],
                           da["sigma1"], depth0=da["depth0"], depth1=da["depth1"], **kw)
            # the grouped call over every batch (only batch g's rows compared)
            Rall, tall = Rg.clone(), tg.clone().view(-1, 3, 1)
            Rall[sl(g)], tall[sl(g)] = Ra, ta.view(-1, 3, 1)
            b = ic.iterate((Rall, tall), dg["x0"], dg["x1"], dg["invD0"], dg["invD1"], K / 2 ** l, dg["sigma0"],
                           dg["sigma1"], depth0=dg["depth0"], depth1=dg["depth1"], group=B, **kw)
            assert torch.equal(a[4], b[4][sl(g)]), f"batch {g} level {l} invalid counts"
            torch.testing.assert_close(b[2][sl(g)], a[2], rtol=2e-6, atol=1e-6 * a[2].abs().max().item())


# ------------------------------------------------------------------------------ cfg3
@pytest.mark.parametrize("groups", [0, 16])
def test_cfg3_distinct_pairs_match_reference(groups):
    """8 distinct pairs in one call (groups = 0), and the bench's launch: 16 batches of the
    same 8 pairs in one grouped call, every batch solved as its own reference call -- R and
    t of every pair within 1e-4 of the fp32 and fp64 reference runs of the 8-pair batch."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg3_b8_640x480_c32")
    G = max(1, groups)
    B = case["B"]
    rep = lambda x: x.repeat(G, *([1] * (x.dim() - 1))) if G > 1 else x
    levels = [{k: rep(v) for k, v in d.items()} for d in _solver_levels(case, dev, True)]
    solver = ic.PyramidSolver(levels, rep(torch.from_numpy(case["K"]).to(dev)), iters=3, remove_tru_sigma=True,
                              group=B if G > 1 else None)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    R, t = rep(R0).contiguous(), rep(t0.reshape(-1, 3)).contiguous()
    solver.run(R, t)
    torch.cuda.synchronize()
    ic.check_status(solver.status)
    for g in range(G):
        _assert_on_reference(R[g * B:(g + 1) * B], t[g * B:(g + 1) * B], z, what=f"cfg3 batch {g}")


@pytest.mark.parametrize("pack", [True, False])
def test_cfg3_iterations_from_reference_pose(pack):
    _restart_iterations("cfg3_b8_640x480_c32", _dev(), pack)


# the bench's eval stream: batch q -> the reference's own run of it (batches 0, 2, 7 cover flip
# codes 0-3: recipe.stream_batch_spec)
CFG3_STREAM = {0: "cfg3_b8_640x480_c32", 2: "cfg3_b8q2_640x480_c32", 7: "cfg3_b8q7_640x480_c32"}


@pytest.mark.parametrize("name", ["cfg3_b8q2_640x480_c32", "cfg3_b8q7_640x480_c32"])
def test_cfg3_flipped_batches_iterations_from_reference_pose(name):
    """The flipped stream batches (left-right, up-down and both) restarted from the reference's
    poses: exact invalid counts, normal equations and one step to rounding."""
    _restart_iterations(name, _dev(), True)


def test_cfg3_bench_call_matches_reference():
    """The bench's own call at N = 1 (bench.make_batches: stream batches 0..15 = 128 pairs as 16
    independent 8-pair batches in ONE grouped PyramidSolver call, channel-quad features):
    batches 0, 2 and 7 -- unflipped, flip codes 0/1, and 2/3 -- against the reference's own
    runs of those batches.  The fixture inputs are checked to be the bench's, bit for bit; every
    pair lies within its own bound (max(1e-4, 1.5x its noise floor)) of the fp32 and fp64 runs,
    and the restarted iterations' invalid counts of each batch are exact in the grouped launch."""
    import bench
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    B, G = 8, 16
    _, levels, K = bench.make_batches(B, 0, G, dev)
    for q, name in CFG3_STREAM.items():
        case, _ = golden_io.load(name)
        for l in range(case["levels"]):
            for key, ck in (("x0", "x0"), ("x1", "x1"), ("sigma0", "s0"), ("sigma1", "s1"), ("invD0", "invD0"),
                            ("invD1", "invD1")):
                got = levels[l][key][q * B:(q + 1) * B].cpu().numpy()
                assert np.array_equal(got, case[f"{ck}_{l}"]), f"{name}: {key} level {l} is not the bench's batch {q}"
    packed = [dict(d, x0=ic.pack_features(d["x0"]), x1=ic.pack_features(d["x1"])) for d in levels]
    solver = ic.PyramidSolver(packed, K, iters=3, remove_tru_sigma=True, group=B)
    R = torch.eye(3, device=dev).repeat(B * G, 1, 1).contiguous()
    t = torch.zeros(B * G, 3, device=dev)
    solver.run(R, t)
    torch.cuda.synchronize()
    ic.check_status(solver.status)
    for q, name in CFG3_STREAM.items():
        _, z = golden_io.load(name, check_digests=False)
        sl = slice(q * B, (q + 1) * B)
        _assert_within_reference_envelope(R[sl], t[sl], z, what=f"cfg3 bench call, batch {q} ({name})")
    # restarted from the reference's poses inside the grouped launch: batch q's invalid counts exact
    for q, name in CFG3_STREAM.items():
        _, z = golden_io.load(name, check_digests=False)
        i = 0
        for l in reversed(range(len(levels))):
            d = packed[l]
            for it in range(3):
                Rq = torch.eye(3, device=dev).repeat(B * G, 1, 1).contiguous()
                tq = torch.zeros(B * G, 3, 1, device=dev)
                if i:
                    Rq[q * B:(q + 1) * B] = torch.from_numpy(z["f32_R"][i - 1]).to(dev)
                    tq[q * B:(q + 1) * B] = torch.from_numpy(z["f32_t"][i - 1]).to(dev).view(B, 3, 1)
                o = ic.iterate((Rq, tq), d["x0"], d["x1"], d["invD0"], d["invD1"], K / 2 ** l, d["sigma0"],
                               d["sigma1"], first=True, reverse=(it & 1) == 1, remove_tru_sigma=True, group=B)
                inv = o[4][q * B:(q + 1) * B].cpu().numpy()
                assert np.array_equal(inv, z["f32_invalid"][i]), f"{name} iter {i}: {inv} vs {z['f32_invalid'][i]}"
                i += 1


def test_cfg3_grouped_iterations_from_reference_pose():
    """The grouped launch (2 batches of the 8 distinct pairs) restarted from the reference's
    poses: each batch's invalid counts equal the reference's exactly."""
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    case, z = golden_io.load("cfg3_b8_640x480_c32")
    lv = golden_io.levels_torch(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    B, G = case["B"], 2
    rep = lambda x: x.repeat(G, *([1] * (x.dim() - 1)))
    L, i = case["levels"], 0
    for l in reversed(range(L)):
        d = lv[l]
        f0, f1 = rep(ic.pack_features(d["f0"])), rep(ic.pack_features(d["f1"]))
        for it in range(3):
            if i == 0:
                R, t = golden_io.init_pose(case, torch.float32, dev)
            else:
                R, t = torch.from_numpy(z["f32_R"][i - 1]).to(dev), torch.from_numpy(z["f32_t"][i - 1]).to(dev)
            o = ic.iterate((rep(R), rep(t.reshape(-1, 3, 1))), f0, f1, rep(d["invD0"]), rep(d["invD1"]),
                           rep(K) / 2 ** l, rep(d["s0"]), rep(d["s1"]), first=True, remove_tru_sigma=True, group=B)
            inv = o[4].cpu().numpy()
            for g in range(G):
                assert np.array_equal(inv[g * B:(g + 1) * B], z["f32_invalid"][i]), f"iter {i} batch {g}"
            i += 1


# ------------------------------------------------------------------------------ cfg4
CFG4 = ["cfg4_pert00_160x120_c8", "cfg4_pert05_160x120_c8", "cfg4_pert10_160x120_c8", "cfg4_pert20_160x120_c8"]


@pytest.mark.parametrize("name", CFG4)
@pytest.mark.parametrize("pack", [True, False])
def test_cfg4_solve_from_perturbed_start(name, pack):
    """Masks, 4 levels at 160x120, C = 8, from the fixture's start.  Every iteration
    restarted from the reference's pose gives its invalid counts exactly and its next pose
    to 2e-5; every iteration of the chained solve, and the solve's final pose, lie within
    each pair's own bound (max(1e-4, 1.5x its noise floor), _assert_within_reference_envelope)."""
    from deep_prob_feature_track_amd import convergence_basin as cb
    dev = _dev()
    case, z = golden_io.load(name)
    _restart_iterations(name, dev, pack)
    if pack:
        _assert_chain_within_envelope(name, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    R, t = cb.solve_from_starts(_solver_levels(case, dev, pack), torch.from_numpy(case["K"]).to(dev), R0[None],
                                t0[None])
    _assert_within_reference_envelope(R[0], t[0], z, what=name)


def test_cfg4_start_sets_in_one_grouped_call():
    """The four fixture start sets as four independent batches of one call
    (solve_from_starts): each lands on its reference run (fp32 and fp64), and the
    convergence counts against the identity-start solve equal the reference's own counts
    exactly (convergence_basin.basin_counts on the reference's final poses)."""
    from deep_prob_feature_track_amd import convergence_basin as cb
    dev = _dev()
    zs = [golden_io.load(n) for n in CFG4]
    case = zs[0][0]
    R0 = torch.stack([golden_io.init_pose(c, torch.float32, dev)[0] for c, _ in zs])
    t0 = torch.stack([golden_io.init_pose(c, torch.float32, dev)[1] for c, _ in zs])
    R, t = cb.solve_from_starts(_solver_levels(case, dev, True), torch.from_numpy(case["K"]).to(dev), R0, t0)
    for p, (_, z) in enumerate(zs):
        _assert_within_reference_envelope(R[p], t[p], z, what=CFG4[p])
    ref_R = torch.from_numpy(np.stack([z["f32_R"][-1] for _, z in zs])).to(dev)
    ref_t = torch.from_numpy(np.stack([z["f32_t"][-1] for _, z in zs])).to(dev)
    n_gpu, m_gpu = cb.basin_counts(R, t, R[0], t[0], rot_thresh=0.02, trans_thresh=0.02)
    n_ref, m_ref = cb.basin_counts(ref_R, ref_t, ref_R[0], ref_t[0], rot_thresh=0.02, trans_thresh=0.02)
    print("cfg4 fixture starts: convergence counts (GPU / reference):", n_gpu.tolist(), n_ref.tolist(),
          "smallest |margin|:", float(np.minimum(np.abs(m_ref["rot_margin"]), np.abs(m_ref["trans_margin"])).min()))
    assert np.array_equal(n_gpu, n_ref), f"counts {n_gpu} vs reference {n_ref}"
    assert n_gpu[0] == case["B"]


SWEEP_TARGET = "cfg4_sweep256_160x120_c8"  # the basin's target: the reference's identity-start solve
BASIN_THRESH = 0.01  # rad / m (compute_RPE_loss errors)


def _target(dev):
    _, zt = golden_io.load(SWEEP_TARGET, check_digests=False)
    return tuple(torch.from_numpy(zt[f"f32_{k}"][-1]).to(dev) for k in ("R", "t"))


def _reference_decisions(z, tgt_R, tgt_t, dev):
    """The reference's own convergence decision per pair (its fp32 run's final pose against
    the target), and the pairs whose decision the reference cannot make stably: a margin
    (threshold - error) no larger than 1.5x how far that margin moves in the reference's own
    rounding-only runs (golden_io.noise_runs) -- every run whose decision differs is in it."""
    from deep_prob_feature_track_amd import convergence_basin as cb

    def margins(R, t):
        _, m = cb.convergence_counts(torch.from_numpy(np.ascontiguousarray(R)).to(dev),
                                     torch.from_numpy(np.ascontiguousarray(t)).to(dev), tgt_R, tgt_t,
                                     BASIN_THRESH, BASIN_THRESH)
        return m["rot_margin"], m["trans_margin"], m["converged"]
    rm, tm, conv = margins(z["f32_R"][-1], z["f32_t"][-1])
    Rs, ts = golden_io.noise_runs(z)
    drm = np.zeros_like(rm)
    dtm = np.zeros_like(tm)
    flips = np.zeros(rm.shape, bool)
    for n in range(Rs.shape[0]):
        a, b, c = margins(Rs[n, -1], ts[n, -1])
        drm, dtm = np.maximum(drm, np.abs(a - rm)), np.maximum(dtm, np.abs(b - tm))
        flips |= c != conv
    undecided = (np.abs(rm) <= FLOOR_FACTOR * drm) | (np.abs(tm) <= FLOOR_FACTOR * dtm) | flips
    return conv, undecided


SWEEP_STARTS = ["cfg4_sweep256_rotx10_160x120_c8", "cfg4_sweep256_tz10_160x120_c8"]
BASIN_STARTS = ["cfg4_sweep256_ry011_160x120_c8", "cfg4_sweep256_tz012_160x120_c8"]


@pytest.mark.parametrize("name", SWEEP_STARTS + BASIN_STARTS)
def test_cfg4_b256_start_set_matches_reference(name):
    """cfg4's 256-pair masked batch from one start set (convergence_basin.py:337-418's 1-D
    axes applied to the identity start: 0.1 rad about x and 0.1 m along z, outside the
    basin; 0.011 rad about y and 0.012 m along z, inside its decision band), against the
    reference's own run from that start: every iteration restarted from the reference's pose
    exact (invalid counts) and to rounding; every iteration of the chained solve and the
    grouped solve's final pose within each pair's own bound; and the convergence decision
    against the basin's target (the reference's identity-start solve) equal to the
    reference's pair by pair -- exact counts over the pairs the reference decides stably,
    the others listed.  The in-basin start sets' reference counts lie strictly between 0 and
    B, so the comparison can fail."""
    from deep_prob_feature_track_amd import convergence_basin as cb
    dev = _dev()
    _restart_iterations(name, dev, True)
    case, z = golden_io.load(name)
    _assert_chain_within_envelope(name, dev)
    R0, t0 = golden_io.init_pose(case, torch.float32, dev)
    R, t = cb.solve_from_starts(_solver_levels(case, dev, True), torch.from_numpy(case["K"]).to(dev), R0[None],
                                t0[None])
    _assert_within_reference_envelope(R[0], t[0], z, what=name)
    tgt_R, tgt_t = _target(dev)
    B = case["B"]
    n_gpu, m_gpu = cb.convergence_counts(R[0], t[0], tgt_R, tgt_t, BASIN_THRESH, BASIN_THRESH)
    conv_ref, undecided = _reference_decisions(z, tgt_R, tgt_t, dev)
    n_ref = int(conv_ref.sum())
    conv_gpu = m_gpu["converged"]
    dec = ~undecided
    print(f"{name}: converged {n_gpu} (GPU) / {n_ref} (reference) of {B}; over the {int(dec.sum())} pairs the "
          f"reference decides stably: {int(conv_gpu[dec].sum())} / {int(conv_ref[dec].sum())}; undecided pairs "
          f"(reference margin within 1.5x its own rounding spread): {np.flatnonzero(undecided).tolist()}")
    if name in BASIN_STARTS:
        assert 0 < n_ref < B, f"{name}: the reference's count {n_ref} must lie strictly between 0 and {B}"
        assert 0 < int(conv_ref[dec].sum()) < int(dec.sum())
    diff = np.flatnonzero(dec & (conv_gpu != conv_ref))
    assert diff.size == 0, f"{name}: convergence decisions differ from the reference's on decided pairs {diff.tolist()}"
    assert int(conv_gpu[dec].sum()) == int(conv_ref[dec].sum())


def test_cfg4_sweep_b256():
    """cfg4's batch: 256 masked pairs at 160x120, C = 8 (80 distinct: tests/golden/recipe.py
    sweep_spec), against the reference's own run of that batch (cfg4_sweep256_160x120_c8):
    every iteration restarted from the reference's pose gives its invalid counts exactly; every
    iteration of the chained identity-start solve and the grouped solve (the basin's target) lie
    within each pair's own bound.  Then a 1-D sweep of perturbed starts around the target (6 axes
    x 7 offsets: +-0.006 / +-0.012 rad or m inside the basin's decision band, and the outer
    +-0.2 rad / +-0.15 m of the reference's sweep range, convergence_basin.py defaults -- 42
    start sets = 10752 solves in grouped calls of 8 start sets): start sets solved in one grouped
    call equal the same sets solved one call each (the far starts too: exact invalid counts and
    JtJ at a common pose), the counts at the in-band offsets are neither all 0 nor all B, and the
    pairs whose margin is below the pose uncertainty are reported."""
    from deep_prob_feature_track_amd import convergence_basin as cb
    from deep_prob_feature_track_amd import ic
    dev = _dev()
    name = "cfg4_sweep256_160x120_c8"
    _restart_iterations(name, dev, True)
    case, z = golden_io.load(name)
    _assert_chain_within_envelope(name, dev)
    B = case["B"]
    K = torch.from_numpy(case["K"]).to(dev)
    lv = _solver_levels(case, dev, True)
    I = torch.eye(3, device=dev).repeat(1, B, 1, 1)
    Rt, tt = cb.solve_from_starts(lv, K, I, torch.zeros(1, B, 3, device=dev))
    Rt, tt = Rt[0], tt[0]
    dev_pose, floor = _assert_within_reference_envelope(Rt, tt, z, what=name)
    bound = np.maximum(SE3_TOL, FLOOR_FACTOR * floor)
    # offsets inside the basin's decision band (the in-basin fixtures: 0.011 rad / 0.012 m
    # bring part of the batch back), so the counts there are neither 0 nor B, plus the far ends
    # of the reference's sweep (0.2 rad, 0.15 m: large-baseline starts through the grouped solver)
    NO = 7
    rot = np.array([-0.2, -0.012, -0.006, 0.0, 0.006, 0.012, 0.2])
    trs = np.array([-0.15, -0.012, -0.006, 0.0, 0.006, 0.012, 0.15])
    Rs, ts = cb.perturbed_starts(Rt, tt, rot, trs)
    assert Rs.shape[:2] == (6 * NO, B)
    Rf, tf = cb.solve_from_starts(lv, K, Rs, ts)
    # the zero-offset start sets of the three rotation axes are the same starts (the target
    # through an Euler round trip), those of the three translation axes the target itself,
    # each solved as a different batch of the grouped calls (every call the same size: a short
    # last round is padded): each pair's schedule is identical, so each group of three must
    # agree bit for bit -- a difference would be cross-batch interference (shared counters /
    # extrema slots)
    zero = [a * NO + 3 for a in range(6)]
    assert torch.equal(Rs[zero[3]], Rt) and torch.equal(ts[zero[3]], tt.reshape(B, 3))
    for grp in (zero[:3], zero[3:]):
        for zz in grp[1:]:
            assert torch.equal(Rs[zz], Rs[grp[0]]) and torch.equal(ts[zz], ts[grp[0]])
            assert torch.equal(Rf[zz], Rf[grp[0]]) and torch.equal(tf[zz], tf[grp[0]]), f"start set {zz} vs {grp[0]}"
    G = 8
    far_sets = [k for k in range(6 * NO) if k % NO in (0, NO - 1)]
    # in-band start sets (the round-5 sets 0, 13, 29 of the 5-offset grid: -0.012 rad about x,
    # +0.006 rad about z, +0.012 m along z), then far ones (-0.2 rad about x, +0.15 m along z)
    for p in (1, 18, 40, 0, 41):
        far = p in far_sets
        # grouped = one call per start set: at a common pose (the grouped solve's result) one
        # no-update iteration per level gives the same invalid counts exactly and the same
        # normal equations up to the fp32 grouping of the workgroup sums (fewer records per
        # pair in the larger launch); the chained poses then agree within the bound below
        Ra, ta = cb.solve_from_starts(lv, K, Rs[p:p + 1], ts[p:p + 1])
        close = torch.maximum((Rf[p] - Ra[0]).abs().amax((1, 2)), (tf[p] - ta[0]).abs().amax(1)).cpu().numpy()
        # two fp32 groupings of the same GPU solve are two rounding samples of each other (not the
        # reference contract of golden_io.envelope): each pair within its bound, but for as many
        # pairs as one of the reference's own rounding-only runs exceeds against the others'
        # floors, which stay within 1.5x the batch floor
        over = np.flatnonzero(close > bound)
        print(f"start set {p}{' (far)' if far else ''}: grouped vs alone chained poses: "
              f"{int((close <= 1e-5).sum())} of {B} pairs within 1e-5, max {close.max():.2e}")
        if far:  # a non-converging far start wanders; pinned at the common pose below instead
            over = over[:0]
            close = np.zeros_like(close)
        assert over.size <= golden_io.loo_exceedances(z, -1, FLOOR_FACTOR, SE3_TOL), \
            f"start set {p}: grouped vs alone, {over.size} pairs beyond their bound (max {close.max():.2e})"
        assert (close <= max(SE3_TOL, FLOOR_FACTOR * float(floor.max()))).all(), \
            f"start set {p}: grouped vs alone {close.max():.2e}"
        g0 = (p // G) * G
        for l in range(len(lv)):
            d = lv[l]
            kw = dict(first=True, update=False, remove_tru_sigma=True, obj_mask0=d["obj_mask0"],
                      obj_mask1=d["obj_mask1"])
            pose = (Rf[p].contiguous(), tf[p].reshape(B, 3, 1).contiguous())
            a = ic.iterate(pose, d["x0"], d["x1"], d["invD0"], d["invD1"], K / 2 ** l, d["sigma0"], d["sigma1"], **kw)
            rep = lambda v: v.repeat(G, *([1] * (v.dim() - 1)))
            Rall = torch.cat([Rf[min(g0 + q, Rf.shape[0] - 1)] for q in range(G)]).contiguous()
            tall = torch.cat([tf[min(g0 + q, tf.shape[0] - 1)] for q in range(G)]).reshape(G * B, 3, 1).contiguous()
            q = p - g0
            b = ic.iterate((Rall, tall), rep(d["x0"]), rep(d["x1"]), rep(d["invD0"]), rep(d["invD1"]),
                           rep(K) / 2 ** l, rep(d["sigma0"]), rep(d["sigma1"]), group=B,
                           **dict(kw, obj_mask0=rep(d["obj_mask0"]), obj_mask1=rep(d["obj_mask1"])))
            sl = slice(q * B, (q + 1) * B)
            assert torch.equal(a[4], b[4][sl]), f"start set {p} level {l}: invalid counts grouped vs alone"
            rel = ((b[2][sl] - a[2]).abs().amax((1, 2)) / a[2].abs().amax((1, 2))).max().item()
            assert rel <= 1e-5, f"start set {p} level {l}: JtJ grouped vs alone rel {rel:.2e}"
    counts, m = cb.basin_counts(Rf, tf, Rt, tt, rot_thresh=0.01, trans_thresh=0.01)
    near = (np.abs(m["rot_margin"]) < bound[None]) | (np.abs(m["trans_margin"]) < bound[None])
    assert len(set(counts[zero[:3]].tolist())) == 1 and len(set(counts[zero[3:]].tolist())) == 1
    print("cfg4 sweep counts (6 axes x 7 offsets):", counts.reshape(6, NO).tolist(),
          "undecided (margin < uncertainty):", near.sum(1).reshape(6, NO).tolist())
    assert (counts[far_sets] < B).all(), "a far start set converged entirely"
    nonzero = np.array([k for k in range(6 * NO) if k % NO not in (0, 3, NO - 1)])
    assert (counts[nonzero] > 0).any() and (counts[nonzero] < B).any(), "degenerate sweep counts"
    assert any(0 < c < B for c in counts[nonzero]), "no start set inside the basin's decision band"
