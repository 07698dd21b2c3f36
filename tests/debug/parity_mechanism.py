"""Why a chained GPU pose leaves 1e-4 of the reference's run: the truncated-sigma extremum flip.

CPU analysis of gpurun_out/parity_dump.npz (tools/parity_dump.py on the GPU box: every iteration
of the GPU's chained solve per fixture).  The truncated-sigma mask (algorithms.py:1975-1980) flags
the pixels whose sigma_r = sigma1(warp) equals the BATCH-global min or max of sigma_r; their
weighted residual becomes 1e-6, which changes JtR of the pair that holds them (J is unmasked).
For every iteration i of a fixture this script evaluates, with the oracle's fp32 restatement of
the reference (oracle/ic_oracle.py -- test infrastructure; the GPU's warp and sampler are
bit-exact against it, tests/test_gpu_parity.py), the extremum pixel sets at the GPU's start pose
(its chained pose after iteration i - 1) and at the reference's own start pose (the fixture's fp32
pose after i - 1), and reports the first iteration where the two sets differ: the pixels, their
pairs, the sigma_r of the competing pixels at both poses and their distance in fp32 ulps.  For
each pair that ends beyond 1e-4 of the reference's fp32 run it names the iteration of its first
jump (deviation > 10x the one-step deviation) and whether the extremum set differed there in a
pixel of that pair (a direct flip) or elsewhere (the pair then moves through the coupled
iterations that follow).

  python tests/debug/parity_mechanism.py [--dump gpurun_out/parity_dump.npz] [--out DESIGN-ready json] NAME...
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import golden_io  # noqa: E402
from oracle import ic_oracle as O  # noqa: E402  (test infrastructure: the oracle is the checker here)


def ulps(a, b):
    """Distance of two fp32 values in units in the last place (same sign assumed)."""
    ia = np.array([a], np.float32).view(np.int32)[0]
    ib = np.array([b], np.float32).view(np.int32)[0]
    return abs(int(ia) - int(ib))


def sigma_r(level, K, R, t):
    """sigma_r = bilinear(sigma1, warp) [B,H,W] (fp32) at pose (R [B,3,3], t [B,3])."""
    B, _, H, W = level["f0"].shape
    x, y = O.pixel_rays(B, H, W, K)
    u, v, _ = O.warp_inverse_depth(x, y, level["invD0"], R, t.reshape(B, 3, 1), K)
    return O.bilinear(level["s1"][:, :1], u, v)[:, 0]


def extrema(sr):
    """(min, max, set of (pair, y, x) attaining min, set attaining max, runner-up below max,
    runner-up above min)."""
    flat = sr.reshape(-1)
    mn, mx = flat.min().item(), flat.max().item()
    B, H, W = sr.shape
    idx = lambda m: {(int(b), int(yy), int(xx)) for b, yy, xx in zip(*np.nonzero(m.numpy()))}  # noqa: E731
    smin, smax = idx(sr == mn), idx(sr == mx)
    below = flat[flat < mx]
    above = flat[flat > mn]
    return mn, mx, smin, smax, (below.max().item() if below.numel() else mx), (above.min().item() if above.numel() else mn)


def analyse(name, dump):
    case, z = golden_io.load(name, check_digests=False)
    lv = golden_io.levels_torch(case, torch.float32, "cpu")
    K0 = torch.from_numpy(case["K"])
    cR, ct = dump[f"{name}__chain_R"], dump[f"{name}__chain_t"]
    iters = cR.shape[0]
    L = case["levels"]
    R0, t0 = golden_io.init_pose(case, torch.float32, "cpu")
    step_dev = dump[f"{name}__step_dev"]
    dev_chain = np.stack([golden_io.pose_deviation(cR[i], ct[i], z, "f32", i) for i in range(iters)])  # [iters, B]
    rows, first_diff = [], None
    per_iter_sets = []
    for i in range(iters):
        l = L - 1 - i // 3
        K = K0 / 2 ** l
        if i == 0:
            starts = {"gpu": (R0, t0.reshape(-1, 3)), "ref": (R0, t0.reshape(-1, 3))}
        else:
            starts = {"gpu": (torch.from_numpy(cR[i - 1]), torch.from_numpy(ct[i - 1])),
                      "ref": (torch.from_numpy(z["f32_R"][i - 1]), torch.from_numpy(z["f32_t"][i - 1]))}
        ex = {k: extrema(sigma_r(lv[l], K, *v)) for k, v in starts.items()}
        g, r = ex["gpu"], ex["ref"]
        same = g[2] == r[2] and g[3] == r[3]
        info = {"iter": i, "level": l, "sets_equal": bool(same),
                "gpu_max": g[1], "ref_max": r[1], "gpu_min": g[0], "ref_min": r[0],
                "gpu_max_pixels": sorted(g[3])[:6], "ref_max_pixels": sorted(r[3])[:6],
                "gpu_min_pixels": sorted(g[2])[:6], "ref_min_pixels": sorted(r[2])[:6],
                "max_margin_ulps_gpu": ulps(g[1], g[4]), "max_margin_ulps_ref": ulps(r[1], r[4]),
                "min_margin_ulps_gpu": ulps(g[0], g[5]), "min_margin_ulps_ref": ulps(r[0], r[5])}
        per_iter_sets.append((set(p for p, _, _ in g[2] | g[3]), set(p for p, _, _ in r[2] | r[3]), same))
        rows.append(info)
        if not same and first_diff is None:
            first_diff = info
    final = dev_chain[-1]
    pairs = []
    for b in np.flatnonzero(final > 1e-4):
        onestep = max(float(step_dev[:, b].max()), 1e-7)
        jump = np.flatnonzero(dev_chain[:, b] > 10 * onestep)
        i0 = int(jump[0]) if jump.size else None
        direct = None
        if i0 is not None:
            gp, rp, same = per_iter_sets[i0]
            direct = (not same) and (b in gp or b in rp)
        pairs.append({"pair": int(b), "final_dev": float(final[b]), "first_jump_iter": i0,
                      "jump_dev": float(dev_chain[i0, b]) if i0 is not None else None,
                      "extremum_sets_differ_at_jump": None if i0 is None else (not per_iter_sets[i0][2]),
                      "pair_holds_a_differing_extremum_pixel": direct})
    return {"fixture": name, "B": int(cR.shape[1]), "iters": iters, "first_set_difference": first_diff,
            "iterations_with_set_difference": [r_["iter"] for r_ in rows if not r_["sets_equal"]],
            "pairs_beyond_1e-4": pairs, "per_iteration": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--dump", default=os.path.join(ROOT, "gpurun_out", "parity_dump.npz"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dump = np.load(a.dump, allow_pickle=False)
    res = []
    torch.set_num_threads(8)
    for name in a.names:
        r = analyse(name, dump)
        res.append(r)
        fd = r["first_set_difference"]
        print(f"{name}: set differences at iterations {r['iterations_with_set_difference']}")
        if fd:
            print(f"  first at iter {fd['iter']} (level {fd['level']}): max {fd['ref_max']:.9g} ref / "
                  f"{fd['gpu_max']:.9g} gpu, pixels ref {fd['ref_max_pixels']} gpu {fd['gpu_max_pixels']}; "
                  f"min pixels ref {fd['ref_min_pixels']} gpu {fd['gpu_min_pixels']}; margins (ulps) max "
                  f"{fd['max_margin_ulps_ref']}/{fd['max_margin_ulps_gpu']}, min {fd['min_margin_ulps_ref']}/"
                  f"{fd['min_margin_ulps_gpu']}")
        for p in r["pairs_beyond_1e-4"]:
            print(f"  pair {p['pair']}: final {p['final_dev']:.2e}, first jump at iter {p['first_jump_iter']} "
                  f"({p['jump_dev']}), sets differ there: {p['extremum_sets_differ_at_jump']}, "
                  f"pair holds a differing extremum pixel: {p['pair_holds_a_differing_extremum_pixel']}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1, default=float)


if __name__ == "__main__":
    main()
