"""The marching kernel's band schedule covers every (strip, row) unit of a pair exactly once
(ADVICE r5): a line-by-line Python replica of ic_reduce_kernel's split (csrc/dpft_ic.hip: the
row-band grid, the hybrid split with its phased pool, the grid + pool split, the strip-major
fallback) and of unit_pos_run, enumerated for every wave of a pair over a range of strip counts,
heights, waves per pair, band skews and both marching directions.  A unit visited twice would be
double-counted in J^T J; one never visited would be missing -- the GPU suite only sees the shapes
the fixtures have.
"""
import itertools

import pytest

GRID_WASTE = 4  # DPFT_GRID_WASTE (csrc/dpft_tuning.h)


def split_start(bnd, n, length, skew):
    h = n >> 1
    sk = skew if n >= 2 else 0
    wsum = (64 + sk) * min(bnd, h) + (64 - sk) * max(bnd - h, 0)
    wtot = (64 + sk) * h + (64 - sk) * (n - h)
    return (length * wsum) // wtot


def wave_units(band, nw, S, H, skew, reverse):
    """The (strip, row) units wave `band` of a pair marches, in marching order (the kernel's
    schedule and unit_pos_run)."""
    U = S * H
    K_ = nw // S
    grid = K_ >= 2 and (nw - K_ * S) * 64 <= nw * GRID_WASTE
    hyb = (not grid) and S < nw < 2 * S
    hh = nw >> 1
    hsk = skew if nw >= 2 else 0
    hwt = (64 + hsk) * hh + (64 - hsk) * (nw - hh)
    hTf, hTu = min(H, (U * (64 + hsk)) // hwt), min(H, (U * (64 - hsk)) // hwt)
    hnf = min(hh, S)
    hpool = hyb and band >= S
    hpNp, hpJ = max(nw - S, 1), band - S
    hpFs = S // hpNp
    hpRb = hpFs * hpNp
    hT = lambda s: hTf if s < hnf else hTu  # noqa: E731
    hpF = hpX0 = hpX1 = 0
    if hpool:
        PU = sum(H - hT(s) for s in range(S))
        RU = sum(H - hT(s) for s in range(S) if s >= hpRb)
        wt = sum(64 + hsk if S + i < hh else 64 - hsk for i in range(hpNp))
        ws = cf = x = 0
        for i in range(hpJ + 1):
            fi = sum(H - hT(r * hpNp + i) for r in range(hpFs))
            wi = 64 + hsk if S + i < hh else 64 - hsk
            x1 = RU if i == hpNp - 1 else max(x, min(max((PU * (ws + wi)) // wt - (cf + fi), 0), RU))
            if i == hpJ:
                hpF, hpX0, hpX1 = fi, x, x1
            ws += wi
            cf += fi
            x = x1
    Kg = -(-nw // S)
    Eg = Kg * S - nw
    gpool = (not grid) and (not hyb) and Kg >= 3

    def gp_w(n):
        return (64 + hsk) * min(n, hh) + (64 - hsk) * min(max(n - hh, 0), nw - hh) + 64 * max(n - nw, 0)

    def gp_cut(k):
        return (H * gp_w(k * S)) // gp_w(Kg * S)
    gk, gs = band // S, band % S
    gr0, gr1 = (gp_cut(gk), gp_cut(gk + 1)) if gpool else (0, 0)
    gL0 = gp_cut(Kg - 1) if gpool else 0
    gHL = H - gL0
    gPU = Eg * gHL
    gpb = (gPU * band) // nw if gpool else 0
    gpe = (gPU * (band + 1)) // nw if gpool else 0
    if gpool:
        ubeg, uend, vband = 0, (gr1 - gr0) + (gpe - gpb), gk
    elif hyb and not hpool:
        ubeg, uend, vband = band * H, band * H + (hTf if band < hh else hTu), 0
    elif hpool:
        ubeg, uend, vband = 0, hpF + hpX1 - hpX0, 1
    elif grid:
        k, s = band // S, band % S
        ubeg = s * H + split_start(k, K_, H, skew) if k < K_ else 0
        uend = s * H + split_start(k + 1, K_, H, skew) if k < K_ else 0
        vband = k
    else:
        ubeg, uend, vband = split_start(band, nw, U, skew), split_start(band + 1, nw, U, skew), band
    nrows = uend - ubeg
    up = ((vband & 1) != 0) != bool(reverse)
    out = []
    for k in range(nrows):
        u = uend - 1 - k if up else ubeg + k
        if gpool:
            m = gr1 - gr0
            if k < m:
                strip, y = gs, (gr1 - 1 - k if up else gr0 + k)
            else:
                j = gpe - 1 - (k - m) if up else gpb + (k - m)
                sp = j // gHL
                strip, y = S - Eg + sp, gL0 + (j - sp * gHL)
        elif hpool:
            if k < hpF:
                kk, r = k, 0
                while r + 1 < hpFs and kk >= H - hT(r * hpNp + hpJ):
                    kk -= H - hT(r * hpNp + hpJ)
                    r += 1
                strip = r * hpNp + hpJ
                ylo = hT(strip)
                y = H - 1 - kk if up else ylo + kk
            else:
                kc = k - hpF
                v = hpX1 - 1 - kc if up else hpX0 + kc
                s, base = hpRb, 0
                while s + 1 < S and v >= base + (H - hT(s)):
                    base += H - hT(s)
                    s += 1
                strip, y = s, hT(s) + (v - base)
        else:
            strip, y = u // H, u % H
        out.append((strip, y))
    return out


def check_cover(nw, S, H, skew, reverse):
    seen = {}
    for band in range(nw):
        for unit in wave_units(band, nw, S, H, skew, reverse):
            seen[unit] = seen.get(unit, 0) + 1
    want = {(s, y) for s in range(S) for y in range(H)}
    twice = {u for u, c in seen.items() if c > 1}
    extra = set(seen) - want
    missing = want - set(seen)
    assert not twice and not extra and not missing, (nw, S, H, skew, reverse, sorted(twice)[:5], sorted(extra)[:5],
                                                     sorted(missing)[:5])


def split_kind(nw, S):
    K_ = nw // S
    grid = K_ >= 2 and (nw - K_ * S) * 64 <= nw * GRID_WASTE
    if grid:
        return "grid"
    if S < nw < 2 * S:
        return "hybrid"
    return "gpool" if -(-nw // S) >= 3 else "strip-major"


@pytest.mark.parametrize("reverse", [0, 1])
@pytest.mark.parametrize("skew", [0, 2, 10])
def test_every_unit_marched_exactly_once(skew, reverse):
    kinds = set()
    for S, H, nw in itertools.product(range(1, 13), (2, 7, 15, 33, 60, 120, 240, 480), (4, 8, 12, 16, 20, 24, 32, 48, 64)):
        check_cover(nw, S, H, skew, reverse)
        kinds.add(split_kind(nw, S))
    assert kinds == {"grid", "hybrid", "gpool", "strip-major"}, kinds


def test_the_shipped_shapes():
    """The bench's launches: 640x480 level 0 (11 strips) and level 1 (6 strips) at 16 waves per
    pair (128 pairs: the hybrid split and the grid + pool split), 32 waves (64 pairs: grid + pool),
    256 waves (8 pairs: the grid, 23 x 11 of 256 waves)."""
    assert split_kind(16, 11) == "hybrid" and split_kind(16, 6) == "gpool" and split_kind(32, 11) == "gpool"
    assert split_kind(256, 11) == "grid"
    for nw, S, H in ((16, 11, 480), (16, 6, 240), (32, 11, 480), (256, 11, 480), (16, 3, 120), (16, 2, 60)):
        for skew, rev in itertools.product((0, 2, 10), (0, 1)):
            check_cover(nw, S, H, skew, rev)
