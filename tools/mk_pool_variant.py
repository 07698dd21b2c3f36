"""Write tools/_var/pool.hip: the shipped kernel source with a PHASED pool for the hybrid band
split (A/B experiment).

The hybrid split (S < waves < 2S per pair: level 0 of a 128-pair launch, 16 waves over 11
strips) gives wave s < S rows [0, T_s) of strip s and lets the nw - S pool waves split the
bottom rows [T_s, H) of all strips strip-major, so horizontally adjacent strips' bottoms
are marched far apart in time and their shared lines are fetched twice.  Phased: pool wave
j marches the bottoms of strips j, j + np, j + 2 np, ... (np = nw - S pool waves), so in
each phase the pool waves march np adjacent strips side by side; the S mod np remaining
strips' bottoms are split strip-major into the per-wave chunks that balance the waves.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")).read()

old_split = """    } else if (hpool) {
      const int PU = hnf * hLf + (S_ - hnf) * hLu, np = nw - S_, j = band - S_;
      int wt = 0, ws0 = 0, ws1 = 0;  // weighted split over the pool waves S .. nw - 1
      for (int i = 0; i < np; ++i) {
        const int wi = (S_ + i) < hh ? 64 + hsk : 64 - hsk;
        wt += wi;
        ws0 += i < j ? wi : 0;
        ws1 += i <= j ? wi : 0;
      }
      ubeg = (PU * ws0) / wt;
      uend = (PU * ws1) / wt;
      vband = 1;
"""
assert old_split in src
new_split = """    } else if (hpool) {
      ubeg = 0;
      uend = hpF + hpX1 - hpX0;
      vband = 1;
"""
src = src.replace(old_split, new_split)

anchor = "    const bool hpool = hyb && band >= S_;\n"
assert anchor in src
phased = anchor + """    // phased pool: wave j marches the bottoms of strips j, j + np, ... (hpFs full rounds), then
    // its chunk [hpX0, hpX1) of the remaining strips' bottoms (strip-major from strip hpRb);
    // the chunks make each wave's total its weighted share of the pool units
    const int hpNp = max(nw - S_, 1), hpJ = band - S_;
    const int hpFs = S_ / hpNp, hpRb = hpFs * hpNp;
    auto hT = [&](int s) { return s < hnf ? hTf : hTu; };
    int hpF = 0, hpX0 = 0, hpX1 = 0;
    if (hpool) {
      int PU = 0, RU = 0;
      for (int s = 0; s < S_; ++s) {
        PU += H - hT(s);
        RU += s >= hpRb ? H - hT(s) : 0;
      }
      int wt = 0;
      for (int i = 0; i < hpNp; ++i) wt += (S_ + i) < hh ? 64 + hsk : 64 - hsk;
      int ws = 0, cf = 0, x = 0;  // running: weight, full-round units, chunk start (a running max)
      for (int i = 0; i <= hpJ; ++i) {
        int fi = 0;
        for (int r = 0; r < hpFs; ++r) fi += H - hT(r * hpNp + i);
        const int wi = (S_ + i) < hh ? 64 + hsk : 64 - hsk;
        const int x1 = i == hpNp - 1 ? RU : max(x, min(max((PU * (ws + wi)) / wt - (cf + fi), 0), RU));
        if (i == hpJ) {
          hpF = fi;
          hpX0 = x;
          hpX1 = x1;
        }
        ws += wi;
        cf += fi;
        x = x1;
      }
    }
"""
src = src.replace(anchor, phased)

old_map = """        if (hpool) {
          const int uf = hnf * hLf;
          if (u < uf) {
            strip = u / max(hLf, 1);
            y = hTf + (u - strip * hLf);
            ytop = hTf;
          } else {
            const int s2 = (u - uf) / max(hLu, 1);
            y = hTu + (u - uf - s2 * hLu);
            strip = hnf + s2;
            ytop = hTu;
          }
        } else {"""
assert old_map in src
new_map = """        if (hpool) {
          // k in marching order: the full rounds' strips first (every pool wave in the same
          // phase), then the chunk; each segment walked in the marching direction
          if (k < hpF) {
            int kk = k, r = 0;
            while (r + 1 < hpFs && kk >= H - hT(r * hpNp + hpJ)) {
              kk -= H - hT(r * hpNp + hpJ);
              ++r;
            }
            strip = r * hpNp + hpJ;
            ylo = hT(strip);
            yhi = H;
            y = up ? H - 1 - kk : ylo + kk;
          } else {
            const int kc = k - hpF;
            const int v = up ? hpX1 - 1 - kc : hpX0 + kc;  // unit of the remaining strips' bottoms
            int s = hpRb, base = 0;
            while (s + 1 < S_ && v >= base + (H - hT(s))) {
              base += H - hT(s);
              ++s;
            }
            strip = s;
            ylo = hT(s) + max(0, hpX0 - base);
            yhi = hT(s) + min(H - hT(s), hpX1 - base);
            y = hT(s) + (v - base);
          }
          strt = y == (up ? yhi - 1 : ylo);
          xs = strip * kTileOut - 1 + lane;
          run = min(up ? y - ylo + 1 : yhi - y, nrows - k);
          return;
        } else {"""
src = src.replace(old_map, new_map)
os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
open(os.path.join(ROOT, "tools", "_var", "pool.hip"), "w").write(src)
print("tools/_var/pool.hip")
