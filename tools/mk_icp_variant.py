"""Write tools/_var/icppipe.hip: the shipped source with icp_records_kernel's pixel loop
software-pipelined (A/B experiment): the next pixel's depth0, geometry and four normal-map
tap loads are issued before the current pixel's term, two pixels alternating in A / B
registers (no loop-carried copies), the pixels still accumulated in order."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")).read()
old = src[src.index("    int pix = beg + tid, y = pix / W, x = pix - y * W;  // then advanced by kThreads without a division"):
          src.index("  if (tab && p.rc_taps)\n    pixels(std::true_type{}, std::true_type{});")]
new = r"""    // software-pipelined: pixel k + 1's depth0, geometry and normal-map taps are issued
    // before pixel k's term (two stages, A / B registers alternating: no loop-carried
    // copies); past the range the loads are clamped to its last pixel and not accumulated
    if (end <= beg) return;
    struct Stage {
      IcpGeo g;
      IcpTaps q;
      float d0;
      bool m0;
    };
    auto issue = [&](Stage& S, int pix, int x, int y) {
      const int pc = min(pix, end - 1);
      S.m0 = m0b ? (m0b[pc] != 0) : true;
      S.d0 = d0b[pc];
      S.g = icp_geo(ncx(x), ncy(min(y, H - 1)), S.d0, Rm, tv, fx, fy, cx, cy, H, W, RC ? rsxy : nullptr);
      S.q = icp_load(S.g, nd1);
    };
    auto term = [&](const Stage& S) {
      const IcpTapXY n{ncx(S.g.x0), ncx(S.g.x1), ncy(S.g.y0), ncy(S.g.y1)};
      const IcpTerm ic = icp_term(S.g, S.q, n, S.d0, Rm, !S.m0, m1b, p.icp_w);
      int kq = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
#pragma unroll
        for (int j = i; j < 6; ++j) acc[kq++] += ic.J[i] * ic.J[j];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[21 + i] += ic.J[i] * ic.r;
    };
    auto advance = [&](int& pix, int& x, int& y) {
      pix += kThreads;
      x += kThreads;
      while (x >= W) {
        x -= W;
        ++y;
      }
    };
    int pix = beg + tid, y = pix / W, x = pix - y * W;  // then advanced by kThreads without a division
    Stage A, Bs;
    issue(A, pix, x, y);
    for (;;) {
      const int pa = pix;
      advance(pix, x, y);
      issue(Bs, pix, x, y);
      if (pa < end) term(A);
      if (pix >= end) break;
      const int pb = pix;
      advance(pix, x, y);
      issue(A, pix, x, y);
      if (pb < end) term(Bs);
      if (pix >= end) break;
    }
  };
"""
src = src.replace(old, new)
os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
open(os.path.join(ROOT, "tools", "_var", "icppipe.hip"), "w").write(src)
print("tools/_var/icppipe.hip")
