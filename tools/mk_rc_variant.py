"""Write tools/_var/rc.hip: the shipped source with the marching kernel's two tap divisions
u / ((W-1)/2), v / ((H-1)/2) done by div_const (one product, one FMA correction with the
hoisted reciprocal: equal to the IEEE division on every input for the verified image sizes,
tools/div_check.c) where p.rc_taps, as the combine_ICP pass already does (A/B experiment;
round 4 measured it slower when the kernel spilled more SGPRs).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")).read()
old = """      F.tp[r] = make_taps(F.wp[r].u, F.wp[r].v, H, W);
      F.pw[r] = pair_weights(F.tp[r]);"""
assert old in src
new = """      if (rcxy) {
        int a_, b_, c_, d_;
        F.tp[r] = make_taps_xy<true>(F.wp[r].u, F.wp[r].v, H, W, a_, b_, c_, d_, rcxy);
      } else {
        F.tp[r] = make_taps(F.wp[r].u, F.wp[r].v, H, W);
      }
      F.pw[r] = pair_weights(F.tp[r]);"""
src = src.replace(old, new)
old = """  auto make_frame_xy = [&](int xs, int y0, const float (&dv)[R], Frame& F, bool s0_rows, const float* xyr = nullptr) {"""
assert old in src
src = src.replace(old, """  const float rcxy_v[2] = {1.0f / ((float)(W - 1) * 0.5f), 1.0f / ((float)(H - 1) * 0.5f)};
  const float* rcxy = (kWin && p.rc_taps) ? rcxy_v : nullptr;
""" + old)
os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
out = os.path.join(ROOT, "tools", "_var", "rc.hip")
open(out, "w").write(src)
print(out)
