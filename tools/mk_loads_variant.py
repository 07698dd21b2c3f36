"""Write tools/_var/loads.hip: the shipped source with the channel-quad marching body's
arithmetic removed and EVERY load kept ("set the bound first").

The access-pattern replay at the bench's real shape: the same kernel, launch shape, band / pool
schedule, tap cache, cross-row prefetch, window in LDS and all six inputs (f0 rows, f1 tap pairs,
the invD1 / sigma1 gathers, the sigma0 / invD0 rows) -- the frame's warp and tap arithmetic stay,
since they generate the gather addresses -- but the per-channel Sobel, residual and channel sums
and the per-pixel 27-term epilogue are gone: each loaded vector is consumed by an empty
`asm volatile` (forces the load and its wait, emits no instruction).  Time it with
`tools/kbench.py --mode reduce --from-solve --c4 --groups 16` (records only, no finalize: the
poses stay at the solved ones) against the shipped library in the same mode; its FETCH_SIZE with
tools/pmc_l0.py --mode reduce.  The records it writes are meaningless.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")).read()

# 1. the channel loop: no Sobel / residual / sums, the loaded vectors consumed by an empty asm
a = src.index("        const f32x4 wtop = *s0p, wmid = *s1p;      // rows above / at the pixel in marching order")
b = src.index("        *s0p = wmid;  // window (y, y + dir)")
body = src[a:b]
assert "Q[8] += res;" in body
src = src[:a] + """        const f32x4 wtop = *s0p, wmid = *s1p;
        asm volatile("" ::"v"(wtop), "v"(wmid), "v"(cur.f), "v"(cur.t[0]), "v"(cur.t[1]), "v"(cur.P), "v"(tc[q][0]),
                     "v"(tc[q][1]));
""" + src[b:]

# 2. the pixel epilogue of the marching step: the frame's gathers and sigma0 rows consumed
a = src.index("      PixelTerms T;\n      pixel_terms(F, T);\n      Sums S;\n      float q[9];")
b = src.index("      finish_pixels(F, T, S, &d0e);\n    };\n    for (int k = 0; k < nrows; ++k) step(k);")
src = src[:a] + """      asm volatile("" ::"v"(F.gd1[0].a), "v"(F.gd1[0].b), "v"(F.gd1[0].c), "v"(F.gd1[0].d), "v"(F.gs1[0].a),
                   "v"(F.gs1[0].b), "v"(F.gs1[0].c), "v"(F.gs1[0].d), "v"(F.s0r[0]), "v"(F.s0r[1]), "v"(F.s0r[2]),
                   "v"(d0e), "v"(Q[0]));
""" + src[b + len("      finish_pixels(F, T, S, &d0e);\n"):]

os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
out = os.path.join(ROOT, "tools", "_var", "loads.hip")
open(out, "w").write(src)
print(out)
