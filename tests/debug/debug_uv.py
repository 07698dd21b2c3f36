import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch, golden_io
from oracle import ic_oracle as O
from deep_prob_feature_track_amd import ic
dev = torch.device("cuda:0")
case, z = golden_io.load(sys.argv[1])
lvg = golden_io.levels_torch(case, torch.float32, dev)[0]
lvc = golden_io.levels_torch(case, torch.float32)[0]
R, t = golden_io.init_pose(case, torch.float32)
K = torch.from_numpy(case["K"])
dbg = ic.debug_pixels((R.to(dev), t.to(dev)), lvg["f0"], lvg["f1"], lvg["invD0"], lvg["invD1"], K.to(dev),
                      lvg["s0"], lvg["s1"]).cpu()
B, C, H, W = lvc["f0"].shape
x, y = O.pixel_rays(B, H, W, K)
u, v, iz = O.warp_inverse_depth(x, y, lvc["invD0"], R, t.view(-1, 3, 1), K)
for nm, a, bb in (("u", dbg[:, 0], u[:, 0]), ("v", dbg[:, 1], v[:, 0])):
    ne = (a != bb).nonzero()
    print(nm, len(ne))
    for (b_, yy, xx) in ne[:6].tolist():
        print(b_, yy, xx, float(a[b_, yy, xx]).hex(), float(bb[b_, yy, xx]).hex(), "d", float(lvc["invD0"][b_, 0, yy, xx]).hex())
np.save("gpurun_out/uv_dbg.npy", dbg.numpy())
