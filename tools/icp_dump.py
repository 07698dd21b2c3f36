"""Dump combine_ICP normal equations at fixed poses (A/B of library builds: DPFT_LIB=...).
python tools/icp_dump.py OUT.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
from deep_prob_feature_track_amd import _native  # noqa: E402
if os.environ.get("DPFT_LIB"):
    _native.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
import golden_io  # noqa: E402
from deep_prob_feature_track_amd import ic  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for name in ("icp_640x480_c32", "icp_160x120_c8"):
    case, z = golden_io.load(name)
    lv = golden_io.levels_torch(case, torch.float32, dev)
    K = torch.from_numpy(case["K"]).to(dev)
    i = 0
    for l in reversed(range(case["levels"])):
        d = lv[l]
        for it in range(3):
            R = torch.from_numpy(z["f32_R"][i]).to(dev)
            t = torch.from_numpy(z["f32_t"][i]).to(dev).reshape(-1, 3, 1)
            for pack in (True, False):
                f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
                o = ic.iterate((R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                               update=False, remove_tru_sigma=True, combine_icp=True, depth0=d["depth0"],
                               depth1=d["depth1"])
                out[f"{name}_{i}_{int(pack)}_jtj"] = o[2].cpu().numpy()
                out[f"{name}_{i}_{int(pack)}_jtr"] = o[3].cpu().numpy()
                out[f"{name}_{i}_{int(pack)}_inv"] = o[4].cpu().numpy()
            i += 1
np.savez(sys.argv[1], **out)
print("saved", len(out))
