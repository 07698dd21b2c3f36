"""Diagnostic: NCHW vs channel-quad kernels on identical poses, every level of a golden case."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch
import golden_io
from deep_prob_feature_track_amd import ic
name = sys.argv[1] if len(sys.argv) > 1 else "cfg2_640x480_c32"
dev = torch.device("cuda:0")
case, z = golden_io.load(name)
lv = golden_io.levels_torch(case, torch.float32, dev)
R0, t0 = golden_io.init_pose(case, torch.float32, dev)
K = torch.from_numpy(case["K"]).to(dev)
i = 0
for l in reversed(range(case["levels"])):
    d = lv[l]
    for it in range(3):
        R = torch.from_numpy(z["f32_R"][i - 1] if i else R0.cpu().numpy()).to(dev)
        t = torch.from_numpy(z["f32_t"][i - 1] if i else t0.cpu().numpy()).to(dev).view(-1, 3, 1)
        out = []
        for pack in (False, True):
            f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
            o = ic.iterate((R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"], first=True,
                           remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                           obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                           combine_icp=bool(z["opt_combine_icp"]))
            out.append([x.cpu().numpy() for x in o])
        a, b = out
        rel = np.abs(a[2] - b[2]).max() / np.abs(a[2]).max()
        print(f"level {l} it {it}: invalid {a[4]} vs {b[4]} golden {z['f32_invalid'][i] if 'f32_invalid' in z else '-'}; "
              f"JtJ rel {rel:.2e}; dR {np.abs(a[0]-b[0]).max():.2e}", flush=True)
        i += 1

print("--- chained traces")
import test_gpu_c4 as T
for pack in (False, True):
    _, _, tr = T._trace(name, dev, pack)
    for i, x in enumerate(tr):
        gi = z["f32_invalid"][i] if "f32_invalid" in z else None
        print(f"pack={pack} iter {i}: invalid {x['invalid']} golden {gi} dR {np.abs(x['R'] - z['f32_R'][i]).max():.2e} "
              f"dt {np.abs(x['t'] - z['f32_t'][i]).max():.2e}", flush=True)
