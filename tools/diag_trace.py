"""Per-iteration GPU trace of a golden case against the reference's fp32 run (GPU box).

python tools/diag_trace.py NAME [NAME ...] [--nchw]

chained: the GPU's own trajectory (ic.iterate from its previous pose), |dR| / |dt| and the
invalid-count difference against the reference per iteration; restart: every iteration
from the reference's pose of the previous one -- invalid counts, JtJ / JtR relative error
and the one-step pose error.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import golden_io  # noqa: E402
from deep_prob_feature_track_amd import ic  # noqa: E402


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("--")]
    pack = "--nchw" not in sys.argv
    dev = torch.device("cuda:0")
    for name in names:
        case, z = golden_io.load(name)
        lv = golden_io.levels_torch(case, torch.float32, dev)
        R0, t0 = golden_io.init_pose(case, torch.float32, dev)
        K = torch.from_numpy(case["K"]).to(dev)
        kw = lambda d: dict(remove_tru_sigma=bool(z["opt_remove_tru_sigma"]), obj_mask0=d.get("mask0"),
                            obj_mask1=d.get("mask1"), depth0=d.get("depth0"), depth1=d.get("depth1"),
                            combine_icp=bool(z["opt_combine_icp"]))
        R, t = R0.clone(), t0.reshape(-1, 3, 1).clone()
        i = 0
        print(f"== {name} ({'c4' if pack else 'nchw'})", flush=True)
        for l in reversed(range(case["levels"])):
            d = lv[l]
            f0, f1 = (ic.pack_features(d["f0"]), ic.pack_features(d["f1"])) if pack else (d["f0"], d["f1"])
            for it in range(3):
                R, t, jc, rc, nc = ic.iterate((R, t), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"], d["s1"],
                                              first=(it == 0), reverse=(it & 1) == 1, **kw(d))
                Rr = torch.from_numpy(z["f32_R"][i - 1]).to(dev) if i else R0
                tr = (torch.from_numpy(z["f32_t"][i - 1]).to(dev) if i else t0).reshape(-1, 3, 1)
                Rn, tn, jr, rr, nr = ic.iterate((Rr, tr), f0, f1, d["invD0"], d["invD1"], K / 2 ** l, d["s0"],
                                                d["s1"], first=True, reverse=(it & 1) == 1, **kw(d))
                zj, zr = z["f32_jtj"][i], z["f32_jtr"][i]
                print(f"l{l} it{it}: chained |dR| {np.abs(R.cpu().numpy() - z['f32_R'][i]).max():.2e} "
                      f"|dt| {np.abs(t.cpu().numpy().reshape(-1, 3) - z['f32_t'][i]).max():.2e} "
                      f"dinv {(nc.cpu().numpy() - z['f32_invalid'][i]).tolist()} | restart "
                      f"dinv {(nr.cpu().numpy() - z['f32_invalid'][i]).tolist()} "
                      f"JtJ {np.abs(jr.cpu().numpy() - zj).max() / np.abs(zj).max():.1e} "
                      f"JtR {np.abs(rr.cpu().numpy() - zr).max() / np.abs(zr).max():.1e} "
                      f"step |dR| {np.abs(Rn.cpu().numpy() - z['f32_R'][i]).max():.1e} "
                      f"|dt| {np.abs(tn.cpu().numpy().reshape(-1, 3) - z['f32_t'][i]).max():.1e}", flush=True)
                i += 1


if __name__ == "__main__":
    main()
