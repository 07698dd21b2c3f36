"""Debug helper: compare one HIP iteration with the oracle on a golden case (GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np, torch
import golden_io
from oracle import ic_oracle as O
from deep_prob_feature_track_amd import ic
dev = torch.device("cuda:0")
for name in sys.argv[1:] or ["cfg1_160x120_c8"]:
    case, z = golden_io.load(name)
    L = case["levels"]
    for tru in (False, True):
        lvg = golden_io.levels_torch(case, torch.float32, dev)[L - 1]
        lvc = golden_io.levels_torch(case, torch.float32)[L - 1]
        R, t = golden_io.init_pose(case, torch.float32)
        K = torch.from_numpy(case["K"]) / 2 ** (L - 1)
        tr = []
        O.solve_level(R, t.view(-1, 3, 1), lvc["f0"], lvc["f1"], lvc["s0"], lvc["s1"], lvc["invD0"],
                      lvc["invD1"], K, iters=1, remove_tru_sigma=tru, mask0=lvc.get("mask0"),
                      mask1=lvc.get("mask1"), trace=tr)
        Rg, tg, jtj, jtr, inv = ic.iterate((R.to(dev), t.to(dev).view(-1, 3, 1)), lvg["f0"], lvg["f1"], lvg["invD0"],
                                           lvg["invD1"], K.to(dev), lvg["s0"], lvg["s1"], first=True,
                                           remove_tru_sigma=tru, obj_mask0=lvg.get("mask0"), obj_mask1=lvg.get("mask1"))
        loss_g = ic.residual_level((R.to(dev), t.to(dev)), lvg["f0"], lvg["f1"], lvg["invD0"], lvg["invD1"], K.to(dev),
                                   lvg["s0"], lvg["s1"], remove_tru_sigma=tru, obj_mask0=lvg.get("mask0"),
                                   obj_mask1=lvg.get("mask1"))
        loss_o = O.residual_loss(R, t, lvc["f0"], lvc["f1"], lvc["s0"], lvc["s1"], lvc["invD0"],
                                 lvc["invD1"], K, remove_tru_sigma=tru, mask0=lvc.get("mask0"),
                                 mask1=lvc.get("mask1"))
        print(f"== {name} tru={tru}")
        print(" invalid hip", inv.cpu().numpy(), "oracle", tr[0]["invalid"].numpy())
        print(" jtr hip   ", jtr.cpu().numpy())
        print(" jtr oracle", tr[0]["JtR"].numpy())
        print(" jtj diag hip   ", np.diagonal(jtj.cpu().numpy(), axis1=1, axis2=2))
        print(" jtj diag oracle", np.diagonal(tr[0]["JtJ"].numpy(), axis1=1, axis2=2))
        print(" loss hip", loss_g.cpu().numpy(), "oracle", loss_o.numpy())

# per-pixel comparison at the initial pose
for name in sys.argv[1:] or ["cfg1_160x120_c8"]:
    case, z = golden_io.load(name)
    L = case["levels"]
    lvg = golden_io.levels_torch(case, torch.float32, dev)[L - 1]
    lvc = golden_io.levels_torch(case, torch.float32)[L - 1]
    R, t = golden_io.init_pose(case, torch.float32)
    K = torch.from_numpy(case["K"]) / 2 ** (L - 1)
    dbg = ic.debug_pixels((R.to(dev), t.to(dev)), lvg["f0"], lvg["f1"], lvg["invD0"], lvg["invD1"], K.to(dev),
                          lvg["s0"], lvg["s1"], obj_mask0=lvg.get("mask0"), obj_mask1=lvg.get("mask1")).cpu()
    B, C, H, W = lvc["f0"].shape
    x, y = O.pixel_rays(B, H, W, K)
    u, v, iz = O.warp_inverse_depth(x, y, lvc["invD0"], R, t.view(-1, 3, 1), K)
    sr = O.bilinear(lvc["s1"], u, v)
    inv = O.occlusion(iz, lvc["invD1"], u, v)
    for nm, a, bb in (("u", dbg[:, 0], u[:, 0]), ("v", dbg[:, 1], v[:, 0]), ("sr", dbg[:, 2], sr[:, 0]),
                      ("s0", dbg[:, 3], lvc["s0"][:, 0]), ("occ", dbg[:, 4], inv[:, 0].float())):
        ne = (a != bb)
        print(f"{nm}: {int(ne.sum())} mismatches; first:", ne.nonzero()[:5].tolist(),
              a[ne][:5].tolist(), bb[ne][:5].tolist())
