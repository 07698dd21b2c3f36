"""Debug helper: one random case, HIP vs fp32 / fp64 oracle (GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import torch
from oracle import ic_oracle as O
from deep_prob_feature_track_amd import ic
from test_gpu_parity import _random_case
dev = torch.device("cuda:0")
B, C, Cs, H, W, tru, masks = [int(a) for a in sys.argv[1:8]]
f0, f1, s0, s1, invD0, invD1, K, m0, m1 = _random_case(B, C, Cs, H, W, seed=B * 1000 + C * 10 + W, masks=bool(masks))
R = torch.eye(3).repeat(B, 1, 1); t = torch.zeros(B, 3, 1)
cu = lambda a: a.to(dev) if a is not None else None
for dt in (torch.float32, torch.float64):
    tr = []
    dd = lambda a: a.to(dt) if a is not None and a.dtype == torch.float32 else a
    O.solve_level(R.to(dt), t.to(dt), dd(f0), dd(f1), dd(s0), dd(s1), dd(invD0), dd(invD1), K.to(dt), iters=1,
                  remove_tru_sigma=bool(tru), mask0=m0, mask1=m1, trace=tr)
    print(dt, "oracle jtr", tr[0]["JtR"].numpy(), "inv", tr[0]["invalid"].numpy())
Rg, tg, jtj, jtr, inv = ic.iterate((cu(R), cu(t)), cu(f0), cu(f1), cu(invD0), cu(invD1), cu(K), cu(s0), cu(s1),
                                   first=True, remove_tru_sigma=bool(tru), obj_mask0=cu(m0), obj_mask1=cu(m1))
print("hip jtr", jtr.cpu().numpy(), "inv", inv.cpu().numpy())
print("hip jtj diag", torch.diagonal(jtj, dim1=1, dim2=2).cpu().numpy(), "oracle", torch.diagonal(tr[0]["JtJ"], dim1=1, dim2=2).numpy())
dbg = ic.debug_pixels((cu(R), cu(t)), cu(f0), cu(f1), cu(invD0), cu(invD1), cu(K), cu(s0), cu(s1),
                      obj_mask0=cu(m0), obj_mask1=cu(m1)).cpu()
x, y = O.pixel_rays(B, H, W, K)
u, v, iz = O.warp_inverse_depth(x, y, invD0, R, t, K)
occ = O.occlusion(iz, invD1, u, v)
if m0 is not None: occ = occ | ~m0
if m1 is not None: occ = occ | ~(O.bilinear(m1.float(), u, v) > 0)
for nm, a, bb in (("u", dbg[:, 0], u[:, 0]), ("v", dbg[:, 1], v[:, 0]), ("occ", dbg[:, 4], occ[:, 0].float())):
    ne = a != bb
    print(nm, int(ne.sum()), ne.nonzero()[:5].tolist(), a[ne][:5].tolist(), bb[ne][:5].tolist())
