"""Host-independent numpy emulation of the reference's fp32 CPU arithmetic for
the warp and the bilinear sampler (test infrastructure).

torch-CPU results depend on the host's vector ISA (the fixtures were made on an
AVX-512 host; a GPU box's host may differ), so bit-exact tests compare the HIP
kernels with this emulation instead: every op is an IEEE fp32 op in numpy, and
the fused multiply-adds torch's kernels use are emulated exactly (an fp32
product is exact in fp64, and the fp64 sum rounded once to fp32 is the fused
result for these magnitudes).  Pinned against torch on the fixture host by
tests/test_ref_arith.py.

  geometry.py:63-85    px = (u - cx) / fx
  geometry.py:312-321  torch.bmm(R, [px,py,1]) = fma(R1, py, R0*px) + R2; + t*invD;
                       u = (X / Z) * fx + cx; iz = invD / Z
  geometry.py:359-364  grid = u / ((W-1)/2) - 1 -> grid_sample(border, align_corners)
                       ix = (g + 1) * ((W-1)/2), weights by distance products,
                       value = fma(d, se, fma(c, sw, fma(b, ne, a * nw)))
"""
import numpy as np

f32, f64 = np.float32, np.float64


def fma(a, b, c):
    return (np.asarray(a, f64) * np.asarray(b, f64) + np.asarray(c, f64)).astype(f32)


def warp(H, W, invD0, R, t, K):
    """invD0 [H,W], R [3,3], t [3], K [4] (this level) -> u, v, iz, px, py (fp32 [H,W])."""
    fx, fy, cx, cy = (f32(k) for k in K)
    u = np.arange(W, dtype=f32)[None, :].repeat(H, 0)
    v = np.arange(H, dtype=f32)[:, None].repeat(W, 1)
    px = ((u - cx) / fx).astype(f32)
    py = ((v - cy) / fy).astype(f32)
    R = R.astype(f32)
    t = t.astype(f32)
    d = invD0.astype(f32)
    P = [((fma(R[i, 1], py, (R[i, 0] * px).astype(f32)) + R[i, 2]).astype(f32) + (t[i] * d).astype(f32)).astype(f32)
         for i in range(3)]
    uu = (((P[0] / P[2]).astype(f32) * fx).astype(f32) + cx).astype(f32)
    vv = (((P[1] / P[2]).astype(f32) * fy).astype(f32) + cy).astype(f32)
    iz = (d / P[2]).astype(f32)
    return uu, vv, iz, px, py


def sample(F, u, v):
    """Bilinear border sample of F [C,H,W] at fp32 u, v [H',W'] -> [C,H',W']."""
    C, H, W = F.shape
    sx, sy = f32((W - 1) / 2), f32((H - 1) / 2)
    ix = ((((u / sx).astype(f32) - f32(1)).astype(f32) + f32(1)).astype(f32) * sx).astype(f32)
    iy = ((((v / sy).astype(f32) - f32(1)).astype(f32) + f32(1)).astype(f32) * sy).astype(f32)
    ix = np.clip(np.nan_to_num(ix, nan=0.0), 0, W - 1).astype(f32)
    iy = np.clip(np.nan_to_num(iy, nan=0.0), 0, H - 1).astype(f32)
    x0, y0 = np.floor(ix), np.floor(iy)
    w = (ix - x0).astype(f32)
    e = (f32(1) - w).astype(f32)
    n = (iy - y0).astype(f32)
    s = (f32(1) - n).astype(f32)
    nw, ne, sw, se = ((s * e).astype(f32), (s * w).astype(f32), (n * e).astype(f32), (n * w).astype(f32))
    xi, yi = x0.astype(np.int64), y0.astype(np.int64)
    x1, y1 = np.minimum(xi + 1, W - 1), np.minimum(yi + 1, H - 1)
    F = F.astype(f32)
    a, b, c, d = F[:, yi, xi], F[:, yi, x1], F[:, y1, xi], F[:, y1, x1]
    return fma(d, se, fma(c, sw, fma(b, ne, (a * nw).astype(f32))))


def occlusion(u, v, iz, invD1):
    """True where invalid (geometry.py:341-350)."""
    H, W = invD1.shape
    d1w = sample(invD1[None], u, v)[0]
    ok = (iz > (d1w - f32(0.1)).astype(f32)) & (u > 0) & (u < W) & (v > 0) & (v < H)
    return ~ok
