"""Golden vectors for the evaluation metrics (reference code/models/criterions.py).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_metrics_golden.py   (build container only)

Seeded random poses / depth / intrinsics -> the reference's compute_RPE_loss,
compute_RT_EPE_loss (with an invalid mask and a NaN pixel), batch_mat2euler /
batch_euler2mat over every axis convention and batch_create_transform;
saved with their inputs in tests/golden/metrics.npz.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main():
    from gen_golden import import_reference
    torch, _ = import_reference()
    import models.criterions as Cr  # noqa: E402  (reference, read-only)
    import models.geometry as G  # noqa: E402
    g = torch.Generator().manual_seed(5)
    B, H, W = 3, 12, 16
    a = (torch.rand(B, 3, generator=g) - 0.5) * 0.4
    R_est = G.batch_euler2mat(a[:, 0], a[:, 1], a[:, 2])
    a2 = a + (torch.rand(B, 3, generator=g) - 0.5) * 0.02
    R_gt = G.batch_euler2mat(a2[:, 0], a2[:, 1], a2[:, 2])
    t_est = torch.rand(B, 3, generator=g) - 0.5
    t_gt = t_est + (torch.rand(B, 3, generator=g) - 0.5) * 0.05
    depth = 0.5 + 3 * torch.rand(B, 1, H, W, generator=g)
    depth[0, 0, 2, 3] = float("nan")
    K = torch.tensor([[20.0, 21.0, 7.5, 5.5]]).repeat(B, 1)
    invalid = torch.rand(B, 1, H, W, generator=g) > 0.8
    ang, trs = Cr.compute_RPE_loss(R_est, t_est, R_gt, t_gt)
    epe = Cr.compute_RT_EPE_loss(R_est, t_est, R_gt, t_gt, depth, K, invalid=invalid)
    epe_noinv = Cr.compute_RT_EPE_loss(R_est, t_est, R_gt, t_gt, depth, K)
    eul = torch.stack(G.batch_mat2euler(R_gt), 1)
    # every Euler axis convention both ways (convergence_basin.py:27 imports both), including a
    # gimbal-locked matrix (the reference's degenerate branch), and kf_vo.py's 4x4 transforms
    axes = sorted(G._AXES2TUPLE)
    ang3 = (torch.rand(4, 3, generator=g, dtype=torch.float64) - 0.5) * 2.0
    ang3[3, 1] = np.pi / 2
    e2m = np.stack([G.batch_euler2mat(ang3[:, 0], ang3[:, 1], ang3[:, 2], axes=ax).numpy() for ax in axes])
    m2e = np.stack([torch.stack(G.batch_mat2euler(torch.from_numpy(e2m[k]), axes=ax), 1).numpy()
                    for k, ax in enumerate(axes)])
    xform = G.batch_create_transform(t_est, R_est).numpy()
    xform_np = G.batch_create_transform(t_est[0].numpy(), R_est[0].numpy())
    np.savez(os.path.join(HERE, "metrics.npz"), R_est=R_est.numpy(), t_est=t_est.numpy(), R_gt=R_gt.numpy(),
             t_gt=t_gt.numpy(), depth=depth.numpy(), K=K.numpy(), invalid=invalid.numpy(), ang=ang.numpy(),
             trs=trs.numpy(), epe=epe.numpy(), epe_noinv=epe_noinv.numpy(), euler=eul.numpy(),
             euler_axes=np.array(axes), euler_angles=ang3.numpy(), euler2mat=e2m, mat2euler=m2e,
             create_transform=xform, create_transform_np=xform_np)
    print("ang", ang.numpy(), "epe", epe.numpy())


if __name__ == "__main__":
    main()
