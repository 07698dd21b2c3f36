"""Generate the golden parity fixtures by running the REFERENCE solver.

Run in the build container only (needs /root/reference; refuses otherwise):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [case ...]
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py --noise case ...   (noise-floor runs)
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py --noise-more=N case ...   (N more such runs)

No reference code is copied: the reference package is imported read-only from
/root/reference/code with the import shims of SURVEY.md Appendix A (stub
cv2 / torchvision / tensorboard modules, torch-1.x float `>>`).  The solver
used is the reference's own `TrustRegionInverseWUncertainty`
(`code/models/algorithms.py:579-997`), driven level by level exactly as
`LeastSquareTracking.forward` does (`code/models/LeastSquareTracking.py:345-445`:
levels 3 -> 0, K / 2^l, pose chained).  Per level and iteration the harness
records JtJ, JtR, the updated pose and the invalid-pixel count by wrapping the
instance's `GN_solver` and the module-level `compute_inverse_residuals`; it
also records `forward_residuals` losses (`algorithms.py:725-786`) at the level's
start and end pose.  Each case runs twice: fp32 and fp64.  With object masks the fp64
run needs one harness-side cast: the reference samples `obj_mask1.float()` on the
pose's (double) grid (algorithms.py:2006), which grid_sample refuses, so the harness
casts the sampled map to the grid's dtype inside `geometry.warp_features` (a 0/1 mask is
exact in both precisions; every other call already has matching dtypes).

`--noise` adds the reference's own fp32 noise floor to a fixture, per iteration (tests bound
chained trajectories by it where it exceeds 1e-4): NOISE_TRIALS runs in which EVERY
Gauss-Newton update's pose (R and t entries) is moved by fresh U(+-JITTER_ABS) noise --
JITTER_ABS is the measured one-step deviation of the HIP solve from the reference (3.4e-8,
tests/test_oracle_golden.py), applied where and as often as that deviation arises (after
each step: an fp32 solve that sums in another order differs from the reference by that much
at every iteration; a moved START would instead leave the identity pose, where the warp is
exact and the clipped sigma plateaus sit at the batch extrema, a discontinuity the solve
itself never crosses) -- and one run on a single thread (SURVEY App. B's 1-vs-N-thread
spread).  `--noise64` adds the fp64
floor the same way (1e-16: the truncated-sigma equality tests make the fp64 trajectory
chaotic too).

Outputs: tests/golden/<case>.npz holding the outputs plus the SHA-256 of every
input tensor (inputs are regenerated from `recipe.py`).
"""
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/code"
sys.path.insert(0, HERE)
import recipe  # noqa: E402

# case name -> solver options
OPTIONS = {
    "cfg1_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg1b_160x120_c8_f04": dict(remove_tru_sigma=False, combine_icp=False),
    "batch4_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "masks_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "icp_160x120_c8": dict(remove_tru_sigma=True, combine_icp=True),
    "cfg2_640x480_c32": dict(remove_tru_sigma=True, combine_icp=False),
    "icp_640x480_c32": dict(remove_tru_sigma=True, combine_icp=True),
    "cfg3_b8_640x480_c32": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg3_b8q2_640x480_c32": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg3_b8q7_640x480_c32": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_pert00_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_pert05_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_pert10_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_pert20_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_sweep256_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_sweep256_rotx10_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_sweep256_tz10_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_sweep256_ry011_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
    "cfg4_sweep256_tz012_160x120_c8": dict(remove_tru_sigma=True, combine_icp=False),
}


def import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("gen_golden.py needs the reference at /root/reference (build container only)")
    sys.dont_write_bytecode = True
    for name in ["cv2", "torchvision", "torchvision.models", "torchvision.transforms", "torch.utils.tensorboard"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    cv2 = sys.modules["cv2"]
    cv2.COLORMAP_JET, cv2.COLORMAP_WINTER, cv2.WINDOW_NORMAL = 2, 3, 0
    sys.modules["torchvision"].models = sys.modules["torchvision.models"]
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torch.utils.tensorboard"].SummaryWriter = object
    import torch
    rs = torch.Tensor.__rshift__
    torch.Tensor.__rshift__ = lambda s, n: s / (2 ** n) if s.is_floating_point() else rs(s, n)
    sys.path.insert(0, REF)
    import models.algorithms as A  # noqa: E402
    return torch, A


def run_case(torch, A, name, dtype, perturb_updates=None):
    """perturb_updates: (numpy Generator, amplitude) -- every update's pose moved by fresh
    uniform noise of that amplitude (the --noise / --noise64 runs); None: the plain run."""
    spec = recipe.CASES[name]
    opt = OPTIONS[name]
    case = recipe.make_case(**spec)
    G = sys.modules["models.geometry"]
    orig_wf = G.warp_features
    if dtype == torch.float64:  # the mask sampling of algorithms.py:2006 (see the module docstring)
        G.warp_features = lambda F, u, v: orig_wf(F.to(u.dtype), u, v)
    try:
        return _run_case(torch, A, name, dtype, spec, opt, case, perturb_updates)
    finally:
        G.warp_features = orig_wf


def _run_case(torch, A, name, dtype, spec, opt, case, perturb_updates=None):
    L = case["levels"]
    B, C = case["B"], case["C"]
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dtype)

    log = {"jtj": [], "jtr": [], "R": [], "t": [], "invalid": []}
    orig_cir = A.compute_inverse_residuals

    def cir(*a, **k):
        out = orig_cir(*a, **k)
        log["invalid"].append(out[3].reshape(out[3].shape[0], -1).sum(1).numpy().astype(np.int64))
        return out

    A.compute_inverse_residuals = cir
    try:
        solvers = []
        for _ in range(L):
            s = A.TrustRegionInverseWUncertainty(
                max_iter=3,
                mEst_func=A.DeepRobustEstimator("None"),
                solver_func=A.DirectSolverNet("Direct-Nodamping"),
                combine_icp=opt["combine_icp"],
                scale_func=A.ScaleNet("None"),
                remove_tru_sigma=opt["remove_tru_sigma"],
            )
            orig_gn = s.GN_solver

            def gn(JtJ, JtR, pose0, direction="inverse", _o=orig_gn):
                out = _o(JtJ, JtR, pose0)
                if perturb_updates is not None:  # every update moved by fresh U(+-amplitude) noise
                    rng, amp = perturb_updates
                    dR = torch.from_numpy(rng.uniform(-amp, amp, size=tuple(out[0].shape))).to(out[0].dtype)
                    dt = torch.from_numpy(rng.uniform(-amp, amp, size=tuple(out[1].shape))).to(out[1].dtype)
                    out = [out[0] + dR, out[1] + dt]
                log["jtj"].append(JtJ.detach().numpy().copy())
                log["jtr"].append(JtR.detach().numpy().reshape(-1, 6).copy())
                log["R"].append(out[0].detach().numpy().copy())
                log["t"].append(out[1].detach().numpy().reshape(-1, 3).copy())
                return out

            s.GN_solver = gn
            solvers.append(s)

        pose = [tt(case["R_init"]), tt(case["t_init"]).view(B, 3, 1)]
        K = tt(case["K"])
        loss_start, loss_end = [], []
        wprior = None
        with torch.no_grad():
            for l in reversed(range(L)):
                Kl = K >> l
                args = dict(
                    x0=tt(case[f"x0_{l}"]), x1=tt(case[f"x1_{l}"]),
                    invD0=tt(case[f"invD0_{l}"]), invD1=tt(case[f"invD1_{l}"]), K=Kl,
                    sigma0=tt(case[f"s0_{l}"]).repeat(1, C, 1, 1),
                    sigma1=tt(case[f"s1_{l}"]).repeat(1, C, 1, 1),
                    depth0=tt(case[f"depth0_{l}"]) if f"depth0_{l}" in case else None,
                    depth1=tt(case[f"depth1_{l}"]) if f"depth1_{l}" in case else None,
                    obj_mask0=torch.from_numpy(case[f"mask0_{l}"]) if f"mask0_{l}" in case else None,
                    obj_mask1=torch.from_numpy(case[f"mask1_{l}"]) if f"mask1_{l}" in case else None,
                )
                if wprior is None:
                    wprior = torch.ones(args["invD0"].shape, dtype=dtype) * 0.001
                s = solvers[l]
                n_inv = len(log["invalid"])
                loss_start.append(s.forward_residuals(pose, wPrior=wprior, vis_res=False, **args).reshape(B).numpy())
                del log["invalid"][n_inv:]
                out = s.forward(pose, wPrior=wprior, vis_res=False, **args)
                pose, wprior = out[0], out[1]
                n_inv = len(log["invalid"])
                loss_end.append(s.forward_residuals(pose, wPrior=wprior, vis_res=False, **args).reshape(B).numpy())
                del log["invalid"][n_inv:]
    finally:
        A.compute_inverse_residuals = orig_cir

    res = {
        "jtj": np.stack(log["jtj"]),          # [L*3, B, 6, 6] in solve order (level L-1 first)
        "jtr": np.stack(log["jtr"]),          # [L*3, B, 6]
        "R": np.stack(log["R"]),              # [L*3, B, 3, 3]
        "t": np.stack(log["t"]),              # [L*3, B, 3]
        "invalid": np.stack(log["invalid"]),  # [L*3, B]
        "loss_start": np.stack(loss_start),   # [L, B]
        "loss_end": np.stack(loss_end),       # [L, B]
    }
    return case, res


NOISE_TRIALS, JITTER_ABS = 8, 3.4e-8


def add_noise_floor(torch, A, name, append=0):
    """The reference's own fp32 noise floor of a case (see the module docstring): appends
    f32_jitter_R [N, iters, B, 3, 3] / f32_jitter_t [N, iters, B, 3] (every iteration of
    NOISE_TRIALS runs in which every Gauss-Newton update's R and t are moved by fresh
    U(+-JITTER_ABS) noise) and f32_t1_R / f32_t1_t [iters, B, ...] (the unperturbed run on
    one thread) to the case's fixture."""
    path = os.path.join(HERE, f"{name}.npz")
    out = dict(np.load(path, allow_pickle=False))
    if append:  # more runs of the same kind (fresh seeds) beside the existing ones
        n0 = out["f32_jitter_R"].shape[0]
        rng = np.random.default_rng(1000 * n0 + sum(ord(c) for c in name))
        Rs, ts = list(out["f32_jitter_R"]), list(out["f32_jitter_t"])
        for _ in range(append):
            _, res = run_case(torch, A, name, torch.float32, perturb_updates=(rng, JITTER_ABS))
            Rs.append(res["R"])
            ts.append(res["t"])
        out["f32_jitter_R"], out["f32_jitter_t"] = np.stack(Rs), np.stack(ts)
        np.savez_compressed(path, **out)
        print(f"{name}: {len(Rs)} per-update jitter runs", flush=True)
        return
    rng = np.random.default_rng(sum(ord(c) for c in name))
    Rs, ts = [], []
    for _ in range(NOISE_TRIALS):
        _, res = run_case(torch, A, name, torch.float32, perturb_updates=(rng, JITTER_ABS))
        Rs.append(res["R"])
        ts.append(res["t"])
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        _, res1 = run_case(torch, A, name, torch.float32)
    finally:
        torch.set_num_threads(nthreads)
    out["f32_jitter_R"], out["f32_jitter_t"] = np.stack(Rs), np.stack(ts)
    out["f32_t1_R"], out["f32_t1_t"] = res1["R"], res1["t"]
    out["meta_jitter_abs"] = np.array(JITTER_ABS)
    np.savez_compressed(path, **out)
    dev = max(np.abs(out["f32_jitter_R"][:, -1] - out["f32_R"][-1]).max(),
              np.abs(out["f32_jitter_t"][:, -1] - out["f32_t"][-1]).max())
    dev1 = max(np.abs(res1["R"][-1] - out["f32_R"][-1]).max(), np.abs(res1["t"][-1] - out["f32_t"][-1]).max())
    print(f"{name}: reference final pose moves by up to {dev:.2e} under {JITTER_ABS:g} per-update jitter, "
          f"{dev1:.2e} on one thread")


NOISE64_ABS = 1e-16


def add_noise_floor64(torch, A, name):
    """The reference's fp64 noise floor (NOISE_TRIALS fp64 runs in which every update's R and
    t are moved by fresh U(+-NOISE64_ABS) noise: the truncated-sigma equality tests flip
    pixels in fp64 too): appends f64_jitter_R / f64_jitter_t [N, iters, B, ...]."""
    path = os.path.join(HERE, f"{name}.npz")
    out = dict(np.load(path, allow_pickle=False))
    rng = np.random.default_rng(7 + sum(ord(c) for c in name))
    Rs, ts = [], []
    for _ in range(NOISE_TRIALS):
        _, res = run_case(torch, A, name, torch.float64, perturb_updates=(rng, NOISE64_ABS))
        Rs.append(res["R"])
        ts.append(res["t"])
    out["f64_jitter_R"], out["f64_jitter_t"] = np.stack(Rs), np.stack(ts)
    out["meta_jitter64_abs"] = np.array(NOISE64_ABS)
    np.savez_compressed(path, **out)
    dev = max(np.abs(out["f64_jitter_R"][:, -1] - out["f64_R"][-1]).max(),
              np.abs(out["f64_jitter_t"][:, -1] - out["f64_t"][-1]).max())
    print(f"{name}: fp64 reference final pose moves by up to {dev:.2e} under {NOISE64_ABS:g} per-update jitter", flush=True)


def main(names):
    torch, A = import_reference()
    if names and names[0] == "--noise64":
        for name in names[1:]:
            add_noise_floor64(torch, A, name)
        return
    if names and names[0] == "--noise":
        for name in names[1:]:
            add_noise_floor(torch, A, name)
        return
    if names and names[0].startswith("--noise-more="):  # --noise-more=N case ...: N more runs each
        n = int(names[0].split("=", 1)[1])
        for name in names[1:]:
            add_noise_floor(torch, A, name, append=n)
        return
    nthreads = torch.get_num_threads()
    for name in names:
        t0 = time.time()
        out = {}
        for tag, dtype in (("f32", torch.float32), ("f64", torch.float64)):
            case, res = run_case(torch, A, name, dtype)
            for k, v in res.items():
                out[f"{tag}_{k}"] = v
        dig = recipe.input_digests(case)
        out["digest_keys"] = np.array(sorted(dig))
        out["digest_vals"] = np.array([dig[k] for k in sorted(dig)])
        out["meta_torch"] = np.array(torch.__version__)
        out["meta_threads"] = np.array(nthreads)
        out["opt_remove_tru_sigma"] = np.array(OPTIONS[name]["remove_tru_sigma"])
        out["opt_combine_icp"] = np.array(OPTIONS[name]["combine_icp"])
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        ref = "f64" if "f64_R" in out else "f32"
        d = np.abs(out["f32_R"][-1] - out[f"{ref}_R"][-1]).max()
        dt = np.abs(out["f32_t"][-1] - out[f"{ref}_t"][-1]).max()
        print(f"{name}: {time.time() - t0:.1f}s  final t({ref}) pair 0={out[ref + '_t'][-1][0].tolist()}  "
              f"|f32-f64| R {d:.2e} t {dt:.2e}  invalid(last)={out['f32_invalid'][-1].tolist()}")


if __name__ == "__main__":
    main(sys.argv[1:] or list(recipe.CASES))
