"""Load a golden fixture and rebuild its inputs (test infrastructure)."""
import os

import numpy as np
import torch

import recipe

GOLDEN = os.path.dirname(os.path.abspath(recipe.__file__))


def load(name, check_digests=True):
    z = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    case = recipe.make_case(**recipe.CASES[name])
    if check_digests:
        dig = recipe.input_digests(case)
        for k, v in zip(z["digest_keys"], z["digest_vals"]):
            assert dig[str(k)] == str(v), f"{name}: input {k} does not match its recorded SHA-256"
    return case, z


def levels_torch(case, dtype=torch.float32, device="cpu", repeat_sigma=False):
    """Per-level dicts of torch tensors (oracle / solver argument names)."""
    out = []
    C = case["C"]
    for l in range(case["levels"]):
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dtype)
        d = dict(f0=t(case[f"x0_{l}"]), f1=t(case[f"x1_{l}"]), s0=t(case[f"s0_{l}"]), s1=t(case[f"s1_{l}"]),
                 invD0=t(case[f"invD0_{l}"]), invD1=t(case[f"invD1_{l}"]))
        if repeat_sigma:
            d["s0"] = d["s0"].repeat(1, C, 1, 1)
            d["s1"] = d["s1"].repeat(1, C, 1, 1)
        for k in ("depth0", "depth1"):
            if f"{k}_{l}" in case:
                d[k] = t(case[f"{k}_{l}"])
        for k in ("mask0", "mask1"):
            if f"{k}_{l}" in case:
                d[k] = torch.from_numpy(case[f"{k}_{l}"]).to(device)
        out.append(d)
    return out


def init_pose(case, dtype=torch.float32, device="cpu"):
    R = torch.from_numpy(case["R_init"]).to(device=device, dtype=dtype)
    t = torch.from_numpy(case["t_init"]).to(device=device, dtype=dtype)
    return R, t


def noise_floor(z, prec="f32"):
    """The reference's own `prec` noise floor per iteration, [iters, B] (None if the
    fixture has none): how far its trajectory moves when only rounding changes -- max over
    the jittered-start runs (start translation moved by U(+-3.4e-8), the measured one-step
    deviation of the HIP solve from the reference) and the one-thread run of max(|dR|, |dt|)
    against the fixture's fp32 run (tests/golden/gen_golden.py --noise); prec="f64": the
    fp64 jittered-start runs (start moved by U(+-1e-15), --noise64)."""
    if f"{prec}_jitter_R" not in z:
        return None
    R, t = z[f"{prec}_R"], z[f"{prec}_t"]
    dR = np.abs(z[f"{prec}_jitter_R"] - R[None]).max(axis=(0, 3, 4))
    dt = np.abs(z[f"{prec}_jitter_t"] - t[None]).max(axis=(0, 3))
    fl = np.maximum(dR, dt)
    if prec == "f32" and "f32_t1_R" in z:
        fl = np.maximum(fl, np.maximum(np.abs(z["f32_t1_R"] - R).max(axis=(2, 3)), np.abs(z["f32_t1_t"] - t).max(axis=2)))
    # per iteration, the largest move of any pair: which pair a rounding change hits is itself
    # chance (the batch-global sigma_r extrema sit in one pair's pixels; B = 256 shows it: the
    # trials move a few pairs each, different ones), so the floor is the batch's, not a pair's
    return np.broadcast_to(fl.max(axis=1, keepdims=True), fl.shape).copy()


def pose_deviation(R, t, z, prec="f32", i=-1):
    """Per pair max(|dR|, |dt|) of poses (R [B,3,3], t [B,3(,1)], numpy or torch) against the
    fixture's `prec` run at iteration i."""
    R = np.asarray(R.cpu() if hasattr(R, "cpu") else R).reshape(-1, 3, 3)
    t = np.asarray(t.cpu() if hasattr(t, "cpu") else t).reshape(-1, 3)
    return np.maximum(np.abs(R - z[f"{prec}_R"][i]).max(axis=(1, 2)), np.abs(t - z[f"{prec}_t"][i]).max(axis=1))
