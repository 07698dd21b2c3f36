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
