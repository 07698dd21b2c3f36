"""The TUM fr1/desk example pairs the reference ships, and deterministic stand-in weights.

The reference's only real image data are five RGB-D frames of fr1/desk
(`code/data/data_examples/TUM/{color,depth}`, 640x480, no ground-truth poses); they are
stored here as arrays (`data/tum_fr1_desk_frames.npz`: color uint8 [5,480,640,3], depth
uint16 [5,480,640]).  Loading follows `code/data/SimpleLoader.py:77-80`: colour / 255,
depth / 5000 clipped to [0.5, 5] m; intrinsics are the Kinect defaults of `code/test.py:68`.
The trained checkpoints are absent (`.MISSING_LARGE_BLOBS:1-2`), so `synthetic_weights`
gives every state_dict entry a deterministic value (integer hashing and exactly-rounded
fp32 ops: the same bits on every host).

Used by the evaluation CLI (`evaluate.py`); the parity fixtures' recipe
(tests/golden/recipe.py) builds on the same loaders.
"""
import os

import numpy as np

FRAMES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "tum_fr1_desk_frames.npz")
K_FULL = np.array([525.0, 525.0, 319.5, 239.5], dtype=np.float32)  # code/test.py:68
ORDERED_PAIRS = [(i, j) for i in range(5) for j in range(5) if i != j]  # the 20 ordered pairs of the 5 frames

_frames_cache = {}


def frames():
    """(color uint8 [5,H,W,3], depth uint16 [5,H,W]) of the five example frames."""
    if "f" not in _frames_cache:
        z = np.load(FRAMES, allow_pickle=False)
        _frames_cache["f"] = (z["color"], z["depth"])
    return _frames_cache["f"]


def depth_m(idx, base_down=1):
    """Depth of frame idx in metres, [H, W] (nearest subsampling by base_down)."""
    _, depth = frames()
    d = depth[idx][::base_down, ::base_down].astype(np.float32) / np.float32(5e3)
    return np.clip(d, np.float32(0.5), np.float32(5.0)).astype(np.float32)


def color_float(idx, base_down=1):
    """[3, H, W] RGB in [0, 1] (nearest subsampling; uint8 / 255 in fp32)."""
    color, _ = frames()
    c = color[idx][::base_down, ::base_down].astype(np.float32)
    return (np.moveaxis(c, -1, 0) / np.float32(255.0)).astype(np.float32)


def synthetic_weights(key, shape, gain=1.5):
    """Deterministic stand-in for trained weights (the checkpoints are absent).

    Conv / linear weights: hashed-integer uniform values with variance
    gain^2 / fan_in; biases 0; BatchNorm at identity statistics.  Integer mixing
    and exactly-rounded float32 ops only, so every host produces the same bits."""
    shape = tuple(int(v) for v in shape)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, np.int64)
    if leaf in ("running_mean", "bias"):
        return np.zeros(shape, np.float32)
    if leaf == "running_var":
        return np.ones(shape, np.float32)
    if len(shape) == 1:  # BatchNorm weight
        return np.ones(shape, np.float32)
    if "sigma_conv" in key:  # keep the uncertainty heads off their clamps
        gain = 0.1
    n = int(np.prod(shape))
    fan_in = n // shape[0]
    seed = np.uint64(sum((k + 1) * ord(ch) for k, ch in enumerate(key)))
    h = np.arange(n, dtype=np.uint64) * np.uint64(2654435761) + seed * np.uint64(40503)
    h &= np.uint64(0xFFFFFFFF)
    for sh in (16, 13, 16):  # integer avalanche mix (exact, host-independent)
        h ^= h >> np.uint64(sh)
        h = (h * np.uint64(0x45D9F3B)) & np.uint64(0xFFFFFFFF)
    u = (h >> np.uint64(8)).astype(np.float32) / np.float32(16777216.0) - np.float32(0.5)  # [-0.5, 0.5)
    scale = np.float32(gain * np.sqrt(12.0 / fan_in))
    return (u * scale).astype(np.float32).reshape(shape)


def load_synthetic_weights(net):
    """Fill every state_dict entry of `net` with synthetic_weights (in place); returns net."""
    import torch
    sd = {k: torch.from_numpy(np.asarray(synthetic_weights(k, v.shape))).to(v.dtype)
          for k, v in net.state_dict().items()}
    net.load_state_dict(sd)
    return net
