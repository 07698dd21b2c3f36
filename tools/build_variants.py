"""Build compile-time variants of libdpft_ic.so under tools/libs/ for A/B runs on the GPU box
(select one with DPFT_LIB=tools/libs/libdpft_<name>.so; tools/kbench.py, bench.py and
tools/variant_pytest.py honour it).

python tools/build_variants.py name=-DFLAG=V[,-DFLAG2=V] ...

The shipped source has no alternative code paths; a variant only moves the numeric operating
point of csrc/dpft_tuning.h (DPFT_SPLIT_MAX_PIXELS, DPFT_SPLIT_MAX_LAUNCH_PIXELS,
DPFT_MARCH_SKEW, DPFT_GRID_WASTE, DPFT_MARCH_MIN_ROWS, DPFT_RING_Q, DPFT_MM_GRID, DPFT_MM_LOADS, DPFT_PROBE_GRID, DPFT_PROBE_DEPTH).
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deep_prob_feature_track_amd import build as B  # noqa: E402


def one(spec):
    name, flags = spec.split("=", 1)
    out = os.path.join(ROOT, "tools", "libs", f"libdpft_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{B.INC}", f"-I{os.path.dirname(B.SRC)}",
           *[f for f in flags.split(",") if f], "-o", out, B.SRC]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
