"""Build compile-time variants of libdpft_ic.so under tools/libs/ for A/B runs on the GPU box
(select one with DPFT_LIB=tools/libs/libdpft_<name>.so; tools/kbench.py, bench.py and
tools/variant_pytest.py honour it).

python tools/build_variants.py name=-DFLAG=V[,-DFLAG2=V] ...
python tools/build_variants.py name=@path/to/experiment.hip[:-DFLAG=V,...] ...   (an experimental copy of the source)

The shipped source has no alternative code paths; a variant only moves the numeric operating
point of csrc/dpft_tuning.h (DPFT_SPLIT_MAX_PIXELS, DPFT_SPLIT_MAX_LAUNCH_PIXELS,
DPFT_MARCH_SKEW, DPFT_GRID_WASTE, DPFT_MARCH_MIN_ROWS, DPFT_RING_Q, DPFT_ICP_SUB, DPFT_MM_GRID, DPFT_MM_LOADS, DPFT_PROBE_GRID, DPFT_PROBE_DEPTH).
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
    src = B.SRC
    if flags.startswith("@"):  # an experimental copy of the source (A/B of code changes)
        src, _, flags = flags[1:].partition(":")
    out = os.path.join(ROOT, "tools", "libs", f"libdpft_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{B.INC}", f"-I{os.path.dirname(B.SRC)}",
           "-Rpass-analysis=kernel-resource-usage", *[f for f in flags.split(",") if f], "-o", out, src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        raise subprocess.CalledProcessError(r.returncode, cmd)
    res = B.kernel_resources(r.stderr)
    for k, v in res.items():
        if k.startswith("void (anonymous namespace)::ic_reduce_kernel<32, true, true, 0, true>"):
            print(f"{name}: L0 kernel {v.get('VGPRs')} VGPRs, {v.get('AGPRs', 0)} AGPRs, "
                  f"{v.get('Occupancy [waves/SIMD]')} waves/SIMD, spill {v.get('VGPRs Spill', 0)}", flush=True)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
