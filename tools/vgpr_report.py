"""Per-kernel register / LDS / scratch report of libdpft_ic.so (compiler view).

python tools/vgpr_report.py [extra hipcc flags...]

Compiles the library once more with -Rpass-analysis=kernel-resource-usage and
prints one line per kernel instantiation: VGPRs (+AGPRs), the waves per SIMD those
registers allow (MI355X_MICROARCH.md, register-file table), LDS bytes, scratch.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deep_prob_feature_track_amd import build as B  # noqa: E402


def waves_per_simd(regs):
    alloc = (regs + 7) // 8 * 8
    return min(8, 512 // max(alloc, 1))


def report(extra=()):
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-c", f"-I{B.INC}",
           "-Rpass-analysis=kernel-resource-usage", *extra, "-o", os.devnull, B.SRC]
    out = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2)
        if key == "Function Name":
            cur = {"name": subprocess.run(["c++filt", val], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[key] = int(val)
    return rows


if __name__ == "__main__":
    for r in report(sys.argv[1:]):
        regs = r.get("VGPRs", 0) + r.get("AGPRs", 0)
        name = r["name"].replace("(anonymous namespace)::", "")
        print(f"{regs:4d} regs  {r.get('Occupancy [waves/SIMD]', waves_per_simd(regs))} waves/SIMD  "
              f"LDS {r.get('LDS Size [bytes/block]', 0):6d}  spill {r.get('VGPRs Spill', 0):3d}  "
              f"scratch {r.get('ScratchSize [bytes/lane]', 0):4d}  {name}")
