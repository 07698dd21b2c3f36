"""Build libdpft_ic.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

The compile also emits the compiler's per-kernel resource report
(-Rpass-analysis=kernel-resource-usage); the build fails if a hot kernel lost its
occupancy -- the channel-quad marching kernels sit a few VGPRs under the 256 that
allow 2 waves per SIMD (one register more halves their residency and, measured,
costs ~70 % on the level-0 launch), and nothing at run time would notice: the grid
is sized from the occupancy query, so results stay right and only speed drops.
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "dpft_ic.hip")
OUT = os.path.join(HERE, "libdpft_ic.so")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DPFT_OFFLOAD_ARCH", "gfx950")

# kernel-name pattern -> minimum waves per SIMD, no register spills
OCCUPANCY_FLOOR = {
    r"^void \(anonymous namespace\)::ic_reduce_kernel<(16|32), true, (true|false), [012], true>": 2,
    r"^void \(anonymous namespace\)::ic_split_kernel<": 4,
}


def kernel_resources(stderr):
    """Parse -Rpass-analysis=kernel-resource-usage remarks -> {demangled name: {field: int}}."""
    out, cur = {}, None
    for line in stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|"
                      r"ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2)
        if key == "Function Name":
            name = subprocess.run(["c++filt", val], capture_output=True, text=True).stdout.strip() or val
            cur = out.setdefault(name, {})
        elif cur is not None:
            cur[key] = int(val)
    return out


def check_occupancy(res):
    bad = []
    for pat in OCCUPANCY_FLOOR:
        if not any(re.search(pat, name) for name in res):
            bad.append(f"no kernel matches {pat!r} (renamed? the guard would check nothing)")
    for name, r in res.items():
        for pat, floor in OCCUPANCY_FLOOR.items():
            if re.search(pat, name):
                occ, spill = r.get("Occupancy [waves/SIMD]", 0), r.get("VGPRs Spill", 0)
                if occ < floor or spill:
                    bad.append(f"{name}: {r.get('VGPRs')} VGPRs, {occ} waves/SIMD (floor {floor}), {spill} spilled")
    if bad:
        raise RuntimeError("occupancy regression:\n  " + "\n  ".join(bad))


LLVM_BIN = "/opt/rocm/lib/llvm/bin"
ISA_OUT = os.path.join(HERE, "libdpft_ic.isa.json")
# the level-0/1 marching kernel of the bench (C = 32, one sigma plane, remove_tru_sigma, U_IC, channel quads)
L0_KERNEL = "_ZN12_GLOBAL__N_116ic_reduce_kernelILi32ELb1ELb1ELi0ELb1EEEvNS_10IterParamsE"
# the combine_ICP pass that runs in front of it in a cfg5 (bench.py --icp) iteration
ICP_KERNEL = "_ZN12_GLOBAL__N_118icp_records_kernelENS_10IterParamsEPf"


def isa_hashes(so_path=OUT):
    """{mangled kernel name: SHA-256 of its gfx950 instruction text} from the library's
    device code object (llvm-objdump; addresses and encodings dropped, branch offsets are
    relative).  A per-launch PMC measurement names the hash of the kernel it measured, so
    it stays valid while that kernel's machine code is unchanged, whatever else changes
    in the source file."""
    import hashlib
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", so_path, os.path.join(d, "x.so")],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM_BIN, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                        f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}"], check=True, capture_output=True)
        dis = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                             check=True, capture_output=True, text=True).stdout
    out, name, body = {}, None, []
    for line in dis.splitlines() + ["<end>:"]:
        m = re.match(r"^<(\S+)>:$", line)
        if m:
            if name is not None:
                out[name] = hashlib.sha256("\n".join(body).encode()).hexdigest()
            name, body = m.group(1), []
        elif name is not None and line.strip():
            body.append(line.split("//")[0].strip())
    out.pop("end", None)
    return out


def write_isa_hashes():
    """Best effort: the hashes only let bench.py match a committed PMC measurement to the
    kernel built here; a missing LLVM tool must not make the library unusable."""
    import json
    import warnings
    try:
        json.dump(isa_hashes(OUT), open(ISA_OUT, "w"), indent=0, sort_keys=True)
    except (OSError, subprocess.CalledProcessError) as e:
        warnings.warn(f"ISA hashes not written ({e}); bench.py will report roofline.traffic = null")


def build(force=False, verbose=False):
    deps = [SRC, os.path.join(HERE, "csrc", "dpft_tuning.h"), os.path.join(INC, "dpft_ic.h"), __file__]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        if not os.path.exists(ISA_OUT) or os.path.getmtime(ISA_OUT) < os.path.getmtime(OUT):
            write_isa_hashes()
        return OUT
    # -Wshadow: a local that shadows a buffer resource of the marching body compiles to a
    # silently wrong kernel (round 2: `rs0`, JtJ off by 1e8); every warning is an error
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{INC}",
           "-Wall", "-Wextra", "-Wshadow", "-Werror",
           "-Rpass-analysis=kernel-resource-usage", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        raise subprocess.CalledProcessError(r.returncode, cmd)
    check_occupancy(kernel_resources(r.stderr))
    os.replace(OUT + ".tmp", OUT)
    write_isa_hashes()
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
