"""Audit a kernel's machine code for reads of registers whose vector-memory load has not
been waited for -- the check that hand-counted `s_waitcnt vmcnt(N)` after inline-asm loads
needs (hipcc does not count those loads: cdna_hip_programming.md §5.7).

    python tools/vmcnt_check.py LIB.so [kernel-substring]

Dataflow over the kernel's control-flow graph: the state is the ordered list of in-flight
loads (their destination registers, oldest first); a load appends, `s_waitcnt vmcnt(N)`
keeps the N youngest, a join keeps per position (counted from the youngest) the union of
the predecessors' registers (conservative).  Every instruction that reads or writes a
register of an in-flight load is reported.  Stores count in vmcnt too (no destination).
"""
import re
import subprocess
import sys
import tempfile
import os

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(so, kernel_sub):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so, os.path.join(d, "x.so")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                             text=True).stdout
    out, cur, name = [], None, None
    for line in txt.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            if cur is not None and kernel_sub in name:
                return name, cur
            name, cur = m.group(2), []
            continue
        m = re.match(r"\s+(\S+)(.*?)//\s*([0-9A-F]+):", line)
        if m and cur is not None:
            tgt = re.search(r"<\S+\+0x([0-9a-f]+)>", line)
            cur.append((int(m.group(3), 16), m.group(1), m.group(2).strip(), int(tgt.group(1), 16) if tgt else None))
    if cur is not None and kernel_sub in (name or ""):
        return name, cur
    raise SystemExit(f"no kernel matching {kernel_sub!r}")


def regs(text):
    """Registers named in an operand string -> set of 'v12' / 's4' / 'a3'."""
    out = set()
    for kind, a, b in re.findall(r"\b([vsa])\[(\d+):(\d+)\]", text):
        out.update(f"{kind}{i}" for i in range(int(a), int(b) + 1))
    text = re.sub(r"\b[vsa]\[\d+:\d+\]", "", text)
    out.update(re.findall(r"\b([vsa]\d+)\b", text))
    return out


def classify(op, args):
    """(is_vm_load, is_vm_store, dest regs, source regs)."""
    parts = [p.strip() for p in re.split(r",(?![^\[]*\])", args) if p.strip()]
    if op.startswith(("buffer_load", "global_load", "flat_load", "scratch_load")):
        lds = " lds" in args
        return True, False, (set() if lds else regs(parts[0])), regs(",".join(parts[0 if lds else 1:]))
    if op.startswith(("buffer_store", "global_store", "flat_store", "scratch_store", "buffer_atomic", "global_atomic")):
        return False, True, set(), regs(args)
    if op.startswith(("s_waitcnt", "s_nop", "s_branch", "s_cbranch", "s_endpgm", "s_barrier", "s_setprio", "s_sleep")):
        return False, False, set(), set()
    if not parts:
        return False, False, set(), set()
    if op.startswith(("ds_write", "ds_store")) or op.startswith("s_store"):
        return False, False, set(), regs(args)
    return False, False, regs(parts[0]), regs(",".join(parts[1:]))


def merge(a, b):
    n = max(len(a), len(b))
    out = []
    for i in range(n, 0, -1):
        s = set()
        if i <= len(a):
            s |= a[-i]
        if i <= len(b):
            s |= b[-i]
        out.append(frozenset(s))
    return out


def main():
    so = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "ic_reduce_kernelILi32ELb1ELb1ELi0ELb1E"
    name, ins = disasm(so, sub)
    base = ins[0][0]
    idx = {a: i for i, (a, *_rest) in enumerate(ins)}
    # successors
    succ = []
    for i, (a, op, args, tgt) in enumerate(ins):
        s = []
        if op.startswith("s_cbranch") or op == "s_branch":
            if tgt is not None and tgt + base in idx:
                s.append(idx[tgt + base])
            if op.startswith("s_cbranch") and i + 1 < len(ins):
                s.append(i + 1)
        elif op == "s_endpgm":
            pass
        elif i + 1 < len(ins):
            s.append(i + 1)
        succ.append(s)
    state = {0: []}
    work = [0]
    bad = {}
    seen_in = {}
    while work:
        i = work.pop()
        st = list(state[i])
        a, op, args, _ = ins[i]
        load, store, dst, src = classify(op, args)
        if op.startswith("s_waitcnt"):
            m = re.search(r"vmcnt\((\d+)\)", args)
            if m:
                st = st[len(st) - int(m.group(1)):] if int(m.group(1)) < len(st) else st
            elif re.fullmatch(r"0", args.strip()) or args.strip() == "0x0":
                st = []
        else:
            inflight = set().union(*st) if st else set()
            hit = (src | (dst if not load else set())) & inflight
            if hit:
                bad.setdefault(a - base, (op, args, sorted(hit)))
            if load:
                st.append(frozenset(dst))
            elif store:
                st.append(frozenset())
        for j in succ[i]:
            new = merge(state[j], st) if j in state else st
            if j not in state or [set(x) for x in new] != [set(x) for x in state[j]]:
                if len(new) > 64:  # vmcnt saturates at 63 outstanding
                    new = new[-64:]
                state[j] = new
                if j not in work:
                    work.append(j)
    print(f"{name}: {len(ins)} instructions, {len(bad)} read(s) / write(s) of in-flight load registers")
    for off, (op, args, hit) in sorted(bad.items())[:60]:
        print(f"  +0x{off:x}: {op} {args}    in flight: {' '.join(hit[:8])}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
