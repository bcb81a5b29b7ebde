"""Static check of the gfx950 store-data hazard in the SHIPPED library.

Round 4 found a `buffer_store_dwordx4` whose data VGPRs the compiler rewrote two wait states after
issue, before the store had read them: the stored values were torn. The library keeps every drain's
store data live until the next barrier (`keep_vgprs`) and waits for the stores of the element /
record kernels (`store_fence`). This checker disassembles the gfx950 code object inside
libfemasm.so and reports every 12- or 16-byte vector-memory store (buffer / global / flat /
scratch `_dwordx3` / `_dwordx4`) whose data VGPRs an instruction writes within WINDOW instructions
after it (counted in wait states: one per instruction, k + 1 for `s_nop k`), with no
`s_waitcnt vmcnt(0)` or `s_barrier` in between, on any control-flow path: `s_branch` continues at
its target, `s_cbranch_*` at its target and at the next instruction (round 6; the round-5 checker
followed address order only).

Exempt (reported, not failed): scratch stores (the compiler's own register spills), rocPRIM's
kernels (third-party, used by the sparsity build, whose pattern fa_check_pattern validates) and the
HBM probe kernels `k_hbm_*` (measurement only; their stored values are never read).

Usage: python tools/store_hazard.py [libfemasm.so] [--window N]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WINDOW = 16
_STORE = re.compile(r"^(buffer|global|flat|scratch)_store_dwordx([34])$")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def disassemble(so: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fatbin.bin"), os.path.join(td, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", so, os.path.join(td, "x.so")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                       check=True, capture_output=True)
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                           text=True)
        return r.stdout


def vregs(tok: str):
    m = _VREG.match(tok.strip())
    if not m:
        return None
    if m.group(1) is not None:
        v = int(m.group(1))
        return set([v])
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def _operands(rest: str):
    rest = rest.split("//")[0]
    return [t.strip() for t in rest.split(",")] if rest.strip() else []


def dest_vgprs(op: str, ops):
    """VGPRs an instruction writes (its first operand for the forms that have a VGPR destination)."""
    if not ops or op.startswith("s_"):
        return set()
    if op.startswith("ds_"):
        has = op.startswith(("ds_read", "ds_load", "ds_swizzle", "ds_permute", "ds_bpermute", "ds_append",
                             "ds_consume")) or "_rtn" in op
        return (vregs(ops[0]) or set()) if has else set()
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        if "_store" in op:
            return set()
        if "_atomic" in op and not re.search(r"\b(sc0|glc)\b", " ".join(ops)):
            return set()
        return vregs(ops[0]) or set()
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    return vregs(ops[0]) or set()


def store_data(op: str, ops):
    if op.startswith("buffer_"):
        return vregs(ops[0])
    return vregs(ops[1]) if len(ops) > 1 else None


_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")


def parse(text: str):
    """[(fn, op, ops, line, address or None)] in address order."""
    fn = None
    insts = []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            fn = m.group(1)
            continue
        s = line.strip()
        if not s or s.startswith(";") or fn is None or not line.startswith("\t"):
            continue
        parts = s.split(None, 1)
        a = _ADDR.search(s)
        insts.append((fn, parts[0], _operands(parts[1]) if len(parts) > 1 else [], s.split("//")[0].strip(),
                      int(a.group(1), 16) if a else None))
    return insts


def successors(insts, at, j):
    """Indices that can execute after instruction j (control flow: s_branch goes to its target only,
    s_cbranch_* to its target and the next instruction; s_endpgm / s_setpc end the path). A branch
    target is the instruction at address + 4 + 4 * simm16 (SOPP); without addresses (or a target
    outside the function) a branch is followed by the next instruction only."""
    f, op, ops, _, addr = insts[j]
    nxt = [j + 1] if j + 1 < len(insts) and insts[j + 1][0] == f else []
    if op in ("s_endpgm", "s_setpc_b64", "s_endpgm_saved"):
        return []
    if op == "s_branch" or op.startswith("s_cbranch_"):
        tgt = None
        if addr is not None and ops:
            try:
                k = int(ops[0].split()[0], 0)
                k = k - 65536 if k >= 32768 else k
                tgt = at.get((f, addr + 4 + 4 * k))
            except ValueError:
                tgt = None
        if tgt is None:
            return nxt
        return [tgt] if op == "s_branch" else sorted(set(nxt + [tgt]))
    return nxt


def check(text: str, window: int = WINDOW):
    """[(function, store line, writer line, distance)] of every hazard site: from each 12/16-B store,
    every control-flow path (successors()) is walked for `window` wait states; the first write of a
    data VGPR on any path is a site, a path ends at s_barrier, s_endpgm or s_waitcnt vmcnt(0)."""
    sites = []
    insts = parse(text)
    at = {(f, a): k for k, (f, _, _, _, a) in enumerate(insts) if a is not None}
    for i, (f, op, ops, ln, _) in enumerate(insts):
        if not _STORE.match(op):
            continue
        data = store_data(op, ops)
        if not data:
            continue
        best = {}  # instruction index -> fewest wait states it is reached with
        work = [(j, 0) for j in successors(insts, at, i)]
        hit = None
        while work:
            j, ws = work.pop()
            if ws >= window or best.get(j, window) <= ws:
                continue
            best[j] = ws
            f2, op2, ops2, ln2, _ = insts[j]
            if op2 == "s_barrier" or op2 == "s_endpgm" or (op2 == "s_waitcnt" and "vmcnt(0)" in " ".join(ops2)):
                continue
            if dest_vgprs(op2, ops2) & data:
                if hit is None or ws + 1 < hit[1]:
                    hit = (ln2, ws + 1)
                continue
            step = int(ops2[0], 0) + 1 if op2 == "s_nop" and ops2 else 1
            work.extend((k, ws + step) for k in successors(insts, at, j))
        if hit:
            sites.append((f, ln, hit[0], hit[1]))
    return sites


def exempt(fn: str, store: str) -> bool:
    return store.startswith("scratch_") or "rocprim" in fn or fn.startswith("_Z11k_hbm_") or "k_hbm_" in fn


def product_sites(so: str, window: int = WINDOW):
    """The hazard sites that are not exempt (the CPU / GPU tests require none)."""
    return [s for s in check(disassemble(so), window) if not exempt(s[0], s[1])]


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    so = args[0] if args else "fem-libraries_amd/femasm/lib/libfemasm.so"
    w = WINDOW
    if "--window" in sys.argv:
        w = int(sys.argv[sys.argv.index("--window") + 1])
    sites = check(disassemble(so), w)
    names = demangle([s[0] for s in sites]) if sites else []
    bad = 0
    for (f, ln, ln2, d), n in zip(sites, names):
        ex = exempt(f, ln)
        bad += not ex
        print(f"{'exempt' if ex else 'SITE  '} {d:3d}  {n[:90]}\n       {ln}\n       {ln2}")
    print(f"{len(sites)} site(s) within {w} wait states, {bad} not exempt")
    sys.exit(1 if bad else 0)
