"""Per-kernel VGPR / AGPR / scratch / occupancy from the library's gfx950 assembly
(`make -C fem-libraries_amd/csrc asm`). Usage: python tools/kernel_resources.py [pattern]"""
import re
import subprocess
import sys

ASM = "fem-libraries_amd/csrc/femasm-gfx950.s"


def kernels(path=ASM):
    name = None
    out = {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            name = m.group(1)
            continue
        m = re.match(r"^; (NumVgprs|NumAgprs|ScratchSize|Occupancy|NumSgprs): (\d+)", line)
        if m and name:
            out.setdefault(name, {})[m.group(1)] = int(m.group(2))
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


if __name__ == "__main__":
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    ks = kernels()
    names = list(ks)
    for n, d in zip(names, demangle(names)):
        if pat in d:
            r = ks[n]
            print(f"{r.get('NumVgprs', 0):4d} v {r.get('NumAgprs', 0):3d} a {r.get('ScratchSize', 0):5d} scr occ {r.get('Occupancy', 0)}  {d[:110]}")
