"""Measurement variants of the HIP library without measurement code in the product source.

Each variant is a list of (old, new) text substitutions applied to a copy of
fem-libraries_amd/csrc/femasm.hip; the copy is compiled to abl/libfemasm_<name>.so (bench with
FEMASM_LIB=abl/libfemasm_<name>.so). Timing-only variants compute wrong matrices.

usage: python tools/r4/variant.py NAME [NAME ...]      (build in parallel)
       python tools/r4/variant.py --list
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "fem-libraries_amd", "csrc", "femasm.hip")
OUT = os.path.join(ROOT, "abl")

# k_gather_lin (FIX = fixed-point / FP64 both): ablations keep the block arithmetic live
V = {
    # no LDS accumulate (the values feed a never-true store so the arithmetic stays)
    "lin_noadd": [(
        "                atomicAdd(reinterpret_cast<unsigned long long*>(ap + i * GD + kk), q);",
        "                if (q == 0x123456789ull) ap[i * GD + kk] = 1.0;"), (
        "              for (int kk = 0; kk < GD; ++kk) atomicAdd(ap + i * GD + kk, G[i][kk]);",
        "              for (int kk = 0; kk < GD; ++kk) if (G[i][kk] == 1.2345e-300) ap[i * GD + kk] = 1.0;")],
    # no chunk stores to HBM (every store offset past the range)
    "lin_nostore": [(
        "NT * u < lim ? base : OOB, 16 * NT * u,", "OOB, 16 * NT * u,"), (
        "(tid == 0 && h) ? 0 : OOB, 0, NTS);", "OOB, 0, NTS);"), (
        "(tid == 1 && ((nv - h) & 1)) ? 8 * (nv - 1) : OOB, 0, NTS);", "OOB, 0, NTS);")],
    # no accumulator zeroing in the drain
    "lin_nozero": [(
        "    for (int u = 0; u < SW; ++u)\n      if (tid + NT * u < np) acc2[h + tid + NT * u] = dv2{0.0, 0.0};",
        "    for (int u = 0; u < SW; ++u)\n      if (tid + NT * u < np && hv == 1.2345e-300) acc2[h + tid + NT * u] = dv2{0.0, 0.0};")],
    # no reference-tensor table reads (constants instead)
    "lin_notab": [(
        "          for (int e = 0; e < BS2; ++e) Bn[e] = Ah0[b1 * BS2 + e];",
        "          for (int e = 0; e < BS2; ++e) Bn[e] = 0.1 * e + b1;"), (
        "        for (int e = 0; e < BS2; ++e) Bn[e] = Ah0[b * BS2 + e];",
        "        for (int e = 0; e < BS2; ++e) Bn[e] = 0.2 * e + b;")],
}


def build(name):
    src = open(SRC).read()
    for old, new in V[name]:
        if old not in src:
            raise SystemExit(f"variant {name}: pattern not found:\n{old}")
        src = src.replace(old, new)
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(ROOT, "fem-libraries_amd", "csrc", f"_variant_{name}.hip")
    open(path, "w").write(src)
    return subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                             "-munsafe-fp-atomics", "-o", os.path.join(OUT, f"libfemasm_{name}.so"), path]), path


if __name__ == "__main__":
    if sys.argv[1:] == ["--list"]:
        print("\n".join(V))
        raise SystemExit(0)
    procs = [build(n) for n in sys.argv[1:]]
    rc = 0
    for p, path in procs:
        rc |= p.wait()
        os.remove(path)
    raise SystemExit(rc)
