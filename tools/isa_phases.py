"""Static ISA accounting of wave_kernel<N, KS> per phase: compiles csrc/mpcqp_wave.hip for one
horizon with -DMPCQP_ISA_MARKS (WV_MARK ids become assembly comments) and counts, between
consecutive marks in program order, VALU / fp64 FMA / DPP / accvgpr moves / LDS / scratch ops.

  python tools/isa_phases.py [--n 10] [--ks 1] [--defs -DFOO] [--keep /tmp/w.s]
"""
import argparse
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "go1-qp-mpc-controller_amd", "csrc", "mpcqp_wave.hip")


def compile_asm(n, defs, out, src=SRC):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-strict-aliasing",
           "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-DMPCQP_ISA_MARKS", f"-DMPCQP_WAVE_FOR_EACH_N(X)=X({n})", "--cuda-device-only", "-S", src,
           "-o", out] + defs
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def classify(ins):
    op = ins.split()[0]
    c = {}
    if op.startswith("v_"):
        if op.startswith("v_accvgpr"):
            c["acc"] = 1
        else:
            c["valu"] = 1
            if "f64" in op and ("fma" in op or "fmac" in op):
                c["fma64"] = 1
            if "_dpp" in op or "row_" in ins or "quad_perm" in ins:
                c["dpp"] = 1
    elif op.startswith("ds_"):
        c["lds"] = 1
    elif op.startswith("scratch_"):
        c["scratch"] = 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        c["vmem"] = 1
    elif op.startswith("s_"):
        c["salu"] = 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--ks", type=int, default=1)
    ap.add_argument("--defs", nargs="*", default=[])
    ap.add_argument("--keep", default=None)
    ap.add_argument("--src", default=SRC)
    a = ap.parse_args()
    out = a.keep or os.path.join(tempfile.mkdtemp(), "w.s")
    compile_asm(a.n, a.defs, out, a.src)
    s = open(out).read()
    m = re.search(r"^(_ZN5mpcqp2wv11wave_kernelILi%dELi%dEE\S*):" % (a.n, a.ks), s, re.M)
    body = s[m.end(): s.index(".Lfunc_end", m.end())].splitlines()
    keys = ["valu", "fma64", "dpp", "acc", "lds", "scratch", "vmem", "salu"]
    seg, tot, rows = "entry", {k: 0 for k in keys}, []
    cur = {k: 0 for k in keys}
    for line in body:
        t = line.strip()
        mm = re.match(r";WV_MARK (\d+)", t)
        if mm:
            rows.append((seg, cur))
            seg, cur = "mark " + mm.group(1), {k: 0 for k in keys}
            continue
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        for k, v in classify(t).items():
            cur[k] += v
            tot[k] += v
    rows.append((seg, cur))
    print("%-10s" % "segment" + "".join("%8s" % k for k in keys))
    for seg, c in rows:
        print("%-10s" % seg + "".join("%8d" % c[k] for k in keys))
    print("%-10s" % "total" + "".join("%8d" % tot[k] for k in keys))


if __name__ == "__main__":
    main()
