#!/usr/bin/env python3
"""Static hazard check of the wave kernels' gfx950 ISA (compiled code + inline asm together).

The solve kernels issue hand-written DPP / permlane / LDS instructions from inline asm, which the
compiler's hazard recognizer and waitcnt pass do not see into.  This tool reads the assembly of
csrc/mpcqp_wave.hip (the inline asm is printed verbatim between ;;#ASMSTART / ;;#ASMEND) and checks,
in program order, the hazards that can corrupt a value silently:

  dpp        a DPP instruction whose DPP source (src0) was written by a VALU instruction fewer than
             2 wait states before (CDNA3/4 ISA, "manually inserted wait states": VALU write VGPR ->
             VALU DPP read of it), or after a VALU write of EXEC (v_cmpx) fewer than 5 before;
  permlane   v_permlane16/32_swap reading a VGPR a VALU wrote in the previous wait state;
  trans      a VALU reading the result of a transcendental (v_rcp/v_sqrt/v_rsq/... ) with no
             instruction in between (TransUseHazard);
  untracked  a VGPR loaded by an inline-asm ds_read (invisible to the waitcnt pass) that any
             instruction reads or writes before an s_waitcnt lgkmcnt that has retired that load
             (LDS returns in order: a wait for lgkmcnt(k) retires every load issued more than k
             LDS instructions before it).  A copy, spill or reuse of such a register before the
             wait reads stale data or is overwritten when the load lands (the suspected
             mechanism behind the round-3 `mu` clobbers).

Wait states: every instruction issued counts 1, `s_nop N` counts N + 1.  The scan is linear inside
each kernel; a label resets nothing (conservative for fall-through, approximate across branches).

  python tools/isa_hazards.py [--asm /tmp/wave.s] [--n 10] [--kernels wave_kernelILi10ELi1E ...]
Exit status 1 if any hazard is found (the build's static check).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "go1-qp-mpc-controller_amd", "csrc", "mpcqp_wave.hip")

REG = re.compile(r"\b([vas])(\d+)\b|\b([vas])\[(\d+):(\d+)\]")
DPP_CTRL = ("row_newbcast", "quad_perm", "row_shl", "row_shr", "row_ror", "row_bcast", "row_share",
            "row_xmask", "row_mirror", "row_half_mirror", "wave_shl", "wave_shr", "wave_rol", "wave_ror")
TRANS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_", "v_rcp_iflag")


def regs(text):
    out = []
    for m in REG.finditer(text):
        if m.group(1):
            out.append((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.extend((k, i) for i in range(a, b + 1))
    return out


def split_operands(rest):
    parts, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


class Ins:
    __slots__ = ("op", "ops", "text", "asm", "line", "defs", "uses", "ws")

    def __init__(self, text, asm, line):
        self.text = text
        self.asm = asm
        self.line = line
        self.ws = 1
        t = text.split(";")[0].strip()
        m = re.match(r"s_nop\s+(\w+)", t)
        if m:
            self.ws = int(m.group(1), 0) + 1
        self.op = t.split()[0] if t else ""
        rest = t[len(self.op):].strip()
        self.ops = split_operands(rest) if rest else []
        self.defs, self.uses = [], []
        op = self.op
        if not op:
            return
        writes_first = (op.startswith("v_") and not op.startswith(("v_cmp_", "v_cmpx_"))
                        or op.startswith(("ds_read", "ds_load", "global_load", "buffer_load", "flat_load",
                                          "scratch_load", "s_load", "s_buffer_load", "s_mov", "s_and", "s_or",
                                          "s_xor", "s_andn2", "s_orn2", "s_cselect", "s_add", "s_sub", "s_mul",
                                          "s_lshl", "s_lshr", "s_bfe", "s_getreg", "s_memtime", "s_memrealtime",
                                          "v_readlane", "v_readfirstlane")))
        if op.startswith("v_permlane") and "swap" in op:  # both operands are read and written
            for o in self.ops[:2]:
                self.defs += regs(o)
                self.uses += regs(o)
            return
        if writes_first and self.ops:
            self.defs = regs(self.ops[0])
            srcs = self.ops[1:]
        else:
            srcs = self.ops
        for o in srcs:
            if any(o.startswith(c) for c in DPP_CTRL) or o.startswith(("offset", "row_mask", "bank_mask")):
                continue
            self.uses += regs(o)
        if op.startswith(("v_fmac", "v_mac")) and self.ops:  # the accumulator is read too
            self.uses += regs(self.ops[0])

    @property
    def is_valu(self):
        return self.op.startswith("v_") and not self.op.startswith("v_accvgpr") or self.op.startswith("v_accvgpr")

    @property
    def is_dpp(self):
        return "_dpp" in self.op or any(c in self.text for c in DPP_CTRL)

    @property
    def writes_exec(self):  # by a VALU (v_cmpx): SALU writes of EXEC need no DPP wait states
        return self.op.startswith("v_cmpx") or (self.op.startswith("v_") and bool(self.ops)
                                                 and self.ops[0].startswith("exec"))

    @property
    def is_trans(self):
        return self.op.startswith(TRANS)

    @property
    def is_lds(self):
        return self.op.startswith("ds_")


def kernels(asm_text, names):
    for nm in names:
        m = re.search(r"^(_ZN5mpcqp2wv\d+%s\S*):" % re.escape(nm), asm_text, re.M)
        if not m:
            raise SystemExit(f"kernel {nm} not found")
        end = asm_text.index(".Lfunc_end", m.end())
        yield nm, asm_text[m.end():end].splitlines(), asm_text[:m.end()].count("\n") + 1


def check(lines, first_line):
    ins, in_asm = [], False
    for k, raw in enumerate(lines):
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        # an asm block may hold several instructions separated by newlines already (verbatim)
        ins.append(Ins(s, in_asm, first_line + k))
    problems = []
    pending = []  # untracked LDS loads: [defs set, lds index, line, text]
    lds_count = 0
    for i, x in enumerate(ins):
        # ---- dpp / permlane / trans hazards: look back over the previous instructions
        def since_def(regset, pred, limit):
            w = 0
            for j in range(i - 1, max(-1, i - 12), -1):
                y = ins[j]
                if pred(y) and set(y.defs) & regset:
                    return w
                w += y.ws
                if w >= limit:
                    return w
            return limit
        if x.is_dpp and x.ops and len(x.ops) > 1 and x.op.startswith("v_"):
            src0 = set(regs(x.ops[1]))
            w = since_def(src0, lambda y: y.op.startswith("v_"), 2)
            if w < 2:
                problems.append(("dpp", x.line, f"{x.text}  <- DPP src written {w} wait states before"))
            w = 0
            for j in range(i - 1, max(-1, i - 12), -1):
                if ins[j].writes_exec:
                    if w < 5:
                        problems.append(("dpp-exec", x.line, f"{x.text}  <- EXEC written {w} wait states before"))
                    break
                w += ins[j].ws
                if w >= 5:
                    break
        if x.op.startswith("v_permlane") and "swap" in x.op:
            w = since_def(set(x.uses), lambda y: y.op.startswith("v_") and not y.op.startswith("v_permlane"), 1)
            if w < 1:
                problems.append(("permlane", x.line, f"{x.text}  <- operand written by VALU just before"))
        if x.op.startswith("v_") and i > 0 and ins[i - 1].is_trans and set(ins[i - 1].defs) & set(x.uses):
            problems.append(("trans", x.line, f"{x.text}  <- reads {ins[i - 1].op} result with no wait state"))
        # ---- untracked LDS loads
        m = re.match(r"s_waitcnt\b.*lgkmcnt\((\d+)\)", x.text)
        if x.op == "s_waitcnt" and ("lgkmcnt" in x.text or x.text.strip() == "s_waitcnt 0"):
            k = int(m.group(1)) if m else 0
            pending = [p for p in pending if p[1] >= lds_count - k]
        elif x.op in ("s_endpgm", "s_setpc_b64"):
            pending = []
        else:
            touched = set(x.defs) | set(x.uses)
            for p in pending:
                hit = p[0] & touched
                if hit:
                    problems.append(("untracked", x.line,
                                     f"{x.text}  <- touches {sorted(hit)[:4]} of the asm load at line {p[2]} "
                                     f"({p[3]}) before its s_waitcnt"))
            if x.is_lds:
                if x.asm and x.op.startswith(("ds_read", "ds_load")):
                    pending.append([set(x.defs), lds_count, x.line, x.text])
                lds_count += 1
    return problems, len(ins)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=None, help="assembly file (default: compile csrc/mpcqp_wave.hip)")
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--all", action="store_true",
                    help="the product build's every horizon (N = 1..20: wave_kernel<N, 1> for N <= 10, "
                         "wave_kernel<N, 0> and scale_kernel<N> for all) from one compile")
    ap.add_argument("--defs", nargs="*", default=[])
    ap.add_argument("--kernels", nargs="*", default=None)
    ap.add_argument("--max-report", type=int, default=40)
    a = ap.parse_args()
    path = a.asm
    if path is None:
        path = os.path.join(tempfile.mkdtemp(), "w.s")
        nflag = [] if a.all else [f"-DMPCQP_WAVE_FOR_EACH_N(X)=X({a.n})"]
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-strict-aliasing",
                        "-mllvm", "-amdgpu-mfma-vgpr-form"]
                       + nflag + ["--cuda-device-only", "-S", SRC, "-o", path] + a.defs
                       + os.environ.get("ISA_EXTRA_FLAGS", "").split(),
                       check=True, stderr=subprocess.DEVNULL)
    text = open(path).read()
    if a.kernels:
        names = a.kernels
    elif a.all:
        names = [f"wave_kernelILi{n}ELi1E" for n in range(1, 11)] + [f"wave_kernelILi{n}ELi0E" for n in range(1, 21)] \
            + [f"scale_kernelILi{n}E" for n in range(1, 21)]
    else:
        names = ([f"wave_kernelILi{a.n}ELi1E"] if a.n <= 10 else []) + [f"wave_kernelILi{a.n}ELi0E", f"scale_kernelILi{a.n}E"]
    total = 0
    seen = 0
    for nm, lines, l0 in kernels(text, names):
        seen += 1
        probs, nins = check(lines, l0)
        kinds = {}
        for kd, _, _ in probs:
            kinds[kd] = kinds.get(kd, 0) + 1
        print(f"{nm}: {nins} instructions, hazards {kinds if kinds else 'none'}")
        for kd, ln, msg in probs[:a.max_report]:
            print(f"  [{kd}] line {ln}: {msg}")
        total += len(probs)
    if seen < len(names):
        print(f"only {seen} of the {len(names)} kernels found in the assembly")
        return 1
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
