"""Static audit of the scan kernels' gfx950 assembly for the hazards hipcc does
not pad around inline-asm MFMAs (cdna_hip_programming.md §5.7 item 2).

The LUT16 scan issues v_smfmac_i32_32x32x64_i8 as an asm statement (its B
operand lives in AGPRs), so the compiler neither knows it is an XDL op nor
inserts its wait states.  This script compiles smx_kernels.hip to assembly
and checks every lut16_scan_kernel instantiation:

  1. VALU write -> smfmac read: no VALU instruction in the 2 issue slots
     before an smfmac writes a register the smfmac reads (A, B, index, C).
  2. smfmac D -> other reader: at least 18 wait states (instructions, an
     s_nop N counting N+1) between an smfmac and any instruction other than
     an smfmac taking the same accumulator whole as C that reads or writes
     its D registers.
  3. no v_accvgpr_read/write outside the asm blocks (the B fragments must
     stay in AGPRs, not be copied per use), no VGPR spills, no scratch.

    python tools/audit_isa.py [path/to/kernels.s]
Exit status 1 on any finding.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XDL_STATES = 18
PATTERN = os.environ.get("AUDIT_KERNEL", "lut16_scan")

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+))\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((kind, r))
    return out


def split_operands(line):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]
    return parts[0], ops


def compile_asm():
    out = "/tmp/smx_kernels_audit.s"
    cmd = [os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"),
           "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "--cuda-device-only", "-S", "-o", out,
           os.path.join(ROOT, "scann_amd", "csrc", "smx_kernels.hip")]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return out


def kernels(path):
    """(name, [instruction lines], metadata lines) of each scan kernel."""
    text = open(path).read().split("\n")
    found = []
    i = 0
    while i < len(text):
        line = text[i]
        m = re.match(r"^(_Z\S*" + PATTERN + r"\S*):", line)
        if m:
            name = m.group(1)
            body = []
            i += 1
            while i < len(text) and not text[i].startswith(".Lfunc_end"):
                body.append(text[i])
                i += 1
            meta = [t for t in text if t.startswith(f"\t.set {name}.")]
            found.append((name, body, meta))
        i += 1
    return found


def audit(name, body, meta):
    issues = []
    for t in meta:
        if (".private_seg_size" in t and not t.rstrip().endswith(" 0")):
            issues.append(f"scratch: {t.strip()}")
    insts = []   # (text, in_asm)
    in_asm = False
    for raw in body:
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(";") or s.endswith(":") or s.startswith("."):
            continue
        insts.append((s, in_asm))
    for k, (s, in_asm) in enumerate(insts):
        op, ops = split_operands(s)
        if op.startswith("v_accvgpr") and not in_asm:
            issues.append(f"compiler AGPR copy: {s}")
        if not op.startswith("v_smfmac"):
            continue
        dst = regs(ops[0])
        srcs = set().union(*(regs(o) for o in ops[1:])) | dst
        # 1. VALU write -> smfmac read within 2 slots
        for j in range(max(0, k - 2), k):
            pop, pops = split_operands(insts[j][0])
            if pop.startswith("v_") and not pop.startswith(("v_smfmac", "v_mfma", "v_readfirstlane",
                                                             "v_cmp")) and pops:
                if regs(pops[0]) & srcs:
                    issues.append(f"VALU->smfmac within 2 slots: {insts[j][0]}  ->  {s}")
        # 2. D -> reader within XDL_STATES
        states = 0
        for j in range(k + 1, len(insts)):
            t, _ = insts[j]
            top, tops = split_operands(t)
            if top.startswith("s_nop"):
                states += int(tops[0], 0) + 1 if tops else 1
            elif top.startswith("v_smfmac") and regs(tops[0]) == dst:
                break   # the chain's next MFMA takes it whole as C
            else:
                touched = set().union(*(regs(o) for o in tops)) if tops else set()
                if touched & dst and states < XDL_STATES:
                    issues.append(f"smfmac D read after {states} states: {s}  ->  {t}")
                    break
                states += 1
            if states >= XDL_STATES:
                break
            if top.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
                break   # (straight-line check only)
    return issues


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    bad = 0
    ks = kernels(path)
    for name, body, meta in ks:
        issues = audit(name, body, meta)
        short = re.sub(r"^_ZN3smx12_GLOBAL__N_1", "", name)
        print(f"{short}: {'ok' if not issues else f'{len(issues)} findings'}")
        for i in issues[:20]:
            print("   ", i)
        bad += len(issues)
    if not ks:
        print("no scan kernels found")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
