#!/usr/bin/env python3
"""Static check: does any inline-asm block read a VGPR that an MFMA wrote too few
wait states earlier?

The compiler's hazard recognizer inserts the wait states CDNA needs between an
MFMA writing a VGPR and a VALU reading it (the hardware does not interlock), but
it cannot see inside inline asm.  mv_common.h's cvt_pk_bf16 used to be an
inline-asm v_cvt_pk_bf16_f32: where the compiler kept MFMA accumulators in
VGPRs (mv_stem.hip's stem_fwd_kernel at __launch_bounds__(256, 2)) it read the
accumulators zero wait states after the MFMA and produced garbage (NaN).

Usage: python scripts/check_mfma_asm_hazards.py [files.hip ...]
Compiles each source for gfx950 to assembly (device only) and scans every
function linearly (branches ignored: conservative for straight-line epilogues).
Exit status 1 if a hazard is found.
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
# XDL (MFMA) VGPR write -> VALU read wait states on CDNA3/4: 2-pass 5, 4-pass 7,
# 8-pass 11, 16-pass 19; use the 16-pass bound for 32x32 shapes, 8-pass otherwise
NEED_16x16 = 11
NEED_32x32 = 19

_LABEL = re.compile(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$")
_REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _regs(operand_text: str):
    out = set()
    for m in _REG.finditer(operand_text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan_asm(text: str):
    """[(function, line, asm text, register, wait states seen, needed)]"""
    problems = []
    fn = None
    pending = {}          # vgpr -> (wait states elapsed, needed)
    in_asm = False
    for ln, raw in enumerate(text.splitlines(), 1):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        m = _LABEL.match(raw)
        if m and not raw.startswith("."):
            fn, pending = m.group(1), {}
            continue
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith((".", "s_endpgm")):
            continue
        op = line.split()[0]
        if in_asm:
            srcs = _regs(line.split(",", 1)[1]) if "," in line else set()
            for r in srcs:
                if r in pending and pending[r][0] < pending[r][1]:
                    problems.append((fn, ln, line, r, pending[r][0], pending[r][1]))
        # advance wait states
        adv = 1
        if op == "s_nop":
            try:
                adv = int(line.split()[1], 0) + 1
            except (IndexError, ValueError):
                adv = 1
        for r in list(pending):
            w, need = pending[r]
            w += adv
            if w >= need:
                del pending[r]
            else:
                pending[r] = (w, need)
        if op.startswith("v_mfma") and not in_asm:
            dst = line.split()[1].rstrip(",")
            if dst.startswith("v"):          # AGPR destinations (a[..]) are read via accvgpr_read
                need = NEED_32x32 if "32x32" in op else NEED_16x16
                for r in _regs(dst):
                    pending[r] = (0, need)
    return problems


def check_file(src: str, extra=()):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17",
               "--cuda-device-only", "-S", "-I", os.path.dirname(src), *extra, "-o", out, src]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-2000:])
        return scan_asm(open(out).read())


def main(argv):
    files = argv or sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")) +
                           glob.glob(os.path.join(ROOT, "csrc", "comm", "*.hip")))
    bad = 0
    for f in files:
        probs = check_file(f)
        for fn, ln, text, reg, w, need in probs[:20]:
            print(f"{os.path.basename(f)}:{ln} {fn}: `{text}` reads v{reg} {w} wait states "
                  f"after an MFMA wrote it (needs {need})")
        bad += len(probs)
        print(f"{os.path.basename(f)}: {len(probs)} hazard(s)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
