"""Static VALU instruction mix of a kernel's hottest loop, from the gfx950 code
object of build/native/device.o (llvm-objdump). Used to price K2's issue
ceiling by instruction class (bench.py `roofline.issue_ceiling`).

    python tools/isa_mix.py [--kernel k_score16fILi32ELb1ELb1E] [--json out.json]

Classes (measured in profiles/r2_valu_issue.json, tools/microbench/valu_issue.hip):
  fast VOP2  the e32 forms of add/sub/subrev/mul/fmac (f32/f16/u16/u32),
             max/min (f16/u16/i16), and/or/xor, lshr/ashr, mov: ~2.27 shader
             cycles per wave64 instruction alone, ~3.44 in VOP3P-heavy streams
  VOP3 class every other VALU instruction (VOP3/VOP3P/SDWA/DPP, 32-bit
             max/min, cndmask, perm, bfi, ...): ~4.16 cycles
The hottest loop is the backward branch enclosing the most VALU instructions
(K2's column loop, unrolled by two columns).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(REPO, "build", "native", "device.o")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
FAST = re.compile(r"^v_(add|sub|subrev|mul|fmac)_(f32|f16|u16|u32)_e32$|^v_(max|min)_(f16|u16|i16)_e32$|"
                  r"^v_(and|or|xor)_b32_e32$|^v_(lshrrev|ashrrev)_[bi]32_e32$|^v_mov_b32_e32$")


def disassemble(obj: str = OBJ) -> list[str]:
    bundle = obj + ".0.hipv4-amdgcn-amd-amdhsa--gfx950"
    if not os.path.exists(bundle) or os.path.getmtime(bundle) < os.path.getmtime(obj):
        subprocess.run([OBJDUMP, "--offloading", obj], check=True, capture_output=True)
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", bundle], check=True, capture_output=True, text=True)
    return out.stdout.splitlines()


def kernel_body(lines: list[str], pattern: str) -> list[tuple[int, str, str]]:
    """(address, mnemonic, text) of the first kernel whose symbol matches."""
    body, inside = [], False
    for ln in lines:
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", ln)
        if m:
            if inside:
                break
            inside = pattern in m.group(2)
            continue
        if not inside:
            continue
        m = re.match(r"^\s+([sv]_\w+)(.*?)//\s*([0-9A-F]+):", ln)
        if m:
            body.append((int(m.group(3), 16), m.group(1), ln))
    if not body:
        raise SystemExit(f"kernel {pattern!r} not found")
    return body


def hottest_loop(body):
    best = None
    for i, (addr, mn, text) in enumerate(body):
        if not mn.startswith("s_cbranch") and mn != "s_branch":
            continue
        target = None
        # llvm-objdump prints the branch target as <symbol+offset>
        t = re.search(r"<\S+\+0x([0-9a-f]+)>", text)
        if t:
            target = body[0][0] + int(t.group(1), 16)
        if target is None or target >= addr:
            continue
        seg = [b for b in body if target <= b[0] <= addr]
        valu = sum(1 for b in seg if b[1].startswith("v_"))
        if best is None or valu > best[0]:
            best = (valu, seg)
    if best is None:
        raise SystemExit("no backward branch found")
    return best[1]


def blocks(body, seg):
    """Basic blocks of a loop (leaders: its start, branch targets, fall-throughs)."""
    base = body[0][0]
    leaders = {seg[0][0]}
    for i, (a, mn, t) in enumerate(seg):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tt = re.search(r"<\S+\+0x([0-9a-f]+)>", t)
            if tt:
                leaders.add(base + int(tt.group(1), 16))
            if i + 1 < len(seg):
                leaders.add(seg[i + 1][0])
    out, cur = [], []
    for x in seg:
        if x[0] in leaders and cur:
            out.append(cur)
            cur = []
        cur.append(x)
    out.append(cur)
    return out


def mix(seg) -> dict:
    fast = vop3 = other = 0
    ops: dict[str, int] = {}
    for _, mn, _ in seg:
        ops[mn] = ops.get(mn, 0) + 1
        if mn.startswith("v_"):
            if FAST.match(mn):
                fast += 1
            else:
                vop3 += 1
        else:
            other += 1
    return {"valu": fast + vop3, "fast_vop2": fast, "vop3_class": vop3, "non_valu": other,
            "ops": dict(sorted(ops.items(), key=lambda kv: -kv[1]))}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_score16fILi32ELb1ELb1E")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    body = kernel_body(disassemble(), a.kernel)
    seg = hottest_loop(body)
    # the column bodies: the loop's straight-line blocks of >= 100 VALU
    # instructions (the rest is the END-column path and the fill/drain tests,
    # taken in a few percent of the columns)
    hot = [x for b in blocks(body, seg) if sum(1 for y in b if y[1].startswith("v_")) >= 100 for x in b]
    out = {"kernel": a.kernel, "loop_bytes": seg[-1][0] - seg[0][0], "loop": mix(seg),
           "column_bodies": {"count": sum(1 for b in blocks(body, seg)
                                          if sum(1 for y in b if y[1].startswith("v_")) >= 100), **mix(hot)}}
    text = json.dumps(out, indent=1)
    print(text)
    if a.json:
        with open(a.json, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    sys.exit(main())
