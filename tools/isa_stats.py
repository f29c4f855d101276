#!/usr/bin/env python3
"""Per-kernel ISA summary of a `hipcc --cuda-device-only -S` listing: registers, scratch, and the
instruction mix (MFMA / VALU / LDS / waits) of every basic block -- the quick check that a kernel
edit removed VALU work or spills before spending GPU time on it.

--loops: every loop (a backward branch to an earlier label) with its instruction mix and top opcodes --
the census behind round 6's K7 VALU work (docs/DESIGN.md §6d): the forward / backward loop bodies' VALU
count per tile, slot-address adds, NaN canonicalisations (v_max_f32 x, x).

usage: tools/isa_stats.py file.s [kernel-substring] [--blocks] [--loops]"""
from __future__ import annotations

import collections
import re
import sys


def kernels(text: str):
    for m in re.finditer(r"^(_Z\S+):\s*(?:;.*)?$", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        yield name, text[m.end():end], text


def meta(text: str, name: str, key: str):
    m = re.search(rf"\.set {re.escape(name)}\.{key}, (\d+)", text)
    return int(m.group(1)) if m else None


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    show_blocks = "--blocks" in sys.argv
    text = open(args[0]).read()
    sub = args[1] if len(args) > 1 else ""
    for name, body, _ in kernels(text):
        if sub not in name:
            continue
        tot = collections.Counter()
        blocks, cur = [], ["entry", collections.Counter()]
        blocks.append(cur)
        for raw in body.split("\n"):
            line = raw.split(";")[0].strip()
            if not line or line.startswith("."):
                if re.match(r"^\.LBB\S+:$", line):
                    cur = [line[:-1], collections.Counter()]
                    blocks.append(cur)
                continue
            c = classify(line.split()[0])
            cur[1][c] += 1
            tot[c] += 1
        regs = {k: meta(text, name, k) for k in ("num_vgpr", "num_agpr", "private_seg_size")}
        print(f"{name[:90]}\n  regs {regs}  total {dict(tot)}")
        if show_blocks:
            for bname, cnt in blocks:
                if sum(cnt.values()):
                    print(f"    {bname:12s} {dict(cnt)}")
        if "--loops" in sys.argv:
            loops(body)


def loops(body: str, min_len: int = 100) -> None:
    """Loops of one kernel body: label .. backward branch, longest form per header, with their mix."""
    lines = body.split("\n")
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    seen = {}
    for i, l in enumerate(lines):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seen[m.group(1)] = i  # the last back edge to a header spans the whole loop
    for head, end in seen.items():
        a = labels[head]
        if end - a < min_len:
            continue
        mix, ops = collections.Counter(), collections.Counter()
        for raw in lines[a:end + 1]:
            line = raw.split(";")[0].strip()
            if not line or line.startswith(".") or line.endswith(":"):
                continue
            op = line.split()[0]
            mix[classify(op)] += 1
            ops[op] += 1
            if op == "v_max_f32_e32" and len(set(line.replace(",", " ").split()[2:4])) == 1:
                ops["(canonicalise)"] += 1
        print(f"    loop {head} ({end - a} lines): {dict(mix)}")
        print("      " + "  ".join(f"{o}:{n}" for o, n in ops.most_common(24)))


if __name__ == "__main__":
    main()
