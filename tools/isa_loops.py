#!/usr/bin/env python3
"""Per-loop instruction census of one kernel in a gfx950 assembly file.

usage: isa_loops.py FILE.s KERNEL_SUBSTRING
Finds backward branches (loops) in the kernel body and prints, per loop, the
instruction count by class (VALU full/half rate per tools/ubench_ops.hip,
s_nop, DPP, LDS, scratch, SALU) and an issue-cycle estimate per wave.
"""
import re
import sys

FULL = re.compile(r"^v_(add|sub|subrev)_(u32|f32|u16|f16|co_u32)?(_e32|_e64)?$|^v_(and|or|xor|not)_b32|^v_mul_f32|^v_(max|min)_(i16|u16|f16)|^v_mov_b32(_e32)?$")


def main(path, name):
    lines = open(path).read().split("\n")
    # kernel body
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            seg = body[labels[m.group(2)]:i + 1]
            cnt = {}
            cyc = 0
            for s in seg:
                s = s.strip()
                if not s or s.startswith((".", ";")) or s.endswith(":"):
                    continue
                op = s.split()[0]
                if op == "s_nop":
                    k = "s_nop"; c = 4 * (1 + int(s.split()[1], 0))
                elif op.startswith("v_") and ("dpp" in s or "row_" in s or "wave_" in s):
                    k = "valu_dpp"; c = 4
                elif op.startswith("v_"):
                    if FULL.match(op):
                        k = "valu_full"; c = 2
                    else:
                        k = "valu_half"; c = 4
                elif op.startswith("ds_"):
                    k = "lds"; c = 4
                elif op.startswith(("scratch_", "buffer_")):
                    k = "scratch/buffer"; c = 4
                elif op.startswith("s_"):
                    k = "salu"; c = 1
                else:
                    k = "other:" + op; c = 4
                cnt[k] = cnt.get(k, 0) + 1
                cyc += c
            print(f"loop {m.group(2)} lines {labels[m.group(2)]}-{i}: {dict(sorted(cnt.items()))} est_issue_cyc/wave={cyc}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
