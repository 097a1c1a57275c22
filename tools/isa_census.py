#!/usr/bin/env python3
"""Instruction census of the benchmarked kernels' inner loops (gfx950 ISA).

Compiles csrc/dispatch.hip to assembly (device only) and, for each kernel the
bench plans name, finds the column-step loop (the loop carrying the DPP
lane hand-offs) with the fewest VALU instructions — the common path — and
records VALU instructions per step.  bench.py turns that into the VALU
issue roofline (achieved wave-instructions/s against 1024 SIMDs x 2.4 GHz /
2 cycles).  Output: profiles/isa_census.json.

usage: python tools/isa_census.py [--asm FILE]
"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# plan name (gasalx_describe_plan) -> (kernel symbol, rows per lane R, group G, pairs per lane)
PLANS = {
    # plan name: (kernel symbol, R, G, pairs per lane, step axis)
    "wavefront16_local_G8R19": ("_ZN2gx11wf16_kernelILi0ELi8ELi19EEEvNS_6WfArgsE", 19, 8, 2, "target"),
    "wavefront16_local_G8R20": ("_ZN2gx11wf16_kernelILi0ELi8ELi20EEEvNS_6WfArgsE", 20, 8, 2, "target"),
    "wavefront16_global_G16R20": ("_ZN2gx11wf16_kernelILi1ELi16ELi20EEEvNS_6WfArgsE", 20, 16, 2, "target"),
    "wavefront16_semi_G8R23": ("_ZN2gx11wf16_kernelILi2ELi8ELi23EEEvNS_6WfArgsE", 23, 8, 2, "query"),
    "wavefront_local_keys_G8R20": ("_ZN2gx9wf_kernelILi0ELb1ELb0ELi8ELi20EEEvNS_6WfArgsE", 20, 8, 1, "target"),
    "wavefront16_global_tb_G16R20": ("_ZN2gx11wf16_kernelILi3ELi16ELi20EEEvNS_6WfArgsE", 20, 16, 2, "target"),
    "wavefront_global_tb_G16R20": ("_ZN2gx9wf_kernelILi1ELb0ELb1ELi16ELi20EEEvNS_6WfArgsE", 20, 16, 1, "target"),
    "wavefront_semi_keys_G8R20": ("_ZN2gx9wf_kernelILi2ELb1ELb0ELi8ELi20EEEvNS_6WfArgsE", 20, 8, 1, "target"),
}


def loops(lines, name):
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            seg = [s.strip() for s in body[labels[m.group(2)]:i + 1]]
            ins = [s for s in seg if s and not s.startswith((".", ";")) and not s.endswith(":")]
            valu = [s for s in ins if s.split()[0].startswith("v_")]
            dpp = [s for s in valu if "row_" in s or "wave_" in s or "_dpp" in s.split()[0]]
            nops = [s for s in ins if s.split()[0] == "s_nop"]
            vmem = [s for s in ins if s.split()[0].startswith(("global_", "buffer_", "scratch_"))]
            yield dict(valu=len(valu), dpp=len(dpp), s_nop=len(nops), vmem=len(vmem), lines=len(seg))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    args = ap.parse_args()
    asm = args.asm
    if not asm:
        asm = "/tmp/gx_dispatch_census.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "genomics-gpu_amd", "csrc"),
                        "-S", "--cuda-device-only", os.path.join(ROOT, "genomics-gpu_amd", "csrc", "dispatch.hip"),
                        "-o", asm], check=True)
    lines = open(asm).read().split("\n")
    out = {}
    for plan, (sym, R, Gs, ppl, axis) in PLANS.items():
        # the column-step loop: DPP hand-offs and at least ~5 VALU per row
        cands = [l for l in loops(lines, sym) if l["dpp"] >= 2 and l["dpp"] % 2 == 0
                 and l["valu"] / (l["dpp"] // 2) >= 5 * R]
        if not cands:
            continue
        best = min(cands, key=lambda l: l["valu"] / (l["dpp"] // 2))
        steps = best["dpp"] // 2
        out[plan] = dict(kernel=sym, R=R, G=Gs, pairs_per_lane=ppl, step_axis=axis, steps_per_iteration=steps,
                         valu_per_step=best["valu"] / steps, s_nop_per_step=best["s_nop"] / steps,
                         valu_per_padded_cell=best["valu"] / steps / (64 * R * ppl))
    path = os.path.join(ROOT, "profiles", "isa_census.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
