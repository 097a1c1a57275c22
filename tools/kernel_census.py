#!/usr/bin/env python3
"""VALU instruction mix of one kernel's steady loop, from the built library (gfx950 ISA).

usage: kernel_census.py LIB.so|OBJ.co KERNEL_SYMBOL|"demangled name" [RATES.json]

Extracts the gfx950 code object from the library's fat binary, disassembles the kernel,
finds its loops (backward branches) and takes the one with the most VALU instructions as
the steady state.  Each VALU instruction is priced by the issue-cost table measured with
tools/ubench_issue.hip (cycles per wave64 instruction per SIMD at 8 waves per SIMD, bank-
separated operands, s_memtime; profiles/r04_valu_issue_rates.json), by opcode, else by
encoding class.  Prints JSON: counts per opcode, the VALU count and the average issue
cycles per VALU instruction of the loop -- what tools/pmc_summary.py multiplies with the
launch's SQ_INSTS_VALU to get the kernel's VALU issue cycles.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, tmp):
    """The gfx950 code objects of the library: its .hip_fatbin section holds one offload bundle per
    HIP translation unit (dispatch.hip, local_rs.hip, rclass.hip, ...), each unbundled apart."""
    fat = os.path.join(tmp, "fat.bin")
    # an explicit output file: with the input alone llvm-objcopy rewrites the library in place,
    # which changed its sha256 (and so unmatched the PMC summaries that record it)
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, lib, os.path.join(tmp, "copy.so")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [i for i in range(len(data)) if data.startswith(magic, i)] if len(data) < (1 << 28) else [0]
    cos = []
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(data)
        part = os.path.join(tmp, f"fat{k}.bin")
        open(part, "wb").write(data[a:b])
        co = os.path.join(tmp, f"k{k}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            cos.append(co)
    return cos


def code_object(lib, tmp, sym=None):
    """The code object holding kernel `sym` (mangled), or the first one."""
    cos = code_objects(lib, tmp)
    if sym is not None:
        for co in cos:
            out = subprocess.run([f"{LLVM}/llvm-objdump", "-t", co], check=True, capture_output=True, text=True).stdout
            if any(ln.split()[-1] == sym for ln in out.splitlines() if ln.split()):
                return co
    return cos[0]


def disasm(co, sym):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--disassemble-symbols=" + sym, co],
                         check=True, capture_output=True, text=True).stdout
    ins = []   # (address, text, branch target offset or None); "<text>  // ADDR: RAW <sym+0xOFF>"
    for line in out.splitlines():
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", line)
        if m:
            t = re.search(r"<\S+\+0x([0-9a-f]+)>", line)
            ins.append((int(m.group(2), 16), m.group(1).strip(), int(t.group(1), 16) if t else None))
    return ins


def rates_table(path):
    if not os.path.exists(path):
        return {}
    d = json.load(open(path))
    return {op: v.get("W2") for op, v in d["ops"].items()}   # the SIMD rate (see the file's "reading")


def price(op, text, table):
    base = re.sub(r"_e(32|64)$", "", op)
    if "dpp" in text or "row_" in text or "wave_" in text:
        return table.get("v_mov_b32_dpp", table.get("v_pk_add_u16", 4.0))
    if base in table:
        return table[base]
    if base.startswith("v_pk_"):
        return table.get("v_pk_add_u16", 4.0)
    if base.startswith(("v_add3", "v_and_or", "v_or3", "v_bitop3", "v_lshl_add", "v_add_lshl", "v_lshl_or",
                        "v_perm", "v_mad", "v_fma", "v_max3", "v_min3", "v_med3", "v_maximum3", "v_cndmask",
                        "v_cmp", "v_mul_lo", "v_mul_hi")):
        return table.get("v_add3_u32", 4.0) if not base.startswith("v_mul_lo") else 8.0
    if base.startswith(("v_add_", "v_sub_", "v_subrev_", "v_and_", "v_or_", "v_xor_", "v_not_", "v_mov_",
                        "v_mul_f32", "v_add_f32")):
        return table.get("v_add_u32", 2.0)
    return 4.0


def mangled(lib, name):
    """The code object's kernel symbol whose demangled form is `name` (as rocprofv3 prints it)."""
    with tempfile.TemporaryDirectory() as tmp:
        out = ""
        for co in ([lib] if lib.endswith(".co") else code_objects(lib, tmp)):
            out += subprocess.run([f"{LLVM}/llvm-objdump", "-t", co], check=True, capture_output=True, text=True).stdout
    syms = sorted({ln.split()[-1] for ln in out.splitlines() if " F " in ln and ln.split()[-1].startswith("_Z")})
    dem = subprocess.run(["c++filt"], input="\n".join(syms), check=True, capture_output=True, text=True).stdout.split("\n")
    for m, d in zip(syms, dem):
        if d.strip() == name.strip():
            return m
    raise SystemExit(f"no kernel symbol demangles to {name!r}")


def census(lib, sym, rates):
    table = rates_table(rates)
    with tempfile.TemporaryDirectory() as tmp:
        ins = disasm(lib if lib.endswith(".co") else code_object(lib, tmp, sym), sym)   # .co: a gfx950 code object
    addr = {a: i for i, (a, _, _) in enumerate(ins)}
    loops = []
    for i, (a, t, off) in enumerate(ins):
        if not t.startswith(("s_cbranch", "s_branch")) or off is None:
            continue
        tgt = ins[0][0] + off    # targets print relative to the symbol
        if tgt in addr and addr[tgt] < i:
            loops.append(ins[addr[tgt]:i + 1])
    if not loops:
        raise SystemExit("no loop found in " + sym)
    # the steady column loop: the innermost loop carrying the DPP lane hand-offs (wavefront
    # sweeps); kernels without them (band pass, thread-per-pair): the loop with the most packed
    # or fp32 arithmetic, the shorter on ties
    def dpp(seg):
        return any(x.startswith("v_") and ("dpp" in x or "wave_shr" in x or "row_" in x) for _, x, _ in seg)

    def arith(seg):
        return sum(1 for _, x, _ in seg if x.startswith(("v_pk_", "v_fma", "v_fmac", "v_mul_f32", "v_perm")))
    # innermost loops (no backward branch inside) carrying the DPP lane hand-offs (wavefront sweeps);
    # of them the densest in cell arithmetic per VALU instruction: the same sweep with capture or
    # boundary code, or a sweep the launch's plan does not take (the round-2 LOCAL sweep beside the
    # e-drift one in the same kernel: 446 against 345 VALU at G8R19), is less dense.  Without DPP
    # loops (band pass, thread-per-pair kernels): the densest innermost loop.
    def inner(seg):
        lo, hi = seg[0][0], seg[-1][0]
        return not any(t.startswith(("s_cbranch", "s_branch")) and o is not None and lo <= ins[0][0] + o < a
                       for a, t, o in seg[:-1])
    nvalu = lambda g: max(1, sum(1 for _, x, _ in g if x.startswith("v_")))
    innermost = [g for g in loops if inner(g)] or loops
    with_dpp = [g for g in innermost if dpp(g) and arith(g) > 0]
    pool = with_dpp or [g for g in innermost if arith(g) > 0]
    if not pool:   # no loop carries the cell arithmetic (e.g. nv16_kernel): no steady loop to price
        return {"kernel": sym, "loop_valu": None, "cycles_per_valu": None,
                "note": "no innermost loop with packed or fp32 cell arithmetic: the steady loop is not "
                        "identified, so no issue-priced figure", "rates": os.path.relpath(rates, ROOT)}
    seg = max(pool, key=lambda g: (arith(g) / nvalu(g), -len(g)))
    best = (0, seg)
    # static census: conditionally executed blocks (divergent captures, resets) are counted
    # too, although the hardware skips them while no lane enters (s_cbranch_execz); the
    # dynamic count is the PMC's SQ_INSTS_VALU
    counts, cyc, nv, ns = {}, 0.0, 0, 0
    for a, t, off in best[1]:
        op = t.split()[0]
        ns += op.startswith("s_")
        if not op.startswith("v_"):
            continue
        counts[op] = counts.get(op, 0) + 1
        cyc += price(op, t, table)
        nv += 1
    return {"kernel": sym, "loop_valu": nv, "loop_salu": ns, "loop_issue_cycles": round(cyc, 2),
            "cycles_per_valu": round(cyc / max(nv, 1), 4), "counts": dict(sorted(counts.items(), key=lambda x: -x[1])),
            "rates": os.path.relpath(rates, ROOT)}


RATES = os.path.join(ROOT, "profiles", "r04_valu_issue_rates.json")

if __name__ == "__main__":
    rates = sys.argv[3] if len(sys.argv) > 3 else RATES
    sym = sys.argv[2] if sys.argv[2].startswith("_Z") else mangled(sys.argv[1], sys.argv[2])
    print(json.dumps(census(sys.argv[1], sym, rates), indent=1))
