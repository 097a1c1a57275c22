#!/usr/bin/env python3
"""Summarise a scripts/pmc_session.sh run into profiles/pmc_<workload>.json.

usage: pmc_summary.py RUN_DIR WORKLOAD PAIRS_PER_LAUNCH
For the dominant kernel of the bench step (its longest dispatch), records every counter of every pass and the derived:
  hbm_bytes_per_launch   = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes; gfx950
                           FETCH_SIZE tallies 128-B requests at 64 B, see
                           MI355X_MICROARCH.md, HBM section)
  valu_insts_per_launch  = SQ_INSTS_VALU (wave instructions)
plus the plan and libgasal sha256 the passes ran (bench.py uses the file only for the
same build and plan) and the dominant dispatch's duration (kernel_ns).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(run_dir, workload, pairs):
    per = collections.defaultdict(dict)   # kernel -> counter -> value (its longest dispatch in the pass)
    dur = {}
    for path in sorted(glob.glob(os.path.join(run_dir, "p*", "run_counter_collection.csv"))):
        rows = list(csv.DictReader(open(path)))
        agg = collections.defaultdict(float)
        pdur = {}
        for r in rows:
            k = r["Kernel_Name"]
            d = int(r["Dispatch_Id"])
            agg[(k, d, r["Counter_Name"])] += float(r["Counter_Value"])
            pdur[(k, d)] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        # a kernel launched twice per step (WITH_START: forward and reverse pass)
        # is summarised by its longest dispatch, the forward pass
        longest = {}
        for (k, d), t in pdur.items():
            if t > pdur.get((k, longest.get(k, -1)), -1):
                longest[k] = d
        dur.update(pdur)
        for (k, d, c), v in agg.items():
            if d == longest[k]:
                per[k][c] = v
    # dominant kernel: longest last dispatch
    best = max(per, key=lambda k: max(v for (kk, _), v in dur.items() if kk == k))
    c = per[best]
    out = {"workload": workload, "kernel": best, "pairs_per_launch": int(pairs), "counters": c}
    # the bench lines the passes printed: their plan and library hash (bench.py accepts this
    # file only for a run of the same build and plan)
    for path in sorted(glob.glob(os.path.join(run_dir, "p*.json"))):
        try:
            line = [ln for ln in open(path) if ln.startswith("{")][-1]
            cfg = json.loads(line)["config"]
            out["plan"], out["lib_sha256"] = cfg.get("plan"), cfg.get("lib_sha256")
            break
        except Exception:
            continue
    out["kernel_ns"] = min(v for (kk, _), v in dur.items() if kk == best)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["hbm_bytes_per_launch"] = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU" in c:
        out["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
    # the steady loop's instruction mix priced by the measured issue table (kernel_census.py), of the
    # same library the passes ran (bench.py: the per-class issue-bound fraction)
    lib = os.path.join(ROOT, "genomics-gpu_amd", "lib", "libgasal.so")
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import hashlib
        import kernel_census as KC
        if hashlib.sha256(open(lib, "rb").read()).hexdigest() == out.get("lib_sha256"):
            c = KC.census(lib, KC.mangled(lib, best), KC.RATES)
            out["census"] = {k: c[k] for k in ("kernel", "loop_valu", "loop_salu", "loop_issue_cycles",
                                               "cycles_per_valu", "rates")}
    except (Exception, SystemExit) as e:   # noqa: BLE001 -- the census is an addition, never a failure
        out["census_error"] = str(e)
    out["note"] = ("separate rocprofv3 --pmc passes (scripts/pmc_session.sh); FETCH_SIZE x2 per the gfx950 "
                   "correction; counters of the longest dispatch of the dominant kernel")
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path, {k: out[k] for k in out if k not in ("counters", "note")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
