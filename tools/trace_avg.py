#!/usr/bin/env python3
"""Per-call durations of one kernel from a rocprofv3 kernel trace, split into the bench's warmup and
timed launches, so a bench line's ms_per_step can be set beside the trace of the same command.

usage: trace_avg.py RUN_kernel_trace.csv KERNEL_SUBSTRING TIMED_CALLS [BENCH_LINE.json]

The last TIMED_CALLS launches of the kernel are the timed steps (bench.py launches the dominant
kernel once per step and runs its warmup first).  Prints JSON: every call's duration, the average,
minimum and maximum of the timed calls and of all calls, and, given the bench line, its ms_per_step
and the ratio ms_per_step / timed average (>= 1: the step cannot be shorter than its kernel).
"""
import csv
import json
import sys


def main():
    path, sub, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    if not ms:
        sys.exit(f"no launch of a kernel matching {sub!r}")
    timed = ms[-k:]
    out = {"kernel": rows[0]["Kernel_Name"], "calls": len(ms), "timed_calls": len(timed),
           "timed_avg_ms": round(sum(timed) / len(timed), 4), "timed_min_ms": round(min(timed), 4),
           "timed_max_ms": round(max(timed), 4), "all_avg_ms": round(sum(ms) / len(ms), 4),
           "per_call_ms": [round(x, 4) for x in ms]}
    if len(sys.argv) > 4:
        line = json.loads([ln for ln in open(sys.argv[4]) if ln.startswith("{")][-1])
        out["bench_ms_per_step"] = line["ms_per_step"]
        out["bench_value"] = line["value"]
        out["step_over_timed_avg"] = round(line["ms_per_step"] / out["timed_avg_ms"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
