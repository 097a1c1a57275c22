#!/bin/bash
# round 4, session S: what the driver runs at round end, on the final library: smoke(), then the
# default bench line.
# Output: gpurun_out/r04s/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04s; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_default.err; exit $rc; }
python3 - $O/bench_default.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["metric"], d["value"], d["unit"], "roofline", d["roofline"]["frac"], d["roofline"]["traffic"], "cpu", d["cpu_baseline"]["value"])
PY
