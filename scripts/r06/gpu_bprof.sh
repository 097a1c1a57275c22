#!/bin/bash
# round 6: kernel + copy trace of the boundary benchmark (tools/boundary_bench, test_prog pattern)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/${TAG:-r06g}; mkdir -p $O
G=$ROOT/tests/golden
cd /tmp && export TMPDIR=/tmp
for T in ${THREADS:-4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/bprof_t$T -o run -- \
    $ROOT/tools/boundary_bench --repl 50 --warm 1 --reps 2 -y local -n $T $G/query_batch.fasta.gz $G/target_batch.fasta.gz \
    > $O/bprof_t$T.json 2> $O/bprof_t$T.err
  rc=$?; echo "[bprof t$T] rc=$rc $(cat $O/bprof_t$T.json)"; [ $rc -eq 0 ] || exit $rc
done
