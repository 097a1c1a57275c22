#!/bin/bash
# round 6: tools/boundary_bench probes (test_prog pattern, 20K sample pairs x 50): thread counts,
# poll back-off, batch sizes; one JSON line per run
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/${TAG:-r06h}; mkdir -p $O
G=$ROOT/tests/golden
run() {  # name args...
  local name=$1; shift
  timeout -k 10 120 $ROOT/tools/boundary_bench --repl 50 --warm 1 --reps 5 "$@" -y local \
    $G/query_batch.fasta.gz $G/target_batch.fasta.gz > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "[$name] rc=$rc $(grep -o '"best_ms": [0-9.]*, "gcups": [0-9.]*' $O/$name.json)"
  [ $rc -eq 0 ] || exit $rc
}
for T in 1 2 4 8; do run t${T} -n $T; run t${T}_poll20 -n $T --poll-us 20; done
run t4_b10k -n 4 --batch 10000
run t4_b20k -n 4 --batch 20000
run t4_s3 -n 4 --storages 3
