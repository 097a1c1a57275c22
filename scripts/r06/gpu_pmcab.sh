#!/bin/bash
# round 6: WRITE_SIZE / FETCH_SIZE passes (separate rocprofv3 --pmc runs, no traces) of one workload
# under the default library and variants.  Usage: TAG=x VARS="name|ENV;..." ARGS="bench args" gpu_pmcab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/${TAG:-r06pmc}; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra V <<< "${VARS:-def|}"
for spec in "${V[@]}"; do
  IFS='|' read -r name envs <<< "$spec"
  for pass in WRITE_SIZE FETCH_SIZE; do
    env $envs timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/${name}_$pass -o run -- \
      python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --parity-pairs 1000 ${ARGS:-} > $O/${name}_$pass.json 2> $O/${name}_$pass.err
    rc=$?; echo "[$name $pass] rc=$rc"; if fatal $rc; then exit $rc; fi
  done
done
exit 0
