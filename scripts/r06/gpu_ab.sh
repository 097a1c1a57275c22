#!/bin/bash
# round 6 A/B session: an optional pytest -k selection, then bench lines under env settings, then an
# optional kernel trace.  Usage: TAG=x SEL="pytest -k expr" LINES="name|ENV=..|bench args;..." PROF="name|ENV|args" gpu_ab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/${TAG:-r06ab}; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -n "${SEL:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "$SEL" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; echo "[pytest] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra L <<< "${LINES:-}"
for spec in "${L[@]}"; do
  IFS='|' read -r name envs args <<< "$spec"
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py $args > $O/$name.json 2> $O/$name.err
  rc=$?
  echo "[$name] rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/$name.json | head -1)"
  if fatal $rc; then echo "fatal in $name"; exit $rc; fi
done
if [ -n "${PROF:-}" ]; then
  IFS=';' read -ra P <<< "$PROF"
  cd /tmp && export TMPDIR=/tmp
  for spec in "${P[@]}"; do
    IFS='|' read -r name envs args <<< "$spec"
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
      python3 $ROOT/bench.py $args > $O/prof_$name.json 2> $O/prof_$name.err
    rc=$?; echo "[prof $name] rc=$rc"; if fatal $rc; then exit $rc; fi
  done
fi
exit 0
