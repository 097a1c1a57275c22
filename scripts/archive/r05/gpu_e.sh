#!/bin/bash
# round 5, session E: bisect the LOCAL sample-data mismatch (scripts/r05/bisect_local.py)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
timeout -k 10 600 python scripts/r05/bisect_local.py
