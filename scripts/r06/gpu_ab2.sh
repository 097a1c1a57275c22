#!/bin/bash
# round 6: VERDICT r05 items 4 and 6 -- LOCAL+TB on the 3-wave G16R12 shape and 300 x 300 LOCAL with
# the segment keys' best in registers, each A/B'd against the default on one box (alternating),
# plus their PMC traffic passes.  Output: gpurun_out/r06i/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
export TAG=${TAG:-r06i}
SEL="three_wave_shape or segments_in_registers or packed_local_traceback or test_local_long_targets" \
LINES="ltb_def|GASALX_X=0|--workload sw_local_tb --no-cpu --no-e2e;ltb_g16|GASALX_LTBD_G16=1|--workload sw_local_tb --no-cpu --no-e2e;ltb_def2|GASALX_X=0|--workload sw_local_tb --no-cpu --no-e2e;ltb_g16_2|GASALX_LTBD_G16=1|--workload sw_local_tb --no-cpu --no-e2e;s300_def|GASALX_X=0|--workload sw_local_300 --no-cpu --no-e2e;s300_reg|GASALX_KSEG_REG=1|--workload sw_local_300 --no-cpu --no-e2e;s300_def2|GASALX_X=0|--workload sw_local_300 --no-cpu --no-e2e;s300_reg2|GASALX_KSEG_REG=1|--workload sw_local_300 --no-cpu --no-e2e" \
  bash scripts/r06/gpu_ab.sh || exit $?
GASALX_KSEG_REG=1 bash scripts/pmc_session.sh s300reg --workload sw_local_300 --parity-pairs 1000 || exit $?
bash scripts/pmc_session.sh s300def --workload sw_local_300 --parity-pairs 1000 || exit $?
GASALX_LTBD_G16=1 bash scripts/pmc_session.sh ltbg16 --workload sw_local_tb --parity-pairs 1000 --streams 1 || exit $?
exit 0
