#!/bin/bash
# PMC calibration passes (one counter group per pass) of traffic_calib and of
# the config-3 search (scripts/ablate.py); outputs under gpurun_out/calib.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/calib_p$i -o pmc -- $R/scripts/calib/traffic_calib > $OUT/calib_p$i.log 2>&1 || exit $?
  if [ -z "$NO_SEARCH" ]; then
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_" --output-format csv -d $OUT/search_p$i -o pmc -- python3 $R/scripts/ablate.py c3 > $OUT/search_p$i.log 2>&1 || exit $?
  fi
done <<'CTRS'
FETCH_SIZE
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum
TCC_REQ_sum TCC_READ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
CTRS
echo calib done
