#!/bin/bash
# rocprofv3 evidence for every BASELINE workload: kernel-trace stats of a bench run + FETCH_SIZE /
# WRITE_SIZE passes (tools/gpu_profile_workload.sh).  Usage: tools/gpu_profile_all.sh ROUNDTAG [workloads...]
set -u
TAG=$1; shift
WS=${@:-syn200 synstr200 rdw_narrow wide_odo}
for W in $WS; do
  bash $GRAFT_REPO_ROOT/tools/gpu_profile_workload.sh $TAG $W views || { echo "profile $W failed"; exit 1; }
done
echo PROFILE_ALL_OK
