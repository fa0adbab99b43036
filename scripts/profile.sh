#!/bin/bash
# GPU-box profile of the bench command: kernel-trace stats, then one PMC pass
# each for FETCH_SIZE and WRITE_SIZE (separate passes: TCC slot limits).
# Output: gpurun_out/prof/<TAG>_{trace,fetch,write}/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
BARGS=${BARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
mkdir -p gpurun_out/prof
set -o pipefail
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -s KILL "$to" "$@" > "gpurun_out/prof/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/prof/${TAG}_$name.log"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG}_trace -o run -- python3 bench.py $BARGS
[ -n "$NO_PMC" ] && exit 0
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/${TAG}_fetch -o run -- python3 bench.py $BARGS
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/${TAG}_write -o run -- python3 bench.py $BARGS
exit 0
