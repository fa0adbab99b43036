#!/bin/bash
# GPU-box run for the key hashing kernel: tests, bench (two key-length mixes),
# rocprofv3 kernel stats and FETCH_SIZE / WRITE_SIZE passes of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1kh}
mkdir -p gpurun_out/prof
set -o pipefail
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/${TAG}_$name.log"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step tests 300 python -u -m pytest tests/test_keyhash.py -x -v --timeout 120 --timeout-method thread
step bench_short 120 python -u scripts/bench_keyhash.py
step bench_long 120 python -u scripts/bench_keyhash.py --min-len 64 --max-len 160 --keys 4000000
step trace 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG}_trace -o run -- python3 scripts/bench_keyhash.py
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/${TAG}_fetch -o run -- python3 scripts/bench_keyhash.py
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/${TAG}_write -o run -- python3 scripts/bench_keyhash.py
exit 0
