#!/bin/bash
# GPU-box run: tests, smoke, short bench.  Stops at the first step that
# faults / aborts / times out (exit 124,134,137,139 or >128); plain test
# failures (exit 1) do not stop later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench}
[[ $STEPS == *tests* ]] && run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *smoke* ]] && run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python -u bench.py ${BENCH_ARGS:-}
exit 0
