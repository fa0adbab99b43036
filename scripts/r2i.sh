#!/bin/bash
# round-2 final build: GPU suite, smoke, default bench, rocprofv3 kernel stats + FETCH/WRITE passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -qE "[0-9]+ failed" gpurun_out/gpu_tests.log || { echo TESTS-FAILED; exit 1; }
TAG=${TAG:-r2i} bash scripts/profile.sh || exit $?
