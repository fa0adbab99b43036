#!/bin/bash
# routed pipeline at world 1 without the loopback collectives: route tests + survey
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.txt 2>&1 || { tail -20 gpurun_out/r3w_tests.txt; exit 1; }
tail -2 gpurun_out/r3w_tests.txt
RUNS="mixed:routed tb_zipf:routed mixed:routed tb_zipf:routed" STEPS=30 bash scripts/survey.sh
