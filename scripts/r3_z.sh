#!/bin/bash
# scaled MSD digit (256 full buckets): GPU suite + survey
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_tests.txt 2>&1 || { tail -30 gpurun_out/r3z_tests.txt; exit 1; }
tail -2 gpurun_out/r3z_tests.txt
RUNS="mixed: fw_uniform: sw_bursty: tb_zipf: mixed: fw_uniform: sw_bursty: mixed:routed" STEPS=20 bash scripts/survey.sh
