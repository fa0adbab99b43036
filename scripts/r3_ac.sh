#!/bin/bash
# predicted grouping-sort plan (k_sort_local alone when the last plan fit LDS): GPU suite + survey
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -k "predicted or sort_local" > gpurun_out/r3ac_tests0.txt 2>&1 || { tail -30 gpurun_out/r3ac_tests0.txt; exit 1; }
tail -1 gpurun_out/r3ac_tests0.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ac_tests.txt 2>&1 || { tail -30 gpurun_out/r3ac_tests.txt; exit 1; }
tail -1 gpurun_out/r3ac_tests.txt
RUNS="mixed: fw_uniform: sw_bursty: tb_zipf: tb_zipf15: mixed: fw_uniform: sw_bursty: tb_zipf:" STEPS=20 bash scripts/survey.sh
