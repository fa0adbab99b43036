#!/bin/bash
# One GPU call's worth of named measurement steps (replaces round 4's one-off
# scripts/steps_r4*.txt files).  Usage, on the gpurun box:
#
#   bash scripts/steps.sh TAG SET [SET ...] [-- EXTRA_STEPS_FILE [PREFIX]]
#
# Each step runs under its own time limit through scripts/gpusteps.sh (output
# in gpurun_out/TAG_<step>.out/.err); a step that times out, aborts or faults
# ends the call.  Sets:
#   gpu     the GPU test suite (pytest -m gpu, thread timeouts)
#   smoke   __graft_entry__.smoke()
#   bench   the driver's command (configs[1], 1 GPU, 20 timed steps)
#   survey  the other workloads: configs[0] FW uniform, configs[2] SW bursty,
#           configs[3] mixed, Zipf 1.5, one hot key, routed mixed / configs[1]
#           at world 1 (buckets in place) and routed mixed with the RCCL
#           loopback exchange (the N > 1 step's work)
#   hot     Zipf 1.5 and one hot key only
#   routed  the three routed lines only
#   e2e     configs[4] through the coalescer (lib/rl_bench_e2e)
#   grpc    configs[4] through the native gRPC server
#   prof    rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the
#           driver's command (scripts/profile.sh, TAG_zipf)
#   proft   the kernel trace only
# EXTRA_STEPS_FILE [PREFIX]: further "<name> <seconds> <command>" lines (ad-hoc
# A/Bs; scripts/ab_r5.txt holds this round's), only those whose name starts
# with PREFIX when one is given.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
shift
F=$(mktemp /tmp/steps.XXXXXX)
B="--steps 20 --warmup 5 --no-cpu-baseline --lat-batches 0"
while [ $# -gt 0 ]; do
    case "$1" in
    gpu) echo "${TAG}_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" ;;
    smoke) echo "${TAG}_smoke 200 python -u -c \"import __graft_entry__ as g; g.smoke()\"" ;;
    bench) echo "${TAG}_bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5" ;;
    survey | hot | routed)
        if [ "$1" = survey ]; then
            echo "${TAG}_mixed 240 python -u bench.py --workload mixed $B"
            echo "${TAG}_sw 240 python -u bench.py --workload sw_bursty $B"
            echo "${TAG}_fw 240 python -u bench.py --workload fw_uniform $B"
        fi
        if [ "$1" != routed ]; then
            echo "${TAG}_z15 200 python -u bench.py --workload tb_zipf15 $B"
            echo "${TAG}_hot 200 python -u bench.py --workload tb_hot $B"
        fi
        if [ "$1" != hot ]; then
            echo "${TAG}_rtm 240 python -u bench.py --ingress routed --workload mixed $B"
            echo "${TAG}_rtm_x 240 python -u bench.py --ingress routed --route-exchange --workload mixed $B"
            echo "${TAG}_rtz 240 python -u bench.py --ingress routed --workload tb_zipf $B"
        fi ;;
    e2e) echo "${TAG}_e2e 200 distributed-rate-limiter_amd/lib/rl_bench_e2e --qps 1e5,1e6,3e6,1e7 --seconds 2" ;;
    grpc) echo "${TAG}_grpc 400 python -u bench.py --grpc" ;;
    prof) echo "${TAG}_prof 700 TAG=${TAG}_zipf BARGS=\"--steps 20 --warmup 5\" bash scripts/profile.sh" ;;
    proft) echo "${TAG}_proft 300 TAG=${TAG}_zipf NO_PMC=1 BARGS=\"--steps 20 --warmup 5\" bash scripts/profile.sh" ;;
    --) shift
        if [ $# -ge 2 ]; then grep -E "^$2" "$1"; shift; else cat "$1"; fi ;;
    *) echo "unknown set $1" >&2; exit 2 ;;
    esac
    shift
done > "$F"
cat "$F"
bash scripts/gpusteps.sh "$F"
