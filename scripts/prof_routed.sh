cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r2f_routed_trace -o run -- python3 bench.py --workload mixed --ingress routed --steps 10 --warmup 2 --no-cpu-baseline --lat-batches 0 > gpurun_out/prof/r2f_routed.log 2>&1
echo rc=$?
