# native gRPC front end on the GPU engine (tests + configs[4] levels) and the routed kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r3h}
timeout -k 10 300 python -u -m pytest tests/test_grpc_native.py tests/test_grpc.py tests/test_coalescer.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 400 python bench.py --grpc --seconds 3 > gpurun_out/${T}_grpc.json 2> gpurun_out/${T}_grpc.err || { tail -30 gpurun_out/${T}_grpc.err; exit 1; }
grep '^{' gpurun_out/${T}_grpc.err || true
TAG=${T}_routed bash scripts/prof_routed.sh
