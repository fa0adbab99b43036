# per-table GC budget + table-kernel warm-up: coalescer/gRPC GPU tests, gRPC levels incl. AllowBatch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp RL_SERVER_STATS=1
mkdir -p gpurun_out
T=${T:-r3t}
timeout -k 10 400 python -u -m pytest tests/test_coalescer.py tests/test_grpc.py tests/test_grpc_native.py tests/test_gpu_parity.py -m gpu -q -x --timeout 150 --timeout-method thread -k "coalescer or grpc or gc or reset" > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 400 python bench.py --grpc --seconds 3 --grpc-unary 35000,100000,150000,200000 --grpc-batched 2000,4000,8000,16000 > gpurun_out/${T}_grpc.json 2> gpurun_out/${T}_grpc.err || { tail -20 gpurun_out/${T}_grpc.err; exit 1; }
grep '^{' gpurun_out/${T}_grpc.err | cut -c1-420
