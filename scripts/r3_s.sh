# AllowBatch overload investigation: server stats + coalescer batch trace at 2M decisions/s through gRPC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp RL_SERVER_STATS=1
mkdir -p gpurun_out
for lv in 4000 6000 8000; do
  timeout -k 10 200 python bench.py --grpc --seconds 3 --grpc-unary "" --grpc-batched $lv > gpurun_out/r3s_$lv.json 2> gpurun_out/r3s_$lv.err || { tail -20 gpurun_out/r3s_$lv.err; exit 1; }
  grep '^{' gpurun_out/r3s_$lv.err | cut -c1-600
done
