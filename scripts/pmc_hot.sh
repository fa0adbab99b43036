cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 python bench.py --workload tb_hot --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/hot.json || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc/a -o run -- python3 bench.py --workload tb_hot --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/b -o run -- python3 bench.py --workload tb_hot --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/b.log 2>&1 || exit $?
