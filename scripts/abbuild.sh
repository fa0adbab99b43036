#!/bin/bash
# build an A/B variant of librl_amd.so: $1 = name, rest = extra hipcc flags
set -e
cd /root/repo/distributed-rate-limiter_amd
name=$1; shift
/opt/rocm/bin/hipcc -O${OPT:-3} -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall ${ENGINEFLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp} "$@" -c csrc/rl_engine.hip -o build/rl_engine_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/librl_amd_$name.so build/rl_engine_$name.o build/rl_keyhash.o build/rl_route.o build/ratelimiter.o build/coalescer.o build/decorators.o
