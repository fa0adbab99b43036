#!/bin/bash
# Build the engine from a git revision (default HEAD) as lib/librl_amd_base.so
# next to the working tree's lib/librl_amd.so, for same-box A/Bs (scripts/ab.sh).
set -e
REV=${1:-HEAD}
cd "$(dirname "$0")/../distributed-rate-limiter_amd"
rm -rf build/base && mkdir -p build/base/x/csrc
ln -sfn "$PWD/../include" build/base/include
for f in $(git ls-files csrc | grep -E '\.(h|hip)$'); do git show "$REV:distributed-rate-limiter_amd/$f" > build/base/x/$f; done
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC"
/opt/rocm/bin/hipcc $HIPFLAGS -c build/base/x/csrc/rl_engine.hip -o build/base/rl_engine.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/librl_amd_base.so build/base/rl_engine.o \
    build/rl_keyhash.o build/rl_route.o build/ratelimiter.o build/coalescer.o build/decorators.o
echo "lib/librl_amd_base.so from $REV"
