#!/bin/bash
# Build kernel microbench variants: build.sh NAME "-DFLAG=1 ..." [source]
set -e
cd "$(dirname "$0")"
mkdir -p bin
src=${3:-fa_bench.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form $2 "$src" -o bin/$1
