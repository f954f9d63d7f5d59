#!/bin/bash
# Build kernel microbench variants: build.sh NAME "-DFLAG=1 ..." [source]
# Flags follow the production build (ops/_build.py): flash-attention sources get
# -amdgpu-mfma-vgpr-form (FILE_FLAGS), the others do not.
set -e
cd "$(dirname "$0")"
mkdir -p bin
src=${3:-fa_bench.hip}
extra=""
case "$src" in fa*) extra="-mllvm -amdgpu-mfma-vgpr-form" ;; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics $extra \
  -I../../service_account_auth_improvements_amd/ops/csrc $2 "$src" -o bin/$1
