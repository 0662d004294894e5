#!/bin/bash
# Build a tuning variant of the library: tools/build_variant.sh NAME "-DEGM_WALK_STACK=512 ..."
# -> emqx_amd/libemqx_gpu_match_NAME.so (select with EGM_LIB=...)
set -e
name=$1; flags=$2
d=/tmp/egm_variant_$name; mkdir -p $d
R=$(cd "$(dirname "$0")/.." && pwd)
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -Wno-unused-value $flags -c $R/emqx_amd/csrc/egm_kernels.hip -o $d/k.o
g++ -O3 -fPIC -std=c++17 -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $flags -c $R/emqx_amd/csrc/egm_table.cpp -o $d/t.o
g++ -O3 -fPIC -std=c++17 -pthread -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $flags -c $R/emqx_amd/csrc/egm_capi.cpp -o $d/c.o
g++ -O3 -fPIC -std=c++17 -pthread -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $flags -c $R/emqx_amd/csrc/egm_retain.cpp -o $d/r.o
hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o $R/emqx_amd/libemqx_gpu_match_$name.so $d/k.o $d/t.o $d/c.o $d/r.o
echo built $R/emqx_amd/libemqx_gpu_match_$name.so
