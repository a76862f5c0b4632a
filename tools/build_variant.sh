#!/bin/bash
# Build a libat2v variant with extra kernel defines for in-process A/B runs (tools/ab_bench.py):
#   tools/build_variant.sh <tag> -DAT2V_BWIN=20 -DAT2V_INV_GROUP=4 ...
# -> at2-node_amd/at2v/variants/libat2v_<tag>.so (the API/host objects are the product's own)
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/at2-node_amd/csrc
O=$R/at2-node_amd/at2v/variants
mkdir -p $O
make -s -C $R/at2-node_amd >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function "$@" -c $C/at2v_kernels.hip -o $O/k_$TAG.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread $O/k_$TAG.o $C/at2v_api.o $C/at2v_host.o $C/at2v_cpu.o -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -o $O/libat2v_$TAG.so
rm -f $O/k_$TAG.o
echo $O/libat2v_$TAG.so
