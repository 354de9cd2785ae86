#!/bin/bash
# Diagnostic build: rows_pp.o and api.o with -DLDPC_STAMPS -> ab/libldpc_hip_ppst.so (make clean-ab when done)
# (rows_pp.o with the product's loop alignment and machine scheduler, as the Makefile builds it)
set -eu
cd "$(dirname "$0")/.."
L=ldpcsimulation_amd/lib; V=ab; mkdir -p $V/obj_ppst
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ildpcsimulation_amd/csrc -Wall -Wno-unused-result -DLDPC_STAMPS -DLDPC_AB_BUILD ${EXTRA:-}"
$H -Xclang -target-feature -Xclang -load-store-opt -falign-loops=32 -mllvm -amdgpu-sched-strategy=max-memory-clause \
    -c -o $V/obj_ppst/rows_pp.o ldpcsimulation_amd/csrc/rows_pp.hip 2>/dev/null
$H -c -o $V/obj_ppst/api.o ldpcsimulation_amd/csrc/api.cpp 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $V/libldpc_hip_ppst.so $L/obj/kernels.o $L/obj/rows_fast.o \
    $V/obj_ppst/rows_pp.o $L/obj/gdbf.o $L/obj/bp.o $L/obj/nb.o $L/obj/nb_api.o $L/obj/nb_graph.o $V/obj_ppst/api.o $L/obj/graph.o
