#!/bin/bash
# Build a variant libmisort with schedule switches for A/B probes:
#   tools/build_variant.sh NAME "-DMISORT_SPAN_PRE=0 -DMISORT_SPAN_POST=0"
# -> parallel-computing-mpi_amd/lib/variants/libmisort_NAME.so (bench: MISORT_LIBRARY=...)
set -e
HERE="$(cd "$(dirname "$0")/.." && pwd)"
C="$HERE/parallel-computing-mpi_amd/csrc"; L="$HERE/parallel-computing-mpi_amd/lib"; O="$L/variants/$1"
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$HERE/include -I$C $2"
/opt/rocm/bin/hipcc $F -c "$C/sort_u32.hip" -o "$O/sort_u32.o" &
/opt/rocm/bin/hipcc $F -c "$C/sort_u64.hip" -o "$O/sort_u64.o" &
/opt/rocm/bin/hipcc $F -c "$C/kernels.hip" -o "$O/kernels.o" &
/opt/rocm/bin/hipcc $F -c "$C/runs.hip" -o "$O/runs.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$L/variants/libmisort_$1.so" "$O/kernels.o" "$O/sort_u32.o" "$O/sort_u64.o" "$L/codec.o" "$O/runs.o" "$L/runtime.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$O"
