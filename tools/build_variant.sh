#!/bin/bash
# Build a variant libmisort with build-time switches for A/B probes:
#   tools/build_variant.sh NAME "-DMISORT_MK_NT=256"
# -> parallel-computing-mpi_amd/lib/variants/libmisort_NAME.so (bench: MISORT_LIBRARY=...)
set -e
HERE="$(cd "$(dirname "$0")/.." && pwd)"
C="$HERE/parallel-computing-mpi_amd/csrc"; L="$HERE/parallel-computing-mpi_amd/lib"; O="$L/variants/$1"
mkdir -p "$O"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$HERE/include -I$C $2"
for src in sort_u32 sort_u64 kernels runs runsk runsk_fg6 codec; do
  /opt/rocm/bin/hipcc $F -c "$C/$src.hip" -o "$O/$src.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$L/variants/libmisort_$1.so" "$O/kernels.o" "$O/sort_u32.o" \
  "$O/sort_u64.o" "$O/codec.o" "$O/runs.o" "$O/runsk.o" "$O/runsk_fg6.o" "$L/runtime.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$O"
