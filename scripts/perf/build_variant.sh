#!/bin/bash
# A/B builds of the library: scripts/perf/build_variant.sh TAG SOURCE "DEFINES"
# recompiles one source file of csrc/ with extra defines and links it with the
# other objects of the default build into lib/libbsm_hip_TAG.so, e.g.
#   scripts/perf/build_variant.sh p8 kernels_tiled.hip "-DBSM_SUM_PART=8"
# then on one box: BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_p8.so python bench.py ...
set -euo pipefail
TAG=$1 SRC=$2 DEFS=${3:-}
cd "$(dirname "$0")/../../basic_sparse_matrix_amd/csrc"
make -s -j8
base=${SRC%.hip}
mkdir -p build_var
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -Wall -Wno-unused-function -Wno-unused-result"
/opt/rocm/bin/hipcc $HIPFLAGS $DEFS -c "$SRC" -o "build_var/${base}_$TAG.o"
objs=""
for o in build/*.o; do
  [ "$o" = "build/$base.o" ] && objs="$objs build_var/${base}_$TAG.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../lib/libbsm_hip_$TAG.so" $objs \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/libbsm_hip_$TAG.so"
