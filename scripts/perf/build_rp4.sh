#!/bin/bash
# A/B build of band_chol5 with FOUR rows per wave (4 waves, RP = 4) for
# b in (497, 1009]: lib/libbsm_hip_rp4.so, selected at run time by
# BSM_CHOL_RPW=4 (scripts/chol_stress.py --rpw 4, scripts/chol_rp4_debug.py).
# The product instantiates RP = 2 only; this copies kernels_solve.hip, adds
# the RP = 4 dispatch line and links it with the other objects of the default
# build (round 5: RP = 4's wrong bits were a v_readlane of lanes that an
# exec-masked copy had left stale, fixed in the shared template).
set -euo pipefail
cd "$(dirname "$0")/../../basic_sparse_matrix_amd/csrc"
make -s -j8
mkdir -p build_var
python3 - <<'PY'
s = open("kernels_solve.hip").read()
old = "    else if (w4 <= 1024) rc = launch_chol5<T, 16, 2>(bd, prog.as<int>(), status, s, tr);\n"
assert s.count(old) == 1
new = ("    else if (w4 <= 1024 && getenv(\"BSM_CHOL_RPW\") && atoi(getenv(\"BSM_CHOL_RPW\")) == 4)\n"
       "        rc = launch_chol5<T, 16, 4>(bd, prog.as<int>(), status, s, tr);\n") + old
open("build_var/kernels_solve_rp4.hip", "w").write(s.replace(old, new))
PY
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -Wall -Wno-unused-function -Wno-unused-result -I."
/opt/rocm/bin/hipcc $HIPFLAGS -c build_var/kernels_solve_rp4.hip -o build_var/kernels_solve_rp4.o
objs=$(ls build/*.o | grep -v kernels_solve)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libbsm_hip_rp4.so $objs build_var/kernels_solve_rp4.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/libbsm_hip_rp4.so"
