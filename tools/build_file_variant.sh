# tools/_var/libsde_NAME.so: the library with one source file rebuilt with extra flags (A/B timing).
# usage: bash tools/build_file_variant.sh FILE.hip NAME [hipcc flags...]
#        SRC=path/to/other.hip bash tools/build_file_variant.sh FILE.hip NAME ...  (FILE.hip replaced by SRC)
set -e
cd "$(dirname "$0")/.."
F=$1; NAME=$2; shift 2
C=scenedepthestimation_amd/csrc
O=scenedepthestimation_amd/_obj
mkdir -p tools/_var
EXTRA=""
[ "$F" = "cv_row.hip" ] && EXTRA="-fno-honor-nans -mno-amdgpu-ieee"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
  -Wno-unused-function -Iinclude -I$C $EXTRA "$@" -c ${SRC:-$C/$F} -o tools/_var/v_$NAME.o
OBJS=""
for o in $O/*.o; do
  [ "$(basename $o)" = "${F%.hip}.o" ] || OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libsde_$NAME.so tools/_var/v_$NAME.o $OBJS
rm tools/_var/v_$NAME.o
