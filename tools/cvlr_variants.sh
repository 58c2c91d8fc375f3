# Profiling builds of cvlr_row_kernel with parts switched off (CVLR_SKIP bits: 1 L stores,
# 2 R stores, 4 dots, 8 loads) -> tools/_var/libsde_<bits>.so.  Run here (CPU), then time on
# the GPU with tools/cvlr_variants.py.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_var
O=scenedepthestimation_amd/_obj
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
    -Iinclude -Iscenedepthestimation_amd/csrc -DCVLR_SKIP=$v -c scenedepthestimation_amd/csrc/cost_volume.hip \
    -o tools/_var/cv_$v.o &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libsde_$v.so tools/_var/cv_$v.o \
    $O/cbca.o $O/cv_row.o $O/sgm.o $O/tower.o
done
ls tools/_var/*.so
