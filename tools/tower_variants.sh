# Profiling builds of the persistent tower kernel -> tools/_var/libsde_t<name>.so, each built with
# the -D options given as NAME=OPTS arguments (e.g. t2="-DTOWER_DIAG=2" r4="-DXP_RING_F16=4").
# TOWER_DIAG bits: 1 stager HBM loads, 2 all stager work, 4 MFMAs, 8 MFMA-wave LDS reads,
# 16 middle-layer output stores, 512 staged values replaced by constants (loads kept).  Run here (CPU), then time on the GPU with tools/tower_variants.py.
set -e
cd "$(dirname "$0")/.."
rm -rf tools/_var; mkdir -p tools/_var
O=scenedepthestimation_amd/_obj
for a in "$@"; do
  n=${a%%=*}; d=${a#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
    -Iinclude -Iscenedepthestimation_amd/csrc $d -c scenedepthestimation_amd/csrc/tower.hip \
    -o tools/_var/tower_$n.o &
done
wait
for a in "$@"; do
  n=${a%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libsde_$n.so tools/_var/tower_$n.o \
    $O/cbca.o $O/cv_row.o $O/sgm.o $O/cost_volume.o
  rm tools/_var/tower_$n.o
done
ls tools/_var/*.so
