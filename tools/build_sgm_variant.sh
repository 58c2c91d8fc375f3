# Build tools/_var/libsde_sgm_NAME.so from one sgm.hip source (A/B timing with tools/sgm_variants.py).
# usage: bash tools/build_sgm_variant.sh NAME path/to/sgm.hip [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; shift 2
C=scenedepthestimation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
  -Wno-unused-function -Iinclude -I$C -I$(dirname $SRC) "$@" -shared -o tools/_var/libsde_sgm_$NAME.so $SRC
