# PMC of the tower's layer-3 launch for the library and each tools/_var/libsde_*.so (tools/tower_layer3.py; one
# rocprofv3 --pmc pass per counter group of tools/pmc_kernel.py), then tools/tower_variants.py timing.
# usage: gpurun --timeout 900 -- bash tools/gpu_pmc_variants.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcvar}; mkdir -p $O
for so in lib tools/_var/libsde_*.so; do
  n=$(basename $so .so)
  timeout -k 10 200 python tools/pmc_kernel.py run $O/$n -- python tools/tower_layer3.py $so f16x3 5 || exit 1
  python tools/pmc_kernel.py sum $O/$n "conv64_h16_kernel" > $O/$n.txt || exit 1
  echo "== $n"; cat $O/$n.txt
done
timeout -k 10 400 python -u tools/tower_variants.py 1024 > $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; exit 1; }
grep -E "us |clock" $O/variants.txt | grep -E "layer3 f16x3  |pair f16x3 |clock" | grep -v 'm32\|split\|wino'
echo done
