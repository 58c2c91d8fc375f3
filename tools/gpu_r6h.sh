set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 300 python -u tools/tower_phase.py tools/_var/libsde_phase*.so > $O/phase.txt 2>&1 || { tail -20 $O/phase.txt; exit 1; }
cat $O/phase.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u tools/sgm_skew_probe.py 8 > $O/sgm_skew.txt 2>&1 || { tail -20 $O/sgm_skew.txt; exit 1; }
cat $O/sgm_skew.txt | grep -v amdgpu.ids
