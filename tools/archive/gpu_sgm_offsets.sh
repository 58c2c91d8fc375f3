set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sgm_off; mkdir -p $O
timeout -k 10 240 python -u tools/sgm_offsets.py > $O/off.log 2>&1 || { tail -20 $O/off.log; exit 1; }
grep -v amdgpu.ids $O/off.log
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/sgm_offsets.py > $O/off_prof.log 2>&1 || { tail -20 $O/off_prof.log; exit 1; }
echo traced
