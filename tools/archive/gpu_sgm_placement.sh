# SGM pair time per HBM placement of its volumes (tools/sgm_placement.py), plain and under a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sgm_place; mkdir -p $O
timeout -k 10 240 python -u tools/sgm_placement.py 4 contig > $O/place.log 2>&1 || { tail -20 $O/place.log; exit 1; }
grep -v amdgpu.ids $O/place.log
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python tools/sgm_placement.py 4 contig > $O/place_prof.log 2>&1 || { tail -20 $O/place_prof.log; exit 1; }
echo traced
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python tools/sgm_placement.py 2 contig > $O/place_pmc.log 2>&1 || { tail -20 $O/place_pmc.log; exit 1; }
echo pmc done
