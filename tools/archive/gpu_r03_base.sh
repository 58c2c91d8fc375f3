# Round-3 baseline: default bench line, PMC of the certified CV+WTA row kernel and of the CBCA scan.
# usage: gpurun --timeout 900 -- bash tools/gpu_r03_base.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03base}
mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 400 $O/bench_default.json
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc_cvrow -- python tools/cv_only.py 1024 1024 192 certified && \
python tools/pmc_kernel.py sum $O/pmc_cvrow "cv_wta_row" > $O/pmc_cv_wta_row.txt && cat $O/pmc_cv_wta_row.txt
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc_cbca -- python tools/cbca_only.py 1024 1024 192 14 1 && \
python tools/pmc_kernel.py sum $O/pmc_cbca "cbca_scan" > $O/pmc_cbca.txt && cat $O/pmc_cbca.txt
