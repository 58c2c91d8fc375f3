# Round-5 probes: tower tests, tower diagnostic builds (tools/tower_variants.py), north-star bench A/B of
# the two 64->64 tower kernels, the SGM pair's gap probe (plain process and under rocprofv3), the CBCA
# fp32-chain timing probe.  usage: gpurun --timeout 1100 -- bash tools/gpu_probe5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-p5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "tower or smoke or cv_wta_split or row_band" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/tower_variants.py 1024 > $O/tower_variants.txt 2>&1 || { tail -20 $O/tower_variants.txt; exit 1; }
grep -E "us |clock" $O/tower_variants.txt | grep -v "sgmgap\|cbca" | tail -20
for p in f16x3 f16x3m32 f16x3; do
  timeout -k 10 300 python bench.py --tower-precision $p --no-cpu-baseline --steps 50 > $O/bench_$p.json 2> $O/bench_$p.err || { tail -20 $O/bench_$p.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$p.json').read().splitlines()[-1]); s=d['stages']; r=s['reference_gpu_path']; print('$p', round(d['ms_per_step'],4), 'tower', round(s['tower_ms_pair'],4), 'l3', round(s['conv_layer3_ms'],4), 'cv', round(s['cv_wta_ms'],4), 'agg', round(r['cv_aggregation_aggregate']['ms'],3), {k[:5]: round(v['ms'],3) for k,v in r['cv_aggregation_kernels'].items()})"
done
timeout -k 10 200 python tools/sgm_gap_probe.py > $O/sgm_gap.txt 2>&1 || { tail -20 $O/sgm_gap.txt; exit 1; }
cat $O/sgm_gap.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_sgm_gap -o run --output-format csv -- python tools/sgm_gap_probe.py 2 > $O/sgm_gap_prof.txt 2>&1 || { tail -20 $O/sgm_gap_prof.txt; exit 1; }
grep pair $O/sgm_gap_prof.txt
SDE_VARIANTS='libsde_cbca*.so' timeout -k 10 200 python tools/lib_variants.py cbca > $O/cbca_p32.txt 2>&1 || { tail -20 $O/cbca_p32.txt; exit 1; }
tail -3 $O/cbca_p32.txt
echo done
