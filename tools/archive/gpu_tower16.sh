# Tower A/B: the 16x16x32 kernel (f16x3, default) vs the 32x32x16 one (f16x3m32): tower tests, then
# alternating north-star bench lines, then a rocprofv3 kernel trace of both.
# usage: gpurun --timeout 900 -- bash tools/gpu_tower16.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-t16}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "tower or smoke or cv_wta_split or row_band" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for p in f16x3 f16x3m32; do
    timeout -k 10 300 python bench.py --tower-precision $p --no-cpu-baseline --steps 50 > $O/bench_${p}_$i.json 2> $O/bench_${p}_$i.err || { tail -20 $O/bench_${p}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/bench_${p}_$i.json').read().splitlines()[-1]); s=d['stages']; print('$p', round(d['ms_per_step'],4), 'tower', round(s['tower_ms_pair'],4), 'l3', round(s['conv_layer3_ms'],4), 'frac', round(d['roofline']['frac'],3), 'vs fp32', s.get('tower_${p}_vs_fp32_max_abs'))"
  done
done
for p in f16x3 f16x3m32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$p -o run --output-format csv -- python bench.py --tower-precision $p --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench_$p.json 2> $O/prof_$p.err || { tail -20 $O/prof_$p.err; exit 1; }
done
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc16 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
python tools/pmc_kernel.py sum $O/pmc16 "h16_kernel<false, true, true, false>" > $O/pmc_tower_layer3_h16.txt
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc32 -- python bench.py --tower-precision f16x3m32 --steps 3 --warmup 1 --no-cpu-baseline && \
python tools/pmc_kernel.py sum $O/pmc32 "x6p_kernel<false, false, true, true, true>" > $O/pmc_tower_layer3_m32.txt
echo done
