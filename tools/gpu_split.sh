# Split-activation tower check: the tower GPU tests, tools/tower_variants.py (library vs tools/_var variants),
# the default bench line.  usage: gpurun --timeout 900 -- bash tools/gpu_split.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-sp1}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "tower" --timeout 200 --timeout-method thread > $O/tests_tower.log 2>&1 || { tail -40 $O/tests_tower.log; exit 1; }
tail -3 $O/tests_tower.log
timeout -k 10 300 python tools/tower_variants.py 1024 > $O/tower_variants.txt 2>&1 || { tail -20 $O/tower_variants.txt; exit 1; }
tail -12 $O/tower_variants.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));s=d['stages'];print(d['value'],d['ms_per_step'],s['tower_ms_pair'],s['conv_layer3_ms'],d['roofline']['frac'],s.get('tower_f16x3_vs_fp32_max_abs'),s.get('cv_exact_fixup_pixels'))"
echo done
