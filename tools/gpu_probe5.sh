# Round-5 probes: tower diagnostic builds (tools/tower_variants.py), the SGM pair's gap probe in a plain
# process and under rocprofv3 (per-launch durations).  usage: gpurun --timeout 900 -- bash tools/gpu_probe5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-p5}; mkdir -p $O
timeout -k 10 300 python tools/tower_variants.py 1024 > $O/tower_variants.txt 2>&1 || { tail -20 $O/tower_variants.txt; exit 1; }
grep -E "us|clock" $O/tower_variants.txt | tail -30
timeout -k 10 200 python tools/sgm_gap_probe.py > $O/sgm_gap.txt 2>&1 || { tail -20 $O/sgm_gap.txt; exit 1; }
cat $O/sgm_gap.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_sgm_gap -o run --output-format csv -- python tools/sgm_gap_probe.py 2 > $O/sgm_gap_prof.txt 2>&1 || { tail -20 $O/sgm_gap_prof.txt; exit 1; }
grep pair $O/sgm_gap_prof.txt
echo done
