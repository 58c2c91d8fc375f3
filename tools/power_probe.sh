# Board power and clocks while the tower pair runs in a loop (is the tower power-capped?).
# usage: gpurun -- bash tools/power_probe.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pw1}; mkdir -p $O
timeout -k 10 20 rocm-smi --showpower --showclocks --showmaxpower > $O/idle.txt 2>&1 || true
timeout -k 10 120 python tools/power_load.py 25 > $O/load.txt 2>&1 &
LP=$!
sleep 12
for k in 1 2 3 4 5; do timeout -k 5 15 rocm-smi --showpower --showclocks >> $O/busy.txt 2>&1 || true; sleep 1; done
wait $LP
grep -iE "power|sclk|mclk|fclk|socclk" $O/idle.txt | head -12
echo ---
grep -iE "power|sclk" $O/busy.txt | head -30
tail -3 $O/load.txt
