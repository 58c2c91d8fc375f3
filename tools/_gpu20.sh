set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run --output-format csv -- python tools/tower_only.py 1024 1024 3 > gpurun_out/p20.log 2>&1 && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof20/run_kernel_stats.csv')):
    print(r['Name'][:45], r['Calls'], r['AverageNs'])
"
