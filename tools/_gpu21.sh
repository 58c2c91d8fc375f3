set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp scenedepthestimation_amd/libsde.so /tmp/libsde_base.so
for v in base e3 e4 e5; do
  if [ $v = base ]; then cp /tmp/libsde_base.so scenedepthestimation_amd/libsde.so; else cp _var/libsde_$v.so scenedepthestimation_amd/libsde.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof21_$v -o run --output-format csv -- python tools/tower_only.py 1024 1024 3 > gpurun_out/p21_$v.log 2>&1 || exit 1
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof21_$v/run_kernel_stats.csv')):
    print(r['Name'][:45], r['Calls'], r['AverageNs'])
"
done
