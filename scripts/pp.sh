set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp -o run -- python tools/plan_probe.py > gpurun_out/pp.log 2>&1 || { tail -20 gpurun_out/pp.log; exit 1; }
python3 - <<'P'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/pp/run_kernel_trace.csv')) if 'plan' in r['Kernel_Name'] or 'elementwise' in r['Kernel_Name'] or 'regions' in r['Kernel_Name'] or 'bloom_or' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in rows[-140:]:
    print(r['Kernel_Name'][:40], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
P
