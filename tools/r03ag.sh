#!/bin/bash
# r03ag: per-dispatch timeline of the KKT factor at B = 512 (is the one 182-position leaf on the
# side stream the tail of the leaf level?)
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python tools/bench_kkt.py --batch 512 --reps 3 > $OUT/tr.log 2>&1
echo rc=$?
python3 - <<'PY' > $OUT/timeline.txt
import csv, glob
f = glob.glob('gpurun_out/r03ag/tr/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'k_front_factor' in r['Kernel_Name'] or 'k_inertia_zero' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last factorisation: from the last k_inertia_zero on
idx = [i for i, r in enumerate(rows) if 'k_inertia_zero' in r['Kernel_Name']]
seg = rows[idx[-1]:]
t0 = int(seg[0]['Start_Timestamp'])
for r in seg:
    n = r['Kernel_Name']; i = n.find('k_'); n = n[i:n.find('(', i)]
    print(f"{(int(r['Start_Timestamp'])-t0)/1e3:9.1f} {(int(r['End_Timestamp'])-t0)/1e3:9.1f} us  grid {r.get('Grid_Size','?'):>8}  {n}")
PY
cat $OUT/timeline.txt
find $OUT/tr -name '*kernel_trace.csv' -delete
echo done
