#!/bin/bash
# r03ah: ND plan with the interval-0 closure anchors in the root (every leaf <= 176 positions):
# full GPU tests, KKT factor timing, factor timeline, smoke, default bench
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ah
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03ah] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03ah] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
for b in 512 64 1; do step kkt_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_b$b.json; done
grep -H '"factor_ms"' $OUT/kkt_*.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python tools/bench_kkt.py --batch 512 --reps 3 > $OUT/tr.log 2>&1
python3 - <<'PY' > $OUT/timeline.txt
import csv, glob
f = glob.glob('gpurun_out/r03ah/tr/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'k_front_factor' in r['Kernel_Name'] or 'k_inertia_zero' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_inertia_zero' in r['Kernel_Name']]
seg = rows[idx[-1]:]
t0 = int(seg[0]['Start_Timestamp'])
for r in seg:
    n = r['Kernel_Name']; i = n.find('k_'); n = n[i:n.find('(', i)]
    print(f"{(int(r['Start_Timestamp'])-t0)/1e3:9.1f} {(int(r['End_Timestamp'])-t0)/1e3:9.1f} us  {n}")
PY
find $OUT/tr -name '*kernel_trace.csv' -delete
cat $OUT/timeline.txt
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench 900 python bench.py
tail -c 300 $OUT/bench.log
echo done
