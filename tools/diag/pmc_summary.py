'''
DIAGNOSTIC: per-kernel summary of a rocprofv3 --pmc counter collection (all kernels), sorted by
wave cycles: launches, waves per launch, and per-wave counter values.

    python tools/diag/pmc_summary.py run_counter_collection.csv [top]
'''
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name']
        i = k.find('k_')
        key = k[i:k.find('(', i)] if i >= 0 else k[:60]
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'SQ_WAVES':
            launches[key] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0.0))
    for key, d in rows[:top]:
        w = max(d.get('SQ_WAVES', 1.0), 1.0)
        per = ' '.join(f'{c[8:] if c.startswith("SQ_INSTS") else c[3:]}/w {v / w:.0f}'
                       for c, v in sorted(d.items()) if c != 'SQ_WAVES')
        print(f'{key[:48]:48s} launches {launches[key]:6d} waves/launch {w / max(launches[key], 1):8.0f} {per}')


if __name__ == '__main__':
    main()
