'''
DIAGNOSTIC: per-launch averages of rocprofv3 --pmc counters for the KKT factor kernels.

    python tools/diag/pmc_kernels.py gpurun_out/<run>/pmc_x/run_counter_collection.csv [...]
'''
import collections
import csv
import sys


def main():
    for path in sys.argv[1:]:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            k = r['Kernel_Name']
            if 'k_front_factor' not in k:
                continue
            i = k.index('k_front_factor')
            key = k[i:k.index('(', i)]
            agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
        print(path)
        for key, d in sorted(agg.items()):
            w = sum(d['SQ_WAVES']) / len(d['SQ_WAVES']) if 'SQ_WAVES' in d else 1.0
            per_wave = {c: f'{sum(v) / len(v) / w:.0f}' for c, v in d.items() if c != 'SQ_WAVES'}
            print(f'  {key:36s} waves {w:8.0f} per wave {per_wave}')


if __name__ == '__main__':
    main()
