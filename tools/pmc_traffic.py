'''
HBM traffic of k_eval from rocprofv3 PMC passes, calibrated on known-byte kernels.

Inputs (gpu_check.sh steps `pmc` and `mbpmc` of one run directory):
  pmc_fetch/run_counter_collection.csv   FETCH_SIZE per dispatch (KB) of bench.py
  pmc_write/run_counter_collection.csv   WRITE_SIZE per dispatch (KB) of bench.py
  mb_fetch/, mb_write/                   the same counters on tools/mb_store:
      kE reads exactly 64 MiB with 8-byte-per-lane loads (k_eval's load width)
      kA writes exactly 252.7 MB with 8-byte-per-lane row stores
MI355X_MICROARCH.md: FETCH_SIZE under-reports wide coalesced reads by 2x on gfx950 and other
access widths are uncalibrated -- so the factor is measured here for our width.

    python tools/pmc_traffic.py gpurun_out/r01i [--write profiles/traffic_latest.json]
'''
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path, encoding='utf-8') as fh:
        for r in csv.DictReader(fh):
            if r['Counter_Name'] == counter:
                vals[r['Kernel_Name']].append(float(r['Counter_Value']))
    return vals


def mean_of(vals, key):
    xs = [v for k, lst in vals.items() if key in k for v in lst]
    return sum(xs) / len(xs) if xs else None


def main():
    run = sys.argv[1]
    out = sys.argv[sys.argv.index('--write') + 1] if '--write' in sys.argv else None
    kb = 1024.0
    e_fetch = mean_of(per_kernel(f'{run}/mb_fetch/run_counter_collection.csv', 'FETCH_SIZE'), 'kE')
    a_write = mean_of(per_kernel(f'{run}/mb_write/run_counter_collection.csv', 'WRITE_SIZE'), 'kA')
    known_read = 64 * 1024 * 1024 * 8 / 8 * 1.0       # 8 Mi doubles = 64 MiB
    known_write = 701 * 88 * 512 * 8.0
    fetch_factor = known_read / (e_fetch * kb)
    write_factor = known_write / (a_write * kb)
    f = mean_of(per_kernel(f'{run}/pmc_fetch/run_counter_collection.csv', 'FETCH_SIZE'), 'k_eval')
    w = mean_of(per_kernel(f'{run}/pmc_write/run_counter_collection.csv', 'WRITE_SIZE'), 'k_eval')
    fetch_bytes = f * kb * fetch_factor
    write_bytes = w * kb * write_factor
    res = {
        'kernel': 'k_eval_paired (racetrack 50x4x13, B=512, fp64, interleaved)',
        'batch': 512, 'dtype': 'f64', 'layout': 'interleaved',
        'fetch_size_kb_raw': f, 'write_size_kb_raw': w,
        'calibration': {'fetch_factor_8B_lane': fetch_factor, 'write_factor_8B_lane': write_factor,
                        'kE_fetch_kb': e_fetch, 'kA_write_kb': a_write},
        'hbm_read_bytes_per_launch': fetch_bytes,
        'hbm_write_bytes_per_launch': write_bytes,
        'hbm_bytes_per_launch': fetch_bytes + write_bytes,
        'note': 'FETCH_SIZE counts L2->fabric read requests (Infinity Cache hits included); '
                'factors measured on known-byte kernels of the same access width',
    }
    print(json.dumps(res, indent=1))
    if out:
        with open(out, 'w', encoding='utf-8') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
