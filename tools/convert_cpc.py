'''
One-time asset conversion (build container): the reference's CPC trajectory CSVs
(drone3d/assets/cpc_{race,warmstart}_raceline.csv, produced by the CPC planner) are copied into
the package's assets with the 14 columns utils/cpc_utils.py reads (t, p, q, v, w), text unchanged.

    python tools/convert_cpc.py [/root/reference/drone3d/assets]
'''
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/drone3d/assets'
    dst = os.path.join(ROOT, 'aircraft_trajectory_optimization_amd', 'assets')
    for name in ('cpc_race_raceline.csv', 'cpc_warmstart_raceline.csv'):
        with open(os.path.join(src, name), encoding='utf-8') as f:
            lines = [','.join(line.strip().split(',')[:14]) for line in f if line.strip()]
        with open(os.path.join(dst, name), 'w', encoding='utf-8') as f:
            f.write('\n'.join(lines) + '\n')
        print(name, len(lines) - 1, 'rows')


if __name__ == '__main__':
    main()
