'''
GPU busy fraction of a rocprofv3 kernel trace (--kernel-trace, csv): the union of all kernel intervals
against the span from the first kernel start to the last kernel end, overall and in windows; the top
kernels by time. Used to tell a host-bound solve (gaps between launches) from a device-bound one.

    python tools/diag/busy_fraction.py DIR/run_kernel_trace.csv [--windows 10]
'''
import csv
import sys

import numpy as np


def main():
    path = sys.argv[1]
    nwin = int(sys.argv[sys.argv.index('--windows') + 1]) if '--windows' in sys.argv else 10
    st, en, names = [], [], []
    with open(path, newline='') as fh:
        for r in csv.DictReader(fh):
            st.append(int(r['Start_Timestamp']))
            en.append(int(r['End_Timestamp']))
            names.append(r['Kernel_Name'][:60])
    st, en = np.array(st), np.array(en)
    o = np.argsort(st)
    st, en = st[o], en[o]
    # union of intervals
    busy = 0
    cur_s, cur_e = st[0], en[0]
    edges = []
    for a, b in zip(st[1:], en[1:]):
        if a > cur_e:
            busy += cur_e - cur_s
            edges.append((cur_s, cur_e))
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    busy += cur_e - cur_s
    edges.append((cur_s, cur_e))
    span = en.max() - st.min()
    print(f'kernels {len(st)}, span {span / 1e9:.3f} s, busy {busy / 1e9:.3f} s, busy fraction {busy / span:.3f}')
    t0 = st.min()
    w = span / nwin
    for i in range(nwin):
        a, b = t0 + i * w, t0 + (i + 1) * w
        bb = sum(max(0, min(e, b) - max(s, a)) for s, e in edges)
        print(f'  window {i}: busy {bb / w:.3f}')


if __name__ == '__main__':
    main()
