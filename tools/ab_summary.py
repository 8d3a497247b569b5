'''
One line per solver A/B arm (tools/solver_ab.py JSON files): fig-8 cold starts (status, iterations, lap)
and the config-3 batch (statuses, median iterations, restorations, watchdog, solve time).

    python tools/ab_summary.py gpurun_out/r06a/abl_1.json gpurun_out/r06b/abl_1.json
'''
import json
import sys


def line(path):
    d = json.load(open(path, encoding='utf-8'))
    out = [f"{path}: tag={d.get('tag')!r}"]
    for k in ('fig8_cold_quat', 'fig8_cold_quat_K4', 'fig8_cold_euler'):
        if k in d:
            v = d[k]
            st = v.get('stats', {})
            out.append(f"  {k}: {v['status']} it={v['iterations']} lap={v['lap_s']:.4f} resto={st.get('restorations')} "
                       f"wd={st.get('watchdog')} solve={v['solve_s']:.1f}s")
    if 'config3' in d:
        c = d['config3']
        out.append(f"  config3: {c['statuses']} median_it={c['iterations']['median']} sum_it={c['iterations']['sum']} "
                   f"resto={c['restorations']} wd={c['watchdog']} soft={c['soft_resto']} fact={c['factorizations']} "
                   f"solve={c['solve_s']:.1f}s it/s={c['instance_iterations_per_s']:.0f} "
                   f"lap_med={(c.get('lap_converged') or {}).get('median')}")
    return '\n'.join(out)


if __name__ == '__main__':
    for p in sys.argv[1:]:
        print(line(p))
