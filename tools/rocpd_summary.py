#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite output (run_results.db): per-kernel dispatch
statistics and, for --pmc runs, per-dispatch counter sums.

usage: rocpd_summary.py DB [DB ...]   (prints CSV-like text)
"""
import sqlite3
import sys
from collections import defaultdict


def summarise(path):
    c = sqlite3.connect(path)
    names = dict(c.execute("select id, display_name from rocpd_info_kernel_symbol"))
    rows = list(c.execute("select id, kernel_id, start, end, event_id, grid_size_x, workgroup_size_x "
                          "from rocpd_kernel_dispatch"))
    dur = defaultdict(list)
    for _, k, s, e, _, _, _ in rows:
        dur[names.get(k, str(k))].append((e - s) * 1e-3)  # ns -> us
    print("# %s" % path)
    print("kernel,calls,total_us,avg_us,min_us,max_us")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print('"%s",%d,%.1f,%.2f,%.2f,%.2f' % (k, len(v), sum(v), sum(v) / len(v), min(v), max(v)))
    pmc = dict(c.execute("select id, name from rocpd_info_pmc"))
    ev = defaultdict(lambda: defaultdict(float))
    for eid, pid, val in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        ev[eid][pmc.get(pid, str(pid))] += val
    if ev:
        per = defaultdict(lambda: defaultdict(list))
        for _, k, _, _, eid, _, _ in rows:
            for n, v in ev.get(eid, {}).items():
                per[names.get(k, str(k))][n].append(v)
        print("kernel,counter,dispatches,avg_per_dispatch,min,max")
        for k, d in per.items():
            for n, v in d.items():
                print('"%s",%s,%d,%.6g,%.6g,%.6g' % (k, n, len(v), sum(v) / len(v), min(v), max(v)))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        summarise(p)
