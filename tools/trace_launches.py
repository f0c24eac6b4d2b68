#!/usr/bin/env python3
"""Per-dispatch view of a rocprofv3 kernel trace: for every launch of the kernels matching a
substring, its grid (workgroups -> waves), duration and ns per wave, in dispatch order.
--step: only the last parsimony run (after the second-to-last k_site_score); --last N: the last
N matching launches; --summary: per-kernel launches / time / waves instead of every launch.

    tools/trace_launches.py DIR/.../kernel_trace.csv [substring] [--step] [--last N] [--summary]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"\b(k_\w+(<[^(]*>)?)", name)
    return (m.group(0) if m else name[:40]).replace("(pm::Mode)", "M")


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "k_"
    last = 0
    if "--last" in sys.argv:
        last = int(sys.argv[sys.argv.index("--last") + 1])
    rows = list(csv.DictReader(open(path)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start Timestamp"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End Timestamp"
    rows.sort(key=lambda r: int(r[key_s]))
    if "--step" in sys.argv:   # one parsimony run: after the second-to-last k_site_score up to the last
        marks = [i for i, r in enumerate(rows) if "k_site_score" in r["Kernel_Name"]]
        rows = rows[marks[-2] + 1: marks[-1] + 1] if len(marks) >= 2 else rows
    sel = [r for r in rows if want in r["Kernel_Name"]]
    if last:
        sel = sel[-last:]
    if "--summary" in sys.argv:
        agg = {}
        for r in sel:
            k = short(r["Kernel_Name"])
            a = agg.setdefault(k, [0, 0.0, 0])
            a[0] += 1
            a[1] += (int(r[key_e]) - int(r[key_s])) / 1e3
            a[2] += int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) // 64
        for k, (n, us, w) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{k:48s} launches {n:4d}  {us:9.1f} us  waves {w:9d}")
        print(f"total {sum(a[1] for a in agg.values()):.1f} us over {sum(a[0] for a in agg.values())} launches")
        return
    tot = 0.0
    for r in sel:
        dur = (int(r[key_e]) - int(r[key_s])) / 1e3
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
        waves = gx // 64 if gx else 0
        tot += dur
        per = dur * 1e3 / waves if waves else 0.0
        print(f"{short(r['Kernel_Name']):44s} grid {gx:10d} wg {wx:5d} waves {waves:9d} {dur:9.1f} us {per:7.3f} ns/wave "
              f"vgpr {r.get('Arch_VGPR_Count', r.get('VGPR_Count', '?'))} lds {r.get('LDS_Block_Size', r.get('LDS_Size', '?'))}")
    print(f"total {tot:.1f} us over {len(sel)} launches")


if __name__ == "__main__":
    main()
