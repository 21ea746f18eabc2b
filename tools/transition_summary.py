#!/usr/bin/env python3
"""Move transitions in a rocprofv3 kernel trace of bench.py: from each k_move_end's start to the
start of the next k_select (the device side of a move boundary: root visit counts back to the host,
action choice, k_apply, the next move's k_move_begin and first chunk of Dirichlet draws), and the
median network launch of the same trace (to compare boxes).

Usage: python tools/transition_summary.py gpurun_out/<run>/prof/bench_kernel_trace.csv [--out f.json]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])
                for r in csv.DictReader(open(args.trace)))
    trans = []
    for i, (s, _e, n) in enumerate(ev):
        if 'k_move_end' not in n:
            continue
        j = i + 1
        while j < len(ev) and 'k_select' not in ev[j][2]:
            j += 1
        if j < len(ev):
            trans.append((ev[j][0] - s) / 1e3)
    trans = [t for t in trans if t < 100e3]   # a gap past 100 ms is a phase change (next play, next leg)
    net = sorted((e - s) / 1e3 for s, e, n in ev if 'k_net_y<' in n)
    srt = sorted(trans)
    res = {'transitions': len(trans), 'median_us': srt[len(srt) // 2] if srt else None,
           'sum_ms': sum(trans) / 1e3, 'net_main_median_us': net[len(net) // 2] if net else None}
    print(json.dumps(res))
    if args.out:
        with open(args.out, 'w') as fh:
            json.dump(res, fh, indent=1)


if __name__ == '__main__':
    main()
