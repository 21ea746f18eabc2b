#!/usr/bin/env python3
"""Per-evaluation summary of a `rocprofv3 --kernel-trace` CSV of bench.py (tools/gpu.sh prof).

For each network build (k_net_y / k_net_z) an evaluation is the 4-boards-per-workgroup launch and
the tail launches after it (<., ., 1..3>, which exit at once unless the remainder has that many
boards per CU).  Reports, per build and per step of the bench run (steps are told apart by the
order of the launches: the main step, then the secondary build, then the default-sims step):
the mean main / tail / total time per evaluation, each tail instance's time when active (> 30 us)
and empty, and the median idle gap before each kernel on the stream.
Usage: python tools/trace_summary.py gpurun_out/OUT/prof/bench_kernel_trace.csv [--out FILE]
"""
import argparse
import collections
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--out')
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    net = re.compile(r'void mtaz::(k_net_[yz])(?:<false, \d+, (\d)>|_tail<\d+>)')
    steps = []        # [(build, [evaluation dicts])]
    tails = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        name, st, en = r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])
        short = re.sub(r'\(.*', '', name).replace('void ', '')
        if prev_end is not None:
            gaps[short].append((st - prev_end) / 1e3)
        prev_end = en
        m = net.match(name)
        if not m:
            continue
        build, nvb = m.group(1), int(m.group(2) or 0)   # 0: k_net_y_tail (the three tail instances)
        dur = (en - st) / 1e3
        if nvb == 4:
            if int(r['Grid_Size_X']) < 256 * 64:    # evaluate() of a few positions (code object load)
                continue
            if not steps or steps[-1][0] != build:
                steps.append((build, []))
            steps[-1][1].append({'main': dur, 'tails': 0.0})
        elif steps and steps[-1][0] == build and steps[-1][1]:
            steps[-1][1][-1]['tails'] += dur
            tails[f'{build}<{nvb}>' if nvb else f'{build}_tail'].append(dur)
    out = {'steps': [], 'tail_instances': {}, 'gap_median_us': {}}
    for build, ev in steps:
        n = len(ev)
        out['steps'].append({'build': build, 'evaluations': n,
                             'main_us': sum(e['main'] for e in ev) / n,
                             'tails_us': sum(e['tails'] for e in ev) / n,
                             'total_us': sum(e['main'] + e['tails'] for e in ev) / n})
    for k, v in sorted(tails.items()):
        act = [x for x in v if x > 30]
        emp = sorted(x for x in v if x <= 30)
        hist = collections.Counter(int(x // 50) * 50 for x in act)
        out['tail_instances'][k] = {'launches': len(v), 'active': len(act),
                                    'active_mean_us': sum(act) / len(act) if act else None,
                                    'active_sum_us': sum(act),
                                    'empty_median_us': emp[len(emp) // 2] if emp else None,
                                    # active launches by duration (50-us bins: the 1-, 2- and 3-board
                                    # instances fall in separate clusters)
                                    'active_hist_50us': {str(b): hist[b] for b in sorted(hist)}}
    for k, v in gaps.items():
        if len(v) >= 100:
            out['gap_median_us'][k] = sorted(v)[len(v) // 2]
    s = json.dumps(out, indent=1)
    if args.out:
        open(args.out, 'w').write(s + '\n')
    print(s)


if __name__ == '__main__':
    main()
