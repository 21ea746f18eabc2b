#!/usr/bin/env python3
"""Summarise the `pmc` step of tools/gpu.sh (gpurun_out/OUT/pmc) into profiles/conv_traffic.json.

Per network evaluation (one launch group: the 4-boards-per-workgroup kernel and its three tail
launches, k_net_[yz]<., ., 1..3>, which mostly exit at once; the sums over every dispatch divided
by the number of main launches): HBM-side bytes = 2 x FETCH_SIZE (gfx950 tallies a 16-B/lane streaming
read at half its bytes, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both reported in KB.
FETCH_SIZE also counts Infinity-Cache hits, so this is fabric-side traffic (an upper bound
on HBM bytes).  The L2 hit rate is TCC_HIT / (TCC_HIT + TCC_MISS).
Usage: python tools/pmc_summary.py gpurun_out/pmc [--out profiles/conv_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


KERNELS = set()
MAIN = re.compile(r'k_net_[yz]<false, \d+, 4>')


def read_counters(root):
    """{counter: (sum over every network dispatch, number of main launches)} over every
    counter_collection CSV under root (one pass per counter group)."""
    vals = defaultdict(dict)
    mains = defaultdict(set)
    for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if 'k_net_' not in row.get('Kernel_Name', ''):
                    continue
                KERNELS.update(re.findall(r'k_net_[yz]', row['Kernel_Name']))
                key = (path, row['Dispatch_Id'])
                name = row['Counter_Name']
                vals[name][key] = vals[name].get(key, 0.0) + float(row['Counter_Value'])
                if MAIN.search(row['Kernel_Name']):
                    mains[name].add(key)
    return {k: (sum(v.values()), len(mains[k]), len(v)) for k, v in vals.items()}


def bench_config(root):
    """games / sims of the profiled bench run, from the JSON line in a pass log."""
    logs = glob.glob(os.path.join(root, 'p*.log')) + glob.glob(os.path.join(os.path.dirname(root.rstrip('/')), 'pmc_p*.log'))
    for log in sorted(logs):
        for line in open(log):
            if line.startswith('{') and '"metric"' in line:
                d = json.loads(line)
                return d['config']['games_per_gpu'], d['config']['sims_per_move'], d
    return None, None, None


def bench_hashes(root):
    """The mtaz_src_sha256 of every bench line under `root` (one per PMC pass)."""
    out = set()
    logs = glob.glob(os.path.join(root, 'p*.log')) + glob.glob(os.path.join(os.path.dirname(root.rstrip('/')), 'pmc_p*.log'))
    for log in logs:
        for ln in open(log):
            if ln.startswith('{') and '"mtaz_src_sha256"' in ln:
                out.add(json.loads(ln)['mtaz_src_sha256'])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('--out', default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  'profiles', 'conv_traffic.json'))
    args = ap.parse_args()
    c = read_counters(args.root)
    mean = lambda k: c[k][0] / c[k][1] if c.get(k) and c[k][1] else None   # per evaluation
    fetch_kb, write_kb = mean('FETCH_SIZE'), mean('WRITE_SIZE')
    hit, miss = mean('TCC_HIT_sum'), mean('TCC_MISS_sum')
    mfma, grbm = mean('SQ_VALU_MFMA_BUSY_CYCLES'), mean('GRBM_GUI_ACTIVE')
    wave, wait_any, wait_inst, active = (mean('SQ_WAVE_CYCLES'), mean('SQ_WAIT_ANY'), mean('SQ_WAIT_INST_ANY'),
                                         mean('SQ_ACTIVE_INST_ANY'))
    conf, ldsact = mean('SQ_LDS_BANK_CONFLICT'), mean('SQ_LDS_IDX_ACTIVE')
    games, sims, line = bench_config(args.root)
    out = {
        'kernel': '+'.join(sorted(KERNELS)),
        'games': games, 'sims': sims,
        'dispatches': {k: v[2] for k, v in c.items()},
        'evaluations': {k: v[1] for k, v in c.items()},
        'fetch_size_kb_per_launch': fetch_kb,
        'write_size_kb_per_launch': write_kb,
        'hbm_bytes_per_launch': (2 * fetch_kb + write_kb) * 1024 if fetch_kb is not None and write_kb is not None else None,
        'l2_hit_rate': hit / (hit + miss) if hit is not None and miss else None,
        # MFMA pipe busy per SIMD (SQ_VALU_MFMA_BUSY_CYCLES over the chip's 1024 SIMDs) over the
        # kernel's cycles per XCD (GRBM_GUI_ACTIVE sums the 8 XCDs)
        'mfma_busy_frac': (mfma / 1024) / (grbm / 8) if mfma is not None and grbm else None,
        'sq_wave_cycle_shares': ({'active_inst_any': active / wave, 'wait_inst_any': wait_inst / wave,
                                  'wait_any': wait_any / wave} if wave else None),
        'lds_bank_conflict_frac': conf / ldsact if conf is not None and ldsact else None,
        'method': 'rocprofv3 --pmc, one pass per counter group, --kernel-include-regex k_net_[yz]; per evaluation = '
                  'sums over the main launch and its tail launches / main launches; '
                  'bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 (gfx950 FETCH_SIZE half-count correction); '
                  'mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)',
    }
    if line is not None:
        out['boards_per_launch'] = line['roofline']['flop_per_launch'] / 638245892
        # the library the passes ran (bench.py attaches this file's traffic only to a run of the same one)
        out['mtaz_src_sha256'] = line.get('mtaz_src_sha256')
    hashes = bench_hashes(args.root)
    if len(hashes) > 1:
        raise SystemExit(f'PMC passes ran different libraries: {sorted(hashes)}')
    json.dump(out, open(args.out, 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
