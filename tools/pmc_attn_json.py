"""Summarise the PMC passes of tools/pmc_attn.sh (rocprofv3 --pmc over tools/attn_bench.py at one layer shape) into
profiles/<round>/pmc_attn_<config>.json, which bench.py reports beside the algorithmic attention fraction.

    python tools/pmc_attn_json.py CONFIG OUT.json gpurun_out/pmc_attn_*/run_counter_collection.csv

Per attention kernel (mean over its launches): MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
1024 SIMDs) (SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs), and VALU
instructions per MFMA instruction (SQ_INSTS_VALU counts the MFMAs too: both forms are given)."""
import collections
import csv
import json
import sys


def main():
    config, out = sys.argv[1], sys.argv[2]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sys.argv[3:]:
        for r in csv.DictReader(open(f)):
            name = r.get('Kernel_Name') or r.get('Kernel-Name') or r.get('KernelName')
            if 'attn' not in name:
                continue
            agg[name.split('(')[0].replace('void ', '')][r['Counter_Name']].append(float(r['Counter_Value']))
    res = {'config': config, 'kernels': {}}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {}
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in m and m.get('GRBM_GUI_ACTIVE'):
            e['mfma_busy'] = round(m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024), 4)
        if m.get('SQ_INSTS_MFMA'):
            v = m.get('SQ_INSTS_VALU', 0.0)
            e['valu_per_mfma_incl'] = round(v / m['SQ_INSTS_MFMA'], 2)
            e['valu_per_mfma_excl'] = round((v - m['SQ_INSTS_MFMA']) / m['SQ_INSTS_MFMA'], 2)
        e['counters'] = {c: round(x, 1) for c, x in sorted(m.items())}
        res['kernels'][k] = e
    json.dump(res, open(out, 'w'), indent=1)
    for k, e in res['kernels'].items():
        print(k, {x: y for x, y in e.items() if x != 'counters'})


if __name__ == '__main__':
    main()
