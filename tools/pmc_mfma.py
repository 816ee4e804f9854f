"""MFMA-busy fraction per kernel from rocprofv3 --pmc counter files (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE; GRBM counts per XCD (8), MFMA busy per SIMD (1024 on MI355X))."""
import csv, glob, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for pat in sys.argv[1:]:
    for f in glob.glob(pat):
        for r in csv.DictReader(open(f)):
            agg[r['Kernel_Name'][:60]][r['Counter_Name']].append(float(r['Counter_Value']))
mean = lambda v: sum(v) / len(v) if v else 0.0
for k, cs in agg.items():
    g, mb, mi = mean(cs['GRBM_GUI_ACTIVE']), mean(cs['SQ_VALU_MFMA_BUSY_CYCLES']), mean(cs['SQ_INSTS_MFMA'])
    if not g or not mi:
        continue
    print(f'{k:60s} MFMA busy {100 * mb / 1024 / (g / 8):5.1f}%   VALU/MFMA {mean(cs["SQ_INSTS_VALU"]) / mi:5.1f}')
