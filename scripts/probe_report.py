#!/usr/bin/env python3
"""Per-dispatch PMC report for scripts/otr_rounds_probe.py runs."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.OrderedDict()
for r in rows:
    if 'otr_kernel' not in r['Kernel_Name']:
        continue
    d.setdefault(int(r['Dispatch_Id']), {})[r['Counter_Name']] = float(r['Counter_Value'])
cfgs = [(V, R) for V in (64, 2) for R in (1, 2, 4, 20, 40)]
I = 2e6
for (V, R), (k, v) in zip(cfgs, sorted(d.items())):
    print(f"V={V:2d} R={R:2d} SALU/inst={v['SQ_INSTS_SALU']/I:8.1f} VALU/inst={v['SQ_INSTS_VALU']/I:8.1f} "
          f"LDS/inst={v.get('SQ_INSTS_LDS',0)/I:6.1f} cyc={v['GRBM_GUI_ACTIVE']/8/1e6:7.2f}M")
