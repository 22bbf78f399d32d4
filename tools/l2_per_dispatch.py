import csv, sys, collections
f = sys.argv[1]
rows = list(csv.DictReader(open(f)))
d = collections.OrderedDict()
for r in rows:
    key = int(r['Dispatch_Id'])
    e = d.setdefault(key, {'k': r['Kernel_Name'], 'grid': r.get('Grid_Size', ''), 'HIT': 0.0, 'MISS': 0.0})
    if 'HIT' in r['Counter_Name']: e['HIT'] += float(r['Counter_Value'])
    else: e['MISS'] += float(r['Counter_Value'])
for k, e in d.items():
    if 'als_solve_mfma' not in e['k']: continue
    name = e['k'].split('als_solve_mfma')[1].split('(')[0]
    tot = e['HIT'] + e['MISS']
    if tot < 1e6: continue
    print(k, name, e['grid'], round(e['HIT'] / tot, 3), round(tot / 1e6, 1))
