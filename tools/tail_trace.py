import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if 'many_kernel' in r['Kernel_Name'] or 'tail' in r['Kernel_Name']]
out = collections.defaultdict(list)
for r in sel:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
    out[(r['Kernel_Name'][:40], r.get('Grid_Size_X', r.get('Grid_Size','')))].append(d)
for k, v in sorted(out.items()):
    v.sort()
    print(k, len(v), 'median %.1f' % v[len(v)//2], 'min %.1f' % v[0])
