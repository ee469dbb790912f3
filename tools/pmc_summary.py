import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if sys.argv[2] in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']] += float(r['Counter_Value'])
d = dict(agg)
print(d)
if 'SQ_THREAD_CYCLES_VALU' in d and 'SQ_ACTIVE_INST_VALU' in d:
    print('VALU lane utilisation %.1f%%' % (100 * d['SQ_THREAD_CYCLES_VALU'] / (64 * d['SQ_ACTIVE_INST_VALU'])))
if 'SQ_WAIT_ANY' in d and 'SQ_WAVE_CYCLES' in d:
    print('wait fraction %.1f%%' % (100 * d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']))
