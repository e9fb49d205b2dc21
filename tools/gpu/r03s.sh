# per-task k_prep counters (BGV_PREP_SPLIT=1: three launches) over the isolated roofline call
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
export TMPDIR=/tmp BGV_PREP_SPLIT=1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 tools/gpu/roof_call.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/gpu/roof_call.py > $O/trace.log 2>&1 || exit 1
python - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.defaultdict(set)
for path in glob.glob('gpurun_out/r03s/p*/**/*counter_collection*.csv', recursive=True):
    for r in csv.DictReader(open(path)):
        k=r['Kernel_Name'].split('(')[0]
        if k!='k_prep': continue
        key=(r['Dispatch_Id'], r['Grid_Size'] if 'Grid_Size' in r else '')
        acc[r['Dispatch_Id']][r['Counter_Name']]+=float(r['Counter_Value'] or 0)
for d,c in sorted(acc.items(), key=lambda kv:int(kv[0])):
    w=c.get('SQ_WAVES',0) or 1
    print(d, {k:round(v/1e9,3) if 'SIZE' in k else round(v/w) for k,v in c.items()})
for r in csv.DictReader(open(glob.glob('gpurun_out/r03s/trace/**/*kernel_trace.csv',recursive=True)[0])):
    if r['Kernel_Name'].startswith('k_prep'): print('trace', r['Kernel_Name'][:8], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6)
PY
