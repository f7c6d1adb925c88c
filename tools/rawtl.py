"""Raw kernel-trace listing around the start of the last solve in a rocprofv3
kernel trace (every dispatch, all queues).  usage: rawtl.py <trace dir>"""
import csv,glob,sys
f=glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True)[0]
rows=list(csv.DictReader(open(f)))
print(list(rows[0].keys()))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
inits=[i for i,r in enumerate(rows) if 'k_init' in r['Kernel_Name']]
i0=inits[-4]  # last solve's first init
t0=int(rows[i0]["Start_Timestamp"])
for r in rows[i0-10:i0+40]:
    print("%-40s q=%s start %9.1f end %9.1f"%(r['Kernel_Name'][:40], r.get('Queue_Id','?'), (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-t0)/1e3))
