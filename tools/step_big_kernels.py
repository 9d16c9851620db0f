"""Big kernels (>= 1000 workgroups, heads, offset conv) of one graph-replayed bench step from a rocprofv3
kernel trace: start / end us, queue, workgroups.  Usage: python tools/step_big_kernels.py TRACE.csv"""
import csv, sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'corr_pyramid_reg' in r['Kernel_Name'] and i+1<len(rows) and 'corr_pyramid' not in rows[i+1]['Kernel_Name']]
i0,i1=idx[-3],idx[-2]
t0=int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i1]:
    n=r['Kernel_Name'].replace('(anonymous namespace)::','').replace('void ','')[:46]
    g=1
    for a,b in (('Grid_Size_X','Workgroup_Size_X'),('Grid_Size_Y','Workgroup_Size_Y')): g*=max(1,int(r[a])//max(1,int(r[b])))
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    if g>=1000 or 'rows_kernel<6' in n or 'g3' in n:
        print(f"{s:8.1f} {e:8.1f} q{r['Queue_Id']} {g:5d} {n}")
print((int(rows[i1]['Start_Timestamp'])-t0)/1e3)
