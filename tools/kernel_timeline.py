import csv,sys,glob,os
for d in sorted(glob.glob(sys.argv[1]+'/c*_*/')):
    rows=list(csv.DictReader(open(d+'run_kernel_trace.csv')))
    rows=[r for r in rows if 'k_replay' in r['Kernel_Name'] or 'k_tables' in r['Kernel_Name'] or 'k_finalize' in r['Kernel_Name']]
    fin=[i for i,r in enumerate(rows) if 'k_finalize' in r['Kernel_Name']]
    last=rows[fin[-2]+1:fin[-1]+1]
    t0=min(int(r['Start_Timestamp']) for r in last)
    print(os.path.basename(d[:-1]), ' '.join(f"{r['Kernel_Name'].replace('void k_replay_','').replace('(cdr_launch)','').replace('k_replay_','')[:22]}:{(int(r['Start_Timestamp'])-t0)/1e6:.1f}-{(int(r['End_Timestamp'])-t0)/1e6:.1f}" for r in last if 'replay' in r['Kernel_Name']))
