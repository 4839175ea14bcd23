mkdir -p gpurun_out
timeout -k 10 300 python scripts/debug/graph_diverge.py > gpurun_out/diverge.log 2>&1; echo rc=$?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_graph -o run --output-format csv -- python bench.py --batch 128 --steps 10 --warmup 3 --graph > gpurun_out/prof_graph.log 2>&1; echo rc=$?
find /tmp/prof_graph -name "*kernel_stats.csv" -exec cp {} gpurun_out/graph_kernel_stats.csv \;
f=$(find /tmp/prof_graph -name "*kernel_trace.csv" | head -1); python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
print('kernels', len(rows))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'][:60]) for r in rows[-400:]]
gaps=[t[i+1][0]-t[i][1] for i in range(len(t)-1)]
print('last400 span us',(t[-1][1]-t[0][0])/1e3,'busy us',sum(e-s for s,e,_ in t)/1e3,'mean gap us',sum(gaps)/len(gaps)/1e3)
" > gpurun_out/graph_gaps.log 2>&1
