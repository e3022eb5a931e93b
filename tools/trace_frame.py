"""Print the kernels of one steady-state frame from a rocprofv3 kernel trace (start offset, duration,
queue, name, grid): tools/trace_frame.py gpurun_out/prof/run_kernel_trace.csv [frame_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 500
idx = [i for i, r in enumerate(rows) if 'PredictTail' in r['Kernel_Name']]   # stage B head
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    nm = r['Kernel_Name'].replace('pf::(anonymous namespace)::', '').split('(')[0]
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:6.1f} q{r['Queue_Id']} {nm[:40]:40s} grid={r['Grid_Size_X']}")
