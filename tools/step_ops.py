"""Per-launch list of the last bench step in a rocprofv3 kernel trace (tools/step_pmc.py run):
queue, start / end relative to the step's log-mel launch, duration, kernel, grid, LDS, VGPRs.
usage: python tools/step_ops.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if 'logmel' in r['Kernel_Name']]
win = rows[starts[-1]:]
t0 = int(win[0]['Start_Timestamp'])
tot = 0.0
for r in win:
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    tot += e - s
    n = r['Kernel_Name'].split('(')[0].replace('void a2m::', '').replace('a2m::', '')
    g = int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])
    print(f"q{r['Queue_Id']} {s:8.1f} {e:8.1f} {e - s:7.1f}  {n[:44]:44s} grid={g}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} "
          f"wg={r['Workgroup_Size_X']} lds={r['LDS_Block_Size']} v={r['VGPR_Count']}")
print(f'kernel sum {tot:.1f} us, window {(int(win[-1]["End_Timestamp"]) - t0) / 1e3:.1f} us')
