"""Timeline of the whole-call kernels in a rocprofv3 kernel trace (csv):
name, queue, stream, grid, start / end / duration in ms after the first.
usage: python tools/kernel_timeline.py run_kernel_trace.csv [min duration ms]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wf_" in r["Kernel_Name"] and "<true>" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in rows:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > lo:
        print(f'{r["Kernel_Name"].split("(")[0][-22:]:24s} q{r["Queue_Id"]} s{r["Stream_Id"]} g{r["Grid_Size_X"]:>7s} '
              f'{s:10.2f} {e:10.2f} {e - s:8.2f}')
