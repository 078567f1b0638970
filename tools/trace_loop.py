"""Median in-loop and back-to-back kernel durations from a rocprofv3 kernel trace CSV.

usage: python tools/trace_loop.py <run_kernel_trace.csv>
In-loop = an E-step launch that follows an M2 launch (and that M2); back to back = an E-step
launch that follows another E-step launch (bench.py's roofline launches).
"""
import csv
import statistics
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
is_e = lambda n: any(k in n for k in ("emx_kernel", "eml_kernel", "emb_kernel", "estep"))
is_m2 = lambda n: "m2_kernel" in n
us = lambda r: (r[1] - r[0]) / 1e3
loop = [i for i in range(1, len(rows)) if is_e(rows[i][2]) and is_m2(rows[i - 1][2])]
b2b = [i for i in range(1, len(rows)) if is_e(rows[i][2]) and is_e(rows[i - 1][2])]
if loop:
    print("in loop: E %.2f us, M2 %.2f us, period %.2f us (%d iterations)" % (
        statistics.median(us(rows[i]) for i in loop),
        statistics.median(us(rows[i - 1]) for i in loop),
        statistics.median((rows[i][0] - rows[j][0]) / 1e3 for i, j in zip(loop[1:], loop[:-1])),
        len(loop)))
if b2b:
    print("back to back: E %.2f us (%d launches)" % (statistics.median(us(rows[i]) for i in b2b), len(b2b)))
