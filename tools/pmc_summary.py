"""Average rocprofv3 PMC counters per kernel over a set of pass directories."""
import collections
import csv
import glob
import sys

def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in sorted(glob.glob(root + "/p*/run_kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    for k, cs in acc.items():
        d = dur.get(k, [0])
        print("== %s  (avg dur %.2f us over %d)" % (k, sum(d) / len(d) / 1e3, len(d)))
        for c, v in sorted(cs.items()):
            print("   %-28s %14.1f" % (c, sum(v) / len(v)))

main(sys.argv[1])
