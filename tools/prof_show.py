import csv, glob, sys
for d in sorted(glob.glob("gpurun_out/%s/*/" % sys.argv[1])):
    f = glob.glob(d + "run_kernel_stats.csv")
    if not f: continue
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = []
    for r in rows:
        name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if "estep" in name or "mstep" in name or "loglik" in name:
            out.append("%s %.2fus x%s" % (name, float(r["AverageNs"]) / 1e3, r["Calls"]))
    print(d.split("/")[-2], " | ".join(out))
