"""profiles/pmc_<round>_K<K>.json from a `tools/gpu.sh TAG prof` output directory: HBM bytes per
launch of each kernel of the iteration = 2 x FETCH_SIZE (gfx950: FETCH_SIZE tallies 128-B requests
at 64 B, MI355X_MICROARCH.md) + WRITE_SIZE, both in KiB per dispatch, averaged over the dispatches
of the PMC passes.  The record is stamped with the build id of the library the passes ran (the
`build_id` field of the bench lines they printed, which must all agree): bench.py only reports a
record whose build id equals its own library's.
usage: python tools/pmc_to_traffic.py gpurun_out/<tag> K E_obs B out.json  (from tools/gpu_r03_prof.sh)"""
import collections
import csv
import glob
import json
import sys

NAMES = {"pass_kernel<%d, 0>": "pass_a", "gene_kernel<%d>": "gene", "upd_kernel<%d, false>": "fin",
         "gm_kernel<%d>": "gene",  # (large-K X rows + S partials, round 5: the gene label)
         "ysum_kernel<%d>": "ysum",  # (large-K Y sums, on a second stream beside gene_kernel)
         "gene_sy_kernel<%d>": "gene_sy",  # (large-K S + Y workgroups, the gene label's second launch)
         # small-K kernels (csrc/sk.h), labelled as EMEngine.LABELS names them
         "sky_pass_kernel<%d>": "fused", "sk_pass_kernel<%d, 3>": "fused", "sk_pass_kernel<%d, 0>": "pass_a",
         "sk_pass_kernel<%d, 2>": "pass_b", "sk_fin_kernel<%d, false>": "fin"}


def main(root, K, E_obs, B, out):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    ids = set()
    for f in sorted(glob.glob(root + "/p*.log")):
        for line in open(f, errors="replace"):
            if line.startswith("{") and '"build_id"' in line:
                ids.add(json.loads(line)["build_id"])
    if len(ids) != 1:
        sys.exit("pmc_to_traffic: expected one build id in %s/p*.log, found %s" % (root, sorted(ids)))
    rec = {"K": K, "E_obs": E_obs, "B": B, "source": root, "build_id": ids.pop(),
           "hbm_bytes_per_launch": {}, "counters": {}}
    for pat, key in NAMES.items():
        cs = acc.get(pat % K)
        if not cs:
            continue
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        rec["counters"][key] = mean
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            rec["hbm_bytes_per_launch"][key] = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
    hb = rec["hbm_bytes_per_launch"]
    # the gene label = gene_kernel + the S / Y launches beside or after it
    extra = [k for k in ("ysum", "gene_sy") if k in hb]
    if extra and "gene" in hb:
        hb["gene_kernel_only"] = hb["gene"]
        hb["gene"] += sum(hb[k] for k in extra)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)
    print(json.dumps(rec["hbm_bytes_per_launch"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
