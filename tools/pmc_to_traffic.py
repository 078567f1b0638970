"""profiles/pmc_<round>_K<K>.json from a `tools/gpu.sh TAG prof` output directory: per launch of
each kernel of the iteration, the bytes the XCD L2s exchanged with the fabric, from the PMC
counters FETCH_SIZE and WRITE_SIZE (KiB per dispatch, averaged over the PMC passes' dispatches).

What the figure is (MI355X_MICROARCH.md, FETCH_SIZE):
  * L2 -> fabric bytes, NOT HBM bytes: Infinity-Cache (MALL) hits are counted too;
  * gfx950's FETCH_SIZE tallies the 128-B requests of a wide coalesced streaming read (16 B per
    lane) at 64 B, so FETCH is doubled only for the kernels whose reads are such streams
    (WIDE_STREAM below: gm_kernel stages its partial-row tiles 16 B per lane); every other
    kernel's reads are 8-byte gathers / 4-16-byte record loads, an uncalibrated width, and its
    FETCH is taken as counted (a lower bound if those requests are also tallied at half);
  * beside it, per kernel, the raw counters and the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS).
The record is stamped with the build id of the library the passes ran (the `build_id` field of
the bench lines they printed, which must all agree): bench.py only reports a record whose build
id equals its own library's.
usage: python tools/pmc_to_traffic.py gpurun_out/<tag> K E_obs B out.json"""
import collections
import csv
import glob
import json
import sys

NAMES = {"pass_kernel<%d, 0>": "pass_a", "upd_kernel<%d, false>": "fin",
         # (large-K X rows + S partials; workgroups per part 1-4, X layout halves / GM::Q4)
         **{"gm_kernel<%%d, %d%s>" % (cs, q): "gene" for cs in (1, 2, 3, 4) for q in ("", ", false", ", true")},
         # small-K kernels (csrc/sk.h), labelled as EMEngine.LABELS names them
         "sky_pass_kernel<%d>": "fused", "sk_pass_kernel<%d, 3>": "fused", "sk_pass_kernel<%d, 0>": "pass_a",
         "sk_pass_kernel<%d, 2>": "pass_b", "sk_fin_kernel<%d, false>": "fin"}


# kernels whose reads are wide coalesced streams (16 B per lane): FETCH_SIZE x 2
WIDE_STREAM = {"gene"}


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
           "basis": "L2->fabric bytes (FETCH_SIZE + WRITE_SIZE; Infinity-Cache hits included); FETCH "
                    "doubled for the wide-stream kernels %s only" % sorted(WIDE_STREAM),
           "l2_fabric_bytes_per_launch": {}, "fetch_doubled": {}, "tcc_hit_rate": {}, "counters": {}}
    for pat, key in NAMES.items():
        cs = acc.get(pat % K)
        if not cs or key in rec["counters"]:
            continue
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        rec["counters"][key] = mean
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            wide = key in WIDE_STREAM
            rec["fetch_doubled"][key] = wide
            rec["l2_fabric_bytes_per_launch"][key] = ((2.0 if wide else 1.0) * mean["FETCH_SIZE"]
                                                      + mean["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean and mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"] > 0:
            rec["tcc_hit_rate"][key] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
    with open(out, "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)
    print(json.dumps({"l2_fabric_bytes_per_launch": rec["l2_fabric_bytes_per_launch"],
                      "tcc_hit_rate": rec["tcc_hit_rate"]}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
