"""Instruction mix of one kernel in a hipcc -S device assembly file (measurement aid).

    python tools/isa_stats.py /tmp/mmsbm.s pass_kernelILi10ELi0E [--dump out.s]
"""
import re
import sys

PATTERNS = ["v_mfma", "s_waitcnt", "global_load", "global_store", "ds_read", "ds_write",
            "ds_bpermute", "s_nop", "v_fma_f64", "v_mul_f64", "v_add_f64", "s_cbranch",
            "v_cndmask", "v_accvgpr", "scratch_", "s_barrier", "v_div", "v_rcp_f64"]


def main(path, key, dump=None):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        head = ln.split(";")[0].rstrip()
        if ln.startswith("_Z") and key in head and head.endswith(":"):
            start = i
            break
    if start is None:
        sys.exit("kernel %s not found" % key)
    body = []
    for ln in lines[start:]:
        body.append(ln)
        if "s_endpgm" in ln:
            break
    print("%s: %d lines" % (lines[start].split(":")[0], len(body)))
    for p in PATTERNS:
        n = sum(1 for ln in body if re.search(r"\b" + p, ln))
        if n:
            print("  %-14s %5d" % (p, n))
    if dump:
        with open(dump, "w") as f:
            f.write("\n".join(body))


if __name__ == "__main__":
    a = sys.argv[1:]
    dump = None
    if "--dump" in a:
        i = a.index("--dump")
        dump = a[i + 1]
        del a[i:i + 2]
    main(a[0], a[1], dump)
