"""Per-wave analysis of a raw s_memtime stamp dump (measurement build, MMSBM_STAMP_DUMP=path).

Layout: u64[5 kernels][65536 waves][8 slots]; slots 0-3 = phase boundaries, 6 = pass prologue loads staged, 4 = genes of the
wave's workgroup (stream-0 passes), 5 = chunks of the wave's unit.
"""
import sys

import numpy as np

NAMES = ["passA", "passB", "fin", "spart", "passLL"]


def main(path, bench_json=None):
    n_wg0 = None
    if bench_json:  # the bench line of the same run: stream-0 workgroups come first in the grid
        import json
        line = open(bench_json).read().strip().splitlines()[-1]
        n_wg0 = json.loads(line)["plan"].get("wg_stream0")
    h = np.fromfile(path, dtype=np.uint64).reshape(5, 1 << 16, 10).astype(np.int64)
    for k, name in enumerate(NAMES):
        t = h[k]
        ok = t[:, 0] != 0
        if not ok.any():
            continue
        idx = np.nonzero(ok)[0]
        t = t[ok]
        t0 = t[:, 0].min()
        start, end = t[:, 0] - t0, t[:, 3] - t0
        life = t[:, 3] - t[:, 0]
        ph1, ph2 = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1]
        q = lambda a: " ".join("%6d" % v for v in np.percentile(a, [0, 50, 90, 99, 100]))
        print("%s: %d waves   (percentiles 0/50/90/99/100)" % (name, len(t)))
        print("  start  %s" % q(start))
        print("  end    %s" % q(end))
        print("  life   %s" % q(life))
        print("  phase1 %s" % q(ph1))
        print("  phase2 %s" % q(ph2))
        if name == "fin" and (t[:, 9] != 0).all():
            # small-K fin (sk_fin_kernel): chip-wide start / end against the E-step launch's waves
            # (the same 100 MHz clock): the gap between the two launches and fin's own span
            ea = h[0]
            ea = ea[ea[:, 0] != 0]
            rt0 = ea[:, 8].min() if len(ea) else t[:, 8].min()
            e_end = ea[:, 9].max() if len(ea) else rt0
            print("  start (ns from the E-step's first wave) %s" % q((t[:, 8] - rt0) * 10))
            print("  end   (ns from the E-step's first wave) %s" % q((t[:, 9] - rt0) * 10))
            print("  E-step's last wave ends at %d ns; fin's first wave starts %d ns later, its last "
                  "ends %d ns after that" % ((e_end - rt0) * 10, (t[:, 8].min() - e_end) * 10,
                                             (t[:, 9].max() - e_end) * 10))
            wg = idx // 4
            ngw = int(sys.argv[3]) if len(sys.argv) > 3 else 59  # gene workgroups (P K / 256)
            for pname, sel in (("gene", wg < ngw), ("cell", wg >= ngw)):
                if sel.any():
                    tt = t[sel]
                    print("  [%s] %d waves: start ns %s | end ns %s | life ns %s" % (
                        pname, sel.sum(), q((tt[:, 8] - rt0) * 10), q((tt[:, 9] - rt0) * 10),
                        q((tt[:, 9] - tt[:, 8]) * 10)))
                    for k in (1, 2, 3):  # cycles from the start to marks 1-3 (0: not marked)
                        if (tt[:, k] != 0).any():
                            print("      ->mark%d cycles %s" % (k, q(np.where(tt[:, k] != 0, tt[:, k] - tt[:, 0], 0))))
                    print("      ->end   cycles %s" % q(tt[:, 7] - tt[:, 0]))
            continue
        if name == "fin":
            print("  ->sync %s" % q(t[:, 4] - t[:, 0]))
            print("  ->rows %s" % q(t[:, 5] - t[:, 0]))
        if name in ("passA", "passB", "passLL") and (t[:, 7] != 0).all():
            # small-K kernels (csrc/sk.h): 6 = p staged, 1 = unit prologue done, 2 = chunk loop
            # done, 3 = unit epilogue done, 7 = kernel end (S reduction / likelihood sum)
            print("  ->p    %s" % q(t[:, 6] - t[:, 0]))
            print("  unit prologue %s" % q(t[:, 1] - t[:, 6]))
            print("  chunk loop    %s" % q(t[:, 2] - t[:, 1]))
            print("  epilogue      %s" % q(t[:, 3] - t[:, 2]))
            print("  tail          %s" % q(t[:, 7] - t[:, 3]))
            # chip-wide timeline from s_memrealtime (100 MHz): when waves start and end relative
            # to the first wave of the launch, in ns
            rt0 = t[:, 8].min()
            print("  start (ns from the first wave) %s" % q((t[:, 8] - rt0) * 10))
            print("  end   (ns from the first wave) %s" % q((t[:, 9] - rt0) * 10))
            print("  life  (ns)                     %s" % q((t[:, 9] - t[:, 8]) * 10))
            if n_wg0:  # per stream group: the chip-wide end time and the phases (cycles)
                wg = idx // 8
                for gname, sel in (("stream 0", wg < n_wg0), ("streams 1/2", wg >= n_wg0)):
                    if not sel.any():
                        continue
                    tt = t[sel]
                    print("  [%s] %d waves" % (gname, sel.sum()))
                    print("    end ns    %s" % q((tt[:, 9] - rt0) * 10))
                    print("    life ns   %s" % q((tt[:, 9] - tt[:, 8]) * 10))
                    print("    prologue  %s" % q(tt[:, 1] - tt[:, 0]))
                    print("      ->p     %s" % q(tt[:, 6] - tt[:, 0]))
                    print("      V       %s" % q(tt[:, 1] - tt[:, 6]))
                    print("    chunks    %s" % q(tt[:, 2] - tt[:, 1]))
                    print("    epilogue  %s" % q(tt[:, 3] - tt[:, 2]))
                    print("    tail      %s" % q(tt[:, 7] - tt[:, 3]))
                    # what sets a wave's length: its stretches (V reloads, M flushes), its chunks
                    for ns in np.unique(tt[:, 4]):
                        sel2 = tt[:, 4] == ns
                        cl = tt[sel2, 2] - tt[sel2, 1]
                        print("    stretches %2d: %5d waves, chunks med %3d, chunk loop med %6d p90 %6d, life ns med %6d" % (
                            ns, sel2.sum(), np.median(tt[sel2, 5]), np.median(cl), np.percentile(cl, 90),
                            np.median((tt[sel2, 9] - tt[sel2, 8]) * 10)))
            ch = t[:, 5]
            print("  chunks %s  stretches %s" % (q(ch), q(t[:, 4])))
            if ch.max() > 0 and ch.min() < ch.max():
                a = np.polyfit(ch, ph2, 1)
                print("  chunk loop ~ %.0f cycles/chunk + %.0f" % (a[0], a[1]))
            continue
        if name in ("passA", "passB", "passLL"):
            ch = t[:, 5]
            print("  chunks %s" % q(ch))
            if ch.max() > 0:
                a = np.polyfit(ch, ph2, 1)
                print("  phase2 ~ %.0f cycles/chunk + %.0f" % (a[0], a[1]))
            if name != "passB":
                ng = t[:, 4]
                print("  ->V    %s" % q(t[:, 6] - t[:, 0]))
                a = np.polyfit(ng, t[:, 6] - t[:, 0], 1)
                print("  ->V ~ %.0f cycles/gene + %.0f" % (a[0], a[1]))
                print("  genes  %s" % q(ng))
                a = np.polyfit(ng, ph1, 1)
                print("  phase1 ~ %.0f cycles/gene + %.0f" % (a[0], a[1]))
            last = np.argsort(end)[-8:]
            for i in last:
                print("   late wave %6d wg %5d start %6d ph1 %6d ph2 %6d chunks %3d genes %3d" % (
                    idx[i], idx[i] // 8, start[i], ph1[i], ph2[i], t[i, 5], t[i, 4]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
