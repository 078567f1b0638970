"""The engine's work plan (csrc/plan.h, built by mmsbm_set_links) checked on the CPU: a small
C++ driver (tests/plan_check.cpp) builds plans for synthetic link tables and checks their
invariants — every observation once per stream, one pivot gene per chunk, unit and gene caps,
chunk coverage, V slots, partial-row numbering per (stream, rating, gene), S-partial tiling."""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def plan_check(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("plan") / "plan_check")
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "plan_check.cpp")],
                   check=True)
    return exe


def _links(P, E, seed, R=2, hub=0.0, multi=0.05, both=0.03):
    rng = np.random.default_rng(seed)
    p = np.ones(P)
    if hub:
        p[: max(1, P // 50)] *= hub  # a few genes with very long pivot runs
    p /= p.sum()
    seen, rows = set(), []
    while len(rows) < E:
        t = tuple(sorted(rng.choice(P, 3, p=p).tolist(), key=str))
        if t in seen:
            continue
        seen.add(t)
        c = [0] * R
        r = int(rng.integers(R))
        c[r] = int(rng.integers(2, 5)) if rng.random() < multi else 1
        if rng.random() < both:
            c[1 - r] = 1
        rows.append(list(t) + c)
    return np.array(rows, dtype=np.int64)


@pytest.mark.parametrize("P,E,units,gcap,sp_rows,hub", [
    (40, 600, (1, 1), 33, 16, 0.0),        # one unit per stream: every run split at 64 chunks
    (200, 3000, (3, 5), 4, 16, 0.0),       # tiny gene cap: gene-capped workgroups
    (300, 5000, (1536, 3072), 33, 16, 30.0),   # hub genes, default unit counts
    (120, 4000, (64, 64), 13, 120, 10.0),  # large-K shape: 13 genes, 120 rows per S partial
    (30, 1500, (1536, 3072), 8, 40, 0.0),  # more units than chunks
    # small-K plans (gcap 0; sp_rows = the workgroup target): stretch-capped units, descriptors
    (300, 5000, (1536, 3072), 0, 1024, 30.0),  # hub genes
    (40, 600, (1, 1), 0, 1024, 0.0),           # one unit per stream: runs split at 32 chunks
    (200, 6000, (64, 64), 0, 3, 5.0),          # long units (16 chunks)
    (30, 1500, (1536, 3072), 0, 1024, 0.0),    # more units than chunks
    (200, 6000, (64, 64), -3, 3, 5.0),         # 8 stretches per unit (K <= 10)
    # fill-packed small-K plans (gcap -1 / -2: the fused launch, 8 / 4 stretches): full units, runs
    # split at unit ends
    (300, 5000, (1, 1), -1, 1024, 30.0),       # hub genes
    (1500, 20000, (1, 1), -1, 1024, 0.0),      # fold0-like degree
    (40, 600, (1, 1), -1, 1024, 0.0),          # few genes: long runs
    (1500, 20000, (1, 1), -2, 1024, 0.0),      # 4 stretches (K = 11, 12)
    # fill-packed stream-0 plans with Y entries (gcap -4: SK_Y, the fused small-K E-step of round 4)
    (300, 5000, (1, 1), -4, 1024, 30.0),       # hub genes
    (1500, 20000, (3840, 3840), -4, 1024, 0.0),  # fold0-like degree, 15 units per CU
    (40, 600, (64, 64), -4, 1024, 0.0),        # few genes: long runs
    (500, 40000, (1536, 3072), 5, 120, 0.0),   # K=30-like gene cap, long runs (balanced units)
])
def test_plan_invariants(plan_check, P, E, units, gcap, sp_rows, hub):
    _check(plan_check, P, E, units, gcap, sp_rows, hub)


def _check(plan_check, P, E, units, gcap, sp_rows, hub, env=None):
    links = _links(P, E, seed=P + E, hub=hub)
    head = "%d 2 %d %d %d %d %d\n" % (len(links), P, units[0], units[1], gcap, sp_rows)
    body = "\n".join(" ".join(str(v) for v in row) for row in links)
    res = subprocess.run([plan_check], input=head + body + "\n", capture_output=True, text=True,
                         env=None if env is None else {**os.environ, **env})
    assert res.returncode == 0 and res.stdout.startswith("ok"), res.stdout + res.stderr
    return res.stdout.split()


# large-K plans packed the round-3 way (MMSBM_BALANCE=0: whole runs per unit) keep every invariant
# but the balance; the balanced plans (default, checked above) split each workgroup evenly
@pytest.mark.parametrize("P,E,units,gcap,sp_rows,hub", [
    (40, 600, (1, 1), 33, 16, 0.0),
    (300, 5000, (1536, 3072), 33, 16, 30.0),
    (120, 4000, (64, 64), 13, 120, 10.0),
    (500, 40000, (64, 64), 5, 120, 0.0),       # K=30-like gene cap, long units
])
def test_plan_invariants_unbalanced(plan_check, P, E, units, gcap, sp_rows, hub):
    _check(plan_check, P, E, units, gcap, sp_rows, hub, env={"PLAN_NO_BALANCE": "1"})


# merged partial rows (K >= 25 plans): one per (workgroup, gene), fewer than one per unit stretch
@pytest.mark.parametrize("P,E,units,gcap,sp_rows,hub", [
    (500, 40000, (64, 64), 13, 120, 0.0),
    (300, 5000, (1536, 3072), 13, 120, 30.0),
    (40, 600, (1, 1), 13, 16, 0.0),
])
def test_plan_invariants_merged(plan_check, P, E, units, gcap, sp_rows, hub):
    merged = _check(plan_check, P, E, units, gcap, sp_rows, hub, env={"PLAN_MERGE": "1"})
    plain = _check(plan_check, P, E, units, gcap, sp_rows, hub)
    assert int(merged[4]) <= int(plain[4])  # partial rows


def test_balanced_plan_fewer_workgroups(plan_check):
    # K=30-like: 5 genes per workgroup, runs of ~10 chunks, 64-chunk units: the round-3 plan's
    # units took whole runs up to 64 chunks, so a workgroup's gene cap left most of its 8 units
    # empty; the balanced plan fills all 8 from fewer workgroups
    bal = _check(plan_check, 500, 40000, (64, 64), 5, 120, 0.0)
    old = _check(plan_check, 500, 40000, (64, 64), 5, 120, 0.0, env={"PLAN_NO_BALANCE": "1"})
    assert int(bal[3]) < int(old[3])


# 4-unit workgroups (the K >= 25 pass kernel: 4-wave workgroups, three per CU, gene cap 4), merged
# and plain partial rows, balanced and round-3 packing
@pytest.mark.parametrize("P,E,units,gcap,sp_rows,hub", [
    (500, 40000, (64, 64), 4, 128, 0.0),
    (300, 5000, (1536, 3072), 4, 128, 30.0),
    (40, 600, (1, 1), 4, 16, 0.0),
    (3000, 4000, (1536, 3072), 4, 128, 0.0),
])
@pytest.mark.parametrize("env", [{"PLAN_MERGE": "1"}, {}, {"PLAN_NO_BALANCE": "1"}])
def test_plan_invariants_four_unit_workgroups(plan_check, P, E, units, gcap, sp_rows, hub, env):
    out = _check(plan_check, P, E, units, gcap, sp_rows, hub, env={**env, "PLAN_NW": "4"})
    assert int(out[2]) == 4 * int(out[3])  # units = 4 x workgroups


@pytest.mark.parametrize("cap", [3, 16, 1024])
def test_s_partial_parts_are_capped_per_rating(plan_check, cap):
    """the large-K S partials take R x parts x K^3 doubles per sample, so their number
    is capped per rating (mmsbm_set_links: 1,024 with 128 rows a part) whatever E; past the cap
    the parts grow longer (gm_kernel walks any number of 64-row tiles) and still tile each
    rating's partial rows (plan_check's S-partial tiling check)."""
    out = _check(plan_check, 500, 40000, (1536, 3072), 13, 4, 0.0, env={"PLAN_SP_CAP": str(cap)})
    n_prows, n_sp = int(out[4]), int(out[5])
    assert n_sp <= 2 * cap
    if cap < 16:
        assert n_sp == 2 * cap and n_prows > 4 * n_sp   # capped: longer parts
