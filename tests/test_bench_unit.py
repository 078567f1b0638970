"""bench.py's host-side accounting (no GPU): the per-kernel work table is keyed by the labels the
engine times (EMEngine.LABELS) for every plan family, and the roofline record follows the
headline rule (SURVEY 8d credit, or the executed FLOPs where the credit exceeds the peak)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _labels():
    import ast
    src = open(os.path.join(REPO, "trigenicinteractionpredictor_amd", "engine.py")).read()
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", None) == "LABELS":
            return ast.literal_eval(node.value)
    raise AssertionError("EMEngine.LABELS not found")


PLAN = {"rows_stream0": 76000, "rows": 76000, "partial_rows": 3200, "partial_rows_stream0": 3200,
        "v_genes": 3000, "wg_stream0": 190, "wg_spartial": 200, "y_entries": 144000}


def test_kernel_work_keys_match_engine_labels():
    for fam, labels in _labels().items():
        work = bench.kernel_work(dict(PLAN, small_k=fam), 10, 1500, 2, 1, 72000)
        assert set(work) == set(labels), (fam, work.keys(), labels)
        assert all(f > 0 and b > 0 for f, b in work.values())


def test_roofline_headline_basis():
    plan = dict(PLAN, small_k=0)
    b2b = {"pass_a": 0.1, "gene": 0.05, "fin": 0.01}
    slow = bench.roofline_record(20, 1500, 2, 8, 72000, plan, 1e-3, b2b, "none")
    assert slow["frac_basis"].startswith("SURVEY") and slow["frac"] == slow["credited"]["frac"]
    fast = bench.roofline_record(20, 1500, 2, 8, 72000, plan, 1e-6, b2b, "none")
    assert fast["frac_basis"].startswith("executed") and fast["frac"] == fast["executed"]["frac"]
    assert fast["credited"]["frac"] > 1.0
    assert fast["dominant_kernel"]["kernel"].startswith("pass_kernel<20")
