"""Link tables that notice in-place edits (trigenicinteractionpredictor_amd/tracked.py): the
reference re-reads `links` on every call (src/TrigenicInteractionPredictor.py:987, :959), so
every edit must change the state the device copy is keyed on."""
import copy
import json
import os
import pickle

import numpy as np

from golden_util import GOLDEN
from trigenicinteractionpredictor_amd.model import Model
from trigenicinteractionpredictor_amd.tracked import TrackedLinks, TrackedRow, version_of


def _edits():
    return [
        lambda t: t["0_1_2"].__setitem__(1, 5),
        lambda t: t["0_1_2"].__iadd__([0]),
        lambda t: t["0_1_2"].append(0),
        lambda t: t["0_1_2"].pop(),
        lambda t: t["0_1_2"].sort(),
        lambda t: t["0_1_2"].reverse(),
        lambda t: t.__setitem__("3_4_5", [1, 0]),
        lambda t: t.__delitem__("0_1_2"),
        lambda t: t.pop("0_1_2"),
        lambda t: t.popitem(),
        lambda t: t.update({"7_8_9": [0, 1]}),
        lambda t: t.setdefault("7_8_9", [0, 1]),
        lambda t: t.clear(),
    ]


def test_every_edit_changes_the_version():
    for edit in _edits():
        t = TrackedLinks({"0_1_2": [1, 0], "1_2_3": [0, 1]})
        v0 = version_of(t)
        edit(t)
        assert version_of(t) != v0
    t = TrackedLinks({"0_1_2": [1, 0]})
    v0 = version_of(t)
    _ = t["0_1_2"][0], len(t), list(t.items()), t.get("x")   # reads do not
    t.setdefault("0_1_2", [9, 9])                            # an existing key is a read
    assert version_of(t) == v0


def test_augmented_assignment_through_the_table():
    t = TrackedLinks({"0_1_2": [1, 0]})
    v0 = version_of(t)
    t["0_1_2"][1] += 1                     # the reference's own idiom (:360-368)
    assert t["0_1_2"] == [1, 1] and version_of(t) != v0
    assert isinstance(t["0_1_2"], TrackedRow)


def test_tables_behave_like_plain_dicts():
    t = TrackedLinks({"0_1_2": [1, 0], "1_2_3": [0, 1]})
    assert t == {"0_1_2": [1, 0], "1_2_3": [0, 1]}
    assert isinstance(t, dict) and isinstance(t["0_1_2"], list)
    assert json.loads(json.dumps(t)) == t
    for clone in (copy.deepcopy(t), pickle.loads(pickle.dumps(t))):
        assert clone == t and type(clone) is dict and type(clone["0_1_2"]) is list


def test_model_link_arrays_follow_in_place_edits():
    g = os.path.join(GOLDEN, "tiny")
    m = Model()
    m.get_traintest(os.path.join(g, "train.dat"), os.path.join(g, "test.dat"))
    key0 = (version_of(m._links), version_of(m._test_links))
    ids0, counts0 = m._link_arrays(0)
    k = next(iter(m.links))
    assert (version_of(m._links), version_of(m._test_links)) != key0   # materialised
    key1 = (version_of(m._links), version_of(m._test_links))
    np.testing.assert_array_equal(m._link_arrays(0)[1], counts0)      # still the parsed arrays
    m.links[k][1] += 3
    assert version_of(m._links) != key1[0]
    ids, counts = m._link_arrays(0)
    np.testing.assert_array_equal(ids, ids0)
    assert counts[0, 1] == counts0[0, 1] + 3
    m.test_links = {"0_1_2": [0, 1]}                                   # a new table
    tids, tcounts = m._link_arrays(1)
    assert tids.tolist() == [[0, 1, 2]] and tcounts.tolist() == [[0, 1]]
    m.links = dict(m.links)                                            # assigned plain dict
    assert isinstance(m.links, TrackedLinks)
