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


def test_assigned_dict_stays_aliased():
    """`m.links = d` keeps `d` as the table's source: row edits of `d` are seen at
    once, edits through `m.links` reach `d`, and keys added to `d` itself arrive with
    links_changed()."""
    m = Model()
    m.P = 6
    d = {"0_1_2": [1, 0], "1_2_3": [0, 1]}
    m.links = d
    v0 = version_of(m._links)
    ids0, counts0 = m._link_arrays(0)
    d["0_1_2"][1] += 2                                   # the caller's own dict
    assert version_of(m._links) != v0
    assert m._link_arrays(0)[1].tolist() == [[1, 2], [0, 1]]
    m.links["3_4_5"] = [1, 1]                            # through the model
    assert d["3_4_5"] == [1, 1]
    del m.links["1_2_3"]
    assert "1_2_3" not in d
    d["2_3_4"] = [0, 3]                                  # a new key in the source: declared
    v1 = version_of(m._links)
    m.links_changed()
    assert version_of(m._links) != v1
    ids, counts = m._link_arrays(0)
    assert ids.tolist() == [[0, 1, 2], [3, 4, 5], [2, 3, 4]]
    assert counts.tolist() == [[1, 2], [1, 1], [0, 3]]
    assert m.links == d


def test_model_deepcopy_and_pickle_keep_tracked_tables():
    """copy.deepcopy / pickle of a Model: the copy's tables are tracked (the next
    engine call can read their versions) and equal the original's."""
    g = os.path.join(GOLDEN, "tiny")
    m = Model()
    m.get_traintest(os.path.join(g, "train.dat"), os.path.join(g, "test.dat"))
    _ = m.links                                           # one table materialised, one lazy
    for clone in (copy.deepcopy(m), pickle.loads(pickle.dumps(m))):
        assert isinstance(clone._links, TrackedLinks) and clone._engine is None
        assert version_of(clone._links) and clone.links == m.links
        assert clone.test_links == m.test_links
        np.testing.assert_array_equal(clone._link_arrays(0)[1], m._link_arrays(0)[1])
        clone.links[next(iter(clone.links))][0] += 1     # edits stay seen in the copy
        assert clone._link_arrays(0)[1][0, 0] == m._link_arrays(0)[1][0, 0] + 1


def test_joint_model_deepcopy_and_alias():
    from trigenicinteractionpredictor_amd import joint
    mj = joint.Model()
    d = {"0_1_2": [1, 0]}
    mj.links = d
    d["0_1_2"][0] += 1
    assert mj.links["0_1_2"] == [2, 0]
    d["1_2_3"] = [0, 1]
    mj.links_changed()
    assert "1_2_3" in mj.links
    clone = copy.deepcopy(mj)
    assert isinstance(clone.links, TrackedLinks) and clone.links == mj.links
    assert version_of(clone.links) and version_of(clone.dlinks)


def test_one_dict_backing_two_tables_reaches_both():
    """a dict assigned to two tables (two Models here) keeps one row object per key;
    the rows notify both tables, so `d[k][r] += 1` and an edit through a row reference taken
    before the second assignment reach both devices' keys; a key added through one table reaches
    `d` and the other table at its links_changed()."""
    d = {"0_1_2": [1, 0], "1_2_3": [0, 1]}
    a, b = Model(), Model()
    a.links = d
    row = d["0_1_2"]
    b.links = d
    assert d["0_1_2"] is row and a.links["0_1_2"] is row and b.links["0_1_2"] is row
    va, vb = version_of(a.links), version_of(b.links)
    d["0_1_2"][1] += 1
    assert version_of(a.links) != va and version_of(b.links) != vb
    va, vb = version_of(a.links), version_of(b.links)
    row[0] = 7
    assert version_of(a.links) != va and version_of(b.links) != vb
    assert a.links["0_1_2"] == b.links["0_1_2"] == [7, 1]
    b.links["5_6_7"] = [1, 1]
    assert "5_6_7" in d and "5_6_7" not in a.links
    a.links_changed()
    assert a.links["5_6_7"] == [1, 1] and a.links["5_6_7"] is b.links["5_6_7"]
