"""Link tables that notice in-place edits.

The reference re-reads `self.links` / `self.test_links` on every call
(src/TrigenicInteractionPredictor.py:987 in make_iteration, :959 in
compute_likelihood), so a caller may edit them between iterations:
`model.links[key][1] += 1`, `model.links[key] = [0, 1]`, `del model.links[key]`.
The engine keeps a device copy of each table (its work plan), so it must learn of
such edits.  `TrackedLinks` is a dict whose values are `TrackedRow` lists; every
mutating method of either bumps one shared counter, which the Model compares before
each device call (an O(1) check, no re-scan of the table).

Both types are plain dict / list subclasses: iteration order, equality, `json`,
`copy` and `isinstance(x, dict)` behave as for the reference's objects.
"""
from __future__ import annotations

import itertools

_clock = itertools.count(1)   # one clock for every table: a number is never reused


class Version:
    """`n` changes at every edit and differs between tables, so a tuple of the `n` of the tables
    a device copy was built from identifies exactly that state."""
    __slots__ = ("n",)

    def __init__(self):
        self.n = next(_clock)

    def bump(self):
        self.n = next(_clock)


class TrackedRow(list):
    """The rating counts [n_0, n_1, ...] of one link; edits bump the counter of every table that
    holds this row object (one list shared by two tables, as the same list object in two of the
    reference's dicts would be, is seen by both)."""
    __slots__ = ("_v",)

    def __init__(self, it=(), version: Version = None):
        super().__init__(it)
        self._v = () if version is None else (version,)

    def _own(self, version: Version):
        if all(v is not version for v in self._v):
            self._v += (version,)

    def _bump(self):
        for v in self._v:
            v.bump()

    def __setitem__(self, i, x):
        super().__setitem__(i, x)
        self._bump()

    def __delitem__(self, i):
        super().__delitem__(i)
        self._bump()

    def __iadd__(self, other):
        r = super().__iadd__(other)
        self._bump()
        return r

    def __imul__(self, n):
        r = super().__imul__(n)
        self._bump()
        return r

    def append(self, x):
        super().append(x)
        self._bump()

    def extend(self, it):
        super().extend(it)
        self._bump()

    def insert(self, i, x):
        super().insert(i, x)
        self._bump()

    def pop(self, *a):
        r = super().pop(*a)
        self._bump()
        return r

    def remove(self, x):
        super().remove(x)
        self._bump()

    def reverse(self):
        super().reverse()
        self._bump()

    def sort(self, *a, **kw):
        super().sort(*a, **kw)
        self._bump()

    def clear(self):
        super().clear()
        self._bump()

    def __reduce_ex__(self, protocol):   # pickles / deep-copies as a plain list
        return (list, (list(self),))


class TrackedLinks(dict):
    """`links` / `test_links`: key 'i_j_k' -> TrackedRow of counts.  Any edit of the table or of
    one of its rows bumps `version.n`.

    `alias`: a plain dict the caller assigned (`model.links = d`).  The reference stores that very
    object, so later edits of `d` are edits of `model.links`.  A dict cannot be made to notice its
    own edits, so the table keeps `d` as its source and shares the row objects with it: `d`'s
    values are replaced by the table's TrackedRow rows (equal lists), so `d[k][r] += 1` is seen at
    once; every edit made through the table is applied to `d` too; and a key added to or removed
    from `d` itself is picked up by `resync()` (what `Model.links_changed()` calls).  A dict may
    back several tables (two Models, or `links` and `test_links`): rows already tracked are
    reused, not replaced, and notify every table holding them, so `d[k][r] += 1` reaches all of
    them; a key added or removed through one table reaches `d`, and the others pick it up at
    their own `resync()`, like a key added to `d` directly."""

    def __init__(self, src=None, version: Version = None, alias: dict = None):
        super().__init__()
        self.version = version if version is not None else Version()
        self.src = alias
        if alias is not None:
            src = alias
        if src:
            for k, v in (list(src.items()) if hasattr(src, "items") else src):
                row = self._row(v)
                dict.__setitem__(self, k, row)
                if alias is not None and row is not v:
                    alias[k] = row

    def resync(self):
        """Re-read the aliased source dict (edits made to it directly); no-op without one."""
        if self.src is None:
            return
        dict.clear(self)
        for k, v in list(self.src.items()):
            row = self._row(v)
            dict.__setitem__(self, k, row)
            if row is not v:
                self.src[k] = row
        self.version.bump()

    def _row(self, v):
        if isinstance(v, list):
            if isinstance(v, TrackedRow):
                v._own(self.version)
                return v
            return TrackedRow(v, self.version)
        return v

    def __setitem__(self, k, v):
        row = self._row(v)
        dict.__setitem__(self, k, row)
        if self.src is not None:
            self.src[k] = row
        self.version.bump()

    def __delitem__(self, k):
        dict.__delitem__(self, k)
        if self.src is not None:
            self.src.pop(k, None)
        self.version.bump()

    def setdefault(self, k, default=None):
        if k in self:
            return dict.__getitem__(self, k)
        self[k] = default
        return dict.__getitem__(self, k)

    def update(self, *a, **kw):
        for k, v in dict(*a, **kw).items():
            row = self._row(v)
            dict.__setitem__(self, k, row)
            if self.src is not None:
                self.src[k] = row
        self.version.bump()

    def __ior__(self, other):
        self.update(other)
        return self

    def pop(self, *a):
        r = dict.pop(self, *a)
        if self.src is not None and a:
            self.src.pop(a[0], None)
        self.version.bump()
        return r

    def popitem(self):
        k, v = dict.popitem(self)
        if self.src is not None:
            self.src.pop(k, None)
        self.version.bump()
        return k, v

    def clear(self):
        dict.clear(self)
        if self.src is not None:
            self.src.clear()
        self.version.bump()

    def __reduce_ex__(self, protocol):   # pickles / deep-copies as a plain dict of lists
        return (dict, ({k: list(v) if isinstance(v, list) else v for k, v in self.items()},))


def tracked(value):
    """The table a Model stores for an assigned value: a TrackedLinks as is, None as is (not
    materialised), any other mapping as a TrackedLinks aliasing it."""
    if value is None or isinstance(value, TrackedLinks):
        return value
    if isinstance(value, dict):
        return TrackedLinks(alias=value)
    return TrackedLinks(value)


def version_of(table) -> int:
    """The state number of a tracked table (0 for None: not materialised yet)."""
    return 0 if table is None else table.version.n


class TrackedTable:
    """Class attribute that keeps a TrackedLinks in the instance: assigning a plain dict stores a
    table aliasing it (`tracked`), with a new version."""

    def __set_name__(self, owner, name):
        self.slot = "_tracked_" + name

    def __get__(self, obj, owner=None):
        if obj is None:
            return self
        return obj.__dict__[self.slot]

    def __set__(self, obj, value):
        obj.__dict__[self.slot] = tracked(value)
