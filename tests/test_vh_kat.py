"""Known-answer tests of the NDC VersionHistory / VersionHistories restatement
(oracle/ndc_ref.cpp), restated from the reference's own tests:
common/persistence/versionHistory_test.go:68-665.  These pin the oracle that the GPU
branch-management kernels (cadence_amd/csrc/ndc.hip) are checked against."""
import ctypes as C

import pytest

from cadence_amd import abi


def _L():
    import oracle
    return oracle.lib()


def _items(pairs):
    """[(eventID, version), ...] -> ctypes array of cdr_vh_item"""
    a = (abi.CdrVHItem * max(1, len(pairs)))()
    for i, (e, v) in enumerate(pairs):
        a[i].event_id, a[i].version = e, v
    return a, len(pairs)


def _it(e, v):
    x = abi.CdrVHItem()
    x.event_id, x.version = e, v
    return x


def _dup(pairs, lca):
    a, n = _items(pairs)
    out = (abi.CdrVHItem * 16)()
    m = C.c_uint32()
    rc = _L().cdro_vh_duplicate_until_lca(a, n, _it(*lca), out, C.byref(m))
    return rc, [(out[i].event_id, out[i].version) for i in range(m.value)] if rc == 0 else None


BASE = [(3, 0), (6, 4)]


def test_duplicate_until_lca_success():  # versionHistory_test.go:68-115
    assert _dup(BASE, (2, 0)) == (0, [(2, 0)])
    assert _dup(BASE, (5, 4)) == (0, [(3, 0), (5, 4)])
    assert _dup(BASE, (6, 4)) == (0, [(3, 0), (6, 4)])


@pytest.mark.parametrize("lca", [(4, 0), (2, 1), (5, 3), (7, 5), (7, 4)])
def test_duplicate_until_lca_failure(lca):  # versionHistory_test.go:117-143
    rc, _ = _dup(BASE, lca)
    assert abi.STATUS[rc] == "E_VH_LCA_NOT_CONTAINED"


def test_contains_item():  # versionHistory_test.go:251-292
    a, n = _items(BASE)
    prev = 0
    for e, v in BASE:
        for eid in range(prev + 1, e + 1):
            assert _L().cdro_vh_contains(a, n, _it(eid, v)) == 1
        prev = e
    for e, v in ((4, 0), (3, 1), (7, 4), (6, 5)):
        assert _L().cdro_vh_contains(a, n, _it(e, v)) == 0
    assert _L().cdro_vh_contains(a, n, _it(0, 0)) == 1  # FirstEventID - 1


def test_is_lca_appendable():  # versionHistory_test.go:294-328
    a, n = _items(BASE)
    assert _L().cdro_vh_is_lca_appendable(a, n, _it(6, 4)) == 1
    assert _L().cdro_vh_is_lca_appendable(a, n, _it(6, 7)) == 0
    assert _L().cdro_vh_is_lca_appendable(a, n, _it(7, 4)) == 0


LOCAL = [(3, 0), (5, 4), (7, 6), (9, 10)]


def _lca(local, remote):
    a, n = _items(local)
    b, m = _items(remote)
    out = abi.CdrVHItem()
    rc = _L().cdro_vh_find_lca(a, n, b, m, C.byref(out))
    return rc, (out.event_id, out.version)


def test_find_lca_item():  # versionHistory_test.go:330-395
    assert _lca(LOCAL, [(3, 0), (7, 4), (8, 8), (11, 12)]) == (0, (5, 4))  # ReturnLocal
    assert _lca(LOCAL, [(3, 0), (5, 4), (6, 6), (11, 12)]) == (0, (6, 6))  # ReturnRemote
    rc, _ = _lca(LOCAL, [(3, 1), (7, 2), (8, 3)])  # Error_NoLCA
    assert abi.STATUS[rc] == "E_VH_NO_LCA"


def _tok(i):
    t = abi.CdrVHToken()
    t.tree, t.branch_lo, t.branch_hi = 7, 1000 + i, 2000 + i
    return t


def _vhs(first):
    """VersionHistories holding `first` as branch 0 (NewVersionHistories)."""
    s = abi.CdrVHS()
    s.items_cap = 16
    pool = (abi.CdrVHItem * (16 * abi.VHS_MAX_BRANCHES))()
    s.n_branches = 1
    s.branch[0].token = _tok(0)
    s.branch[0].n_items = len(first)
    for i, (e, v) in enumerate(first):
        pool[i].event_id, pool[i].version = e, v
    return s, pool


def _add(s, pool, pairs, i):
    a, n = _items(pairs)
    ch, idx = C.c_int(), C.c_uint32()
    rc = _L().cdro_vhs_add(C.byref(s), pool, C.byref(_tok(i)), a, n, C.byref(ch), C.byref(idx))
    return rc, bool(ch.value), idx.value


def _branch(s, pool, b):
    off = b * s.items_cap
    return [(pool[off + i].event_id, pool[off + i].version) for i in range(s.branch[b].n_items)]


def test_add_get_version_history():  # versionHistory_test.go:505-535
    vh2 = [(3, 0), (5, 4), (6, 6), (11, 12)]
    s, pool = _vhs(LOCAL)
    assert s.current == 0
    assert _add(s, pool, vh2, 1) == (0, True, 1)
    assert s.current == 1
    assert _branch(s, pool, 0) == LOCAL and _branch(s, pool, 1) == vh2
    assert bytes(s.branch[1].token) == bytes(_tok(1))


def test_add_version_history_first_item_mismatch():  # versionHistory.go:463-465
    s, pool = _vhs(LOCAL)
    rc, _, _ = _add(s, pool, [(3, 1), (9, 12)], 1)
    assert abi.STATUS[rc] == "E_VH_FIRST_ITEM_MISMATCH"


def _find_lca_index(s, pool, pairs):
    a, n = _items(pairs)
    idx, it = C.c_uint32(), abi.CdrVHItem()
    rc = _L().cdro_vhs_find_lca_index(C.byref(s), pool, a, n, C.byref(idx), C.byref(it))
    return rc, idx.value, (it.event_id, it.version)


INCOMING = [(3, 0), (5, 4), (8, 6), (11, 100)]


def test_find_lca_index_larger_event_id_wins():  # versionHistory_test.go:537-566
    s, pool = _vhs(LOCAL)
    assert _add(s, pool, [(3, 0), (5, 4), (6, 6), (11, 12)], 1)[0] == 0
    assert _find_lca_index(s, pool, INCOMING) == (0, 0, (7, 6))


def test_find_lca_index_same_event_id_shorter_wins():  # versionHistory_test.go:568-596
    s, pool = _vhs(LOCAL)
    assert _add(s, pool, [(3, 0), (5, 4), (7, 6)], 1)[0] == 0
    assert _find_lca_index(s, pool, INCOMING) == (0, 1, (7, 6))


def test_find_first_index_by_item():  # versionHistory_test.go:598-625
    s, pool = _vhs([(3, 0), (5, 4), (7, 6)])
    assert _add(s, pool, LOCAL, 1)[0] == 0
    idx = C.c_uint32()
    assert _L().cdro_vhs_find_first_index_by_item(C.byref(s), pool, _it(8, 10), C.byref(idx)) == 0
    assert idx.value == 1
    assert _L().cdro_vhs_find_first_index_by_item(C.byref(s), pool, _it(4, 4), C.byref(idx)) == 0
    assert idx.value == 0
    assert _L().cdro_vhs_find_first_index_by_item(C.byref(s), pool, _it(41, 4), C.byref(idx)) != 0


def test_is_rebuilt():  # versionHistory_test.go:627-665
    s, pool = _vhs(LOCAL)
    assert _add(s, pool, [(3, 0), (5, 4), (6, 6), (11, 12)], 1) == (0, True, 1)
    assert _L().cdro_vhs_is_rebuilt(C.byref(s), pool) == 0
    s.current = 0
    assert _L().cdro_vhs_is_rebuilt(C.byref(s), pool) == 1
    s.current = 1
    assert _L().cdro_vhs_is_rebuilt(C.byref(s), pool) == 0


def _task(pairs, first, last, version, tok=9):
    t = abi.CdrNdcTask()
    a, n = _items(pairs)
    t.items_off, t.n_items = 0, n
    t.first_event_id = first
    t.last_event_id, t.last_version = last
    t.version = version
    t.new_token = _tok(tok)
    return t, a


def _branch_op(s, pool, t, a):
    d = abi.CdrNdcDecision()
    _L().cdro_ndc_branch(C.byref(t), a, 1, C.byref(s), pool, C.byref(d))
    return d


def test_ndc_handcrafted_multiple_branches_flow():
    """host/ndc/nDC_integration_test.go:310-613: branch 1-14 @21, then eventsBatch3
    (15-20 @30) appended to the current branch, then eventsBatch2 (15 @31) forks at
    (14, 21), becomes a new branch and — higher version than the current branch's last
    write — triggers the conflict-resolution rebuild of events 1-14."""
    s, pool = _vhs([(14, 21)])
    t, a = _task([(14, 21), (20, 30)], 15, (20, 30), 30)
    d = _branch_op(s, pool, t, a)
    assert (d.code, d.action, d.branch_index, d.created) == (0, abi.NDC_APPLY_CURRENT, 0, 0)
    # the applied events extend the current branch (the replay's VH, synchronised)
    s.branch[0].n_items = 2
    pool[1].event_id, pool[1].version = 20, 30
    t, a = _task([(14, 21), (15, 31)], 15, (15, 31), 31)
    d = _branch_op(s, pool, t, a)
    assert (d.code, d.action, d.branch_index, d.created) == (0, abi.NDC_REBUILD, 1, 1)
    assert (d.lca.event_id, d.lca.version) == (14, 21)
    assert d.rebuild_next_event_id == 15
    assert s.n_branches == 2 and s.current == 0  # switched by the rebuild, not by AddVersionHistory
    assert _branch(s, pool, 1) == [(14, 21)] and bytes(s.branch[1].token) == bytes(_tok(9))


def test_ndc_backfill_skip_retry_and_same_version():
    s, pool = _vhs([(14, 21), (20, 30)])
    # lower version fork: non-current branch, VH gets the last event only
    t, a = _task([(14, 21), (16, 25)], 15, (16, 25), 25)
    d = _branch_op(s, pool, t, a)
    assert (d.code, d.action, d.branch_index, d.created) == (0, abi.NDC_BACKFILL, 1, 1)
    assert _branch(s, pool, 1) == [(14, 21), (16, 25)] and s.current == 0
    # duplicate task (already applied events)
    t, a = _task([(14, 21), (20, 30)], 18, (20, 30), 30)
    assert _branch_op(s, pool, t, a).action == abi.NDC_SKIP
    # a gap: retry
    t, a = _task([(14, 21), (20, 30), (25, 30)], 23, (25, 30), 30)
    assert abi.STATUS[_branch_op(s, pool, t, a).code] == "E_NDC_RETRY_TASK"
    # an incoming task whose first event is already on the LCA's branch: duplicate
    t, a = _task([(14, 21), (15, 30)], 15, (15, 30), 30)
    assert _branch_op(s, pool, t, a).action == abi.NDC_SKIP


def test_ndc_same_version_as_current_last_write():
    """A task for a non-current branch with the current branch's last-write version:
    BadRequestError (nDCConflictResolver.go:100-105)."""
    s, pool = _vhs([(14, 21), (20, 30)])
    assert _add(s, pool, [(14, 21), (16, 35)], 1) == (0, True, 1)  # branch 1 becomes current
    t, a = _task([(14, 21), (20, 30), (22, 35)], 21, (22, 35), 35)
    d = _branch_op(s, pool, t, a)
    assert abi.STATUS[d.code] == "E_NDC_SAME_VERSION"
    assert _branch(s, pool, 0) == [(14, 21), (20, 30)]  # unchanged on error
