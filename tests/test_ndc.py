"""NDC conflict resolution on the CPU restatement (oracle/): the reference's hand-crafted
3-branch history and the forked synthetic config 5, through cadence_amd.ndc.replicate
(branch decisions, nDCStateRebuilder rebuild + VersionHistory verification, apply)."""
import collections
import ctypes as C

from cadence_amd import abi, engine, ndc

from . import ndc_fixture


def test_handcrafted_three_branches_oracle():
    import oracle
    base, rebuild, forks, doc = ndc_fixture.handcrafted()
    final, vhs, pool, decs, info = ndc.replicate(oracle.NdcBackend(), base, rebuild, forks)
    ndc_fixture.check_reference_outcome(final, vhs, pool, decs, doc)
    assert info["replayed_events"] == 20 + 14 + 1


def test_forked_config5_oracle_invariants():
    """Every fork A forces a rebuild (its version is above every base version); fork B
    rebuilds or backfills; rebuilt version histories always verify; the final current
    branch holds the highest last-write version (IsRebuilt false) and its items are the
    replayed state's version history."""
    import oracle
    n = 200
    base, rebuild, forks = ndc.synth_forked(5, n, 0x5EED0C05)
    final, vhs, pool, decs, info = ndc.replicate(oracle.NdcBackend(), base, rebuild, forks)
    assert engine.status_histogram(final) == {"OK": n}
    a = collections.Counter(abi.NDC_ACTIONS[decs[0][w].action] for w in range(n) if decs[0][w].code == abi.OK)
    b = collections.Counter(abi.NDC_ACTIONS[decs[1][w].action] for w in range(n) if decs[1][w].code == abi.OK)
    assert a == {"REBUILD": n}
    assert set(b) == {"REBUILD", "BACKFILL"}
    for w in range(n):
        s = vhs[w]
        assert s.n_branches == 3
        assert oracle.lib().cdro_vhs_is_rebuilt(C.byref(s), pool) == 0  # IsRebuilt: current = newest
        last = [ndc.branch_items(vhs, pool, w, k)[-1][1] for k in range(3)]
        assert last[s.current] == max(last)
        cur = ndc.branch_items(vhs, pool, w, s.current)
        assert [(i.event_id, i.version) for i in final.rows(w, "vh")] == cur
        # fork point: every branch shares the base's items up to it
        f = forks[0][1][w].first_event_id - 1
        pre = [it for it in ndc.branch_items(vhs, pool, w, 0) if it[0] < f]
        for k in (1, 2):
            assert ndc.branch_items(vhs, pool, w, k)[:len(pre)] == pre
