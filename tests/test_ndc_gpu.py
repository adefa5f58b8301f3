"""GPU parity of the NDC conflict-resolution path (cadence_amd/csrc/ndc.hip + the replay
kernels) against the CPU restatement (oracle/ndc_ref.cpp, replay_ref.cpp): the branch
kernel on randomised version histories and tasks (every decision and error site), the
forked synthetic config 5 end to end, and the reference's hand-crafted 3-branch history."""
import ctypes as C

import numpy as np
import pytest

from cadence_amd import abi, engine, ndc

from . import ndc_fixture

pytestmark = pytest.mark.gpu


def _vhs_state(vhs, pool, n):
    """The logical VersionHistories of every workflow (slots past a branch's items and
    branches past n_branches are scratch)."""
    out = []
    for w in range(n):
        s = vhs[w]
        out.append((s.current, s.n_branches, tuple(
            (bytes(s.branch[b].token), tuple(ndc.branch_items(vhs, pool, w, b))) for b in range(s.n_branches))))
    return out


def _copy(a):
    b = type(a)()
    C.memmove(b, a, C.sizeof(a))
    return b


def _random_cases(n, seed):
    """Branching version histories built the way replication builds them (a base, forks
    duplicated up to an LCA and extended with higher versions), then tasks derived from
    a random branch: truncated / extended, first event on, before or after the next ID,
    versions below, equal to or above the current branch's last write; 5% of the items
    corrupted (malformed histories)."""
    rng = np.random.default_rng(seed)
    cap = 16
    vhs, pool = ndc.new_vhs(n, cap)
    tasks = (abi.CdrNdcTask * n)()
    items = (abi.CdrVHItem * (n * cap))()
    for w in range(n):
        base, e, v = [], 0, int(rng.integers(1, 4))
        for _ in range(int(rng.integers(1, 5))):
            e += int(rng.integers(1, 20))
            base.append((e, v))
            v += int(rng.integers(1, 15))
        branches = [base]
        for _ in range(int(rng.integers(0, 4 if rng.random() < 0.9 else 9))):
            src = branches[int(rng.integers(len(branches)))]
            k = int(rng.integers(len(src)))
            cut = src[:k + 1]
            if rng.random() < 0.5 and k > 0:
                cut[-1] = (int(rng.integers(cut[-2][0] + 1, cut[-1][0] + 1)), cut[-1][1])
            b = list(cut)
            ee, vv = b[-1]
            for _ in range(int(rng.integers(1, 3))):
                ee += int(rng.integers(1, 10))
                vv += int(rng.integers(1, 30))
                b.append((ee, vv))
            branches.append(b)
        branches = branches[:abi.VHS_MAX_BRANCHES]
        s = vhs[w]
        s.n_branches = len(branches)
        s.current = int(np.argmax([b[-1][1] for b in branches])) if rng.random() < 0.8 else \
            int(rng.integers(len(branches)))
        for bi, b in enumerate(branches):
            s.branch[bi].token.tree = w
            s.branch[bi].token.branch_lo, s.branch[bi].token.branch_hi = bi, 7
            s.branch[bi].n_items = len(b)
            for i, (ee, vv) in enumerate(b):
                pool[s.items_off + bi * cap + i].event_id = ee
                pool[s.items_off + bi * cap + i].version = vv
        # the task: a branch's prefix, extended
        src = branches[int(rng.integers(len(branches)))]
        k = int(rng.integers(len(src)))
        inc = list(src[:k + 1])
        if rng.random() < 0.4 and inc[-1][0] > 1:
            inc[-1] = (int(rng.integers(max(1, inc[-2][0] + 1 if len(inc) > 1 else 1), inc[-1][0] + 1)), inc[-1][1])
        lca_e = inc[-1][0]
        ee, vv = inc[-1]
        cur_last = branches[s.current][-1][1]
        r = rng.random()
        newv = cur_last + int(rng.integers(1, 9)) if r < 0.45 else (cur_last if r < 0.55 else
                                                                   vv + int(rng.integers(0, 3)))
        ee += int(rng.integers(1, 6))
        inc.append((ee, max(newv, vv)))
        if rng.random() < 0.05:
            j = int(rng.integers(len(inc)))
            inc[j] = (inc[j][0], int(rng.integers(0, 100)))
        t = tasks[w]
        t.items_off, t.n_items = w * cap, len(inc)
        for i, (a, b) in enumerate(inc):
            items[w * cap + i].event_id, items[w * cap + i].version = a, b
        t.first_event_id = lca_e + 1 + int(rng.choice([-1, 0, 0, 0, 0, 1]))
        t.last_event_id, t.last_version = inc[-1]
        t.version = inc[-1][1]
        t.new_token.tree, t.new_token.branch_lo, t.new_token.branch_hi = w, 99, 9
    return tasks, items, vhs, pool


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ndc_branch_kernel_matches_oracle(engine_gpu, seed):
    import oracle
    n = 3000
    tasks, items, vhs, pool = _random_cases(n, seed)
    g_vhs, g_pool = _copy(vhs), _copy(pool)
    dec_gpu = ndc.GpuBackend(engine_gpu).branch(tasks, items, g_vhs, g_pool, n)
    dec_ref = oracle.NdcBackend().branch(tasks, items, vhs, pool, n)
    bad = [w for w in range(n) if bytes(dec_gpu[w]) != bytes(dec_ref[w])]
    assert not bad, [(w, abi.STATUS[dec_gpu[w].code], abi.STATUS[dec_ref[w].code]) for w in bad[:5]]
    assert _vhs_state(g_vhs, g_pool, n) == _vhs_state(vhs, pool, n)
    seen = {abi.STATUS[dec_ref[w].code] for w in range(n)} | {abi.NDC_ACTIONS[dec_ref[w].action] for w in range(n)}
    for want in ("OK", "SKIP", "APPLY_CURRENT", "REBUILD", "BACKFILL", "E_NDC_RETRY_TASK", "E_NDC_SAME_VERSION"):
        assert want in seen, (want, seen)


def _same_outputs(batch, a, b, what, tasks=False):
    """Records of every entry (lastDecision is not part of a persisted state)."""
    bad = engine.compare(batch, a, b, last_decision=False)
    if tasks:
        bad += engine.compare_tasks(batch, a, b)
    assert not bad, what + ": " + "\n".join(bad[:10])


def _replicate_both(eng, base, rebuild, forks, items_cap=None):
    """The device pipeline (cdr_ndc_replicate_async per round) against the CPU restatement
    (oracle.ndc_replicate: the rebuilt MutableState kept in memory): final states, version
    histories, decisions, and each round's rebuild (+ refreshTasks) and apply records."""
    import oracle
    rep = ndc.DeviceReplicator(eng, base, rebuild, forks, items_cap=items_cap)
    try:
        got = rep.run()
    finally:
        rep.close()
    ref = oracle.ndc_replicate(base, rebuild, forks, items_cap=items_cap, threads=4)
    n = base.n_wfs
    _same_outputs(base, got[0], ref[0], "final state")
    assert _vhs_state(got[1], got[2], n) == _vhs_state(ref[1], ref[2], n)
    for k, (dg, dr) in enumerate(zip(got[3], ref[3])):
        assert [bytes(dg[w]) for w in range(n)] == [bytes(dr[w]) for w in range(n)], k
        (rg, ag), (rr, ar) = got[4][k], ref[4][k]
        _same_outputs(rebuild, rg, rr, f"round {k} rebuild", tasks=True)
        _same_outputs(forks[k][0], ag, ar, f"round {k} apply")
    return got


def test_handcrafted_three_branches_gpu(engine_gpu):
    base, rebuild, forks, doc = ndc_fixture.handcrafted()
    final, vhs, pool, decs, _ = _replicate_both(engine_gpu, base, rebuild, forks)
    ndc_fixture.check_reference_outcome(final, vhs, pool, decs, doc)


@pytest.mark.parametrize("seed", [0x5EED0C05, 7])
def test_forked_config5_gpu(engine_gpu, seed):
    base, rebuild, forks = ndc.synth_forked(5, 400, seed)
    final, vhs, pool, decs, rounds = _replicate_both(engine_gpu, base, rebuild, forks)
    assert engine.status_histogram(final) == {"OK": 400}
    assert {abi.NDC_ACTIONS[decs[1][w].action] for w in range(400)} == {"REBUILD", "BACKFILL"}


def test_vh_item_capacity_gpu(engine_gpu):
    """Too few VersionHistories item slots: both sides fail the same workflows with
    CDR_E_VHS_CAPACITY (k_vhs_sync / cdro_vhs_sync), the rest replicate identically."""
    base, rebuild, forks = ndc.synth_forked(5, 200, 0x5EED0C07)
    final, *_ = _replicate_both(engine_gpu, base, rebuild, forks, items_cap=4)
    assert engine.status_histogram(final).get("E_VHS_CAPACITY", 0) > 0


@pytest.mark.parametrize("seed", [11, 12])
def test_forked_config5_faults_gpu(engine_gpu, seed):
    """Faulted forks: failing rebuilds / applies leave their errors in the state, later
    rounds skip those workflows — identically on both sides."""
    base, rebuild, forks = ndc.synth_forked(5, 300, seed, error_rate=0.2)
    final, *_ = _replicate_both(engine_gpu, base, rebuild, forks)
    assert len(engine.status_histogram(final)) > 1


def test_in_memory_carry_gpu(engine_gpu):
    """GPU twin of the in-memory carry KAT: the general kernel's carry prologue keeps the
    rebuilt builder's currentVersion when cdr_carry.in_memory says so."""
    import numpy as np
    from . import test_ndc
    suf, pre_out, outs = test_ndc.in_memory_case()
    for mem in (0, 1):
        suf.carry = engine.Carry(src=np.array([0], np.int32), state=pre_out, in_memory=np.array([mem], np.uint8))
        got = engine_gpu.replay(suf)
        bad = engine.compare(suf, got, outs[mem])
        assert not bad, (mem, bad[:5])


def test_forked_config5_1m_digests_gpu(engine_gpu):
    """The device-resident replication run at full size (1M forked config-5 workflows: base
    branch + two rounds, cdr_ndc_replicate_async) against oracle.ndc_replicate: every
    workflow's final persisted state by entry digest (k_digest / digest_ref.cpp), every
    round's decision and the current branch's VersionHistory (bench.py --ndc-forks times the
    same run, profiles/r3_ndc/bench_ndc_forks_1m.json)."""
    import oracle
    n = 1_000_000
    base, rebuild, forks = ndc.synth_forked(5, n, 0x5EED0C05)
    rep = ndc.DeviceReplicator(engine_gpu, base, rebuild, forks)
    try:
        _, g_vhs, g_pool, g_decs, _ = rep.run()
        per_d = rep.dev.alloc(n * 8)
        tot_d = rep.dev.alloc(8)
        rc = abi.lib().cdr_entry_digests_async(engine_gpu.ctx, C.byref(rep.base_db), C.byref(rep.state),
                                               C.c_void_p(per_d), C.c_void_p(tot_d), None)
        assert rc == 0
        got_c = (C.c_uint64 * n)()
        rep.dev.down(got_c, per_d, n * 8)
        got = np.frombuffer(got_c, np.uint64).copy()
    finally:
        rep.close()
    r_state, r_vhs, r_pool, r_decs, _ = oracle.ndc_replicate(base, rebuild, forks, threads=16)
    want, _ = oracle.entry_digests(base, ndc.state_caps_for(base, rebuild, forks), r_state, threads=16)
    assert engine.status_histogram(r_state) == {"OK": n}
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, bad[:10]
    for k in range(len(forks)):
        assert all(bytes(g_decs[k][w]) == bytes(r_decs[k][w]) for w in range(n)), k
    assert all(ndc.branch_items(g_vhs, g_pool, w, g_vhs[w].current) ==
               ndc.branch_items(r_vhs, r_pool, w, r_vhs[w].current) for w in range(n))
