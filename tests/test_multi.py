"""Multi-rank (N>1) path of bench.py on CPU: gloo, world size 2.

The replay shards with no data-path collective: historyShardID = Fingerprint32(wid) %
16384 (common/util.go:249-252), shards -> ranks greedily, each rank replays only its
workflows, and one all-reduce (sum) of {events, entries, ok, checksum} closes the step
(bench.reduce_step, the function bench.main calls).  Here each rank replays its share
with the CPU restatement (oracle/, the parity checker — no GPU in this container) and
hashes it with the restatement of the product checksum (cdr_checksum_async's per-entry
k_digest hash, oracle/digest_ref.cpp); the all-reduced totals must equal a
single-process replay of the whole population."""
import os
import socket

import numpy as np
import pytest

import bench
import oracle
from cadence_amd import abi, engine

TOTAL = 600
SEED = 0x5EED0003


def _stats(batch, out):
    """[events, entries, OK entries, checksum] as bench.main builds them: the checksum is
    cdr_checksum_async's (the sum of per-entry k_digest hashes), restated."""
    n_ev = len(batch.events)
    ok = sum(1 for w in range(batch.n_wfs) if out.result[w].code == abi.OK)
    _, cs = oracle.entry_digests(batch, out.plan, out)
    return [n_ev, batch.n_wfs, ok, cs - 2 ** 64 if cs >= 2 ** 63 else cs]


def _share(mine, cfg):
    b = engine.synth_batch(cfg, len(mine), SEED, index_map=mine)
    return b, oracle.replay(b)


def _rank(rank, world, port, cfg, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine, _ = bench.assign_shards(TOTAL, world, rank, bench.workflow_weights(cfg, TOTAL, SEED))
        b, out = _share(mine, cfg)
        stats, elapsed = bench.reduce_step(dist, torch, torch.tensor(_stats(b, out), dtype=torch.int64),
                                           1.0 + rank)
        owned = [None] * world
        dist.all_gather_object(owned, mine.tolist())
        if rank == 0:
            q.put((stats, elapsed, owned))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("cfg", [3, 4])
def test_two_rank_shards_match_single_process(cfg):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, cfg, q)) for r in range(2)]
    for p in procs:
        p.start()
    stats, elapsed, owned = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the shard->rank assignment partitions the population
    allw = np.sort(np.concatenate([np.array(o, np.int64) for o in owned]))
    assert np.array_equal(allw, np.arange(TOTAL))
    assert all(len(o) > 0 for o in owned)
    # the all-reduced totals equal one process replaying everything; the timed region is
    # the slowest rank's
    b, out = _share(np.arange(TOTAL, dtype=np.uint32), cfg)
    assert stats == _stats(b, out)
    assert elapsed == 2.0


def test_shard_assignment_balances_events():
    lengths = np.random.default_rng(1).lognormal(np.log(200), 1.0, TOTAL)
    loads = []
    for r in range(4):
        mine, load = bench.assign_shards(TOTAL, 4, r, lengths)
        loads.append(lengths[mine].sum())
    assert np.isclose(sum(loads), lengths.sum())
    assert max(loads) / (sum(loads) / 4) < 1.25


# ---- the configs[4] conflict-resolution line and the carry-in line, multi-rank
# (bench.ndc_forks_line / bench.carry_line shard the same way: historyShardID -> greedy
# shard->rank, no data-path collective, one all-reduce of [events, workflows, OK, digest sum])
NDC_TOTAL = 240


def _ndc_stats(mine):
    from cadence_amd import ndc
    base, rebuild, forks = ndc.synth_forked(5, len(mine), SEED, index_map=mine)
    state, _, _, decs, rounds = oracle.ndc_replicate(base, rebuild, forks)
    events = bench.ndc_counts(base, rebuild, forks, rounds, decs)[0]
    ok = sum(1 for w in range(base.n_wfs) if state.result[w].code == abi.OK)
    _, cs = oracle.entry_digests(base, state.plan, state)
    return [events, base.n_wfs, ok, cs - 2 ** 64 if cs >= 2 ** 63 else cs]


def _carry_stats(mine, cfg):
    b = engine.synth_batch(cfg, len(mine), SEED, index_map=mine)
    cut = engine.split_half(b)
    pre, suf = engine.cut_batches(b, cut)
    pre_out = oracle.replay(pre)
    codes = np.array([pre_out.result[w].code for w in range(b.n_wfs)])
    src = np.where((cut > 0) & (codes == abi.OK), np.arange(b.n_wfs), -1).astype(np.int32)
    for w in np.nonzero((cut > 0) & (codes != abi.OK))[0]:
        suf.wfs[w] = b.wfs[w]
    suf.carry = engine.Carry(src=src, state=pre_out)
    out = oracle.replay(suf, tasks=True)
    events = int(sum(suf.wfs[w].ev_len for w in range(suf.n_wfs)))
    ok = sum(1 for w in range(suf.n_wfs) if out.result[w].code == abi.OK)
    _, cs = oracle.entry_digests(suf, out.plan, out)
    return [events, len(mine), ok, cs - 2 ** 64 if cs >= 2 ** 63 else cs]


def _rank_line(rank, world, port, kind, cfg, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total = NDC_TOTAL if kind == "ndc" else TOTAL
        mine, _ = bench.assign_shards(total, world, rank, bench.workflow_weights(cfg, total, SEED))
        st = _ndc_stats(mine) if kind == "ndc" else _carry_stats(mine, cfg)
        stats, elapsed = bench.reduce_step(dist, torch, torch.tensor(st, dtype=torch.int64), 2.0 - rank)
        if rank == 0:
            q.put((stats, elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,cfg", [("ndc", 5), ("carry", 3), ("carry", 5)])
def test_two_rank_lines_match_single_process(kind, cfg):
    """bench.py --ndc-forks / --carry at world size 2: the all-reduced totals of the ranks'
    shards equal one process replicating (replaying) the whole population."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_line, args=(r, 2, port, kind, cfg, q)) for r in range(2)]
    for p in procs:
        p.start()
    stats, elapsed = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = NDC_TOTAL if kind == "ndc" else TOTAL
    everything = np.arange(total, dtype=np.uint32)
    assert stats == (_ndc_stats(everything) if kind == "ndc" else _carry_stats(everything, cfg))
    assert stats[2] > 0
    assert elapsed == 2.0
