"""Carry-in diagnostics: replays the carry-in scenarios of tests/test_carry.py (2DC builders,
the default route and the hand-on chain) on the library named by CDR_LIB (default: the
in-tree one) and, for every entry whose output differs from the oracle, prints the entry's
plan (caps flags = which register-table variant), its result, and the replication-state
fields that differ beside the loaded ones.  This is how the round-6 LastReplicationInfo loss
was narrowed to the 12-activity carry variant before its ISA was read
(tools/isa_execz_lint.py).

usage: [CDR_LIB=variants/libcdr_<name>.so] python tools/carry_probe.py
"""
import os
import sys


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (the HIP runtime libcdr binds to, tests/conftest.py)

from cadence_amd import abi, engine  # noqa: E402
import oracle  # noqa: E402

def scenario(e, name, cfg, n, seed, split_seed, builder=-1, err=0.0, small=False):
    b = engine.synth_batch(cfg, n, seed=seed, builder=builder, error_rate=err)
    pre, cut = engine.split_batch(b, split_seed)
    pre_gpu = e.replay(pre)
    sb = engine.suffix_batch(b, cut, pre, pre_gpu)
    ref = oracle.replay(sb)
    pl = engine.plan(sb)
    if small:
        for w in range(sb.n_wfs):
            if sb.carry.src[w] >= 0 and pl.caps[w].flags & (abi.CAP_REG | abi.CAP_REG2):
                pl.caps[w].flags |= abi.CAP_REG | abi.CAP_REG0
    got = e.replay(sb, pl)
    bad = engine.compare(sb, got, ref, limit=1000)
    print(f"== {name}: {len(bad)} mismatches")
    for line in bad[:40]:
        w = int(line.split()[1].rstrip(":"))
        d = sb.wfs[w]
        print(f"  {line}")
        print(f"    builder={d.builder} newrun={d.newrun} newrun_call={d.newrun_call} parent={d.parent} "
              f"src={sb.carry.src[w]} caps.flags={pl.caps[w].flags:#x} code={got.result[w].code} "
              f"flags={got.result[w].flags:#x} ref.code={ref.result[w].code} ref.flags={ref.result[w].flags:#x}")
        if sb.carry.src[w] >= 0:
            print(f"    loaded lri_mask={pre_gpu.repl[w].lri_mask} got={got.repl[w].lri_mask} ref={ref.repl[w].lri_mask} "
                  f"got.cur={got.repl[w].current_version} ref.cur={ref.repl[w].current_version}")
            ga, ra = got.repl[w], ref.repl[w]
            for f, _ in abi.CdrReplState._fields_:
                x, y = getattr(ga, f), getattr(ra, f)
                x = list(x) if hasattr(x, "__len__") else x
                y = list(y) if hasattr(y, "__len__") else y
                if x != y:
                    print(f"      {f}: got {x} ref {y} loaded {getattr(pre_gpu.repl[w], f) if not hasattr(getattr(pre_gpu.repl[w], f), '__len__') else list(getattr(pre_gpu.repl[w], f))}")
    return len(bad)


def main():
    e = engine.Engine(0)
    e.set_cls(abi.CLS_BUILD)
    tot = 0
    tot += scenario(e, "carry_builders[2DC]", 0, 300, 41 + abi.BUILDER_2DC, abi.BUILDER_2DC + 3,
                    builder=abi.BUILDER_2DC, err=0.2)
    tot += scenario(e, "chain_builders[2DC]", 3, 300, 71 + abi.BUILDER_2DC, abi.BUILDER_2DC + 5,
                    builder=abi.BUILDER_2DC, err=0.15, small=True)
    for cfg in (0, 3, 4):
        tot += scenario(e, f"kernel_tiers[{cfg}] default", cfg, 400, 0x5EED0400 + cfg, cfg + 11,
                        err=0.1 if cfg in (0, 3) else 0.0)
    e.close()
    print("total mismatches", tot)


if __name__ == "__main__":
    main()
