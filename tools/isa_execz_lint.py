"""Exec-zero lint for the gfx950 disassembly of libcdr's kernels.

Why: the ROCm 7.2 compiler (clang 22.0.0git roc-7.2.0) can place a vector register copy
made by the register allocator's live-range splitting in front of the exec-restoring
`s_or_b64 exec, exec, s[..]` that ends a divergent region (the SGPR allocation pass first
rematerialises a scalar constant at the top of that join block, after which the VGPR pass
no longer recognises the exec restore as the block's prologue).  Where that block is
entered from a divergent loop's exit (`s_andn2_b64 exec, exec, ..; s_cbranch_execnz
<loop>`) or from an `s_cbranch_execz` skip, exec is 0 when the copy executes, so the copy
writes no lane and the value is lost (DESIGN.md §3 "Round 6: the LastReplicationInfo loss").

The lint walks every kernel and reports each instruction that writes a VGPR / AGPR while
exec is provably zero: after the fall-through of such a loop exit, or at the target of an
`s_cbranch_execz`, up to the first instruction that writes exec again.  A vector write
there is dead code at best and a lost value at worst; libcdr's build requires none.

usage: python tools/isa_execz_lint.py <disassembly.s | object.o with a HIP fat binary> ...
(exit 1 on findings; cadence_amd/csrc/Makefile runs it on every kernel object it builds)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

FN = re.compile(r"^([0-9a-f]+) <(.*)>:$")
INS = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):")
TGT = re.compile(r"<([^>+]*)(?:\+0x([0-9a-f]+))?>")


def kernels(path):
    cur, name, base = None, None, 0
    for line in open(path):
        m = FN.match(line.rstrip())
        if m:
            if cur:
                yield name, base, cur
            name, base, cur = m.group(2), int(m.group(1), 16), []
            continue
        m = INS.match(line)
        if m and cur is not None:
            cur.append((int(m.group(2), 16), m.group(1), line))
    if cur:
        yield name, base, cur


def writes_exec(text):
    op = text.split()[0]
    args = text[len(op):]
    first = args.split(",")[0].strip() if args.strip() else ""
    return first == "exec" or op.endswith("saveexec_b64") or op.endswith("saveexec_b32") or "exec_lo" == first


def writes_vector(text):
    """The instruction writes a VGPR / AGPR under the exec mask (v_writelane ignores exec)."""
    op = text.split()[0]
    if op.startswith(("s_", "global_store", "buffer_store", "scratch_store", "ds_write", "ds_store",
                      "flat_store", "v_writelane", "v_readlane", "v_readfirstlane", "v_cmp")):
        return False
    args = text[len(op):].strip()
    if not args:
        return False
    first = args.split(",")[0].strip()
    return bool(re.match(r"^[va](\d+|\[\d+:\d+\])$", first))


def _scan(ins, start, stop_ok):
    """Vector writes from ins[start] up to the first exec write (returned if stop_ok(it))."""
    hits = []
    for j in range(start, len(ins)):
        t = ins[j][1]
        if writes_exec(t):
            return hits if stop_ok(t) else []
        if writes_vector(t):
            hits.append(j)
        op = t.split()[0]
        if op in ("s_branch", "s_endpgm", "s_setpc_b64") or op.startswith("s_cbranch"):
            return []
    return []


def lint(path):
    """(kernel, address, instruction) of every vector write executed with exec provably
    zero or narrowed below its region: (1) after a divergent loop's exit
    (`s_andn2_b64 exec, exec, ..` + backward `s_cbranch_execnz`) before exec is restored;
    (2) in the join block of `s_and_saveexec_b64 sN, ..; s_cbranch_execz J` before J's
    `s_or_b64 exec, exec, sN` (there exec is the then-lanes or zero, never the region's)."""
    bad = []
    for name, base, ins in kernels(path):
        addr_idx = {a: i for i, (a, _, _) in enumerate(ins)}
        for i, (a, t, raw) in enumerate(ins):
            op = t.split()[0]
            if i == 0:
                continue
            m = TGT.search(raw)
            tgt = base + int(m.group(2) or "0", 16) if m else None
            if op == "s_cbranch_execnz" and tgt is not None and tgt <= a and \
                    ins[i - 1][1].startswith("s_andn2_b64 exec, exec"):
                hits = _scan(ins, i + 1, lambda t: True)
            elif op == "s_cbranch_execz" and tgt in addr_idx:
                sv = re.match(r"s_and_saveexec_b64 (s\[\d+:\d+\])", ins[i - 1][1])
                if not sv:
                    continue
                end = "s_or_b64 exec, exec, " + sv.group(1)
                hits = _scan(ins, addr_idx[tgt], lambda t, end=end: t.strip() == end)
            else:
                continue
            bad.extend((name, ins[j][0], ins[j][1]) for j in hits)
    return bad


def disassemble(obj, tmp):
    """gfx950 disassembly of the device code in a host object built by hipcc."""
    fb, co, asm = (os.path.join(tmp, os.path.basename(obj) + x) for x in (".fatbin", ".co", ".s"))
    r = subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fb, obj], capture_output=True)
    if r.returncode != 0 or not os.path.exists(fb) or os.path.getsize(fb) == 0:
        return None  # a host-only object (no device code)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                    "--targets=" + TARGET, "--output=" + co], check=True)
    with open(asm, "w") as f:
        subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, stdout=f)
    return asm


def main():
    total = 0
    tmp = tempfile.mkdtemp(prefix="execz_")
    for p in sys.argv[1:]:
        src = disassemble(p, tmp) if p.endswith(".o") else p
        if src is None:
            continue
        bad = lint(src)
        total += len(bad)
        for name, a, t in bad:
            print(f"{p}: {name} @{a:#x}: {t}")
    print(f"exec-zero vector writes: {total}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
