"""Reaching definitions of one VGPR at one instruction of a disassembled gfx950 kernel
(the output of tools/isa.sh, one kernel cut out): builds the CFG from the branch targets
and lists every instruction that writes the register and reaches the use, with its
predecessor chain.  A diagnostic for register-allocation questions (which definitions a
value at a store can come from).

usage: python tools/isa_reach.py kernel.s <use line number (1-based)> <register: v12 | a3>
"""
import re
import sys


def parse(path):
    ins = []  # (line_no, addr, text)
    for i, line in enumerate(open(path), 1):
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            ins.append((i, int(m.group(2), 16), m.group(1), line.rstrip()))
    return ins


def target(line, base):
    m = re.search(r"<[^>+]*\+0x([0-9a-f]+)>", line)
    if m:
        return base + int(m.group(1), 16)
    m = re.search(r"<[^>+]*>", line)
    return base if m else None


def regs_written(text):
    """VGPR numbers the instruction writes (its first operand, for VALU / loads / reads)."""
    op = text.split()[0]
    if op.startswith(("global_store", "buffer_store", "scratch_store", "ds_write", "s_", "flat_store",
                      "global_atomic", "ds_store")) and "_rtn" not in op:
        if not (op.startswith("s_") and False):
            return set()
    if op.startswith("s_"):
        return set()
    args = text[len(op):].strip()
    if not args:
        return set()
    first = args.split(",")[0].strip()
    m = re.match(r"([va])\[(\d+):(\d+)\]$", first)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", first)
    if m:
        return {first}
    return set()


def main():
    path, use_line, reg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    reg = reg if reg[0] in "va" else "v" + reg
    ins = parse(path)
    base = ins[0][1]
    idx_of_addr = {a: k for k, (_, a, _, _) in enumerate(ins)}
    n = len(ins)
    succ = [[] for _ in range(n)]
    for k, (ln, a, t, raw) in enumerate(ins):
        op = t.split()[0]
        if op == "s_branch":
            tg = target(raw, base)
            succ[k].append(idx_of_addr[tg])
        elif op.startswith("s_cbranch"):
            tg = target(raw, base)
            succ[k].append(idx_of_addr[tg])
            if k + 1 < n:
                succ[k].append(k + 1)
        elif op in ("s_endpgm", "s_setpc_b64"):
            pass
        else:
            if k + 1 < n:
                succ[k].append(k + 1)
    pred = [[] for _ in range(n)]
    for k in range(n):
        for s in succ[k]:
            pred[s].append(k)
    use = next(k for k, (ln, _, _, _) in enumerate(ins) if ln == use_line)
    # backward search: from the use, walk predecessors until a def of reg
    seen = set()
    defs = {}
    stack = [(p, use) for p in pred[use]]
    while stack:
        k, frm = stack.pop()
        if k in seen:
            continue
        seen.add(k)
        if reg in regs_written(ins[k][2]):
            defs.setdefault(k, frm)
            continue
        for p in pred[k]:
            stack.append((p, k))
    for k in sorted(defs):
        print(f"line {ins[k][0]}: {ins[k][2]}")


if __name__ == "__main__":
    main()
