#!/usr/bin/env python3
"""Approximate VGPR liveness over a kernel's gfx950 assembly (diagnostic):
backward dataflow over the basic blocks, VALU/DS/VMEM defs and uses parsed
from the operands (partial-exec writes treated as full defs).  Prints the
program points with the most live 32-bit VGPRs and their context, to find
where a kernel's register demand peaks.

usage: tools/vgpr_live.py FILE.s KERNEL_SYMBOL [TOP]"""
import re
import sys


def regs(tok):
    tok = tok.strip()
    m = re.match(r"^-?v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^-?\|?v(\d+)\|?$", tok)
    if m:
        return [int(m.group(1))]
    return []


def split_ops(rest):
    out, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        if ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [o.strip().split()[0] if o.strip() else "" for o in out]


def defs_uses(op, ops):
    d, u = [], []
    allr = [regs(o) for o in ops]
    if op.startswith(("ds_write", "ds_store", "global_store", "buffer_store", "flat_store", "scratch_store")):
        for r in allr:
            u += r
        return d, u
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "s_")):
        for r in allr:
            u += r
        return d, u
    if not allr:
        return d, u
    d = allr[0]
    for r in allr[1:]:
        u += r
    if op.startswith(("v_fmac", "v_mac", "v_writelane")) or "dpp" in op:
        u += d
    return d, u


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    L = open(path).read().split("\n")
    st = [i for i, l in enumerate(L) if l.startswith(sym + ":")][0]
    en = [i for i, l in enumerate(L) if i > st and l.startswith(".Lfunc_end")][0]
    ins, labels = [], {}
    for i in range(st + 1, en + 1):
        t = L[i].split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            labels[t[:-1]] = len(ins)
            continue
        if t.startswith("."):
            continue
        parts = t.split(None, 1)
        ins.append((i, parts[0], split_ops(parts[1]) if len(parts) > 1 else []))
    n = len(ins)
    # basic blocks
    starts = {0} | set(labels.values())
    for k, (_, op, ops) in enumerate(ins):
        if op.startswith(("s_cbranch", "s_branch", "s_setpc")) and k + 1 < n:
            starts.add(k + 1)
    starts = sorted(s for s in starts if s < n)
    bid = {}
    blocks = []
    for j, s0 in enumerate(starts):
        e0 = starts[j + 1] if j + 1 < len(starts) else n
        blocks.append((s0, e0))
        for k in range(s0, e0):
            bid[k] = j
    succ = []
    for j, (s0, e0) in enumerate(blocks):
        _, op, ops = ins[e0 - 1]
        sc = []
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = ops[0] if ops else ""
            if tgt in labels and labels[tgt] in bid:
                sc.append(bid[labels[tgt]])
            if op.startswith("s_cbranch") and j + 1 < len(blocks):
                sc.append(j + 1)
        elif op != "s_endpgm" and j + 1 < len(blocks):
            sc.append(j + 1)
        succ.append(sc)
    du = [defs_uses(op, ops) for (_, op, ops) in ins]
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for j in range(len(blocks) - 1, -1, -1):
            s0, e0 = blocks[j]
            live = set()
            for s in succ[j]:
                live |= live_in[s]
            for k in range(e0 - 1, s0 - 1, -1):
                d, u = du[k]
                live -= set(d)
                live |= set(u)
            if live != live_in[j]:
                live_in[j] = live
                changed = True
    pts = []
    for j, (s0, e0) in enumerate(blocks):
        live = set()
        for s in succ[j]:
            live |= live_in[s]
        for k in range(e0 - 1, s0 - 1, -1):
            d, u = du[k]
            live -= set(d)
            live |= set(u)
            pts.append((len(live), k))
    pts.sort(reverse=True)
    seen = []
    for cnt, k in pts:
        if any(abs(k - s) < 40 for s in seen):
            continue
        seen.append(k)
        line = ins[k][0]
        print("live %d at asm line %d: %s" % (cnt, line + 1, L[line].strip()[:70]))
        if len(seen) >= top:
            break


if __name__ == "__main__":
    main()
