"""Audit hand-counted vmcnt code (device_common.h vld16 / vm_wait) in gfx950
assembly: simulate the wave's vector-memory queue over the control-flow graph
of each kernel and report every instruction that touches (reads or writes) a
VGPR that is still the destination of an in-flight global/buffer load, i.e.
before an `s_waitcnt vmcnt(n)` has retired that load.

A hit means the register allocator moved, copied or reused a register the
hardware will still write: the late data lands in whatever the register holds
by then (an address, a loop counter, ...).

Usage: python tools/vmcnt_audit.py file.s [kernel-substring]
"""
import re
import sys
from collections import defaultdict

VMEM = re.compile(r"^(global_load|global_store|buffer_load|buffer_store|global_atomic|buffer_atomic|"
                  r"flat_load|flat_store|scratch_load|scratch_store)")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(path):
    funcs, cur, name = {}, None, None
    for line in open(path):
        s = line.split(";")[0].rstrip()
        if not s.strip():
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", s) and not s.startswith("\t"):
            lab = s.split(":")[0]
            if lab.startswith("_Z") or (cur is None and not lab.startswith(".")):
                name = lab
                cur = funcs.setdefault(name, [])
            if cur is not None:
                cur.append(("label", lab))
            continue
        if cur is None:
            continue
        t = s.strip()
        if t.startswith(".") or t.startswith("s_endpgm") and False:
            if t.startswith(".Lfunc_end"):
                cur = None
            continue
        cur.append(("ins", t))
        if t.startswith("s_endpgm"):
            pass
    return funcs


def blocks(ins):
    bl, lab_of, cur = [], {}, []
    for kind, v in ins:
        if kind == "label":
            if cur:
                bl.append(cur)
            cur = []
            lab_of[v] = len(bl)
            continue
        cur.append(v)
        if v.startswith("s_branch") or v.startswith("s_cbranch") or v.startswith("s_endpgm") \
                or v.startswith("s_setpc"):
            bl.append(cur)
            cur = []
    if cur:
        bl.append(cur)
    # label -> block index (labels point to the next block)
    succ = defaultdict(list)
    # rebuild with label positions
    return bl, lab_of


def audit(ins, max_states=64):
    # build blocks with label starts
    bl, starts, cur, labels_at = [], {}, [], {}
    for kind, v in ins:
        if kind == "label":
            if cur:
                bl.append(cur)
                cur = []
            starts[v] = len(bl)
            continue
        cur.append(v)
        if re.match(r"s_(branch|cbranch|endpgm|setpc)", v):
            bl.append(cur)
            cur = []
    if cur:
        bl.append(cur)
    succs = []
    for i, b in enumerate(bl):
        last = b[-1]
        s = []
        m = re.match(r"s_(c?branch\w*)\s+(\S+)", last)
        if last.startswith("s_endpgm") or last.startswith("s_setpc"):
            pass
        elif m:
            tgt = starts.get(m.group(2))
            if tgt is not None:
                s.append(tgt)
            if m.group(1) != "branch" and i + 1 < len(bl):
                s.append(i + 1)
        elif i + 1 < len(bl):
            s.append(i + 1)
        succs.append(s)
    seen = defaultdict(set)
    work = [(0, ())]
    hits = []
    while work:
        bi, st = work.pop()
        if st in seen[bi] or len(seen[bi]) >= max_states:
            continue
        seen[bi].add(st)
        q = list(st)
        for insn in bl[bi]:
            op = insn.split()[0]
            pend = set()
            for e in q:
                if e:
                    pend |= set(e)
            m = re.search(r"vmcnt\((\d+)\)", insn) if op == "s_waitcnt" else None
            if m:
                n = int(m.group(1))
                while len(q) > n:
                    q.pop(0)
                continue
            if op == "s_waitcnt" and "vmcnt" not in insn and "lgkmcnt" in insn:
                continue
            used = regs(insn) if op.startswith("v_") or op.startswith("ds_") or VMEM.match(op) or \
                op.startswith("s_") else set()
            if VMEM.match(op):
                operands = insn[len(op):]
                if "load" in op:
                    # global_load_lds: the first operand is the address (the data
                    # goes to LDS); a load's destination may be the destination
                    # of an older in-flight load (loads return in order)
                    lds = "_lds" in op
                    dst = set() if lds else regs(operands.split(",")[0])
                    src = regs(operands) if lds else regs(",".join(operands.split(",")[1:]))
                    bad = src & pend
                    if bad:
                        hits.append((bi, insn, sorted(bad)))
                    q.append(tuple(sorted(dst)))
                else:
                    bad = used & pend
                    if bad:
                        hits.append((bi, insn, sorted(bad)))
                    q.append(())
                continue
            bad = used & pend
            if bad:
                hits.append((bi, insn, sorted(bad)))
        for s in succs[bi]:
            work.append((s, tuple(q)))
    return hits, len(bl)


def _cfg(ins):
    bl, starts, cur = [], {}, []
    for kind, v in ins:
        if kind == "label":
            if cur:
                bl.append(cur)
                cur = []
            starts[v] = len(bl)
            continue
        cur.append(v)
        if re.match(r"s_(branch|cbranch|endpgm|setpc)", v):
            bl.append(cur)
            cur = []
    if cur:
        bl.append(cur)
    succs = []
    for i, b in enumerate(bl):
        last, s = b[-1], []
        m = re.match(r"s_(c?branch\w*)\s+(\S+)", last)
        if last.startswith("s_endpgm") or last.startswith("s_setpc"):
            pass
        elif m:
            tgt = starts.get(m.group(2))
            if tgt is not None:
                s.append(tgt)
            if m.group(1) != "branch" and i + 1 < len(bl):
                s.append(i + 1)
        elif i + 1 < len(bl):
            s.append(i + 1)
        succs.append(s)
    return bl, succs


WRITES_ONLY = "--writes" in sys.argv


def _step(insn, q, hits=None, bi=None):
    """Advance the in-flight queue q (list of dest-register tuples, oldest
    first; () for stores) over one instruction; record hits."""
    op = insn.split()[0]
    pend = set()
    for e in q:
        pend |= set(e)
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", insn)
        if m:
            n = int(m.group(1))
            while len(q) > n:
                q.pop(0)
        return
    used = regs(insn)
    if VMEM.match(op):
        operands = insn[len(op):]
        if "load" in op:
            lds = "_lds" in op
            dst = set() if lds else regs(operands.split(",")[0])
            bad = (used - dst) & pend
            q.append(tuple(sorted(dst)))
        else:
            bad = used & pend
            q.append(())
    else:
        bad = used & pend
        if WRITES_ONLY:
            # the first operand of a VALU / DS read is its destination
            ops = insn[len(op):].split(",")
            dst = regs(ops[0]) if (op.startswith("v_") and not op.startswith("v_cmp")) or \
                op.startswith("ds_read") else set()
            bad = dst & pend
    if bad and hits is not None:
        hits.append((bi, insn, sorted(bad)))


def _wait_only(block):
    return all(i.startswith("s_waitcnt") or i.startswith("s_branch") or i.startswith("s_nop")
               for i in block)


def _merge(bi, ins_states, preds, bl):
    """Join of the in-flight queues of bi's predecessors.  The cases of a
    switch-dispatched vm_wait(n) (blocks holding only a waitcnt) join with the
    strongest case (the count is runtime-uniform and assumed right); every
    other join -- if/else of roles, loop back-edges -- keeps the longest queue
    (a load in flight on some path is in flight)."""
    states = [s for _, s in ins_states]
    fpreds = [pi for pi in preds[bi] if pi < bi]
    if fpreds and all(_wait_only(bl[pi]) for pi in fpreds):
        st = min(states, key=len)
        return st
    return max(states, key=len)


def audit_must(ins, rounds=50):
    """Must-analysis: a load counts as in flight at a forward join only if it is
    in flight on every incoming path (the switch-dispatched vm_wait(n) of
    device_common.h joins its cases this way: the strongest case wins), and on
    a loop back-edge if it is in flight on any.  A hit therefore means a path
    on which NO wait retired the load before the register was touched."""
    bl, succs = _cfg(ins)
    preds = defaultdict(list)
    for i, ss in enumerate(succs):
        for j in ss:
            preds[j].append(i)
    out = [None] * len(bl)
    for _ in range(rounds):
        changed = False
        for bi in range(len(bl)):
            ins_states = []
            for pi in preds[bi]:
                if out[pi] is not None:
                    ins_states.append((pi >= bi, out[pi]))
            if bi == 0:
                st = ()
            elif not ins_states:
                continue
            else:
                st = _merge(bi, ins_states, preds, bl)
            q = list(st)
            for insn in bl[bi]:
                _step(insn, q)
            new = tuple(q)
            if out[bi] != new:
                out[bi] = new
                changed = True
        if not changed:
            break
    hits = []
    for bi in range(len(bl)):
        ins_states = [(pi >= bi, out[pi], pi) for pi in preds[bi] if out[pi] is not None]
        st = _merge(bi, [(b, s2) for b, s2, _ in ins_states], preds, bl) if ins_states else ()
        q = list(st)
        for insn in bl[bi]:
            _step(insn, q, hits, bi)
    return hits, len(bl)


if __name__ == "__main__":
    funcs = parse(sys.argv[1])
    args = [a for a in sys.argv[2:] if not a.startswith("--")]
    filt = args[0] if args else ""
    for name, ins in funcs.items():
        if filt not in name:
            continue
        if not any(k == "ins" and re.search(r"s_waitcnt vmcnt\(([1-9]\d*)\)", v) for k, v in ins):
            continue
        hits, nb = (audit(ins) if "--may" in sys.argv else audit_must(ins))
        uniq = {}
        for bi, insn, r in hits:
            uniq.setdefault(insn, r)
        print(f"{name}: {nb} blocks, {len(uniq)} distinct instructions touching in-flight load registers")
        for insn, r in list(uniq.items())[:40]:
            print(f"    {insn}    <- v{r}")
