"""Static check of the async-load discipline in the LDS kernel's ISA (hipcc -S output).

For every inline-asm global_load (or returning global_atomic) into v[a:b], every control-flow path from the load (following s_branch /
s_cbranch_* targets and fall-through) must reach a counted wait (inline-asm s_waitcnt) or a full vmcnt(0)
drain before any other instruction reads or writes v[a..b]; the only exception is another inline-asm load
into the same registers (its "+v" operand keeps them allocated).  Spills are covered: a scratch_store of such
a register on such a path is a read of it.

Loads tagged "smg:wave0" in the inline asm (the scheduling ticket and the ion descriptor of ion_pipe_kernel) are
issued and waited by wave 0 only, under wave-uniform conditions that hold for every lane of wave 0; the other
waves branch around both with an exec-zero edge (the taken edge of s_cbranch_execz, or the fall-through of
s_cbranch_execnz).  For them the paths are searched twice: without any exec-zero edge (the issuing wave: a use
found there is a VIOLATION), and with them (a use found only there is reported as GUARDED: reached only by a wave
that issued no such load).  Every other load is searched along all
edges.

usage: check_async_regs.py file.s [kernel-symbol-prefix]
Last line: "<n> async loads checked, <v> violations, <g> guarded".
"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
kern = sys.argv[2] if len(sys.argv) > 2 else "_ZN3smg15ion_pipe_kernelILi0E"
bad = total = guarded = 0


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def search(body, in_asm, labels, dst, start, follow_execz=True):
    """First instruction touching ``dst`` on a path from ``start`` that meets no wait (None: every path waits)."""
    seen, stack = set(), [start]
    while stack:
        j = stack.pop()
        while j < len(body) and j not in seen:
            seen.add(j)
            t = body[j]
            if (in_asm[j] and t.startswith("s_waitcnt")) or (t.startswith("s_waitcnt") and "vmcnt(0)" in t):
                break
            if not t or t.startswith((".", ";")) or t.endswith(":") or re.match(r"^\.LBB\w+:", t):
                j += 1
                continue
            toks = [x.strip(",") for x in t.split()]
            touched = set()
            for x in toks[1:]:
                touched |= regs(x)
            if touched & dst and not (in_asm[j] and t.startswith(("global_load", "global_atomic"))):
                return (j, t)
            op = toks[0]
            if op.startswith("s_cbranch") or op == "s_branch":
                tgt = toks[1] if len(toks) > 1 else ""
                # exec-zero edges: the taken edge of s_cbranch_execz, the fall-through of s_cbranch_execnz
                if tgt in labels and (follow_execz or op != "s_cbranch_execz"):
                    stack.append(labels[tgt])
                if op == "s_branch" or (op == "s_cbranch_execnz" and not follow_execz):
                    break
            if op in ("s_endpgm", "s_setpc_b64"):
                break
            j += 1
    return None


for st in [i for i, l in enumerate(src) if l.startswith(kern)]:
    name = src[st].split(":")[0]
    en = next(i for i in range(st, len(src)) if src[i].strip().startswith(".size") and name in src[i])
    body = [l.strip() for l in src[st:en]]
    in_asm, f = [False] * len(body), False
    for i, l in enumerate(body):
        if l.startswith(";;#ASMSTART"):
            f = True
        elif l.startswith(";;#ASMEND"):
            f = False
        in_asm[i] = f
    # labels inside loops carry a trailing comment ("; in Loop: Header=..."): match the name only
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
    dsts = set()
    for i, l in enumerate(body):
        # async loads and the async returning atomic (scheduling ticket): both write their first operand later
        if not (in_asm[i] and (l.startswith("global_load") or (l.startswith("global_atomic") and " sc0" in l))):
            continue
        total += 1
        dst = regs(l.split()[1].rstrip(","))
        dsts |= dst
        wave0 = "smg:wave0" in l
        hit = search(body, in_asm, labels, dst, i + 1, follow_execz=not wave0)
        if hit:
            print("VIOLATION", name[:60], i, l, "->", hit[0], hit[1])
            bad += 1
        elif wave0:
            hit = search(body, in_asm, labels, dst, i + 1, follow_execz=True)
            if hit:
                print("GUARDED", name[:60], i, l, "->", hit[0], hit[1])
                guarded += 1
print(f"{total} async loads checked, {bad} violations, {guarded} guarded")
sys.exit(1 if bad else 0)
