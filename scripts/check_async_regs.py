"""Static check of the async-load discipline in the LDS kernel's ISA: between an inline-asm global_load into
v[a:b] and the next inline-asm s_waitcnt vmcnt (linear order), no other instruction may read or write
v[a..b] except another inline-asm load into the same registers.  usage: check_async_regs.py file.s [kernel]"""
import re, sys

src = open(sys.argv[1]).read().split("\n")
kern = sys.argv[2] if len(sys.argv) > 2 else "_ZN3smg15ion_pipe_kernelILi0E"
bad = total = 0
starts = [i for i, l in enumerate(src) if l.startswith(kern)]
for st in starts:
    en = next(i for i in range(st, len(src)) if src[i].strip().startswith(".size") and kern in src[i])
    body = [l.strip() for l in src[st:en]]
    in_asm = [False] * len(body)
    f = False
    for i, l in enumerate(body):
        if l.startswith(";;#ASMSTART"):
            f = True
        elif l.startswith(";;#ASMEND"):
            f = False
        in_asm[i] = f

    def regs(tok):
        m = re.match(r"v\[(\d+):(\d+)\]", tok)
        if m:
            return set(range(int(m.group(1)), int(m.group(2)) + 1))
        m = re.match(r"v(\d+)$", tok)
        return {int(m.group(1))} if m else set()

    for i, l in enumerate(body):
        if not (in_asm[i] and l.startswith("global_load_dwordx2")):
            continue
        total += 1
        dst = regs(l.split()[1].rstrip(","))
        for j in range(i + 1, len(body)):
            t = body[j]
            if in_asm[j] and t.startswith("s_waitcnt"):
                break
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            toks = [x.strip(",") for x in t.split()]
            touched = set()
            for x in toks[1:]:
                touched |= regs(x)
            if touched & dst and not (in_asm[j] and t.startswith("global_load_dwordx2")):
                print("VIOLATION", kern, i, l, "->", j, t)
                bad += 1
                break
print(f"{total} async loads checked, {bad} violations")
sys.exit(1 if bad else 0)
