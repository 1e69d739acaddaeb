"""Instruction mix of a kernel's loops from its gfx950 assembly (tools/isa.sh output):
    python tools/isa_loops.py <file.s> <kernel-symbol-substring> [--top 8]
Splits the kernel into basic blocks (.LBB labels), finds the natural loops from the back edges (a branch to a
label at or before it), and prints per loop: its blocks' instruction counts by class -- VALU (v_*, transcendental
v_rcp / v_rsq / v_sqrt / v_exp / v_log / v_sin / v_cos counted apart), SALU (s_* other than the classes below),
branches (s_cbranch_* / s_branch), exec-mask moves (s_*_saveexec_*, s_*  exec ...), waits / nops (s_waitcnt,
s_nop, s_sleep, s_setprio), LDS (ds_*), memory (global_* / buffer_* / s_load_* / s_buffer_*) -- and the share of
SALU that manages control flow (exec masks, branches, vcc / scc tests of ballots)."""
import argparse
import re
from collections import Counter

TRANS = ("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")


def classify(ins, ops):
    if ins.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if ins.startswith(("s_waitcnt", "s_nop", "s_sleep", "s_setprio", "s_barrier")):
        return "wait"
    if ins.startswith("ds_"):
        return "lds"
    if ins.startswith(("global_", "buffer_", "flat_", "s_load", "s_buffer", "scratch_")):
        return "mem"
    if ins.startswith("v_"):
        return "trans" if ins.startswith(TRANS) else "valu"
    if ins.startswith("s_"):
        if "saveexec" in ins or "exec" in ops:
            return "exec"
        return "salu"
    return "other"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("asm")
    p.add_argument("kernel")
    p.add_argument("--top", type=int, default=8)
    a = p.parse_args()
    lines = open(a.asm).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and a.kernel in l)
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^_Z\S*:", lines[i]) or lines[i].startswith(".Lfunc_end")), len(lines))
    blocks, cur = [], {"label": "entry", "ins": [], "succ": []}
    for l in lines[start + 1:end]:
        s = l.split(";")[0].strip()
        if not s:
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "ins": [], "succ": []}
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        ins, ops = parts[0], (parts[1] if len(parts) > 1 else "")
        cur["ins"].append((ins, ops))
        if ins.startswith(("s_cbranch", "s_branch")):
            cur["succ"].append(ops.strip())
    blocks.append(cur)
    index = {b["label"]: i for i, b in enumerate(blocks)}
    loops = []
    for i, b in enumerate(blocks):
        for t in b["succ"]:
            j = index.get(t)
            if j is not None and j <= i:
                loops.append((j, i))
    res = []
    for j, i in loops:
        c = Counter()
        for b in blocks[j:i + 1]:
            for ins, ops in b["ins"]:
                c[classify(ins, ops)] += 1
        res.append((sum(c.values()), j, i, c))
    res.sort(reverse=True)
    print(f"{a.kernel}: {len(blocks)} blocks, {sum(len(b['ins']) for b in blocks)} instructions, {len(loops)} back edges")
    for tot, j, i, c in res[:a.top]:
        ctrl = c["exec"] + c["branch"]
        print(f"loop {blocks[j]['label']}..{blocks[i]['label']} ({i - j + 1} blocks, {tot} instr): "
              + ", ".join(f"{k} {c[k]}" for k in ("valu", "trans", "salu", "exec", "branch", "wait", "lds", "mem"))
              + f"; control-flow SALU {ctrl} of {c['salu'] + ctrl} scalar")


if __name__ == "__main__":
    main()
