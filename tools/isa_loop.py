"""Instruction mix of a kernel's main loop from hipcc assembly (dev tool).

    python tools/isa_loop.py <file.s> [kernel-substring]

Prints, per kernel, the basic blocks of the outermost backward-branch loop with their VALU / MFMA
/ LDS / SALU counts, so an edit's effect on the per-tile issue cost is visible
without a GPU run."""
import re
import sys


def blocks(body):
    cur, out = "entry", {}
    order = []
    for ln in body.split("\n"):
        t = ln.strip()
        m = re.match(r"^(\.LBB[\w_]+):", t) or re.match(r"^; (%bb\.\d+):", t)
        if m:
            cur = m.group(1)
            order.append(cur)
            out[cur] = []
            continue
        if not t or t.startswith((";", ".")):
            continue
        out.setdefault(cur, []).append(t.split(";")[0].strip())
        if cur not in order:
            order.append(cur)
    return order, out


def kind(i):
    if i.startswith("v_mfma"):
        return "mfma"
    if i.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
        return "trans"
    if i.startswith("v_"):
        return "valu"
    if i.startswith("ds_"):
        return "lds"
    if i.startswith(("buffer_", "global_")):
        return "vmem"
    if i.startswith("s_"):
        return "salu"
    return "other"


def main():
    s = open(sys.argv[1]).read()
    sel = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
        name, body = m.group(1), m.group(2)
        if sel not in name:
            continue
        order, bl = blocks(body)
        idx = {b: i for i, b in enumerate(order)}
        loop = None
        for b in order:
            for ins in bl[b]:
                mm = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.LBB[\w_]+)", ins)
                if mm and mm.group(1) in idx and idx[mm.group(1)] <= idx[b]:
                    span = (idx[mm.group(1)], idx[b])
                    if loop is None or span[1] - span[0] > loop[1] - loop[0]:
                        loop = span
        print(name)
        if loop is None:
            print("  no loop")
            continue
        tot = {}
        for b in order[loop[0]:loop[1] + 1]:
            c = {}
            for ins in bl[b]:
                k = kind(ins)
                c[k] = c.get(k, 0) + 1
                tot[k] = tot.get(k, 0) + 1
            print(f"  {b:24s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        print("  loop total: " + " ".join(f"{k}={v}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
