"""Instruction mix of a kernel's loops from hipcc assembly (dev tool).

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S <src.hip> -o <file.s> (+ the build flags)
    python tools/isa_loop.py <file.s> <kernel symbol or unique substring> [first last]

Prints every loop (a backward branch to a label of the kernel) with its VALU / transcendental /
packed-fp32 / MFMA / LDS / VMEM / SALU / s_nop / s_waitcnt counts, so an edit's effect on the
per-tile issue cost is visible without a GPU run; with [first last] (instruction
indices printed for a loop) also the per-opcode histogram of that range."""
import collections
import re
import sys


def kind(i):
    op = i.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
        return "trans"
    if op.startswith("v_pk_") and "f32" in op:
        return "pkf32"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    src = open(sys.argv[1]).read()
    names = [m.group(1) for m in re.finditer(r"^([\w.$]+):", src, re.M) if sys.argv[2] in m.group(1)
             and not m.group(1).startswith(".")]
    if not names:
        sys.exit(f"no kernel matching {sys.argv[2]!r}")
    kname = names[0]
    start = src.index("\n" + kname + ":")
    end = src.index(".Lfunc_end", start)
    labels, insts = {}, []
    for ln in src[start:end].split("\n")[1:]:
        t = ln.strip()
        m = re.match(r"^(\.LBB[\w_]+):", t)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        insts.append(t.split(";")[0].strip())
    print(kname)
    for idx, i in enumerate(insts):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)", i)
        if m and labels.get(m.group(2), 1 << 30) <= idx:
            a = labels[m.group(2)]
            c = collections.Counter(kind(x) for x in insts[a:idx + 1])
            print(f"  loop {m.group(2)} [{a}..{idx}] n={idx + 1 - a}: "
                  + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    if len(sys.argv) > 4:
        a, b = int(sys.argv[3]), int(sys.argv[4])
        for k, v in collections.Counter(x.split()[0] for x in insts[a:b + 1]).most_common():
            print(f"{v:5d} {k}")


if __name__ == "__main__":
    main()
