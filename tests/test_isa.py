"""Disassembly check of the M0 contract of the LDS-DMA helpers (CPU: hipcc cross-compiles gfx950).

The buffer / global LDS-DMA helpers in csrc/common.h (``dma16_buf``, ``dma4_buf``, ``glds*``) write
M0 from inline asm and issue the DMA in the same asm block.  M0 is a reserved register to hipcc, so
it cannot be listed as a clobber; instead this test proves, on the code hipcc actually emits for
every product kernel, that the compiler never touches M0 itself:

  * every instruction that names ``m0`` lies inside an inline-asm block (``;;#ASMSTART`` ..
    ``;;#ASMEND``);
  * every LDS-DMA instruction (``buffer_load_* ... lds``, ``global_load_lds_*``) lies inside an asm
    block that wrote M0 before it;
  * no instruction that reads M0 implicitly (movrel, sendmsg, GWS / append / consume, interp) is
    emitted anywhere.

If a future compiler keeps a live value in M0 across these asm blocks, or emits its own LDS-DMA or
M0 user, this test fails instead of the DMA destinations silently moving.
"""
from __future__ import annotations

import concurrent.futures as cf
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "quantizedattention_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"

M0_IMPLICIT = re.compile(r"^\s*(s_movrel|v_movrel|s_sendmsg|ds_gws|ds_append|ds_consume|v_interp|"
                         r"s_ttracedata|v_writelane_b32_e64\s+\S+,\s*m0)")
DMA = re.compile(r"^\s*(buffer_load_\w+\s.*\blds\b|global_load_lds_\w+)")
M0_WRITE = re.compile(r"^\s*s_mov_b32\s+m0\s*,")


def _device_asm(src: Path, out_dir: Path) -> str:
    from quantizedattention_amd.build import CFLAGS, FILE_FLAGS
    flags = [f for f in CFLAGS if f not in ("-fPIC",)]
    out = out_dir / (src.stem + ".s")
    cmd = [HIPCC, *flags, *FILE_FLAGS.get(src.name, []), "--cuda-device-only", "-S", str(src),
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc -S failed for {src.name}:\n{r.stderr[-2000:]}")
    return out.read_text()


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("isa")
    srcs = sorted(CSRC.glob("*.hip"))
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        texts = list(ex.map(lambda s: _device_asm(s, d), srcs))
    return dict(zip((s.name for s in srcs), texts))


def _check(text: str) -> tuple[int, list[str]]:
    """Returns (number of LDS-DMA instructions seen, violations)."""
    bad, n_dma = [], 0
    in_asm, m0_set = False, False
    for no, line in enumerate(text.split("\n"), 1):
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm, m0_set = True, False
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith((";", ".")):
            continue
        code = t.split(";")[0]
        if M0_IMPLICIT.match(code):
            bad.append(f"line {no}: implicit M0 user {code!r}")
        if DMA.match(code):
            n_dma += 1
            if not (in_asm and m0_set):
                bad.append(f"line {no}: LDS-DMA without an M0 write in its own asm block: {code!r}")
        if re.search(r"\bm0\b", code):
            if not in_asm:
                bad.append(f"line {no}: compiler-emitted M0 access {code!r}")
            elif M0_WRITE.match(code):
                m0_set = True
    return n_dma, bad


def test_every_kernel_source_keeps_the_m0_contract(asm):
    total = 0
    for name, text in asm.items():
        n, bad = _check(text)
        total += n
        assert not bad, f"{name}: " + "; ".join(bad[:5])
    assert total > 0, "no LDS-DMA found: the pattern no longer matches the emitted code"


def test_checker_flags_a_compiler_m0_use():
    ok = ";;#ASMSTART\n\ts_mov_b32 m0, s4\n\ts_nop 0\n\tbuffer_load_dwordx4 v1, s[0:3], s5 offen lds\n;;#ASMEND\n"
    assert _check(ok) == (1, [])
    n, bad = _check(ok + "\ts_mov_b32 m0, -1\n\tds_read_b32 v0, v1\n")
    assert bad and "compiler-emitted" in bad[0]
    n, bad = _check(";;#ASMSTART\n\tbuffer_load_dword v1, s[0:3], s5 offen lds\n;;#ASMEND\n")
    assert bad and "without an M0 write" in bad[0]


# A buffer store of more than 64 bits of data, and the instructions after it.  hipcc pads a VALU write
# of the store's data registers only when soffset is not a register; on gfx950 the hazard holds with
# an SGPR soffset too (a record store followed directly by a v_and into its dword-0 register stored
# the new value, run-dependently: tests/test_gpu_int8_ext.py::test_int8_bwd_ws_long_d64).  So every
# such store must use an inline-constant soffset, which the compiler then protects.
WIDE_STORE = re.compile(r"^\s*buffer_store_(dwordx[34]|b96|b128)\s+v\[\d+:\d+\],\s*\S+,\s*s\[\d+:\d+\],\s*(\S+)")


def _wide_store_violations(text: str) -> tuple[int, list[str]]:
    bad, n = [], 0
    for no, line in enumerate(text.split("\n"), 1):
        m = WIDE_STORE.match(line.split(";")[0])
        if m:
            n += 1
            soff = m.group(2).rstrip(",")
            if re.fullmatch(r"s\d+|s\[\d+:\d+\]|m0|vcc\w*|ttmp\d+", soff):
                bad.append(f"line {no}: wide buffer store with a register soffset: {line.strip()!r}")
    return n, bad


def test_wide_buffer_stores_use_a_constant_soffset(asm):
    total = 0
    for name, text in asm.items():
        n, bad = _wide_store_violations(text)
        total += n
        assert not bad, f"{name}: " + "; ".join(bad[:3])
    assert total > 0, "no wide buffer store found: the pattern no longer matches the emitted code"


def test_checker_flags_a_register_soffset():
    assert _wide_store_violations("\tbuffer_store_dwordx4 v[112:115], v117, s[4:7], 0 offen\n") == (1, [])
    n, bad = _wide_store_violations("\tbuffer_store_dwordx4 v[112:115], v137, s[24:27], s58 offen\n")
    assert n == 1 and bad



# The symptom itself, however the store is addressed: the data registers of a > 64-bit store written
# by a VALU within two wait states of the store (s_nop N counts N + 1).  hipcc keeps every padded wide
# store at distance >= 3 (global stores: an s_nop 1 where needed); the pre-fix record store had its
# dword-0 register rewritten by the second instruction after it.  Linear order is checked, which is
# execution order on the fall-through path.
_WIDE_ANY = re.compile(r"^(global_store_dwordx[34]|flat_store_dwordx[34]|buffer_store_dwordx[34]|"
                       r"global_store_b(96|128)|buffer_store_b(96|128))\s")


def _vregs(spec: str) -> set[int]:
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", spec)
    return {int(m.group(1))} if m else set()


def _store_data_overwrites(text: str) -> tuple[int, list[str]]:
    code = [ln.split(";")[0].strip() for ln in text.split("\n")]
    code = [c for c in code if c and not c.startswith(".") and not c.endswith(":")]
    n, bad = 0, []
    for i, c in enumerate(code):
        if not _WIDE_ANY.match(c):
            continue
        n += 1
        ops = [t.strip(",") for t in c.split()[1:]]
        data = _vregs(ops[1] if c.startswith(("global", "flat")) else ops[0])
        dist = 0
        for nxt in code[i + 1:i + 4]:
            dist += int(nxt.split()[1]) + 1 if nxt.startswith("s_nop") else 1
            if dist > 2:
                break
            if (nxt.startswith("v_") and not nxt.startswith(("v_readlane", "v_readfirstlane"))
                    and _vregs(nxt.split()[1].strip(",")) & data):
                bad.append(f"{c!r} then {nxt!r} at distance {dist}")
                break
    return n, bad


def test_no_wide_store_data_overwritten_within_two_wait_states(asm):
    total = 0
    for name, text in asm.items():
        n, bad = _store_data_overwrites(text)
        total += n
        assert not bad, f"{name}: " + "; ".join(bad[:3])
    assert total > 0


def test_checker_flags_a_close_overwrite():
    old = ("\tbuffer_store_dwordx4 v[114:117], v143, s[24:27], s2 offen\n"
           "\tv_and_b32_e32 v97, 0x7fffffff, v70\n\tv_and_b32_e32 v114, 0x7fffffff, v71\n")
    new = ("\tbuffer_store_dwordx4 v[112:115], v117, s[4:7], 0 offen\n\ts_nop 1\n"
           "\tv_and_b32_e32 v112, 0x7fffffff, v68\n")
    assert _store_data_overwrites(old)[1] and not _store_data_overwrites(new)[1]


def _cfg(body: list[str]):
    """Basic blocks of one kernel's assembly: (names, successors, scratch-op count per block).  A
    block starts at a label or after a branch; s_branch has one successor, s_cbranch also falls
    through."""
    names, succ, nscr = [], [], []
    cur = None

    def start(name):
        nonlocal cur
        names.append(name)
        succ.append([])
        nscr.append(0)
        cur = len(names) - 1

    start("entry")
    ended = False
    for line in body:
        lm = re.match(r"^(\.LBB\w+):", line)
        if lm:
            if not ended:
                succ[cur].append(lm.group(1))
            start(lm.group(1))
            ended = False
            continue
        code = line.split(";")[0].strip()
        if not code or code.startswith("."):
            continue
        if ended:   # code after an unconditional branch without a label: unreachable, own block
            start(f"_dead{len(names)}")
            ended = False
        if "scratch_" in code:
            nscr[cur] += 1
        bm = re.match(r"s_(c?)branch\w*\s+(\.LBB\w+)", code)
        if bm:
            succ[cur].append(bm.group(2))
            if bm.group(1):   # conditional: falls through into a new block
                start(f"_ft{len(names)}")
                succ[cur - 1].append(names[cur])
            else:
                ended = True
        elif code.startswith(("s_endpgm", "s_setpc")):
            ended = True
    idx = {n: i for i, n in enumerate(names)}
    return names, [[idx[s] for s in ss if s in idx] for ss in succ], nscr


def _loop_spills(text: str) -> dict:
    """Scratch (spill) instructions that lie on a cycle of the control-flow graph, per kernel (blocks
    in a strongly connected component of more than one block, or with an edge to themselves).  A
    reload block placed after a loop that jumps back to the epilogue is not inside a loop."""
    out = {}
    for m in re.finditer(r"^(\w+):\s*;\s*@\1\n(.*?)^\.Lfunc_end", text, flags=re.S | re.M):
        kernel = m.group(1)
        names, succ, nscr = _cfg(m.group(2).split("\n"))
        # Tarjan's SCC, iterative
        index, low, on, stack, comp = {}, {}, set(), [], [None] * len(names)
        counter = 0
        for root in range(len(names)):
            if root in index:
                continue
            work = [(root, 0)]
            while work:
                v, i = work.pop()
                if i == 0:
                    index[v] = low[v] = counter
                    counter += 1
                    stack.append(v)
                    on.add(v)
                if i < len(succ[v]):
                    work.append((v, i + 1))
                    w = succ[v][i]
                    if w not in index:
                        work.append((w, 0))
                    elif w in on:
                        low[v] = min(low[v], index[w])
                    continue
                if low[v] == index[v]:
                    members = []
                    while True:
                        w = stack.pop()
                        on.discard(w)
                        members.append(w)
                        if w == v:
                            break
                    for w in members:
                        comp[w] = (len(members), v)
                if work:
                    u = work[-1][0]
                    low[u] = min(low[u], low[v])
        n = sum(nscr[b] for b in range(len(names))
                if nscr[b] and (comp[b][0] > 1 or b in succ[b]))
        if n:
            out[kernel] = n
    return out


def test_no_register_spills_in_loops(asm):
    """No product kernel touches scratch inside a loop (a spill there costs a scratch round trip per
    tile, and its VMEM op also makes the loop's counted vmcnt waits drain the ring's DMA).  Round 4
    found this the hard way: the ring-slot unrolled forward spilled 134 VGPRs in its causal
    instantiation (the causal int8 step went from 2.5 to 5.5 ms) before the unroll was restricted.
    A value stored once before a loop and reloaded once after it (a kernel at the 256-VGPR limit
    keeping an epilogue pointer out of the loop's way) costs nothing and is allowed."""
    bad = []
    for name, text in asm.items():
        for kernel, n in _loop_spills(text).items():
            bad.append(f"{name}: {kernel[:90]} has {n} scratch ops inside loops")
    assert not bad, "\n".join(bad)


def test_loop_spill_checker_flags_a_loop_spill():
    text = ("k:  ; @k\n.LBB0_1:\n  v_add_f32 v0, v0, v1\n  scratch_load_dword v2, off, off\n"
            "  s_cbranch_scc1 .LBB0_1\n  scratch_store_dword off, v3, off\n.Lfunc_end0:\n")
    assert _loop_spills(text) == {"k": 1}
    # a reload block laid out after the epilogue that branches back to it: not a loop
    text = ("k:  ; @k\n  scratch_store_dword off, v3, off\n  s_cbranch_scc1 .LBB0_3\n.LBB0_1:\n"
            "  v_add_f32 v0, v0, v1\n  s_endpgm\n.LBB0_3:\n  scratch_load_dword v2, off, off\n"
            "  s_branch .LBB0_1\n.Lfunc_end0:\n")
    assert _loop_spills(text) == {}
