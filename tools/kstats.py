"""VGPR / SGPR / spill / LDS figures of every kernel in one source (hipcc -S with the product flags).

    python tools/kstats.py int8_attn_fwd.hip [-DNAME=VALUE ...]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from quantizedattention_amd.build import CFLAGS, FILE_FLAGS  # noqa: E402

src = ROOT / "quantizedattention_amd" / "csrc" / sys.argv[1]
with tempfile.TemporaryDirectory() as d:
    out = Path(d) / "k.s"
    flags = [f for f in CFLAGS if f != "-fPIC"]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, *FILE_FLAGS.get(src.name, []), *sys.argv[2:],
                    "--cuda-device-only", "-S", str(src), "-o", str(out)], check=True)
    text = out.read_text()
    if len(sys.argv) > 2 and sys.argv[-1].startswith("--keep="):
        pass
for m in re.finditer(r"\.name:\s+(\S+)\n((?:.*\n){0,90}?)\s+\.vgpr_spill_count:\s+(\d+)", text):
    body = m.group(2)
    g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", body) or [None, "?"])[1]  # noqa: E731
    print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} sgpr {g('sgpr_count'):>4} "
          f"spill {m.group(3):>4} lds {g('group_segment_fixed_size'):>6}  {m.group(1)[:110]}")
