"""VGPR / spill counts per kernel from a hipcc -S assembly file.
Usage: python tools/kstats.py file.s [substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
entries = re.split(r"\n  - ", meta)[1:]
for e in entries:
    name = re.search(r"\.name:\s+(\S+)", e)
    if not name:
        continue
    n = name.group(1)
    if len(sys.argv) > 2 and sys.argv[2] not in n:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "?"])[1]
    print(f"{n[:70]:70s} vgpr={g('vgpr_count')} agpr={g('agpr_count')} vspill={g('vgpr_spill_count')} lds={g('group_segment_fixed_size')}")
