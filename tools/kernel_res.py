"""Per-kernel resources (VGPR / AGPR / spill / LDS / scratch) from a hipcc -S
device listing's AMDGPU metadata:  python tools/kernel_res.py listing.s [substring]"""
import re
import sys

t = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
meta = t[t.find("amdhsa.kernels:"):]
for ent in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", ent)
    if not name or sub not in name.group(1):
        continue
    f = {k: (re.search(rf"\.{k}:\s+(\d+)", ent) or [None, "?"])[1]
         for k in ("vgpr_count", "agpr_count", "vgpr_spill_count", "group_segment_fixed_size", "private_segment_fixed_size")}
    print(f"{name.group(1)[:70]:70s} vgpr {f['vgpr_count']:>4} agpr {f['agpr_count']:>3} spill {f['vgpr_spill_count']:>3} "
          f"lds {f['group_segment_fixed_size']:>6} scratch {f['private_segment_fixed_size']}")
