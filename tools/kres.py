"""Print per-kernel resources (VGPR/SGPR/LDS/scratch) from a hipcc -S device assembly."""
import re, subprocess, sys
txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = subprocess.run(["c++filt", f.get("name", "?")], capture_output=True, text=True).stdout.strip()
    print(f"{name[:60]:60s} vgpr {f.get('vgpr_count', '-'):>4} agpr {f.get('agpr_count','0'):>3} sgpr {f.get('sgpr_count', '-'):>4} "
          f"lds {f.get('group_segment_fixed_size', '-'):>6} scratch {f.get('private_segment_fixed_size', '-'):>5} "
          f"maxthr {f.get('max_flat_workgroup_size', '-')}")
