#!/usr/bin/env python3
"""asm_mix.py <file.s> <substr>...: VALU/LDS/VMEM instruction mix of the
kernels whose mangled name contains every substring (static counts)."""
import collections
import re
import sys

src = open(sys.argv[1]).read()
keys = sys.argv[2:]
parts = re.split(r"\n(_Z\S+):\s*;[^\n]*\n", src)
for i in range(1, len(parts), 2):
    name, body = parts[i], parts[i + 1]
    if not all(k in name for k in keys):
        continue
    body = body.split(".Lfunc_end")[0]
    ops = re.findall(r"^\s+([vsdgb][a-z_0-9]+)", body, re.M)
    c = collections.Counter(ops)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name}\n  VALU {valu}  SALU {sum(v for k, v in c.items() if k.startswith('s_'))}  "
          f"LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}  "
          f"VMEM {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))}")
    m = re.search(r"vgpr_count:\s*(\d+)|NumVgprs:\s*(\d+)", body)
    print("  ", ", ".join(f"{k} {v}" for k, v in c.most_common(24) if k.startswith("v_")))
