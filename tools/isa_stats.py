"""Per-kernel instruction statistics of a gfx950 ISA dump (hipcc --cuda-device-only -S).

usage: python tools/isa_stats.py <file.s> [name filter]
"""
import re
import sys

s = open(sys.argv[1]).read()
filt = sys.argv[2] if len(sys.argv) > 2 else ""
starts = [m for m in re.finditer(r"^(_Z\w+):", s, re.M)]
for i, m in enumerate(starts):
    name = m.group(1)
    if filt not in name:
        continue
    end = starts[i + 1].start() if i + 1 < len(starts) else len(s)
    body = s[m.start():end].split(".Lfunc_end")[0]
    ins = [l.strip().split()[0] for l in body.splitlines() if l.startswith("\t") and not l.startswith("\t.")
           and l.strip() and not l.strip().startswith(";")]
    cnt = lambda p: sum(1 for x in ins if x.startswith(p))
    meta = s[end:end + 4000] if False else ""
    print(f"{name[:64]:64s} insts {len(ins):5d} valu {cnt('v_'):5d} salu {cnt('s_'):5d} "
          f"div_scale {cnt('v_div_scale'):3d} rcp {cnt('v_rcp_f32'):3d} sqrt {cnt('v_sqrt_f32'):3d} "
          f"cvt_f16 {cnt('v_cvt_f16') + cnt('v_cvt_pk'):3d} global_ld {cnt('global_load'):3d} ds {cnt('ds_'):3d}")
