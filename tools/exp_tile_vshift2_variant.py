#!/usr/bin/env python3
# usage: tools/exp_tile_vshift2_variant.py <mode> spgemm_new_amd/csrc/maxk_spgemm.hip out.hip
# (build out.hip with -I spgemm_new_amd/csrc and load it via MAXK_LIB).  Development tool.
"""Isolating the wrong results of the TILE VALU-shift variant
(exp_tile_vshift_variant.py, DESIGN.md §4 TILE):
  mode "movbfe": shifts on the VALU, but inside gpr-index mode only a plain
                 v_mov of the indexed selector word; the v_bfe with the VGPR
                 bit offset runs after s_set_gpr_idx_off;
  mode "addr":   only the row-address shift on the VALU (bit offset stays SALU)."""
import re
import subprocess
import sys

mode, src, dst = sys.argv[1], sys.argv[2], sys.argv[3]
here = __file__.rsplit("/", 1)[0]
subprocess.run([sys.executable, here + "/exp_tile_vshift_variant.py", src, dst], check=True)
s = open(dst).read()
a = s.index("__device__ __forceinline__ void tile_groups2(")
b = s.index("__device__ __forceinline__ tile_hdr_t tile_load_hdr(")
body = s[a:b]
if mode == "movbfe":
    out, pend = [], []
    for line in body.split("\n"):
        m = re.match(r'(\s*)"v_bfe_u32 %\[(t\d)\], v48, %\[(o\d)\], 8\\n\\t"', line)
        if m:
            out.append('%s"v_mov_b32 %%[%s], v48\\n\\t"' % (m.group(1), m.group(2)))
            pend.append((m.group(1), m.group(2), m.group(3)))
            continue
        out.append(line)
        if '"s_set_gpr_idx_off\\n\\t"' in line and pend:
            for ind, t, o in pend:
                out.append('%s"v_bfe_u32 %%[%s], %%[%s], %%[%s], 8\\n\\t"' % (ind, t, t, o))
            pend = []
    assert not pend
    body = "\n".join(out)
elif mode == "addr":
    orig = s[a:b]  # undo the bit-offset part: restore s_lshl into s81.. and the SGPR bfe offsets
    om = {"o0": "s81", "o1": "s84", "o2": "s87", "o3": "s90"}
    for o, sg in om.items():
        body = re.sub(r'"v_lshlrev_b32 %%\[%s\], 3, ([^\\]+)\\n\\t"' % o, r'"s_lshl_b32 %s, \1, 3\\n\\t"' % sg, body)
        body = body.replace(", v48, %%[%s], 8" % o, ", v48, %s, 8" % sg)
        body = body.replace('[%s] "=&v"(%s), ' % (o, o), "")
    body = body.replace("uint32_t o0, o1, o2, o3, a0, a1, a2, a3;", "uint32_t a0, a1, a2, a3;")
    body = body.replace('"memory", "scc", ', '"memory", "scc", "s81", "s84", "s87", "s90", ')
elif mode in ("alate", "anop"):
    # "addr", then either the VALU row-address shifts moved after the group's
    # s_set_gpr_idx_off (no gpr-index toggle between their write and the read),
    # or kept in place with s_nop 7 before each SRC0 s_set_gpr_idx_on
    om = {"o0": "s81", "o1": "s84", "o2": "s87", "o3": "s90"}
    for o, sg in om.items():
        body = re.sub(r'"v_lshlrev_b32 %%\[%s\], 3, ([^\\]+)\\n\\t"' % o, r'"s_lshl_b32 %s, \1, 3\\n\\t"' % sg, body)
        body = body.replace(", v48, %%[%s], 8" % o, ", v48, %s, 8" % sg)
        body = body.replace('[%s] "=&v"(%s), ' % (o, o), "")
    body = body.replace("uint32_t o0, o1, o2, o3, a0, a1, a2, a3;", "uint32_t a0, a1, a2, a3;")
    body = body.replace('"memory", "scc", ', '"memory", "scc", "s81", "s84", "s87", "s90", ')
    if mode == "anop":
        body = body.replace('"s_set_gpr_idx_on s80, gpr_idx(SRC0)\\n\\t"',
                            '"s_nop 7\\n\\ts_set_gpr_idx_on s80, gpr_idx(SRC0)\\n\\t"')
    else:
        out, pend = [], []
        for line in body.split("\n"):
            if re.match(r'\s*"v_lshrrev_b32 %\[a\d\], 14, ', line):
                pend.append(line)
                continue
            out.append(line)
            if '"s_set_gpr_idx_off\\n\\t"' in line and pend:
                out.extend(pend)
                pend = []
        assert not pend
        body = "\n".join(out)
else:
    sys.exit("mode: movbfe | addr | alate | anop")
open(dst, "w").write(s[:a] + body + s[b:])
