#!/usr/bin/env python3
# usage: tools/exp_tile_vshift_variant.py spgemm_new_amd/csrc/maxk_spgemm.hip out.hip  (then build out.hip
# with -I spgemm_new_amd/csrc and load it via MAXK_LIB).  Development tool; the variant gave wrong
# results at k = 32 (TILE), kept to reproduce that.
"""Variant of maxk_spgemm.hip: the TILE record shifts for the bit offset and the
row address run on the VALU (VGPR temps) instead of the SALU."""
import re, sys
src = open(sys.argv[1]).read()
a = src.index("__device__ __forceinline__ void tile_groups2(")
b = src.index("__device__ __forceinline__ tile_hdr_t tile_load_hdr(")
body = src[a:b]
om = {"s81": "o0", "s84": "o1", "s87": "o2", "s90": "o3"}
am = {"s82": "a0", "s85": "a1", "s88": "a2", "s91": "a3"}
for s, o in om.items():
    body = re.sub(r'"s_lshl_b32 %s, ([^,]+), 3\\n\\t"' % s, r'"v_lshlrev_b32 %%[%s], 3, \1\\n\\t"' % o, body)
    body = body.replace(", v48, %s, 8" % s, ", v48, %%[%s], 8" % o)
for s, o in am.items():
    body = re.sub(r'"s_lshr_b32 %s, ([^,]+), 14\\n\\t"' % s, r'"v_lshrrev_b32 %%[%s], 14, \1\\n\\t"' % o, body)
    body = body.replace(", 2, %s\\n" % s, ", 2, %%[%s]\\n" % o)
for s in list(om) + list(am):
    assert all(s not in l for l in body.replace('"%s"' % s, "").split("\n") if not l.strip().startswith("//")), s
    body = body.replace(', "%s"' % s, "")
decl = "    uint32_t o0, o1, o2, o3, a0, a1, a2, a3;\n"
outs = ('[o0] "=&v"(o0), [o1] "=&v"(o1), [o2] "=&v"(o2), [o3] "=&v"(o3), '
        '[a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), ')
body = body.replace("    uint64_t ex;\n", "    uint64_t ex;\n" + decl)
body = body.replace(': [t0] "=&v"(t0)', ': ' + outs + '[t0] "=&v"(t0)')
assert body.count(decl) == 2 and body.count(outs) == 2
open(sys.argv[2], "w").write(src[:a] + body + src[b:])
