"""Per-basic-block instruction census of one kernel in a gfx950 .s file (tools/isa_blocks.py).

usage: python tools/isa_blocks.py file.s kernel_substring [min_loads]
Prints the basic blocks with at least min_loads vector-memory loads: instruction count by class.
"""
import re, sys, collections

path, kname = sys.argv[1], sys.argv[2]
min_loads = int(sys.argv[3]) if len(sys.argv) > 3 else 8
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if re.match(r"^_Z\S*:", l) and kname in l:
        start = i
        break
end = len(lines)
for i in range(start + 1, len(lines)):
    if re.match(r"^_Z\S*:", lines[i]) or lines[i].startswith("\t.section") or ".Lfunc_end" in lines[i] and lines[i].endswith(":"):
        end = i
        break
blocks, cur, name = [], [], "entry"
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        blocks.append((name, cur)); cur = []; name = m.group(1); continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith(".") : continue
    cur.append(s.split()[0])
blocks.append((name, cur))
def cls(op):
    if op.startswith("v_pk_"): return "valu_pk"
    if op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos")): return "valu_trans"
    if op.startswith(("v_cvt", "v_mad_u32_u24", "v_mul_u32_u24", "v_lshl_add", "v_fma_mix", "v_med3", "v_min_u32", "v_max_u32", "v_mul_lo", "v_mul_hi", "v_add3", "v_lshl_or", "v_and_or", "v_xad", "v_mad_u64")): return "valu_half"
    if op.startswith("v_"): return "valu_full"
    if op.startswith(("global_load", "buffer_load", "flat_load")): return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store")): return "vmem_st"
    if op.startswith("ds_"): return "lds"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith("s_"): return "salu"
    return "other"
tot = collections.Counter()
for name, ins in blocks:
    c = collections.Counter(cls(o) for o in ins)
    tot.update(c)
    if c["vmem_ld"] >= min_loads:
        ops = collections.Counter(ins)
        print(f"{name}: {len(ins)} insts", dict(c))
        print("   top:", ops.most_common(24))
print("kernel total", sum(tot.values()), dict(tot))
