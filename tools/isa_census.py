#!/usr/bin/env python3
"""Static instruction census of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S).

    python tools/isa_census.py LISTING.s KERNEL_SUBSTRING [--top 40] [--blocks]

Prints VGPR / spill figures from the listing's metadata, the instruction counts by opcode and by
class (VALU scalar FP32 arithmetic, packed FP32, division / square-root helpers, scratch, VMEM,
LDS, SALU, branches), and with --blocks the basic blocks with their instruction counts and loop
back edges -- the static view used beside the PMC counts (k_shade_nee)."""
import argparse
import collections
import re
import sys


def kernel_body(lines, sub):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and sub in l.split(":")[0]:
            start = i
            name = l.split(":")[0]
        elif start is not None and l.startswith(".Lfunc_end"):
            return name, lines[start:i]
    sys.exit(f"kernel {sub} not found")


def meta(lines, name):
    out = {}
    for l in lines:
        m = re.match(r"\s*\.set\s+" + re.escape(name) + r"\.(\w+),\s*(\S+)", l)
        if m:
            out[m.group(1)] = m.group(2)
    return out


def klass(op):
    if op.startswith("scratch_") or op.startswith("buffer_") and "off" in op:
        return "scratch"
    if op.startswith("v_pk_"):
        return "valu_packed"
    if op in ("v_div_scale_f32", "v_div_fmas_f32", "v_div_fixup_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32"):
        return "valu_divsqrt"
    if re.match(r"v_(mul|add|sub|subrev|fma|fmac|mac|mad|max|min)_f32", op):
        return "valu_f32"
    if op.startswith("v_cmp") or op.startswith("v_cndmask"):
        return "valu_cmp_sel"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--blocks", action="store_true")
    a = ap.parse_args()
    lines = open(a.listing).read().splitlines()
    name, body = kernel_body(lines, a.kernel)
    md = meta(lines, name)
    ops = collections.Counter()
    cls = collections.Counter()
    blocks = []
    cur = ["entry", 0, None]
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\S*:", s):
                blocks.append(cur)
                cur = [s.rstrip(":"), 0, None]
            continue
        if re.match(r"^\.LBB\S*:", s):
            blocks.append(cur)
            cur = [s.rstrip(":"), 0, None]
            continue
        op = s.split()[0]
        if op.endswith(":"):
            continue
        ops[op] += 1
        cls[klass(op)] += 1
        cur[1] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            cur[2] = s.split()[-1]
    blocks.append(cur)
    scratch = sum(v for k, v in ops.items() if k.startswith("scratch_"))
    print(f"{name}\n  vgpr {md.get('num_vgpr')}  private_seg_size {md.get('private_seg_size')}  "
          f"instructions {sum(ops.values())}  scratch ops {scratch}")
    for k, v in sorted(cls.items(), key=lambda kv: -kv[1]):
        print(f"  {k:14s} {v}")
    print("  top opcodes:")
    for k, v in ops.most_common(a.top):
        print(f"    {k:28s} {v}")
    if a.blocks:
        idx = {b[0]: i for i, b in enumerate(blocks)}
        for i, (lbl, n, tgt) in enumerate(blocks):
            back = tgt in idx and idx[tgt] <= i
            print(f"  {lbl:12s} {n:5d}" + (f"  -> {tgt} (back edge)" if back else ""))


if __name__ == "__main__":
    main()
