"""Instruction accounting of a blend kernel's inner pair loop from `hipcc -S` output.

    python tools/isa_loop_account.py FILE.s KERNEL_SYMBOL_SUBSTRING

Finds the kernel, then the innermost loop that contains `s_ff1_i32_b64` (the live-mask walk of
the pair steps), and counts its instructions by unit (VALU incl. v_exp / DPP, SALU, LDS, VMEM,
branch) and, for VALU, by role using the operand patterns of render_fwd.hip / render_bwd.hip:
  power   gauss_power (v_sub of the pixel offsets, v_mul / v_fmac on the staged conic)
  exp     r3dg_expf (v_med3 clamp, 0x3fb8aa3b log2e, Cody-Waite 0xbf317200 / 0xb5bfbe8e, the
          polynomial constants, v_lshl_add exponent add) or v_exp_f32
  ...     everything else is reported as 'other' with the instruction list, labelled by hand in
          DESIGN.md.
Blocks are counted once each (both instances of the pair and the accumulate branches)."""
import re
import sys


def kernel_body(text, sym):
    start = None
    lines = text.splitlines()
    for i, ln in enumerate(lines):
        if start is None and ln.startswith("_Z") and sym in ln and ln.rstrip().endswith(sym.split()[-1] + ":") is False:
            pass
        if start is None and re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", ln):
            start = i
        elif start is not None and ".end_amdhsa_kernel" in ln:
            return lines[start:i]
    raise SystemExit(f"kernel {sym} not found")


def inner_loop(body):
    """The blocks of the innermost loop that holds `s_ff1_i32_b64`: its header block and every block
    the compiler annotates `in Loop: Header=<header>` (the latch may fall through to the header)."""
    blocks, cur = [], None
    for ln in body:
        m = re.match(r"^(\.LBB\S+):(.*)$", ln) or re.match(r"^; (%bb\.\d+):(.*)$", ln)
        if m:
            cur = [m.group(1), m.group(2), []]
            blocks.append(cur)
        elif cur is not None:
            if not cur[2] and ln.strip().startswith(";") and "Loop" in ln:
                cur[1] += ln
            else:
                cur[2].append(ln)
    hdr = None
    for i, (name, comment, lines) in enumerate(blocks):
        if any("s_ff1_i32_b64" in x for x in lines) and "Inner Loop Header" in comment:
            hdr = name.lstrip(".").replace("LBB", "BB")
            out = list(lines)
            break
    if hdr is None:
        raise SystemExit("no s_ff1 loop found")
    for name, comment, lines in blocks:
        if f"Header={hdr} " in comment + " " and name.lstrip(".").replace("LBB", "BB") != hdr:
            out += lines
    return out


POWER = re.compile(r"v_(sub|mul|fmac|fma)_f32")
EXP_CONST = ("0x3fb8aa3b", "0xcb400000", "0xbf317200", "0xb5bfbe8e", "0x3ab54ace", "0x3d2aac28", "0x3e2aaa49",
             "0x3efffffe")


def main():
    text = open(sys.argv[1]).read()
    loop = inner_loop(kernel_body(text, sys.argv[2]))
    insts = [ln.strip() for ln in loop if ln.strip() and not ln.strip().startswith((";", ".", "/"))]
    insts = [s for s in insts if not s.startswith(("s_waitcnt", ";;#"))]
    units = {"valu": [], "salu": [], "lds": [], "vmem": [], "branch": []}
    for s in insts:
        op = s.split()[0]
        if op.startswith(("s_cbranch", "s_branch")):
            units["branch"].append(s)
        elif op.startswith("ds_"):
            units["lds"].append(s)
        elif op.startswith(("global_", "buffer_", "flat_")):
            units["vmem"].append(s)
        elif op.startswith("s_"):
            units["salu"].append(s)
        elif op.startswith("v_"):
            units["valu"].append(s)
    exp = [s for s in units["valu"] if s.startswith(("v_exp_f32", "v_med3_f32", "v_lshl_add_u32"))
           or any(c in s for c in EXP_CONST) or re.match(r"v_fma_f32 \S+, \S+, \S+, 1\.0", s)]
    print(f"loop: {len(insts)} instructions")
    for u, v in units.items():
        print(f"  {u:6s} {len(v)}")
    print(f"  VALU in the exp statement: {len(exp)}")
    print("VALU listing:")
    for s in units["valu"]:
        print("   ", s)


if __name__ == "__main__":
    main()
