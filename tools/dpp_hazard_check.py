"""DPP read-after-VALU-write hazard check on compiled gfx950 assembly (development tool).

gfx9 needs 2 wait states between a VALU write of a VGPR and a DPP instruction reading that
VGPR as its DPP source (src0); the hardware does not interlock.  For every DPP instruction in
the given .s file, the two preceding instructions (s_nop N counts as N + 1 wait states; labels
and branches end the window conservatively) must not be VALU writes of that register.
usage: python tools/dpp_hazard_check.py <file.s> [function-name-substring]"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] if len(sys.argv) > 2 else ""
inside = not want
bad = 0
window = []  # (wait states, set of VGPRs written) of the last instructions


def regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


for ln, line in enumerate(src, 1):
    t = line.strip()
    if re.match(r"^[_A-Za-z0-9.$]+:", t):
        if want:
            inside = want in t and not t.startswith(".L") or (inside and t.startswith(".L"))
        window.clear()  # a branch target: be conservative, assume anything came before
        window.append((0, {"any"}))
        continue
    if not inside or not t or t.startswith((";", ".", "//")):
        continue
    op, *rest = t.split(None, 1)
    # operands end where the DPP/SDWA modifiers start (" quad_perm:[1,2,3,0] row_mask:..."):
    # cut them off first, or the last operand keeps the modifier text and matches no register
    body = re.split(r"\s+(?:quad_perm|row_|bank_mask|bound_ctrl|wave_|dst_sel|src0_sel|"
                    r"src1_sel|dst_unused|fi:|offset|sc0|sc1|nt\b)", rest[0])[0] if rest else ""
    args = [a.strip() for a in body.split(",")] if body else []
    if op == "s_nop":
        window.append((int(args[0], 0) + 1, set()))
        continue
    if "_dpp" in op or "quad_perm" in t or "row_" in t:
        # src0 is the DPP source: for VOP2/VOPC forms with vcc, the first VGPR operand after dst(s)
        srcs = [a for a in args[1:] if re.match(r"v(\d+|\[)", a)]
        if op.startswith(("v_add_co_u32", "v_addc_co_u32")):
            srcs = [a for a in args[2:] if re.match(r"v(\d+|\[)", a)]
        dpp_src = regs(srcs[0]) if srcs else set()
        states = 0
        for ws, wr in reversed(window):
            if states >= 2:
                break
            if "any" in wr or wr & dpp_src:
                print(f"{sys.argv[1]}:{ln}: DPP source {srcs[0] if srcs else '?'} written "
                      f"{states} wait state(s) before: {t}")
                bad += 1
                break
            states += max(ws, 1)
    written = regs(args[0]) if op.startswith("v_") and args else set()
    window.append((0, written))
    window = window[-4:]
print("dpp hazards:", bad)
sys.exit(1 if bad else 0)
