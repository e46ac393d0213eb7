"""Static checks of the generated inline asm (lodestar_amd/csrc/fp_asm.h,
tools/gen_fp_asm.py): the header is what the generator writes today, and in
every block each carry SGPR pair read by a VALU instruction (the carry-in of
v_addc/v_subb, the mask of v_cndmask) was written at least 3 slots earlier
(gfx950: 2 wait states between a VALU SGPR write and a VALU read of it; the
hardware does not interlock this hazard, so a violation is a silent wrong
carry).  Also: every carry read has a write before it in the same block, and
no VGPR result is read before it is written."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "lodestar_amd", "csrc", "fp_asm.h")
GEN = os.path.join(ROOT, "tools", "gen_fp_asm.py")


def blocks():
    src = open(HDR).read()
    for m in re.finditer(r'asm\("(.*?)"\s*:\s*(.*?)\s*:\s*(.*?)\);', src, re.S):
        lines = m.group(1).split("\\n\\t")
        outs = [o.strip() for o in m.group(2).replace("\n", " ").split(",") if o.strip()]
        yield lines, outs


def test_header_matches_generator(tmp_path):
    out = tmp_path / "fp_asm.h"
    code = open(GEN).read().replace('OUT = os.path.join(ROOT, "lodestar_amd", "csrc", "fp_asm.h")', f'OUT = {str(out)!r}')
    script = tmp_path / "gen.py"
    script.write_text(code)
    subprocess.check_call([sys.executable, str(script)], cwd=ROOT, stdout=subprocess.DEVNULL)
    assert out.read_text() == open(HDR).read(), "fp_asm.h is stale: run python tools/gen_fp_asm.py"


def test_carry_wait_states_and_order():
    n_blocks = 0
    for lines, outs in blocks():
        n_blocks += 1
        sgpr_ops = {i for i, o in enumerate(outs) if o.startswith('"=&s"')}
        vgpr_outs = {i for i, o in enumerate(outs) if o.startswith('"=&v"')}
        written_at = {}
        vwritten = set()
        for slot, ins in enumerate(lines):
            if ins.startswith("s_nop"):
                continue
            op, args = ins.split(None, 1)
            ops = [int(a.strip()[1:]) for a in args.split(",")]
            if op == "v_cndmask_b32_e64":
                dst, reads_v, reads_s, writes_s = ops[0], ops[1:3], [ops[3]], []
            elif op.endswith("_co_u32_e64") and op.split("_")[1] in ("add", "sub"):
                dst, reads_v, reads_s, writes_s = ops[0], ops[2:4], [], [ops[1]]
            else:  # v_addc / v_subb: dst, carry-out, a, b, carry-in
                dst, reads_v, reads_s, writes_s = ops[0], ops[2:4], [ops[4]], [ops[1]]
            for r in reads_s:
                assert r in sgpr_ops, (ins, "carry operand is not an SGPR output")
                assert r in written_at, (ins, "carry read before any write")
                assert slot - written_at[r] >= 3, (ins, f"only {slot - written_at[r] - 1} wait states")
            for r in reads_v:
                if r in vgpr_outs:
                    assert r in vwritten, (ins, "result register read before it is written")
            for w in writes_s:
                written_at[w] = slot
            vwritten.add(dst)
    assert n_blocks >= 9
