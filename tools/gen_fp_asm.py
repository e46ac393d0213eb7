"""Generate lodestar_amd/csrc/fp_asm.h: gfx950 inline-asm modular additions
and subtractions on 12 x 32-bit limbs with interleaved carry chains.

Why: a 12-limb carry chain compiled from __builtin_addc/subc runs every step
through VCC, and gfx950 wants 2 wait states between a VALU write of a carry
SGPR and the next v_addc/v_subb/v_cndmask reading it, so hipcc pads each step
with `s_nop 1` (k_miller: ~8% of its issue slots are s_nop).  Here each chain
has its own SGPR-pair carry and the chains of independent operations are
interleaved by a small list scheduler that emits `s_nop 0` only where no
instruction is ready, so two independent modular operations (an Fp2 add, the
two components of an Fp2 subtraction, ...) take ~73 slots instead of ~160.

Operations (each r = a OP b mod p, inputs reduced, output reduced):
  ADD : s = a + b (chain X), t = s - p (chain Y), r = borrow(Y) ? s : t
  SUB : t = a - b (chain X), u = t + p (chain Y), r = borrow(X) ? u : t
  LAZY: s = a + b (chain X only; product inputs < 2p, fp.h fp_add_lazy)
p's limbs come in as VGPR operands (carry-in forms take no literal and only one
SGPR on gfx950); hipcc keeps them in registers across a kernel.

    python tools/gen_fp_asm.py   (rewrites lodestar_amd/csrc/fp_asm.h)
"""
import itertools
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "lodestar_amd", "csrc", "fp_asm.h")
NL = 12
SGPR_GAP = 2  # wait states between a VALU carry write and its VALU reader


def schedule(chains):
    """chains: list of lists of (text, reads_carry_of, writes_carry, deps)
    where each instruction is a dict {txt, cin (carry id read or None),
    cout (carry id written or None), after (list of (chain, idx) it needs)}.
    Greedy round-robin list scheduling honouring SGPR_GAP on carries and
    plain order on VGPR dependences."""
    pos = {}  # (chain, idx) -> slot
    carry_slot = {}  # carry id -> slot of its last write
    nxt = [0] * len(chains)
    out = []
    slot = 0
    rr = 0
    while any(nxt[c] < len(chains[c]) for c in range(len(chains))):
        picked = None
        for k in range(len(chains)):
            c = (rr + k) % len(chains)
            i = nxt[c]
            if i >= len(chains[c]):
                continue
            ins = chains[c][i]
            if any(d not in pos for d in ins["after"]):
                continue
            if ins["cin"] is not None and slot - carry_slot[ins["cin"]] <= SGPR_GAP:
                continue
            picked = c
            break
        if picked is None:
            out.append("s_nop 0")
        else:
            c = picked
            ins = chains[c][nxt[c]]
            out.append(ins["txt"])
            pos[(c, nxt[c])] = slot
            if ins["cout"] is not None:
                carry_slot[ins["cout"]] = slot
            nxt[c] += 1
            rr = (c + 1) % len(chains)
        slot += 1
    return out


def gen(ops):
    """ops: tuple of 'add' / 'sub' / 'lazy', one per independent operation.
    Operand numbering: outputs r_k[12] (k = 0..), temps t_k[12] (add/sub),
    carries X_k, Y_k; inputs a_k[12], b_k[12], then p[12] if any reduction."""
    n = len(ops)
    red = [o != "lazy" for o in ops]
    idx = 0
    R, T, CX, CY = {}, {}, {}, {}
    for k in range(n):
        R[k] = list(range(idx, idx + NL)); idx += NL
    for k in range(n):
        if red[k]:
            T[k] = list(range(idx, idx + NL)); idx += NL
    for k in range(n):
        CX[k] = idx; idx += 1
        if red[k]:
            CY[k] = idx; idx += 1
    n_out = idx
    A, B = {}, {}
    for k in range(n):
        A[k] = list(range(idx, idx + NL)); idx += NL
        B[k] = list(range(idx, idx + NL)); idx += NL
    P = list(range(idx, idx + NL)) if any(red) else None
    n_in = idx - n_out

    chains = []
    for k, op in enumerate(ops):
        x = []
        for i in range(NL):
            a, b, r, c = f"%{A[k][i]}", f"%{B[k][i]}", f"%{R[k][i]}", f"%{CX[k]}"
            if op in ("add", "lazy"):
                txt = f"v_add_co_u32_e64 {r}, {c}, {a}, {b}" if i == 0 else f"v_addc_co_u32_e64 {r}, {c}, {a}, {b}, {c}"
            else:
                txt = f"v_sub_co_u32_e64 {r}, {c}, {a}, {b}" if i == 0 else f"v_subb_co_u32_e64 {r}, {c}, {a}, {b}, {c}"
            x.append({"txt": txt, "cin": None if i == 0 else ("X", k), "cout": ("X", k), "after": []})
        cx = len(chains)
        chains.append(x)
        if not red[k]:
            continue
        y = []
        for i in range(NL):
            s, p, t, c = f"%{R[k][i]}", f"%{P[i]}", f"%{T[k][i]}", f"%{CY[k]}"
            if op == "add":
                txt = f"v_sub_co_u32_e64 {t}, {c}, {s}, {p}" if i == 0 else f"v_subb_co_u32_e64 {t}, {c}, {s}, {p}, {c}"
            else:
                txt = f"v_add_co_u32_e64 {t}, {c}, {s}, {p}" if i == 0 else f"v_addc_co_u32_e64 {t}, {c}, {s}, {p}, {c}"
            y.append({"txt": txt, "cin": None if i == 0 else ("Y", k), "cout": ("Y", k), "after": [(cx, i)]})
        cy = len(chains)
        chains.append(y)
        # final select: add keeps s (in r) when s - p borrowed; sub takes t + p (in tmp) when a - b borrowed
        sel = []
        for i in range(NL):
            r, t = f"%{R[k][i]}", f"%{T[k][i]}"
            if op == "add":
                sel.append({"txt": f"v_cndmask_b32_e64 {r}, {t}, {r}, %{CY[k]}", "cin": ("Y", k), "cout": None,
                            "after": [(cy, NL - 1)]})
            else:
                sel.append({"txt": f"v_cndmask_b32_e64 {r}, {r}, {t}, %{CX[k]}", "cin": ("X", k), "cout": None,
                            "after": [(cy, NL - 1)]})
        chains.append(sel)
    lines = schedule(chains)
    # a select reads r (written by the chain) and overwrites it: chains read r
    # before it (the Y chain of the same op is complete by construction)
    return lines, n_out, n_in, R, T, CX, CY, A, B, P


def emit(name, ops, args_doc):
    lines, n_out, n_in, R, T, CX, CY, A, B, P = gen(ops)
    n = len(ops)
    red = [o != "lazy" for o in ops]
    outs, ins = [], []
    for k in range(n):
        outs += [f'"=&v"(r{k}.l[{i}])' for i in range(NL)]
    for k in range(n):
        if red[k]:
            outs += [f'"=&v"(t{k}[{i}])' for i in range(NL)]
    for k in range(n):
        outs.append(f'"=&s"(cx{k})')
        if red[k]:
            outs.append(f'"=&s"(cy{k})')
    for k in range(n):
        ins += [f'"v"(a{k}.l[{i}])' for i in range(NL)]
        ins += [f'"v"(b{k}.l[{i}])' for i in range(NL)]
    if P is not None:
        ins += [f'"v"(P_MOD.l[{i}])' for i in range(NL)]
    params = ", ".join(f"fp_t& r{k}, const fp_t& a{k}, const fp_t& b{k}" for k in range(n))
    body = []
    body.append(f"// {args_doc}: {len(lines)} issue slots ({sum(1 for l in lines if l.startswith('s_nop'))} s_nop)")
    body.append(f"__device__ __forceinline__ void {name}({params}) {{")
    for k in range(n):
        if red[k]:
            body.append(f"  uint32_t t{k}[{NL}];")
    body.append("  uint64_t " + ", ".join(
        [f"cx{k}" for k in range(n)] + [f"cy{k}" for k in range(n) if red[k]]) + ";")
    asm = "\\n\\t".join(lines)
    body.append(f'  asm("{asm}"')
    body.append("      : " + ", ".join(outs))
    body.append("      : " + ", ".join(ins) + ");")
    body.append("}")
    return "\n".join(body)


HEADER = """// GENERATED by tools/gen_fp_asm.py -- do not edit.
// gfx950 inline-asm modular add/sub on 12 x 32-bit limbs with interleaved,
// SGPR-carried chains (see the generator's docstring for the scheme and the
// wait-state rule it schedules for).  Device only; fp.h keeps the portable
// forms for the host build and for BGV_ASM_ADD=0.
#pragma once
#if defined(__HIP_DEVICE_COMPILE__)
namespace bgv {
"""


def main():
    parts = [HEADER]
    names = {"add": "add", "sub": "sub", "lazy": "addnr"}
    for ops in [("add",), ("sub",), ("add", "add"), ("sub", "sub"), ("add", "sub"), ("lazy", "lazy"),
                ("lazy", "sub"), ("add", "add", "add"), ("sub", "sub", "sub")]:
        name = "fpa_" + "_".join(names[o] for o in ops)
        doc = "; ".join(f"r{k} = a{k} {'+' if o != 'sub' else '-'} b{k}{'' if o == 'lazy' else ' mod p'}"
                        for k, o in enumerate(ops))
        parts.append(emit(name, ops, doc))
        parts.append("")
    parts.append("}  // namespace bgv\n#endif")
    open(OUT, "w").write("\n".join(parts) + "\n")
    print(OUT)


if __name__ == "__main__":
    main()
